#!/bin/bash
# r02d: NTH stream variants — parity, interleaved sweep on cfg4/cfg5, PMC bytes per variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step sweep 400 python bench.py --sweep cfg4,cfg5 --sweep-variants "0,0,0,38;0,0,0,40;0,0,0,41;0,0,0,30" --steps 10 --warmup 3 || exit $?
step pmc38 300 python tools/pmc_traffic.py r02d_v38 cfg4 0,0,0,38 || exit $?
step pmc40 300 python tools/pmc_traffic.py r02d_v40 cfg4,cfg5 0,0,0,40 || exit $?
step pmc_tx 400 python tools/pmc_tx.py r02d || exit $?
echo ALLDONE
