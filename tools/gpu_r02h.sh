#!/bin/bash
# r02h: lane kernel pipe 14 (software-pipelined staged loads) vs pipe 12 on
# cfg2; stream kernel without the scratch spill (cfg4/cfg5); parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 12 "$OUT/$name.log"; return $rc; }
step pytest_gpu 480 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep2 300 python bench.py --sweep cfg2 --sweep-counts --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12;1,4,1,14;1,4,1,14,3;1,4,1,14,2' || exit $?
step sweep45 300 python bench.py --sweep cfg4,cfg5 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,39;0,0,0,34' || exit $?
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu || exit $?
echo ALLDONE
