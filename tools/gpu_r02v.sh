#!/bin/bash
# r02v: pruned tree parity + cfg4 FETCH/WRITE bytes of the default (54) vs
# the no-heads / no-stream ablations (46 base)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 12 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
for v in 0,0,0,54 0,0,0,46 0,0,0,446 0,0,0,246; do
  step pmc_$v 300 python tools/pmc_traffic.py r02v cfg4 $v || exit $?
done
echo ALLDONE
