#!/bin/bash
# r02s: span reduced per wave before the LDS atomics (all stream kernels)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep4nc 300 python bench.py --sweep cfg4 --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,54;0,0,0,56;0,0,0,57;0,0,0,646;0,0,0,446;0,0,0,246' || exit $?
step sweep45 400 python bench.py --sweep cfg4,cfg5 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,54;0,0,0,56;0,0,0,57' || exit $?
echo ALLDONE
