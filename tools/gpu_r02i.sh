#!/bin/bash
# r02i: lane pipes 12/14/15 x blocks per CU on cfg2 (parity first)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 12 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "staged or every_kernel or cfg2 or smoke"
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep2 300 python bench.py --sweep cfg2 --sweep-counts --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12;1,4,1,14,3;1,4,1,14,4;1,4,1,15,3;1,4,1,15,2' || exit $?
step sweep2nc 300 python bench.py --sweep cfg2 --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12;1,4,1,14,3;1,4,1,14,4;1,4,1,15,3;1,4,1,15,2' || exit $?
echo ALLDONE
