#!/bin/bash
# r02z: branch-free group kernel (pipes 4/5) on cfg3; parity first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep3 500 python bench.py --sweep cfg3 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '8,2,2,0;8,2,2,4;8,2,2,5;8,2,1,4;8,2,1,5;8,2,2,4,6;8,2,1,4,8;8,2,1,5,6' || exit $?
echo ALLDONE
