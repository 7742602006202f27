#!/bin/bash
# r02o: 32-KiB tail tiles (pipes 49/50) vs 38 on cfg4/cfg5; cfg2 lane default A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep45 400 python bench.py --sweep cfg4,cfg5,cfg3 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,49;0,0,0,50;0,0,0,46;0,0,0,146;0,0,0,246;0,0,0,446;0,0,0,646;8,2,2,0' || exit $?
step sweep2 300 python bench.py --sweep cfg2 --sweep-counts --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12,4;1,4,1,14,2;1,4,1,12,5;1,4,1,14,3' || exit $?
echo ALLDONE
