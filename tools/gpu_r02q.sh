#!/bin/bash
# r02q: pipelined resident stream kernel (52/53: next tile's heads prefetched) vs 38
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep45 400 python bench.py --sweep cfg4,cfg5 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,52;0,0,0,53;0,0,0,52,3;0,0,0,42' || exit $?
echo ALLDONE
