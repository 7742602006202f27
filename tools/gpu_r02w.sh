#!/bin/bash
# r02w: cfg3 group-kernel shapes x blocks/CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 40 "$OUT/$name.log"; return $rc; }
step sweep3 500 python bench.py --sweep cfg3 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '8,2,2,0;8,2,2,0,4;8,2,2,0,6;8,2,2,0,8;8,2,2,15;8,2,2,14;8,4,2,18;8,4,1,18;16,2,2,14;16,2,2,18;8,2,2,26;8,2,2,28;8,2,1,0;4,1,2,0' || exit $?
echo ALLDONE
