#!/bin/bash
# the stream kernel with fewer frames per block on cfg3 and cfg4, against their defaults;
# GPU parity of the count paths (the jumbo default now 32 frames per block)
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|Error" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step pytest_cnt 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_digest.py -k "count_paths or layouts or whole_burst" || exit $?
step sweep_fpb_cfg3 400 python -u bench.py --sweep cfg3 --sweep-counts --steps 20 --warmup 3 --sweep-variants "8,2,2,40;0,0,0,38;0,0,0,338;0,0,0,538;0,0,0,738" || exit $?
step sweep_fpb_cfg4 400 python -u bench.py --sweep cfg4 --sweep-counts --steps 20 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,538;0,0,0,738" || exit $?
