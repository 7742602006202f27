#!/bin/bash
# cfg5: the stream kernel with 256 / 128 / 64 frames per block (pipes 38 / 338 / 538)
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|Error" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step pytest_fpb 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "every_kernel or layouts or generated" || exit $?
step sweep_fpb 400 python -u bench.py --sweep cfg5 --sweep-counts --steps 20 --warmup 3 --sweep-variants "0,0,0,38;0,0,0,338;0,0,0,538;0,0,0,738" || exit $?
