#!/bin/bash
# jumbo stream kernel: 16 frames per block (938) and the probe consumed before
# the stream at 32 (739) against the default 738; parity of every variant and
# the count paths first
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|Error" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step pytest_fpb3 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_digest.py -k "every_kernel or count_paths or whole_burst" || exit $?
step sweep_fpb3_cfg5 400 python -u bench.py --sweep cfg5 --sweep-counts --steps 20 --warmup 3 --sweep-variants "0,0,0,738;0,0,0,938;0,0,0,1138;0,0,0,738;0,0,0,938;0,0,0,1138" || exit $?
