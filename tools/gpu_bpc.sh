#!/bin/bash
# resident blocks per CU for the cfg3 group kernel (grid-stride tail: 52 trips
# for 51.2 of work at 5 per CU, 64 even trips at 4) and the jumbo stream kernel
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|Error" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step sweep_bpc_cfg3 400 python -u bench.py --sweep cfg3 --sweep-counts --steps 20 --warmup 3 --sweep-variants "8,2,2,40,0;8,2,2,40,4;8,2,2,40,3;8,2,2,40,2" || exit $?
step sweep_bpc_cfg5 400 python -u bench.py --sweep cfg5 --sweep-counts --steps 20 --warmup 3 --sweep-variants "0,0,0,938,0;0,0,0,938,4;0,0,0,938,3" || exit $?
