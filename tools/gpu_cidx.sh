#!/bin/bash
# cfg4: what the SH kernel's count-index store costs (1064: no store; 2064:
# stored before the verdict), counts on and off
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep" "$OUT/$name.log" | cut -c1-300; return $rc; }
step sweep_cidx 400 python -u bench.py --sweep cfg4 --sweep-counts --steps 30 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,1064;0,0,0,2064" || exit $?
step sweep_nocnt 400 python -u bench.py --sweep cfg4 --steps 30 --warmup 3 --sweep-variants "0,0,0,64" || exit $?
