#!/bin/bash
# cfg5 (jumbo, stream kernel pipe 38): what the per-thread head and partial-chunk
# loads at the block start cost (ablations 438 / 838 / 1238, wrong verdicts by
# construction), counts on as in the bench; and the cfg4 counts A/B
set -u
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|median|K1" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step sweep_jumbo 400 python -u bench.py --sweep cfg5 --sweep-counts --steps 20 --warmup 3 --sweep-variants "0,0,0,38;0,0,0,438;0,0,0,838;0,0,0,1238" || exit $?
step ab_counts 400 python -u tools/ab_counts.py cfg4,cfg5 5 30 || exit $?
