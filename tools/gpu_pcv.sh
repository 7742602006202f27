#!/bin/bash
# cfg4: what the SH kernel's block-start partial-chunk load costs (pipe 264 =
# pipe 64 without it, wrong verdicts by construction): interleaved sweep with
# and without counts, and the L2 request / hit / miss difference
set -u
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|probe_hit_rate|^probe|^no_probe" "$OUT/$name.log" | cut -c1-400; return $rc; }
step membw 120 tools/membw_cfg2 || exit $?
grep "RDW   U=2 bpc=2" $OUT/membw.log
step sweep_pcv 400 python -u bench.py --sweep cfg4 --steps 30 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,264;0,0,0,160" || exit $?
step sweep_pcv_counts 400 python -u bench.py --sweep cfg4 --sweep-counts --steps 30 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,264" || exit $?
step pmc_pcv 400 python tools/pmc_probe_hits.py cfg4 r03e 264 || exit $?
