#!/bin/bash
# round 6: pipe 16 (pipe 14 + the straight-line lane verdict) — lane parity
# tests, an interleaved cfg2 sweep against pipe 14 (with and without counts),
# and the SQ counters of both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ab}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "lane or udp_port_window or variant" > $OUT/lane16_tests_$TAG.log 2>&1 || { tail -30 $OUT/lane16_tests_$TAG.log; exit 1; }
tail -1 $OUT/lane16_tests_$TAG.log
for c in "" "--sweep-counts"; do
  timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,14;1,4,1,16" $c > $OUT/sweep_l16${c}_$TAG.log 2>&1 || { tail -5 $OUT/sweep_l16${c}_$TAG.log; exit 1; }
  grep "sweep cfg" $OUT/sweep_l16${c}_$TAG.log | tail -2
done
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $P1 --kernel-include-regex lane_kernel -d $OUT/pmc_sq_$TAG -o run \
    -- python3 bench.py --sweep cfg2 --sweep-variants "1,4,1,14;1,4,1,16" --steps 4 --warmup 1 > $OUT/pmc_sq_$TAG.log 2>&1 || { tail -5 $OUT/pmc_sq_$TAG.log; exit 1; }
echo ALLDONE
