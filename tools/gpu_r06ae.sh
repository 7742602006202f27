#!/bin/bash
# round 6: T tiles per trip (pipes 19 / 21 / 22: T = 2 / 3 / 4) — lane parity
# on the RX_DIAG build, an interleaved cfg2 sweep, then the cfg2 bench line
# with pipe 19 forced against the default pipe 14, alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ae}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "lane or udp_port_window" > $OUT/laneT_tests_$TAG.log 2>&1 || { tail -30 $OUT/laneT_tests_$TAG.log; exit 1; }
tail -1 $OUT/laneT_tests_$TAG.log
timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,14;1,4,1,19;1,4,1,21;1,4,1,22;1,4,1,19,3;1,4,1,19,1" --sweep-counts \
    > $OUT/sweep_lT_$TAG.log 2>&1 || { tail -5 $OUT/sweep_lT_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_lT_$TAG.log | tail -6
Q="--workload cfg2 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
R=$OUT/ab19_$TAG.txt; : > $R
for k in 1 2 3; do
  for v in 14 19; do
    timeout -k 10 200 python bench.py $Q --variant 1,4,1,$v > $OUT/ab19_${v}_$k.log 2>&1 || { tail -5 $OUT/ab19_${v}_$k.log; exit 1; }
    echo "pipe $v round $k: $(grep '^{' $OUT/ab19_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel"]["median_ms"], d["roofline"]["kernel"]["frac"], d["digest_ok"], d["counts_match"], d["parity"])')" >> $R
    tail -1 $R
  done
done
echo ALLDONE
