#!/bin/bash
# round 6: the 8-B verdict leg with the lane shapes of the RX_DIAG build
# (pipes 14 / 16 / 19 / 21 / 22), one bench process each, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ak}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
Q="--workload cfg2 --no-cpu --no-sockrate --no-cfg1 --no-tx"
R=$OUT/v8shapes_$TAG.txt; : > $R
for k in 1 2; do
  for v in 14 16 19 21 22; do
    timeout -k 10 200 python bench.py $Q --variant 1,4,1,$v > $OUT/v8s_${v}_$k.log 2>&1 || { tail -5 $OUT/v8s_${v}_$k.log; exit 1; }
    echo "pipe $v round $k: $(grep '^{' $OUT/v8s_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("v16", d["ms_per_step"], d["roofline"]["frac"], "v8", d["verdict8"])')" >> $R
    tail -1 $R
  done
done
echo ALLDONE
