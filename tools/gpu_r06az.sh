#!/bin/bash
# round 6: the cfg2 bench line with pipe 25 (two tiles a grid stride apart)
# against pipe 19 (adjacent tiles), alternating processes, RX_DIAG build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06az}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
Q="--workload cfg2 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
R=$OUT/ab25_$TAG.txt; : > $R
for k in 1 2 3; do
  for v in 19 25; do
    timeout -k 10 200 python bench.py $Q --variant 1,4,1,$v > $OUT/ab25_${v}_$k.log 2>&1 || { tail -5 $OUT/ab25_${v}_$k.log; exit 1; }
    echo "pipe $v round $k: $(grep '^{' $OUT/ab25_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["kernel"]["median_ms"], d["digest_ok"], d["counts_match"], d["parity"])')" >> $R
    tail -1 $R
  done
done
echo ALLDONE
