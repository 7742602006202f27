#!/bin/bash
# round 6: count passes with every trip's index loads in flight (slab pass:
# prefetch across the bin clearing and the next trip, 16-B slab stores fused
# with the wrap check; reduce: 16 loads in flight) against the round-5 passes
# (RXGPU_LIB=librxgpu_cv1.so), alternating processes; count parity + digests
# first, a kernel trace of the new passes last
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06w}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_churn.py tests/test_digest.py -k "count or digest" \
    > $OUT/counttests_$TAG.log 2>&1 || { tail -30 $OUT/counttests_$TAG.log; exit 1; }
tail -1 $OUT/counttests_$TAG.log
Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
R=$OUT/count_ab_$TAG.txt; : > $R
LIBDIR=$PWD/dpdk-tcp-udp_protocol_stack_amd
for k in 1 2 3; do
  for lib in v1 v2; do
    if [ $lib = v1 ]; then export RXGPU_LIB=$LIBDIR/librxgpu_cv1.so; else unset RXGPU_LIB; fi
    timeout -k 10 200 python bench.py $Q > $OUT/cnt${lib}_$k.log 2>&1 || { tail -5 $OUT/cnt${lib}_$k.log; exit 1; }
    echo "count $lib round $k: $(grep '^{' $OUT/cnt${lib}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cfg4", d["ms_per_step"], d["roofline"]["kernel"]["median_ms"], d["counts_match"], d["digest_ok"], "cfg5", d["cfg5"]["ms_per_step"], d["cfg5"].get("kernel_median_ms"), d["cfg5"]["counts_match"], d["cfg5"]["digest_ok"])')" >> $R
    tail -1 $R
  done
done
unset RXGPU_LIB
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_cnt_$TAG -o run \
    -- python3 bench.py $Q --steps 20 > $OUT/cntprof.log 2>&1 || exit 1
echo ALLDONE
