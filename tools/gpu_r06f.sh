#!/bin/bash
# round 6: write-batch depth sweep (RX_DIAG build: pipes 41/43-46 vs 40) with
# a parity check of the diag WB variants, the cfg2 time-batched store ceiling,
# and the bench (socket API: pipelined receive with the earlier wait)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06f}
DL=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
RXGPU_LIB=$DL timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread -k "every_kernel_variant" > $OUT/pytest_wbdiag_$TAG.txt 2>&1
rc=$?; tail -2 $OUT/pytest_wbdiag_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  RXGPU_LIB=$DL timeout -k 10 300 python bench.py --sweep cfg3 --steps 20 --warmup 3 --sweep-counts \
      --sweep-variants "8,2,2,40;8,2,2,41;8,2,2,43;8,2,2,44;8,2,2,45;8,2,2,46" > $OUT/sweep_wbd${k}_$TAG.log 2>&1 || exit $?
  grep sweep $OUT/sweep_wbd${k}_$TAG.log
done
timeout -k 10 200 ./tools/membw_cfg2 > $OUT/membw_cfg2_$TAG.txt 2>&1 || exit $?
head -30 $OUT/membw_cfg2_$TAG.txt
BENCH_DETAIL=$OUT/detail_bench_$TAG.json timeout -k 10 400 python bench.py --workload cfg2 --no-cfg1 --no-tx --no-v8 > $OUT/bench_$TAG.log 2>&1 || exit $?
grep '^{' $OUT/bench_$TAG.log > $OUT/bench_$TAG.json
echo ALLDONE
