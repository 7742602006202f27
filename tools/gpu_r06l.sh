#!/bin/bash
# round 6: the write-batched G=8 kernel with a 16-bit LDS histogram (RX_DIAG
# pipes 47-49) — parity on the diag build (every variant, write-batched
# bursts, the 16-bit bins at their limit), then an interleaved cfg3 sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06l}
DL=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
RXGPU_LIB=$DL timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread -k "write_batched or hist16 or every_kernel_variant" > $OUT/pytest_h16_$TAG.txt 2>&1
rc=$?; tail -3 $OUT/pytest_h16_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for k in 1 2; do
  RXGPU_LIB=$DL timeout -k 10 300 python bench.py --sweep cfg3 --steps 20 --warmup 3 --sweep-counts \
      --sweep-variants "8,2,2,41;8,2,2,47;8,2,2,48;8,2,2,49;8,2,2,40" > $OUT/sweep_h16${k}_$TAG.log 2>&1 || exit $?
  grep sweep $OUT/sweep_h16${k}_$TAG.log
done
echo ALLDONE
