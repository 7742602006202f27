#!/bin/bash
# round 6: the write-batched G=8 kernels (pipes 41/42) — parity, then an
# interleaved cfg3 sweep against pipe 40 (two passes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread -k "write_batched or every_kernel_variant or generated_bursts" > $OUT/pytest_wb_$TAG.txt 2>&1
rc=$?; tail -3 $OUT/pytest_wb_$TAG.txt; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
for k in 1 2; do
  timeout -k 10 300 python bench.py --sweep cfg3 --steps 20 --warmup 3 --sweep-counts \
      --sweep-variants "8,2,2,40;8,2,2,41;8,2,2,42;8,2,2,40;8,2,2,41;8,2,2,42" > $OUT/sweep_wb${k}_$TAG.log 2>&1 || exit $?
  grep sweep $OUT/sweep_wb${k}_$TAG.log
done
echo ALLDONE
