#!/bin/bash
# round 6: cfg3 pipe 48 with the remaining passes of both frames loaded
# together (RX_DIAG pipes 54 / 55 / 56: RI 2 / 4 / 10) — parity, then an
# interleaved cfg3 sweep with counts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ao}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "group_write_batched or every_kernel_variant" > $OUT/ri_tests_$TAG.log 2>&1 || { tail -30 $OUT/ri_tests_$TAG.log; exit 1; }
tail -1 $OUT/ri_tests_$TAG.log
timeout -k 10 300 python bench.py --sweep cfg3 --sweep-variants "8,2,2,48;8,2,2,54;8,2,2,55;8,2,2,56" --sweep-counts \
    > $OUT/sweep_ri_$TAG.log 2>&1 || { tail -5 $OUT/sweep_ri_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_ri_$TAG.log | tail -4
echo ALLDONE
