#!/bin/bash
# round 6: cfg3 at five blocks per CU (RX_DIAG pipes 50-53 against pipe 48),
# interleaved sweeps with and without per-flow counts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06y}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
V="8,2,2,48;8,2,2,50;8,2,2,51;8,2,2,52;8,2,2,53"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
    -k "group_write_batched or hist16_edge" > $OUT/wb5_tests_$TAG.log 2>&1 || { tail -20 $OUT/wb5_tests_$TAG.log; exit 1; }
tail -1 $OUT/wb5_tests_$TAG.log
for c in "" "--sweep-counts"; do
  timeout -k 10 300 python bench.py --sweep cfg3 --sweep-variants "$V" $c > $OUT/sweep_wb5${c}_$TAG.log 2>&1 || { tail -5 $OUT/sweep_wb5${c}_$TAG.log; exit 1; }
  grep "sweep cfg" $OUT/sweep_wb5${c}_$TAG.log | tail -5
done
echo ALLDONE
