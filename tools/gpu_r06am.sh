#!/bin/bash
# round 6: pipe 23 (pipe 19 with both tiles' stores at the trip's end) —
# lane parity on the RX_DIAG build, then an interleaved cfg2 sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06am}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "lane_staged or udp_port_window or every_kernel_variant" > $OUT/l23_tests_$TAG.log 2>&1 || { tail -30 $OUT/l23_tests_$TAG.log; exit 1; }
tail -1 $OUT/l23_tests_$TAG.log
timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,19;1,4,1,25;1,4,1,19;1,4,1,25" --sweep-counts \
    > $OUT/sweep_l23_$TAG.log 2>&1 || { tail -5 $OUT/sweep_l23_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_l23_$TAG.log | tail -3
echo ALLDONE
