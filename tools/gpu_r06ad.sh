#!/bin/bash
# round 6: pipes 18 / 19 (two adjacent tiles per trip, the byte-pattern
# ceiling's shape) — lane parity on the RX_DIAG build, then an interleaved
# cfg2 sweep against pipes 14 / 16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ad}
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
    -k "lane or udp_port_window or variant" > $OUT/lane18_tests_$TAG.log 2>&1 || { tail -30 $OUT/lane18_tests_$TAG.log; exit 1; }
tail -1 $OUT/lane18_tests_$TAG.log
timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,14;1,4,1,16;1,4,1,18;1,4,1,19;1,4,1,18,3" --sweep-counts \
    > $OUT/sweep_l18_$TAG.log 2>&1 || { tail -5 $OUT/sweep_l18_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_l18_$TAG.log | tail -5
echo ALLDONE
