#!/bin/bash
# round 6: pipe 16 at 2 / 3 / 4 blocks per CU, and its no-store ablation
# (RX_DIAG 1604) beside pipe 14's (1404): interleaved cfg2 sweeps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ac}
timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,14;1,4,1,16;1,4,1,16,3;1,4,1,16,4" --sweep-counts \
    > $OUT/sweep_l16bpc_$TAG.log 2>&1 || { tail -5 $OUT/sweep_l16bpc_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_l16bpc_$TAG.log | tail -4
RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so timeout -k 10 300 python bench.py --sweep cfg2 \
    --sweep-variants "1,4,1,14;1,4,1,1404;1,4,1,16;1,4,1,1604" --sweep-counts > $OUT/sweep_l16abl_$TAG.log 2>&1 || { tail -5 $OUT/sweep_l16abl_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_l16abl_$TAG.log | tail -4
echo ALLDONE
