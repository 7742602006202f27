#!/bin/bash
# round 6: what the per-flow counts cost the cfg2 lane kernel (pipe 14), and
# where its time goes (RX_DIAG ablations of pipe 0 beside pipe 0 and 14)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
DL=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
V="1,4,1,14;1,4,1,0;1,4,1,101;1,4,1,104;1,4,1,108;1,4,1,113"
RXGPU_LIB=$DL timeout -k 10 300 python bench.py --sweep cfg2 --steps 50 --warmup 5 --sweep-variants "$V" > $OUT/sweep_cnt0_r06r.log 2>&1 || exit $?
RXGPU_LIB=$DL timeout -k 10 300 python bench.py --sweep cfg2 --steps 50 --warmup 5 --sweep-counts --sweep-variants "$V" > $OUT/sweep_cnt1_r06r.log 2>&1 || exit $?
grep -h sweep $OUT/sweep_cnt0_r06r.log $OUT/sweep_cnt1_r06r.log
echo ALLDONE
