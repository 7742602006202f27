#!/bin/bash
# round 6: where the cfg2 lane kernel's time goes (pipe 14 ablations, RX_DIAG)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
DL=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
V="1,4,1,14;1,4,1,1401;1,4,1,1404;1,4,1,1408;1,4,1,1413"
for c in "" "--sweep-counts"; do
  RXGPU_LIB=$DL timeout -k 10 300 python bench.py --sweep cfg2 --steps 50 --warmup 5 $c --sweep-variants "$V" > $OUT/sweep_abl14_r06u.log 2>&1 || exit $?
  grep sweep $OUT/sweep_abl14_r06u.log
done
echo ALLDONE
