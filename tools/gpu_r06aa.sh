#!/bin/bash
# round 6: SQ counters of the cfg2 lane kernel (pipe 14) and its no-store /
# no-work ablations (RX_DIAG 1404 / 1413): instructions per wave, and how a
# wave's cycles split between issuing and waiting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06aa}
export TMPDIR=/tmp
export RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so
V="1,4,1,14;1,4,1,1404;1,4,1,1413"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
k=1
for P in "$P1" "$P2"; do
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex lane_kernel -d $OUT/pmc_sq_${TAG}_$k -o run \
      -- python3 bench.py --sweep cfg2 --sweep-variants "$V" --steps 4 --warmup 1 > $OUT/pmc_sq_${TAG}_$k.log 2>&1 || { tail -5 $OUT/pmc_sq_${TAG}_$k.log; exit 1; }
  k=$((k+1))
done
echo ALLDONE
