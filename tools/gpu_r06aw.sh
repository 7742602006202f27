#!/bin/bash
# round 6: SQ counters and the effective shader clock (GRBM_GUI_ACTIVE / 8 /
# kernel time, MI355X_MICROARCH.md) of the cfg4 SH kernel and the cfg2 lane
# kernel on this box, to explain the per-box spread of cfg4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06aw}
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
k=1
for P in "$P1" "$P2"; do
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "sh_kernel|lane_kernel" -d $OUT/pmc_clk_${TAG}_$k -o run \
      -- python3 bench.py --sweep cfg4,cfg2 --sweep-variants "0,0,0,67;1,4,1,19" --steps 4 --warmup 1 > $OUT/pmc_clk_${TAG}_$k.log 2>&1 || { tail -5 $OUT/pmc_clk_${TAG}_$k.log; exit 1; }
  k=$((k+1))
done
echo ALLDONE
