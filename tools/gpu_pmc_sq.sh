#!/bin/bash
# SQ occupancy/wait counters of the default classify kernel per workload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${PMC_WL:-cfg4 cfg3 cfg2}; do
  timeout -k 10 300 python tools/pmc_counters.py sq $wl "--no-tx" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
    >> gpurun_out/pmc_sq.log 2>&1 || exit $?
done
echo ALLDONE
