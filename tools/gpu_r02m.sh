#!/bin/bash
# r02m: lane pipes x blocks/CU on cfg2 after the LDS port window; SQ counters
# of the cfg4 default (stream kernel pipe 38)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step sweep2 300 python bench.py --sweep cfg2 --sweep-counts --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12,3;1,4,1,12,4;1,4,1,12,5;1,4,1,12,6;1,4,1,14,2;1,4,1,14,3;1,4,1,15,2' || exit $?
step sweep1 300 python bench.py --sweep cfg1 --steps 20 --warmup 5 \
    --sweep-variants '1,4,1,12,4;1,4,1,14,3' || exit $?
export TMPDIR=/tmp
step sq4 300 python tools/pmc_counters.py sq cfg4 "--no-tx --no-cfg1" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" \
    "SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" || exit $?
echo ALLDONE
