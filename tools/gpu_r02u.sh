#!/bin/bash
# r02u: stream kernels on cfg3 (1500 B) against the G=8 group kernel
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step sweep3 400 python bench.py --sweep cfg3 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '8,2,2,0;0,0,0,38;0,0,0,54;0,0,0,56;0,0,0,57;0,0,0,39;8,2,2,1;16,2,2,0' || exit $?
export TMPDIR=/tmp
step sq3 300 python tools/pmc_counters.py sq cfg3 "--no-tx --no-cfg1" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" || exit $?
echo ALLDONE
