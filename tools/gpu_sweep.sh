#!/bin/bash
# Interleaved variant sweep on the GPU box (tuning; parity first).
#   WL=cfg4,cfg5 V='0,0,0,38;0,0,0,54' [COUNTS=1] [STEPS=10] [SQ=cfg4] bash tools/gpu_sweep.sh
# V: ';'-separated g,p,fpg,pipe[,blocks_per_cu] (see rxgpu.KERNEL_VARIANTS and
# the diagnostic pipes >= 100 in csrc/rx_classify.hip).  SQ: also collect SQ
# instruction counters of the default kernel on that workload.  Each GPU step
# has its own time limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 40 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
C=""; [ "${COUNTS:-1}" = 1 ] && C="--sweep-counts"
step sweep 600 python bench.py --sweep "${WL:-cfg4}" $C --steps "${STEPS:-10}" --warmup 3 \
    --sweep-variants "${V:-}" || exit $?
if [ -n "${SQ:-}" ]; then
  export TMPDIR=/tmp
  step sq 300 python tools/pmc_counters.py sq "$SQ" "--no-tx --no-cfg1" \
      "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" || exit $?
fi
echo ALLDONE
