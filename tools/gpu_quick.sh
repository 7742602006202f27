#!/bin/bash
# Targeted GPU check + interleaved sweep (tuning):
#   K='pytest -k expr' WL=cfg4 V='0,0,0,54;0,0,0,60' [COUNTS=1] bash tools/gpu_quick.sh
# Each GPU step has its own time limit; a failing step ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 25 "$OUT/$name.log"; return $rc; }
if [ -n "${K:-}" ]; then
  step pytest_q 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" || exit $?
fi
if [ -n "${V:-}" ]; then
  C=""; [ "${COUNTS:-1}" = 1 ] && C="--sweep-counts"
  step sweep 600 python bench.py --sweep "${WL:-cfg4}" $C --steps "${STEPS:-10}" --warmup 3 \
      --sweep-variants "$V" || exit $?
fi
echo ALLDONE
