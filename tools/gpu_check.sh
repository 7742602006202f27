#!/bin/bash
# GPU check after a change: the named tests first (K), then the whole -m gpu
# suite, smoke, an optional A/B script (AB) and a short bench line.  Each GPU
# step has its own time limit; a failing step ends the script.
#   K='churn or digest' AB='tools/ab_track.py cfg2,cfg4' bash tools/gpu_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; date +%T; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"; return $rc; }
if [ -n "${K:-}" ]; then
  step pytest_k 420 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" || exit $?
fi
if [ "${FULL:-1}" = 1 ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread || exit $?
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ -n "${AB:-}" ]; then
  step ab 400 python $AB || exit $?
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench 500 python bench.py ${BENCH_ARGS:-} || exit $?
  grep '^{' $OUT/bench.log > $OUT/bench_line.json || true
fi
echo ALLDONE
