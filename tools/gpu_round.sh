#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout (anything but 0/1 from
# pytest, anything but 0 elsewhere) ends the script there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
STEPS=${STEPS:-20}

step() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" ; date +%T
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "$OUT/$name.log"
  return $rc
}

step pytest_gpu 420 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${AB:-}" ]; then
  step ab 400 python tools/ab_tables.py "$AB" ${AB_ROUNDS:-5} || exit $?
fi
if [ -n "${SWEEP:-}" ]; then
  step sweep 300 python bench.py --sweep "$SWEEP" --steps 10 --warmup 3 || exit $?
fi
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 300 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log > $OUT/bench_$TAG.json || true
if [ "${PROF:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
      -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu || exit $?
fi
if [ "${TXPMC:-0}" = 1 ]; then
  step pmc_tx 400 python tools/pmc_tx.py $TAG || exit $?
fi
if [ "${PMC:-0}" = 1 ]; then
  step pmc 600 python tools/pmc_traffic.py $TAG ${PMC_WL:-cfg2,cfg3} || exit $?
fi
echo ALLDONE
