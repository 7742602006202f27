#!/bin/bash
# Round-4 GPU session: parity suite, smoke, the bench line exactly as the
# driver runs it, then rocprofv3 --kernel-trace --stats of the bench on the
# SAME box in the same call, and the table that ties each workload's
# roofline.kernel (per-dispatch HIP events) to the trace
# (tools/roofline_check.py).  Optional: PMC=1 HBM bytes (pmc_traffic, stamped
# with this library's SHA, before the bench so the line carries
# roofline.traffic); N2=1 the N = 2 spawn rehearsal.  Each GPU step has its own
# time limit; a failing step ends the script.
#     TAG=r04a bash tools/gpu_r04.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r04}
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; date +%T; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
if [ "${TESTS:-1}" = 1 ]; then
  # plain test failures (rc 1) still let the bench run; anything else (a
  # timeout, an abort, a fault) ends the session
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  rc=$?; [ $rc -le 1 ] || exit $rc
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
export TMPDIR=/tmp
if [ "${PMC:-0}" = 1 ]; then
  step pmc 900 python tools/pmc_traffic.py $TAG cfg2,cfg3,cfg4,cfg5 || exit $?
  cp $OUT/pmc_$TAG.json profiles/pmc_$TAG.json || exit 1
fi
step bench 420 python bench.py ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log > $OUT/bench_$TAG.json || true
step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 bench.py --no-cpu --no-sockrate --no-v8 --no-cfg1 --no-tx || exit $?
grep '^{' $OUT/rocprof.log > $OUT/bench_profiled_$TAG.json || true
f=$(find $OUT/prof_$TAG -name '*kernel_trace.csv' | head -1)
s=$(find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1)
[ -n "$s" ] && cp "$s" $OUT/kernel_stats_$TAG.csv
if [ -n "$f" ]; then
  python tools/trace_durations.py "$f" > $OUT/trace_durations_$TAG.txt
  python tools/roofline_check.py $OUT/bench_profiled_$TAG.json "$f" $OUT/bench_$TAG.json \
      > $OUT/roofline_check_$TAG.txt 2>&1
  cat $OUT/roofline_check_$TAG.txt
fi
if [ "${N2:-0}" = 1 ]; then
  step n2 400 python bench.py --gpus 2 --steps 5 --warmup 2 || exit $?
  grep '^{' $OUT/n2.log > $OUT/bench_n2_$TAG.json || true
fi
echo ALLDONE
