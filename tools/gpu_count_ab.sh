#!/bin/bash
# Count-path check: parity of the count tests, then kernel traces of cfg4 and
# cfg5 (classify with and without counts, slab and reduce dispatch durations)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "count or stream or generated or fuzzed or layouts" > $OUT/pytest_q.log 2>&1; rc=$?; tail -2 $OUT/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for wl in ${WLS:-cfg4 cfg5}; do
  WL=$wl ARGS="--no-count-stream ${ARGS:-}" bash tools/gpu_trace_wl.sh > /dev/null || exit 1
  echo "== $wl"; sed -n '1,3p;$p' $OUT/trace_$wl.txt; tail -3 $OUT/trace_$wl.txt
done
echo ALLDONE
