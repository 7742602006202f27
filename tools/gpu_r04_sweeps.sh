#!/bin/bash
# Round-4 tuning session: a -k subset of the GPU tests, interleaved variant
# sweeps on cfg4 and cfg5, and the socket-API part of the bench line.  Each
# GPU step has its own time limit; a failing step ends the script.
#   K='...' V4='0,1,1,64;0,1,1,67' V5='0,1,1,938;0,1,1,2938' bash tools/gpu_r04_sweeps.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h "sweep \|passed\|failed\|error" "$OUT/$name.log" | tail -n 12; return $rc; }
if [ -n "${K:-}" ]; then
  step pytest_q 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$K" || exit $?
fi
if [ -n "${V4:-}" ]; then
  step sweep_cfg4 400 python bench.py --sweep cfg4 --sweep-counts --steps 20 --warmup 3 --sweep-variants "$V4" || exit $?
fi
if [ -n "${V5:-}" ]; then
  step sweep_cfg5 400 python bench.py --sweep cfg5 --sweep-counts --steps 20 --warmup 3 --sweep-variants "$V5" || exit $?
fi
if [ "${SOCK:-1}" = 1 ]; then
  step bench_sock 400 python bench.py --workload cfg2 --steps 5 --no-cpu --no-cfg1 --no-v8 --no-tx || exit $?
  python tools/sock_summary.py $OUT/bench_sock.log
fi
echo ALLDONE
