#!/bin/bash
# r02j: cfg2 no-work ceiling (tools/membw_cfg2), then the new default (pipe 14) bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 40 "$OUT/$name.log"; return $rc; }
step membw_cfg2 120 tools/membw_cfg2 || exit $?
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step bench 300 python bench.py --steps 20 --warmup 5 --no-cpu --workload cfg2 || exit $?
echo ALLDONE
