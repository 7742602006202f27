#!/bin/bash
# quick GPU check: the whole -m gpu suite, smoke, and one default bench line
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step bench 420 python bench.py ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log > $OUT/bench_check.json
