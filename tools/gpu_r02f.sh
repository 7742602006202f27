#!/bin/bash
# r02f: 2-B count indices + slab-grouped reduce — parity, then the count path
# A/B (count4B = round-1 count path) interleaved on cfg4/cfg5, rocprof of the
# count kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest_gpu 480 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ab 400 python tools/ab_tables.py cfg4 7 port+1/4,count4B,countR1,count4B+R1 || exit $?
export TMPDIR=/tmp
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r02f -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-cfg1 --workload cfg4,cfg5 || exit $?
echo ALLDONE
