#!/bin/bash
# round 6: six count-index buffers in the count-stream ring (RXG_TT_COUNT_6BUF)
# against the default three, alternating processes; the slab-geometry parity
# test first, a kernel trace of the six-buffer case last
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06v}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "count_slab_geometry" > $OUT/slabgeo_$TAG.log 2>&1 || { tail -20 $OUT/slabgeo_$TAG.log; exit 1; }
tail -1 $OUT/slabgeo_$TAG.log
Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
R=$OUT/ring_ab_$TAG.txt; : > $R
for k in 1 2 3; do
  for tt in 0 32; do
    timeout -k 10 200 python bench.py $Q --tune-tables $tt > $OUT/ring${tt}_$k.log 2>&1 || { tail -5 $OUT/ring${tt}_$k.log; exit 1; }
    echo "tune_tables=$tt round $k: $(grep '^{' $OUT/ring${tt}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cfg4", d["ms_per_step"], d["roofline"]["kernel"]["median_ms"], d["counts_match"], d["digest_ok"], "cfg5", d["cfg5"]["ms_per_step"], d["cfg5"].get("kernel_median_ms"), d["cfg5"]["counts_match"], d["cfg5"]["digest_ok"])')" >> $R
    tail -1 $R
  done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_ring_$TAG -o run \
    -- python3 bench.py $Q --tune-tables 32 --steps 20 > $OUT/ringprof.log 2>&1 || exit 1
echo ALLDONE
