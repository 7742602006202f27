#!/bin/bash
# round 6: cfg4 slab geometry A/B (rxg_tune_tables RXG_TT_SLAB_HALF = 8,
# RXG_TT_SLAB_QUARTER = 16 against the default 256 slab blocks), alternating
# bench processes, then a kernel trace of each to see what overlaps what
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread -k "slab_geometry or count_slab_bin or count_idx16" > $OUT/pytest_slab_$TAG.txt 2>&1
rc=$?; tail -2 $OUT/pytest_slab_$TAG.txt; [ $rc -eq 0 ] || exit $rc
Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
for k in 1 2; do
  for tt in 0 8 16; do
    timeout -k 10 200 python bench.py $Q --tune-tables $tt > $OUT/slab${tt}_$k.log 2>&1 || exit $?
    echo "tt=$tt round $k: $(grep '^{' $OUT/slab${tt}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["kernel"], d["counts_match"], d["digest_ok"], "cfg5", d["cfg5"]["ms_per_step"], d["cfg5"].get("kernel_median_ms"), d["cfg5"]["counts_match"])')"
  done
done | tee $OUT/slab_ab_$TAG.txt
export TMPDIR=/tmp
for tt in 0 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_slab${tt}_$TAG -o run \
      -- python3 bench.py $Q --tune-tables $tt --steps 20 > $OUT/slabprof${tt}.log 2>&1 || exit $?
done
echo ALLDONE
