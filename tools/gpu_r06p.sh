#!/bin/bash
# round 6: the count stream at high priority (the slab pass of burst k ahead
# of burst k+1's classify blocks) against the default, alternating processes,
# then a kernel trace of the high-priority case
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06p}
Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
for k in 1 2 3; do
  for pr in 0 -1; do
    timeout -k 10 200 python bench.py $Q --count-stream-priority $pr > $OUT/prio${pr}_$k.log 2>&1 || exit $?
    echo "prio=$pr round $k: $(grep '^{' $OUT/prio${pr}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cfg4", d["ms_per_step"], d["roofline"]["kernel"]["median_ms"], d["counts_match"], d["digest_ok"], "cfg5", d["cfg5"]["ms_per_step"], d["cfg5"].get("kernel_median_ms"), d["cfg5"]["counts_match"], d["cfg5"]["digest_ok"])')"
  done
done | tee $OUT/prio_ab_$TAG.txt
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_prio_$TAG -o run \
    -- python3 bench.py $Q --count-stream-priority -1 --steps 20 > $OUT/prioprof.log 2>&1 || exit $?
echo ALLDONE
