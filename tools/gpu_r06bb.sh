#!/bin/bash
# round 6: the 8-B verdict leg (rxg_classify_dev8) with pipe 14 against pipe
# 19, alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06bb}
Q="--workload cfg2 --no-cpu --no-sockrate --no-cfg1 --no-tx"
R=$OUT/abv8b_$TAG.txt; : > $R
for k in 1 2; do
  for v in 16 25; do
    timeout -k 10 200 python bench.py $Q --variant 1,4,1,$v > $OUT/abv8b_${v}_$k.log 2>&1 || { tail -5 $OUT/abv8b_${v}_$k.log; exit 1; }
    echo "pipe $v round $k: $(grep '^{' $OUT/abv8b_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("v16", d["ms_per_step"], d["roofline"]["frac"], "v8", d["verdict8"])')" >> $R
    tail -1 $R
  done
done
echo ALLDONE
