#!/bin/bash
# A/B of the count stream (rxg_classify_dev_cs) against counts on the classify
# stream, interleaved bench processes on one box (cfg4, cfg5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload cfg4,cfg5 --no-cpu --no-cfg1 --no-tx --steps 20 > gpurun_out/b_cs$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --workload cfg4,cfg5 --no-cpu --no-cfg1 --no-tx --steps 20 --no-count-stream > gpurun_out/b_sync$i.log 2>&1 || exit 1
done
for f in b_cs1 b_sync1 b_cs2 b_sync2; do
  python3 -c "
import json,sys
for l in open('gpurun_out/$f.log'):
    if l.startswith('cfg'):
        n,j=l.split(' ',1); d=json.loads(j); print('$f', n, d['ms_per_step'], d['count_stream'])
"
done
echo ALLDONE
