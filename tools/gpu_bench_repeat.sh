#!/bin/bash
# the bench line three times in separate processes (per-process spread), cfg2 + cfg4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --workload cfg2,cfg4 --no-cpu --no-cfg1 --no-tx --steps 20 > gpurun_out/b_c2_$i.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/b_c2_$i.log'):
    if l.startswith('{'): d=json.loads(l); print('cfg2', d['ms_per_step'], d['value'], 'cfg4', d['cfg4']['ms_per_step'], d['cfg4']['count_stream'])
"
done
echo ALLDONE
