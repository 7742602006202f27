#!/bin/bash
# A/B of the flow-table load factor (rxg_tune_flow_load) on cfg4, interleaved
# bench processes on one box: --flow-load N = exact-key tables at load <= 2^-N
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for fl in ${FLS:-1 2}; do
    timeout -k 10 200 python bench.py --workload cfg4 --no-cpu --no-cfg1 --no-tx --steps 20 --flow-load $fl > gpurun_out/b_fl${fl}_$i.log 2>&1 || exit 1
    python3 -c "
import json
for l in open('gpurun_out/b_fl${fl}_$i.log'):
    if l.startswith('{'): d=json.loads(l); print('flow_load', $fl, 'rep', $i, 'ms_per_step', d['ms_per_step'], 'kernel_ms', d['kernel_ms_avg'], 'parity', d['parity']['mismatches'])
"
  done
done
echo ALLDONE
