#!/bin/bash
# cfg4 (IMIX) session: parity tests, variant sweep, rocprof kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out
timeout -k 10 480 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload cfg4 --no-cpu --sweep "${WL:-cfg4}" --steps 10 --warmup 3 ${SWARGS:-} \
  --sweep-variants "${VARS:-0,0,0,20;8,2,1,1;8,2,2,0;4,1,2,0;16,2,2,0;1,4,1,5;8,2,1,0}" \
  > gpurun_out/sw4.log 2>&1 || exit $?
grep sweep gpurun_out/sw4.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/p4 -o run \
  -- python3 $R/bench.py --workload ${PWL:-cfg4} --no-cpu --steps 10 --warmup 3 > $R/gpurun_out/p4.log 2>&1 || exit $?
python3 -c "import csv
for r in csv.DictReader(open('$R/gpurun_out/p4/run_kernel_stats.csv')): print(r['Name'][:90], r['Calls'], float(r['AverageNs'])/1e3)"
