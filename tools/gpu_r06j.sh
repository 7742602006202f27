#!/bin/bash
# round 6: why cfg4's next classify starts only after the previous burst's
# reduce: the HIP API trace beside the kernel trace (no counters)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/prof_api_r06j -o run \
    -- python3 bench.py --workload cfg4 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8 --steps 20 > $OUT/apitrace.log 2>&1 || exit $?
ls $OUT/prof_api_r06j
echo ALLDONE
