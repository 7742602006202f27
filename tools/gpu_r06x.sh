#!/bin/bash
# round 6: resident blocks per CU for the final cfg2 / cfg3 defaults
# (interleaved sweep, one process per workload)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06x}
timeout -k 10 300 python bench.py --sweep cfg2 --sweep-variants "1,4,1,14,2;1,4,1,14,3;1,4,1,14,4;1,4,1,14,1" \
    > $OUT/sweep_bpc_cfg2_$TAG.log 2>&1 || { tail -5 $OUT/sweep_bpc_cfg2_$TAG.log; exit 1; }
grep "^sweep\|sweep cfg" $OUT/sweep_bpc_cfg2_$TAG.log | tail -4
timeout -k 10 300 python bench.py --sweep cfg3 --sweep-variants "8,2,2,48,0;8,2,2,48,4;8,2,2,48,3" \
    > $OUT/sweep_bpc_cfg3_$TAG.log 2>&1 || { tail -5 $OUT/sweep_bpc_cfg3_$TAG.log; exit 1; }
grep "sweep cfg" $OUT/sweep_bpc_cfg3_$TAG.log | tail -3
echo ALLDONE
