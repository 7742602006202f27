#!/bin/bash
# round 6: the count stream on CUs of its own (bench --cu-split N: N > 0 one
# CU per 32-CU group, N < 0 the last |N| CUs) against the shared default,
# alternating processes.  Any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06q}
Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
: > $OUT/cus_ab_$TAG.txt
for k in 1 2; do
  for cfg in "0 0" "8 0" "16 16" "-8 0"; do
    set -- $cfg
    timeout -k 10 200 python bench.py $Q --cu-split $1 --tune-tables $2 > $OUT/cus_${1}_${2}_$k.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "cu_split=$1 rc=$rc"; exit $rc; }
    echo "cu_split=$1 tt=$2 round $k: $(grep '^{' $OUT/cus_${1}_${2}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("cfg4", d["ms_per_step"], d["roofline"]["kernel"]["median_ms"], d["counts_match"], d["digest_ok"], "cfg5", d["cfg5"]["ms_per_step"], d["cfg5"].get("kernel_median_ms"), d["cfg5"]["counts_match"], d["cfg5"]["digest_ok"])')" >> $OUT/cus_ab_$TAG.txt
  done
done
cat $OUT/cus_ab_$TAG.txt
echo ALLDONE
