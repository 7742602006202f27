#!/bin/bash
# rocprofv3 kernel trace of one bench workload (diagnostics):
#   WL=cfg4 [ARGS=...] bash tools/gpu_trace_wl.sh   -> gpurun_out/trace_<WL>.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_${WL} -o run \
    -- python3 bench.py --workload ${WL} --no-cpu --no-cfg1 --no-tx --steps 10 --warmup 3 ${ARGS:-} \
    > $OUT/tr_${WL}.log 2>&1 || { tail -20 $OUT/tr_${WL}.log; exit 1; }
f=$(find $OUT/tr_${WL} -name '*kernel_trace.csv' | head -1)
python3 - "$f" > $OUT/trace_${WL}.txt <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "rx_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-40:]:
    nm = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{nm[:60]:60s} start {s/1e3:14.1f} us dur {(e-s)/1e3:9.1f} us")
PY
cat $OUT/trace_${WL}.txt
