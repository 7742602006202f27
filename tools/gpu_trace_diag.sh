#!/bin/bash
# diagnostics: cfg4 trace from the _diag tree (a copy built without the count passes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out
(cd _diag && WL=cfg4 ARGS="--no-count-stream" GRAFT_REPO_ROOT=$R/_diag bash $R/tools/gpu_trace_wl.sh > /dev/null 2>&1; cp gpurun_out/trace_cfg4.txt $R/gpurun_out/trace_cfg4_diag.txt) || exit 1
sed -n '1,3p' gpurun_out/trace_cfg4_diag.txt; tail -3 gpurun_out/trace_cfg4_diag.txt
