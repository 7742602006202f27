#!/bin/bash
# A/B of the count passes: the same cfg4 trace from the pre-session tree
# (_old, a git worktree built in place) and from this tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
(cd _old && WL=cfg4 ARGS="" GRAFT_REPO_ROOT=$R/_old bash $R/tools/gpu_trace_wl.sh > /dev/null 2>&1; cp gpurun_out/trace_cfg4.txt $R/gpurun_out/trace_cfg4_old.txt) || exit 1
WL=cfg4 ARGS="--no-count-stream" bash tools/gpu_trace_wl.sh > /dev/null 2>&1 || exit 1
echo OLD; tail -6 gpurun_out/trace_cfg4_old.txt; echo NEW; tail -6 gpurun_out/trace_cfg4.txt
