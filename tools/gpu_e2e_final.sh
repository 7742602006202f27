#!/bin/bash
# PCIe-inclusive rate (host buffers: pinned H2D, K1, D2H, 3 staging slots) on the final tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 400 python bench.py --e2e --workload cfg2,cfg3 --steps 10 --warmup 3 --no-cpu --no-tx > $OUT/e2e.log 2>&1
rc=$?; grep -E "^e2e|^pcie" $OUT/e2e.log; exit $rc
