#!/bin/bash
# GPU parity tests + the PCIe-inclusive (sync and pipelined) rates
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_all.log 2>&1 || { tail -40 gpurun_out/pt_all.log; exit 1; }
tail -3 gpurun_out/pt_all.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --e2e --no-cpu --workload ${WL:-cfg2,cfg3,cfg4,cfg5} > gpurun_out/e2e.log 2>&1
rc=$?; grep -E "^e2e|^pcie|^\{" gpurun_out/e2e.log | cut -c1-400; exit $rc
