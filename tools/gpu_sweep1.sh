#!/bin/bash
# variant parity + a kernel-variant sweep: SWEEP_WL (workloads) x SWEEP_V (variants)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_kernel_variant" > gpurun_out/pt_var.log 2>&1 || { tail -30 gpurun_out/pt_var.log; exit 1; }
tail -3 gpurun_out/pt_var.log
timeout -k 10 500 python bench.py --sweep "$SWEEP_WL" --sweep-variants "$SWEEP_V" ${SWEEP_COUNTS:+--sweep-counts} --steps 10 --warmup 3 > gpurun_out/sweep1.log 2>&1
rc=$?; grep sweep gpurun_out/sweep1.log; exit $rc
