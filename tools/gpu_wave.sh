#!/bin/bash
# wave-kernel parity (variant + layout tests) and a cfg3/cfg4/cfg5 sweep with
# bpc caps: SWEEP_WL, SWEEP_V
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "every_kernel_variant or layouts" > gpurun_out/pt_wave.log 2>&1 || { tail -40 gpurun_out/pt_wave.log; exit 1; }
tail -3 gpurun_out/pt_wave.log
timeout -k 10 500 python bench.py --sweep "$SWEEP_WL" --sweep-variants "$SWEEP_V" --steps 10 --warmup 3 > gpurun_out/sweep_wave.log 2>&1
rc=$?; grep sweep gpurun_out/sweep_wave.log; exit $rc
