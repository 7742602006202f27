#!/bin/bash
# Stream-kernel session: GPU parity, then an interleaved variant sweep on the
# stream-kernel workloads (cfg4 IMIX, cfg5 jumbo).  VARS / WL override.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu --sweep "${WL:-cfg4,cfg5}" --steps 10 --warmup 3 \
  --sweep-variants "${VARS:-0,0,0,30;0,0,0,32;0,0,0,33;0,0,0,34}" > gpurun_out/sws.log 2>&1 || exit $?
grep sweep gpurun_out/sws.log
