#!/bin/bash
# Flow-table load factor x stream-kernel probe order: GPU parity, then
# interleaved sweeps at load <= 1/4 (default) and <= 1/2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/pt.log 2>&1
rc=$?; tail -3 gpurun_out/pt.log; [ $rc -le 1 ] || exit $rc
for fl in ${LOADS:-2 1 3}; do
  timeout -k 10 300 python bench.py --no-cpu --flow-load $fl --sweep "${WL:-cfg4,cfg5,cfg3}" --steps 10 --warmup 3 \
    --sweep-variants "${VARS:-0,0,0,30;0,0,0,32;0,0,0,33;0,0,0,34;8,2,2,0}" > gpurun_out/fl$fl.log 2>&1 || exit $?
  echo "flow load 2^-$fl"; grep sweep gpurun_out/fl$fl.log
done
