#!/bin/bash
# round 6: the C application (pipelined phase) and the halves/pipelined
# socket tests, then the N = 2 rehearsal of the refactored bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_c_app.py tests/test_gpu_halves.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/pytest_capp_$TAG.txt 2>&1
rc=$?; tail -3 $OUT/pytest_capp_$TAG.txt; [ $rc -eq 0 ] || exit $rc
TAG=$TAG TESTS=0 BENCH=0 N2=1 bash tools/gpu_r05.sh
