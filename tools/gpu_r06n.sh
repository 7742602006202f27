#!/bin/bash
# round 6: K2 (TX checksum) at 64 B — parity of every variant, then the
# sweep of the new 8 / 16 frames-per-group variants against the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06n}
timeout -k 10 300 python -u -m pytest tests/test_tx.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > $OUT/pytest_tx_$TAG.txt 2>&1
rc=$?; tail -2 $OUT/pytest_tx_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tx_sweep.py cfg2 0,13,14,6 0,4,8 > $OUT/tx_sweep_$TAG.txt 2>&1 || exit $?
cat $OUT/tx_sweep_$TAG.txt
echo ALLDONE
