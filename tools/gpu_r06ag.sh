#!/bin/bash
# round 6: K2 with the next trip's descriptors loaded one trip ahead (tx
# variants 13-15) — TX parity, then the interleaved variant sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r06ag}
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_tx.py \
    > $OUT/tx_tests_$TAG.log 2>&1 || { tail -30 $OUT/tx_tests_$TAG.log; exit 1; }
tail -1 $OUT/tx_tests_$TAG.log
timeout -k 10 400 python tools/tx_sweep.py cfg2,cfg3,cfg4,cfg5 0,13,14,2,15,10 > $OUT/tx_sweep_$TAG.txt 2>&1 || { tail -5 $OUT/tx_sweep_$TAG.txt; exit 1; }
cat $OUT/tx_sweep_$TAG.txt | tail -30
echo ALLDONE
