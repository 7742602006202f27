#!/bin/bash
# r02n: stream kernel with interleaved DPP scans + SALU wave offsets; cfg4/cfg5 sweep; SQ cfg4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; return $rc; }
step pytest_gpu 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ]; then exit $rc; fi
step sweep45 400 python bench.py --sweep cfg4,cfg5 --sweep-counts --steps 10 --warmup 3 \
    --sweep-variants '0,0,0,38;0,0,0,39;0,0,0,46;0,0,0,48;0,0,0,33' || exit $?
export TMPDIR=/tmp
step sq4 300 python tools/pmc_counters.py sq cfg4 "--no-tx --no-cfg1" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" || exit $?
echo ALLDONE
