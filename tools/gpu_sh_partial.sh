#!/bin/bash
# the SH kernel with partial last chunks summed in the stream: parity (the
# fallback cases, every variant, generated bursts, whole-burst digests), then
# cfg4 against the HEAD build across bench processes and an interleaved sweep
set -u
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "^sweep|passed|failed|median step|Error|assert" "$OUT/$name.log" | cut -c1-300 | tail -12; return $rc; }
step pytest_sh 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_digest.py -k "fallback or every_kernel or generated or whole_burst or edge or layouts" || exit $?
step sweep_sh 400 python -u bench.py --sweep cfg4 --sweep-counts --steps 30 --warmup 3 --sweep-variants "0,0,0,64;0,0,0,264;0,0,0,60" || exit $?
step ab_lib_sh 600 python -u tools/ab_lib.py tools/librxgpu_head.so cfg4,cfg2 3 || exit $?
