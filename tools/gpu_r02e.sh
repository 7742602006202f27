#!/bin/bash
# r02e: resident-grid stream variants (pipes 42/43) — parity, interleaved sweep
# on cfg4/cfg5 (with and without counts, blocks-per-CU caps), and an N=2
# bench rehearsal with both ranks on the one GPU (gloo control plane + gloo
# count all-reduce, the split path and per-rank parity)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest_gpu 480 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
V="0,0,0,38;0,0,0,42;0,0,0,42,3;0,0,0,42,4;0,0,0,39;0,0,0,43;0,0,0,43,4"
step sweep 400 python bench.py --sweep cfg4,cfg5 --sweep-variants "$V" --steps 10 --warmup 3 || exit $?
step sweepc 400 python bench.py --sweep cfg4,cfg5 --sweep-counts --sweep-variants "$V" --steps 10 --warmup 3 || exit $?
step n2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --workload cfg2,cfg4 || exit $?
grep '^{' $OUT/n2.log > $OUT/bench_n2_r02e.json || true
echo ALLDONE
