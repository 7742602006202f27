#!/bin/bash
# r02y: N=2 bench rehearsal on the final tree, both ranks on the one GPU
# (gloo control plane + gloo count all-reduce; the RSS split + gather path
# and per-rank parity), every workload
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 6 "$OUT/$name.log"; return $rc; }
step n2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 || exit $?
grep '^{' $OUT/n2.log > $OUT/bench_n2_r02y.json || true
echo ALLDONE
