#!/bin/bash
# Final-tree GPU session, in the order the bench line needs: parity suite,
# smoke, PMC HBM bytes of every workload (stamped with this librxgpu.so's SHA
# and copied into profiles/ so the bench publishes roofline.traffic from it),
# the bench line (with the PCIe-inclusive leg), rocprofv3 kernel stats and
# per-workload dispatch durations, and an N = 2 rehearsal.  Each GPU step has its own time limit; a
# failing step ends the script.     TAG=r02ab bash tools/gpu_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r02}
STEPS=${STEPS:-20}
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; date +%T; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread || exit $?
step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
export TMPDIR=/tmp
step pmc 900 python tools/pmc_traffic.py $TAG cfg2,cfg3,cfg4,cfg5 || exit $?
cp $OUT/pmc_$TAG.json profiles/pmc_$TAG.json || exit 1
step bench 420 python bench.py --steps $STEPS --warmup 5 --e2e ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log > $OUT/bench_$TAG.json || true
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu || exit $?
f=$(find $OUT/prof_$TAG -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python tools/trace_durations.py "$f" > $OUT/trace_durations_$TAG.txt
# N = 2 rehearsal of the split path: two ranks on this one GPU (gloo carries
# the counts when the ranks share a GPU; the driver's N-GPU run uses RCCL)
step n2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 || exit $?
grep '^{' $OUT/n2.log > $OUT/bench_n2_$TAG.json || true
echo ALLDONE
