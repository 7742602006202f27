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
timeout -k 10 60 tools/membw_cfg2 > $OUT/membw_cfg2.log 2>&1 && grep "RDW   U=2 bpc=2" $OUT/membw_cfg2.log
step pmc 900 python tools/pmc_traffic.py $TAG cfg2,cfg3,cfg4,cfg5 || exit $?
cp $OUT/pmc_$TAG.json profiles/pmc_$TAG.json || exit 1
step bench 420 python bench.py --steps $STEPS --warmup 5 --e2e ${BENCH_ARGS:-} || exit $?
grep '^{' $OUT/bench.log > $OUT/bench_$TAG.json || true
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
    -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu --no-sockrate --no-v8 || exit $?
f=$(find $OUT/prof_$TAG -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python tools/trace_durations.py "$f" > $OUT/trace_durations_$TAG.txt
# N = 2 rehearsal of the split path: two ranks on this one GPU (gloo carries
# the counts when the ranks share a GPU; the driver's N-GPU run uses RCCL)
step n2 400 python bench.py --gpus 2 --steps 5 --warmup 2 || exit $?
grep '^{' $OUT/n2.log > $OUT/bench_n2_$TAG.json || true
# CEIL=1: the read ceilings of this box (tools/membw_large: plain streams and
# the cfg3 access pattern with no per-frame work) right after the bench, and
# the SQ counters of the cfg3 kernel, for the roofline comparison on one box
if [ "${CEIL:-0}" = 1 ]; then
  step membw 300 ./tools/membw_large || exit $?
  step sq_cfg3 400 python tools/pmc_counters.py $TAG cfg3 "--no-tx --no-sockrate --no-cfg1 --no-v8" \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
    "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" || exit $?
fi
# PROBE=1: L2 hits of the flow-table probes at cfg4 (with vs without the probe)
if [ "${PROBE:-0}" = 1 ]; then
  step probe_hits 400 python tools/pmc_probe_hits.py cfg4 $TAG || exit $?
fi
echo ALLDONE
