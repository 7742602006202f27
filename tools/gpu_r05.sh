#!/bin/bash
# Round-5 GPU session: parity suite, smoke, the bench exactly as the driver
# runs it (compact stdout line + the full detail file), rocprofv3
# --kernel-trace --stats of the bench on the SAME box, and the table tying
# each workload's roofline.kernel to the trace.  Optional: SWING=1 the cfg2
# placement / clock probe (tools/cfg2_swing.py) first thing and again after
# the tests; PMC=1 HBM bytes; N2=1 the N = 2 spawn rehearsal; PROC=1 cfg2 per
# context and process; MEMBW3=1, SWEEPBPC=1 bytes-in-flight sweeps; ABCS=1
# the count stream A/B; SOCKHOST=1 the host socket path alone.  Each GPU step
# has its own time limit; a failing step ends the script.
#     TAG=r05a bash tools/gpu_r05.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r05}
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; date +%T; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log"; return $rc; }
bench() {  # name limit args...: the line and its detail file kept under the name
  local name=$1 t=$2; shift 2
  BENCH_DETAIL=$OUT/detail_${name}_$TAG.json step $name $t python bench.py "$@" || return $?
  grep '^{' $OUT/$name.log > $OUT/${name}_$TAG.json || true
}
if [ "${SWING:-0}" = 1 ]; then
  step swing_first 240 python tools/cfg2_swing.py || exit $?
  grep '^{' $OUT/swing_first.log > $OUT/swing_first_$TAG.json || true
  bench bench_cfg2_first 240 --workload cfg2 --no-cfg1 --no-sockrate --no-tx --no-v8 || exit $?
fi
if [ "${PROC:-0}" = 1 ]; then
  # cfg2 per process: default / second / high-priority stream, a second
  # context, a burst behind a spacer (tools/cfg2_proc.py), in 5 processes
  for k in 1 2 3 4 5; do
    NCTX=6 step proc$k 120 python tools/cfg2_proc.py || exit $?
    grep '^{' $OUT/proc$k.log >> $OUT/proc_$TAG.jsonl || true
  done
  # 6 contexts in one process under the kernel trace: kernel durations vs gaps per case
  NCTX=6 step proctrace 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof_proc_$TAG -o run \
      -- python3 tools/cfg2_proc.py || exit $?
  f=$(find $OUT/prof_proc_$TAG -name '*kernel_trace.csv' | head -1)
  [ -n "$f" ] && python tools/proc_trace.py $OUT/proctrace.log "$f" > $OUT/proc_trace_$TAG.txt 2>&1
  cat $OUT/proc_trace_$TAG.txt
fi
if [ "${SOCKHOST:-0}" = 1 ]; then
  # the host socket path alone (no GPU): drain_all's prefetch variants,
  # interleaved, in place and copy (tools/sock_host_bench.c, tools/Makefile nsv)
  C0=$(python3 -c 'import os; print(sorted(os.sched_getaffinity(0))[0])')
  for r in 1 2; do for v in a4l0 a8l0 a16l0 a4l3 a8l3 a8l1 a2l0 a0l0; do
    echo "== $v round $r" >> $OUT/sockhost_$TAG.txt
    LD_LIBRARY_PATH=tools/nsv/$v:dpdk-tcp-udp_protocol_stack_amd:oracle timeout -k 5 60 ./tools/sock_host_bench 1 $C0 >> $OUT/sockhost_$TAG.txt 2>&1 || exit $?
  done; done
  LD_LIBRARY_PATH=tools/nsv/a4l0:dpdk-tcp-udp_protocol_stack_amd:oracle timeout -k 5 60 ./tools/sock_host_bench 0 $C0 >> $OUT/sockhost_$TAG.txt 2>&1 || exit $?
fi
if [ "${TESTS:-1}" = 1 ]; then
  # plain test failures (rc 1) still let the bench run; anything else (a
  # timeout, an abort, a fault) ends the session
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
  rc=$?; [ $rc -le 1 ] || exit $rc
  step smoke 150 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [ "${SWING:-0}" = 1 ]; then
  step swing_after 240 python tools/cfg2_swing.py || exit $?
  grep '^{' $OUT/swing_after.log > $OUT/swing_after_$TAG.json || true
fi
if [ "${SWINGDIAG:-0}" = 1 ]; then
  # right after the tests (the order the driver and round 4 used): short
  # cfg2 + cfg5 benches back to back, then after a pause, with amd-smi
  # (clocks, power, temperatures) sampled all along
  ( while true; do echo "T $(date +%s.%N)"; timeout 10 amd-smi metric -g 0 -c -p -t 2>/dev/null; sleep 0.2; done ) > $OUT/smi_$TAG.log 2>&1 &
  SMI=$!
  Q="--workload cfg2,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
  for k in 1 2; do echo "T $(date +%s.%N) quick$k" >> $OUT/smi_marks_$TAG.log; bench quick$k 240 $Q || { kill $SMI; exit 1; }; done
  sleep 20
  echo "T $(date +%s.%N) quick3" >> $OUT/smi_marks_$TAG.log
  bench quick3 240 $Q || { kill $SMI; exit 1; }
  echo "T $(date +%s.%N) end" >> $OUT/smi_marks_$TAG.log
  kill $SMI
fi
export TMPDIR=/tmp
if [ "${PMC:-0}" = 1 ]; then
  step pmc 900 python tools/pmc_traffic.py $TAG cfg2,cfg3,cfg4,cfg5 || exit $?
  cp $OUT/pmc_$TAG.json profiles/pmc_$TAG.json || exit 1
fi
if [ "${BENCH:-1}" = 1 ]; then
  bench bench 420 ${BENCH_ARGS:-} || exit $?
  BENCH_DETAIL=$OUT/detail_rocprof_$TAG.json step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run \
      -- python3 bench.py --no-cpu --no-sockrate --no-v8 --no-cfg1 --no-tx || exit $?
  grep '^{' $OUT/rocprof.log > $OUT/bench_profiled_$TAG.json || true
  f=$(find $OUT/prof_$TAG -name '*kernel_trace.csv' | head -1)
  s=$(find $OUT/prof_$TAG -name '*kernel_stats.csv' | head -1)
  [ -n "$s" ] && cp "$s" $OUT/kernel_stats_$TAG.csv
  if [ -n "$f" ]; then
    python tools/trace_durations.py "$f" > $OUT/trace_durations_$TAG.txt
    python tools/roofline_check.py $OUT/detail_rocprof_$TAG.json "$f" $OUT/detail_bench_$TAG.json \
        > $OUT/roofline_check_$TAG.txt 2>&1
    cat $OUT/roofline_check_$TAG.txt
  fi
fi
if [ "${MEMBW3:-0}" = 1 ]; then  # cfg3 access-shape ceilings (tools/membw_cfg3.hip)
  step membw_cfg3 150 ./tools/membw_cfg3 || exit $?
  cp $OUT/membw_cfg3.log $OUT/membw_cfg3_$TAG.txt
fi
if [ "${WC:-0}" = 1 ]; then  # the RX_DIAG build: WC kernel parity, then the interleaved cfg3 sweep
  RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so step pytest_diag 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread -k "wave_contiguous or every_kernel_variant" || exit $?
  RXGPU_LIB=$PWD/dpdk-tcp-udp_protocol_stack_amd/librxgpu_diag.so step sweep_wc 400 python bench.py --sweep cfg3 --steps 20 --warmup 3 --sweep-counts --sweep-variants "8,2,2,40;0,0,0,80;0,0,0,81;0,0,0,82;0,0,0,83;8,2,2,0" || exit $?
  grep sweep $OUT/sweep_wc.log > $OUT/sweep_wc_$TAG.txt || true
fi
if [ "${AB2BUF:-0}" = 1 ]; then  # cfg4: three count-index buffers (default) vs two, alternating
  Q="--workload cfg4 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
  for k in 1 2; do
    bench ab3buf$k 240 $Q || exit $?
    bench ab2buf$k 240 $Q --tune-tables 4 || exit $?
  done
fi
if [ "${SWEEPBPC:-0}" = 1 ]; then  # resident blocks per CU (bytes in flight): cfg3's G=8 kernel, cfg2's lane kernel
  step sweep_bpc3 400 python bench.py --sweep cfg3 --steps 20 --warmup 3 --sweep-counts \
      --sweep-variants "8,2,2,40,0;8,2,2,40,1;8,2,2,40,2;8,2,2,40,3;8,2,2,40,4;8,2,2,40,5;8,2,2,40,6" || exit $?
  step sweep_bpc2 400 python bench.py --sweep cfg2 --steps 50 --warmup 5 --sweep-counts \
      --sweep-variants "1,4,1,14,0;1,4,1,14,1;1,4,1,14,2;1,4,1,14,3;1,4,1,14,4" || exit $?
  grep -h sweep $OUT/sweep_bpc3.log $OUT/sweep_bpc2.log > $OUT/sweep_bpc_$TAG.txt || true
fi
if [ "${ABCS:-0}" = 1 ]; then  # cfg4 (and cfg5): count passes on the count stream (default) vs after K1 on its stream
  Q="--workload cfg4,cfg5 --no-cpu --no-sockrate --no-cfg1 --no-tx --no-v8"
  for k in 1 2; do
    bench abcs$k 240 $Q || exit $?
    bench abnocs$k 240 $Q --no-count-stream || exit $?
  done
fi
if [ "${N2:-0}" = 1 ]; then
  # the N = 2 logic with two ranks on this one GPU: the default per-rank
  # shards, then the split of one global burst (the golden frame digest over
  # both ranks)
  bench n2 400 --gpus 2 --steps 5 --warmup 2 || exit $?
  bench n2split 400 --gpus 2 --steps 5 --warmup 2 --shard-gen split --workload cfg2,cfg3 || exit $?
fi
echo ALLDONE
