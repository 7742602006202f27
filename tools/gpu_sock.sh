#!/bin/bash
# socket layer on the GPU box: delivery parity tests, then the socket-API rate
# leg (three bench processes, workload cfg2 only for the device legs)
set -u
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "== $name: $*"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "passed|failed|Error|socket_api" "$OUT/$name.log" | cut -c1-400 | tail -6; return $rc; }
step pytest_sock 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests -m gpu -k "deliver or nstack or compact or ingest or churn" || exit $?
for i in 1 2 3; do
  step sock_$i 300 python -u bench.py --workload cfg2 --steps 5 --warmup 2 --no-cpu --no-cfg1 --no-v8 --no-tx || exit $?
done
