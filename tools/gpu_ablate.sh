set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ablate2.log
for v in "1,0,1" "1,4,1" "1,101,1" "1,104,1" "1,108,1" "1,113,1"; do
  for c in "" "--no-counts"; do
    timeout -k 10 120 python bench.py --workload cfg2 --variant $v --no-cpu --steps 10 --warmup 3 $c > gpurun_out/o.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.load(open('gpurun_out/o.json')); print('$v $c', d['kernel_ms_avg'], d['value'])" >> gpurun_out/ablate2.log
  done
done
cat gpurun_out/ablate2.log
