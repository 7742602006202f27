set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py tests/test_gpu_parity.py -k "count or stream" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload cfg4,cfg5 --no-cpu --no-cfg1 --no-tx --steps 20 > gpurun_out/b_cs$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py --workload cfg4,cfg5 --no-cpu --no-cfg1 --no-tx --steps 20 --no-count-stream > gpurun_out/b_sync$i.log 2>&1 || exit 1
done
echo ALLDONE
