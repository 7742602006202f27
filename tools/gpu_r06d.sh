mkdir -p gpurun_out
timeout -k 10 200 ./tools/membw_cfg3 > gpurun_out/membw_cfg3_r06d.txt 2>&1 && \
timeout -k 10 200 ./tools/membw_cfg2 > gpurun_out/membw_cfg2_r06d.txt 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_halves.py -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_halves_r06d.txt 2>&1 ; tail -3 gpurun_out/pytest_halves_r06d.txt && \
BENCH_DETAIL=gpurun_out/detail_bench_r06d.json timeout -k 10 400 python bench.py --workload cfg2 --no-cfg1 --no-tx --no-v8 > gpurun_out/bench_r06d.log 2>&1; echo rc=$?
