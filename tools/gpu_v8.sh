set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "edge or every_kernel or generated" > gpurun_out/pytest_v8.txt 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_v8.txt; exit 1; }
tail -3 gpurun_out/pytest_v8.txt
timeout -k 10 300 python -u tools/ab_v8.py cfg2,cfg3,cfg4,cfg5 5 50 > gpurun_out/ab_v8.txt 2>&1 || { echo AB_FAIL; tail -30 gpurun_out/ab_v8.txt; exit 1; }
cat gpurun_out/ab_v8.txt
timeout -k 10 420 python -u tools/ab_lib.py tools/librxgpu_head.so cfg2,cfg4 3 > gpurun_out/ab_lib_head.txt 2>&1 || { echo ABLIB_FAIL; tail -30 gpurun_out/ab_lib_head.txt; exit 1; }
tail -4 gpurun_out/ab_lib_head.txt
