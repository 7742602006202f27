# cfg2 on whatever box this is: the byte-pattern ceilings (membw_cfg2), an
# interleaved sweep of the lane kernels x resident blocks per CU (counts on,
# as in the bench), and the 16-B path of this library against the HEAD build
# (tools/librxgpu_head.so) across bench processes.  Each step has its own limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/membw_cfg2 > gpurun_out/membw_cfg2_box.txt 2>&1 || { echo MEMBW_FAIL; exit 1; }
grep -E "bpc=2|bpc=4" gpurun_out/membw_cfg2_box.txt | head -24
timeout -k 10 300 python -u bench.py --sweep cfg2 --sweep-counts --steps 50 --warmup 5 \
  --sweep-variants "1,4,1,14,2;1,4,1,14,3;1,4,1,14,4;1,4,1,12,2;1,4,1,12,3;1,4,1,12,4;1,4,1,5,4;1,4,1,5,6" \
  > gpurun_out/sweep_cfg2_box.txt 2>&1 || { echo SWEEP_FAIL; tail -20 gpurun_out/sweep_cfg2_box.txt; exit 1; }
grep "sweep cfg2" gpurun_out/sweep_cfg2_box.txt
timeout -k 10 500 python -u tools/ab_lib.py tools/librxgpu_head.so cfg2,cfg4,cfg3 3 > gpurun_out/ab_lib_head.txt 2>&1 || { echo ABLIB_FAIL; tail -30 gpurun_out/ab_lib_head.txt; exit 1; }
tail -6 gpurun_out/ab_lib_head.txt
