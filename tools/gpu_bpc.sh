cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 120 tools/membw_window > gpurun_out/membw_window.txt 2>&1 || exit $?
timeout -k 10 400 python bench.py --sweep cfg3,cfg5 --sweep-variants "8,2,2,0,0;8,2,2,0,2;8,2,2,0,3;8,2,2,0,4;8,2,2,0,6;8,4,2,18,0;8,4,2,18,2;8,4,2,18,4;16,2,2,18,0;16,2,2,18,3;32,2,2,18,0;32,2,2,18,2;64,1,2,18,0;64,1,2,18,4;0,1,1,30,0;0,1,1,30,3" --steps 10 --warmup 3 > gpurun_out/sweep_bpc.log 2>&1
