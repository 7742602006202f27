set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1; echo "list rc=$?"
for v in "1,4,1" "4,1,2"; do
  timeout -k 10 200 python bench.py --workload cfg2 --variant $v --no-cpu --steps 10 >> gpurun_out/ablate.log 2>&1 || exit $?
  timeout -k 10 200 python bench.py --workload cfg2 --variant $v --no-cpu --steps 10 --no-counts >> gpurun_out/ablate.log 2>&1 || exit $?
done
timeout -k 10 100 python -c "
import torch,time
x=torch.empty(1<<30,dtype=torch.uint8,device='cuda'); y=torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(20): y.copy_(x)
torch.cuda.synchronize(); el=(time.perf_counter()-t)/20
print('d2d copy 1GiB: %.1f GB/s (read+write)'%(2*(1<<30)/el/1e9))
" >> gpurun_out/ablate.log 2>&1 || exit $?
for v in "1,4,1" "4,1,2"; do
timeout -k 10 500 python tools/pmc_counters.py r01d cfg2 "--variant $v" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE" >> gpurun_out/pmcx.log 2>&1 || exit $?
done
echo ALLDONE
