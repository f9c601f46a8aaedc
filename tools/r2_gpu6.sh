#!/bin/bash
# oracle-divergence breakdown (small sanity case, then the headline frame) + BDPT counter passes
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u tools/oracle_divergence.py gpurun_out/div_mixed.json 0 mixed 96 64 > gpurun_out/div_mixed.log 2>&1 || { echo "div mixed failed"; tail -20 gpurun_out/div_mixed.log; exit 3; }
cat gpurun_out/div_mixed.log | tail -2
timeout -k 10 400 python3 -u tools/oracle_divergence.py gpurun_out/div_sm.json 0 > gpurun_out/div_sm.log 2>&1 || { echo "div sm failed"; tail -20 gpurun_out/div_sm.log; exit 4; }
tail -2 gpurun_out/div_sm.log
B="python3 bench.py --integrator bdpt --steps 8 --warmup 2 --no-cpu-baseline --no-roofline-model"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmcb_fetch -o f -- $B > gpurun_out/pmcb_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/pmcb_fetch.log; exit 5; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmcb_write -o w -- $B > gpurun_out/pmcb_write.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/pmcb_write.log; exit 5; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmcb_sq1 -o s -- $B > gpurun_out/pmcb_sq1.log 2>&1 || { echo "sq1 pass failed"; tail -5 gpurun_out/pmcb_sq1.log; exit 5; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmcb_sq2 -o t -- $B > gpurun_out/pmcb_sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 gpurun_out/pmcb_sq2.log; exit 5; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcb_grbm -o g -- $B > gpurun_out/pmcb_grbm.log 2>&1 || { echo "grbm pass failed"; tail -5 gpurun_out/pmcb_grbm.log; exit 5; }
echo "bdpt pmc passes done"
