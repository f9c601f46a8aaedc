#!/bin/bash
# round-2 GPU call 2: full-size reference parity, accumulate/filter pins, counters
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_reference_scale.py tests/test_gpu_accumulate.py \
  "tests/test_gpu_bdpt.py::test_bdpt_frames_in_flight" -v --timeout 900 --timeout-method thread > gpurun_out/pytest2.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest2.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
echo "counters rc=$?"
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-roofline-model --no-bdpt"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f -- $B > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/pmc_fetch.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w -- $B > gpurun_out/pmc_write.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/pmc_write.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_sq1 -o s -- $B > gpurun_out/pmc_sq1.log 2>&1 || { echo "sq1 pass failed"; tail -5 gpurun_out/pmc_sq1.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_sq2 -o t -- $B > gpurun_out/pmc_sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 gpurun_out/pmc_sq2.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_grbm -o g -- $B > gpurun_out/pmc_grbm.log 2>&1 || { echo "grbm pass failed"; tail -5 gpurun_out/pmc_grbm.log; exit 5; }
echo "pmc passes done"
