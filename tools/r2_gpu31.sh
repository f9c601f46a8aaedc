#!/bin/bash
# round-2 GPU call 31: full GPU suite, default bench, kernel-trace profile of it, PT counter passes
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/p31_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/p31_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/p31_pytest.log | head -20; exit 3; fi
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 4; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('gather_ceiling'), d.get('bdpt',{}).get('value'))"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d gpurun_out/p31_trace -o t -- python3 bench.py > gpurun_out/p31_trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/p31_trace.log; exit 5; }
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-roofline-model --no-bdpt"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f -- $B > gpurun_out/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/pmc_fetch.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w -- $B > gpurun_out/pmc_write.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/pmc_write.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_sq1 -o s -- $B > gpurun_out/pmc_sq1.log 2>&1 || { echo "sq1 pass failed"; tail -5 gpurun_out/pmc_sq1.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_sq2 -o t -- $B > gpurun_out/pmc_sq2.log 2>&1 || { echo "sq2 pass failed"; tail -5 gpurun_out/pmc_sq2.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_grbm -o g -- $B > gpurun_out/pmc_grbm.log 2>&1 || { echo "grbm pass failed"; tail -5 gpurun_out/pmc_grbm.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE -d gpurun_out/pmc_ta -o a -- $B > gpurun_out/pmc_ta.log 2>&1 || { echo "ta pass failed"; tail -5 gpurun_out/pmc_ta.log; exit 6; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum -d gpurun_out/pmc_tcp -o b -- $B > gpurun_out/pmc_tcp.log 2>&1 || { echo "tcp pass failed"; tail -5 gpurun_out/pmc_tcp.log; exit 6; }
echo "pmc passes done"
