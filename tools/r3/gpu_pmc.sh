#!/bin/bash
# Round 3 counters: (1) FETCH_SIZE calibration on the dependent-gather probe; (2) kernel trace of the
# bench's timed call (its launches = the last dispatch of each kernel: --no-kernel-timing); (3) PMC
# passes of the same command.  Each rocprofv3 pass in its own process, each under its own timeout.
export TMPDIR=/tmp
mkdir -p gpurun_out/cal gpurun_out/timed
C="python3 tools/pmc_calibrate.py"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/cal/fetch -o f -- $C > gpurun_out/cal/fetch.log 2>&1 || { tail -5 gpurun_out/cal/fetch.log; exit 5; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/cal/tcc -o t -- $C > gpurun_out/cal/tcc.log 2>&1 || { tail -5 gpurun_out/cal/tcc.log; exit 5; }
python3 tools/pmc_calibrate.py --summarise gpurun_out/cal > gpurun_out/cal/summary.txt 2>&1 || { tail -20 gpurun_out/cal/summary.txt; exit 6; }
grep -E "factor|hit_rate|misses_per" gpurun_out/cal/summary.txt | head -12
B="python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/timed/trace -o k -- $B > gpurun_out/timed/trace.log 2>&1 || { tail -5 gpurun_out/timed/trace.log; exit 7; }
P="gpurun_out/timed"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/pmc_fetch -o f -- $B > $P/f.log 2>&1 || { tail -5 $P/f.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/pmc_write -o w -- $B > $P/w.log 2>&1 || { tail -5 $P/w.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $P/pmc_sq1 -o s -- $B > $P/s.log 2>&1 || { tail -5 $P/s.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum -d $P/pmc_sq2 -o t -- $B > $P/t.log 2>&1 || { tail -5 $P/t.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc_grbm -o g -- $B > $P/g.log 2>&1 || { tail -5 $P/g.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $P/pmc_ta -o a -- $B > $P/a.log 2>&1 || { tail -5 $P/a.log; exit 8; }
echo "passes done"
