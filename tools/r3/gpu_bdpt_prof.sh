#!/bin/bash
# BDPT: kernel trace (per launch: the four connect classes, the per-depth extends) and PMC passes
# of the bench's BDPT object; each rocprofv3 pass in its own process and timeout.
export TMPDIR=/tmp
P=gpurun_out/bp
mkdir -p $P
B="python3 bench.py --integrator bdpt --steps 16 --warmup 2 --no-kernel-timing --no-cpu-baseline --no-roofline-model"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P/trace -o k -- $B > $P/trace.log 2>&1 || { tail -5 $P/trace.log; exit 7; }
grep -v "^\[\|^W20\|^I20" $P/trace.log | tail -2 | cut -c1-400
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/pmc_fetch -o f -- $B > $P/f.log 2>&1 || { tail -5 $P/f.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/pmc_write -o w -- $B > $P/w.log 2>&1 || { tail -5 $P/w.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $P/pmc_sq1 -o s -- $B > $P/s.log 2>&1 || { tail -5 $P/s.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum -d $P/pmc_sq2 -o t -- $B > $P/t.log 2>&1 || { tail -5 $P/t.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc_grbm -o g -- $B > $P/g.log 2>&1 || { tail -5 $P/g.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $P/pmc_ta -o a -- $B > $P/a.log 2>&1 || { tail -5 $P/a.log; exit 8; }
echo "passes done"
