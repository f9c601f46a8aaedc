#!/bin/bash
# Evidence for the current build: kernel trace + PMC passes of the bench's timed call (the counters
# bench.py reads, profiles/pmc_latest.json), then per-rank scaling emulation (PT 20 steps as one call
# per rank; BDPT band split, 8 frames per call).
export TMPDIR=/tmp
P=gpurun_out/${EV_DIR:-ev}
mkdir -p $P
B="python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P/trace -o k -- $B > $P/trace.log 2>&1 || { tail -5 $P/trace.log; exit 7; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $P/pmc_fetch -o f -- $B > $P/f.log 2>&1 || { tail -5 $P/f.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $P/pmc_write -o w -- $B > $P/w.log 2>&1 || { tail -5 $P/w.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $P/pmc_sq1 -o s -- $B > $P/s.log 2>&1 || { tail -5 $P/s.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum -d $P/pmc_sq2 -o t -- $B > $P/t.log 2>&1 || { tail -5 $P/t.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $P/pmc_grbm -o g -- $B > $P/g.log 2>&1 || { tail -5 $P/g.log; exit 8; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE -d $P/pmc_ta -o a -- $B > $P/a.log 2>&1 || { tail -5 $P/a.log; exit 8; }
echo "passes done"
python3 tools/pmc_json.py $P "$B" 1 pmc_ $P/pmc_latest.json > $P/pmc_json.log 2>&1 || { tail -5 $P/pmc_json.log; exit 9; }
python3 tools/timed_call_trace.py $(find $P/trace -name "*.db" | head -1) > $P/timed_call_trace.txt 2>&1 || { tail -5 $P/timed_call_trace.txt; exit 9; }
cat $P/timed_call_trace.txt | head -12
[ -n "$NO_SCALE" ] && exit 0
timeout -k 10 400 python tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_scale.json 2> $P/pt_scale.err || { tail -5 $P/pt_scale.err; exit 4; }
python -c "import json; d=json.load(open('$P/pt_scale.json')); print('PT', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
timeout -k 10 500 python tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 16 --batch 8 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || { tail -5 $P/bdpt_scale.err; exit 4; }
python -c "import json; d=json.load(open('$P/bdpt_scale.json')); print('BDPT', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
