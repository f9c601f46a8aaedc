#!/bin/bash
# round-2 GPU call 15: sanity subset on the rebuilt library, dependent-fetch ceiling probe
# (tools/probe/chase_probe.hip), and TA/TD/TCP/UTCL1 counters of the bench's traversal kernels.
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace.py tests/test_gpu_render.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p15_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/p15_pytest.log; exit 3; }
tail -1 gpurun_out/p15_pytest.log
P=tools/probe/chase_probe
: > gpurun_out/chase.jsonl
for args in "lane4 20000000 256" "lane4 2000000 256" "lane4 32768 256" "lane1 20000000 256" "quad 20000000 256" \
            "dual4 20000000 256" "lane4 20000000 256 16" "lane4 20000000 256 8" "quad 20000000 256 16" "dual4 20000000 256 16" \
            "quad 2000000 256" "lane1 2000000 256"; do
  timeout -k 5 60 $P $args >> gpurun_out/chase.jsonl 2>> gpurun_out/chase.err || { echo "probe $args failed"; cat gpurun_out/chase.err; exit 4; }
done
cat gpurun_out/chase.jsonl
B="python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-roofline-model --no-bdpt"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE -d gpurun_out/p15_ta -o a -- $B > gpurun_out/p15_ta.log 2>&1 || { echo "ta pass failed"; tail -5 gpurun_out/p15_ta.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum -d gpurun_out/p15_tcp1 -o b -- $B > gpurun_out/p15_tcp1.log 2>&1 || { echo "tcp1 pass failed"; tail -5 gpurun_out/p15_tcp1.log; exit 5; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum -d gpurun_out/p15_tcp2 -o c -- $B > gpurun_out/p15_tcp2.log 2>&1 || { echo "tcp2 pass failed"; tail -5 gpurun_out/p15_tcp2.log; exit 5; }
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_UTCL1_TRANSLATION_MISS_sum -d gpurun_out/p15_chase1 -o d -- $P lane4 20000000 256 32 1 > gpurun_out/p15_chase1.log 2>&1 || { echo "chase pmc failed"; tail -5 gpurun_out/p15_chase1.log; exit 5; }
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE -d gpurun_out/p15_chase2 -o e -- $P lane4 20000000 256 32 1 > gpurun_out/p15_chase2.log 2>&1 || { echo "chase pmc2 failed"; tail -5 gpurun_out/p15_chase2.log; exit 5; }
echo "pmc passes done"
for d in p15_ta p15_tcp1 p15_tcp2; do
  for f in $(find gpurun_out/$d -name '*.db'); do python3 tools/pmc_summary.py $f k_shadow_extend k_primary | tail -4; done
done
for d in p15_chase1 p15_chase2; do
  for f in $(find gpurun_out/$d -name '*.db'); do python3 tools/pmc_summary.py $f k_lane4 | tail -2; done
done
