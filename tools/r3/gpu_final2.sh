#!/bin/bash
# final tree: full GPU suite, smoke, default bench, kernel trace of the timed call
export TMPDIR=/tmp
SUITE_DIR=${F_DIR:-final2} bash tools/r3/gpu_suite.sh || exit 3
B1_DIR=${F_DIR:-final2} bash tools/r3/gpu_bench1.sh || exit 4
P=gpurun_out/${F_DIR:-final2}
timeout -s KILL 300 rocprofv3 --kernel-trace -d $P/tt -o k -- python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model > $P/tt.log 2>&1 || { tail -5 $P/tt.log; exit 5; }
python3 tools/timed_call_trace.py $(find $P/tt -name "*.db" | head -1) > $P/timed_call_trace.txt && tail -1 $P/timed_call_trace.txt
rm -rf $P/tt
