#!/bin/bash
# default bench (PT headline + BDPT object) and its kernel-trace profile
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench5.json 2> gpurun_out/bench5.err || { echo "bench failed"; tail -20 gpurun_out/bench5.err; exit 3; }
cat gpurun_out/bench5.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o bench -- python3 bench.py > gpurun_out/prof5.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof5.log; exit 4; }
find gpurun_out/prof5 -name "*.csv" | head
