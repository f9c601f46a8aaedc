#!/bin/bash
# round-2 GPU check: tests, bench, kernel-trace profile
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 3; }
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --no-roofline-model > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 4; }
find gpurun_out/prof -name "*stats*" | head
