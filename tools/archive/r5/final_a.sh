# Round-5 final tree, part A: GPU suite + smoke, the driver's bench (N = 1) under a kernel trace, the
# depth-5 lines.  Outputs under gpurun_out/r5fin.
export TMPDIR=/tmp
P=gpurun_out/r5fin; mkdir -p $P
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit "${3:-3}"; }
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || fail suite $P/pytest_gpu.log 3
tail -1 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || fail smoke $P/smoke.log 4
tail -1 $P/smoke.log
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err || fail bench $P/bench.err 4
python3 tools/bench_summary.py $P/bench.json
python3 tools/rocpd_stats.py $(find $P/bench_trace -name "*.db" | head -1) > $P/rocprof_kernel_stats_bench.csv
python3 tools/timed_call_trace.py $(find $P/bench_trace -name "*.db" | head -1) > $P/bench_timed_call_trace.txt 2>&1 || true
find $P/bench_trace -name "*.db" -delete
timeout -k 10 600 python3 bench.py --max-depth 5 > $P/bench_d5.json 2> $P/bench_d5.err || fail d5 $P/bench_d5.err 4
timeout -k 10 600 python3 bench.py --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/bench_d5_rr.err || fail d5rr $P/bench_d5_rr.err 4
python3 tools/bench_summary.py $P/bench_d5.json $P/bench_d5_rr.json
echo ALLOK
