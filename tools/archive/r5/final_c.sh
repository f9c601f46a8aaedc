# Round-5 final tree, evidence in dependency order: counters first (PT timed call, BDPT calls; copied
# into profiles/ on the box so the bench line's `traffic` reads THIS tree's counters), then the
# driver's bench under a kernel trace.  Outputs under gpurun_out/r5fc.
export TMPDIR=/tmp
P=gpurun_out/r5fc; mkdir -p $P
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit "${3:-3}"; }
bash tools/gpu_task.sh evidence r5fc/evidence > $P/evidence.log 2>&1 || fail evidence $P/evidence.log 5
bash tools/gpu_task.sh bdpt-prof r5fc/bdpt_prof > $P/bdpt_prof.log 2>&1 || fail bdpt_prof $P/bdpt_prof.log 5
find $P/evidence $P/bdpt_prof -name "*.db" -delete
cp $P/evidence/pmc_latest.json profiles/pmc_latest.json && cp $P/bdpt_prof/pmc_bdpt.json profiles/pmc_bdpt.json || fail copy /dev/null 6
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err || fail bench $P/bench.err 4
python3 tools/bench_summary.py $P/bench.json
python3 tools/rocpd_stats.py $(find $P/bench_trace -name "*.db" | head -1) > $P/rocprof_kernel_stats_bench.csv
python3 tools/timed_call_trace.py $(find $P/bench_trace -name "*.db" | head -1) > $P/bench_timed_call_trace.txt 2>&1 || true
find $P/bench_trace -name "*.db" -delete
cat $P/evidence/timed_call_trace.txt
echo ALLOK
