# Round-5 evidence on the final tree: the driver's bench (N = 1) under a kernel trace, the depth-5
# sensitivity lines, counters of the PT timed call and of the BDPT calls, the per-rank scaling
# emulation and every BASELINE config.  Outputs under gpurun_out/r5final.
export TMPDIR=/tmp
P=gpurun_out/r5final; mkdir -p $P
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit "${3:-3}"; }
# 1. the driver's command, as the driver runs it, under rocprofv3 --kernel-trace --stats
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $P/bench_trace -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err || fail bench $P/bench.err 4
python3 tools/bench_summary.py $P/bench.json
python3 tools/rocpd_stats.py $(find $P/bench_trace -name "*.db" | head -1) > $P/rocprof_kernel_stats_bench.csv
python3 tools/timed_call_trace.py $(find $P/bench_trace -name "*.db" | head -1) > $P/bench_timed_call_trace.txt 2>&1 || true
find $P/bench_trace -name "*.db" -delete
# 2. depth 5: PT (the reference's pinned path), PT with Russian roulette, and the BDPT object
timeout -k 10 600 python3 bench.py --max-depth 5 > $P/bench_d5.json 2> $P/bench_d5.err || fail d5 $P/bench_d5.err 4
timeout -k 10 600 python3 bench.py --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/bench_d5_rr.err || fail d5rr $P/bench_d5_rr.err 4
python3 tools/bench_summary.py $P/bench_d5.json $P/bench_d5_rr.json
# 3. counters: the PT timed call and the BDPT calls
bash tools/gpu_task.sh evidence r5final/evidence > $P/evidence.log 2>&1 || fail evidence $P/evidence.log 5
bash tools/gpu_task.sh bdpt-prof r5final/bdpt_prof > $P/bdpt_prof.log 2>&1 || fail bdpt_prof $P/bdpt_prof.log 5
find $P/evidence -name "*.db" -size +30M -delete
# 4. per-rank scaling emulation
timeout -k 10 500 python3 tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_scale.json 2> $P/pt_scale.err || fail pt_scale $P/pt_scale.err 4
timeout -k 10 600 python3 tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 32 --batch 16 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || fail bdpt_scale $P/bdpt_scale.err 4
# 5. every BASELINE config
bash tools/gpu_task.sh configs r5final/configs > $P/configs.log 2>&1 || fail configs $P/configs.log 5
tail -6 $P/configs.log
echo ALLOK
