export TMPDIR=/tmp
P=gpurun_out/r5a; Q=gpurun_out/r5b; mkdir -p $P $Q
T="python -u -m pytest -x -v --timeout 580 --timeout-method thread"
timeout -k 10 400 $T tests/test_gpu_quant_nodes.py tests/test_gpu_trace.py > $P/quant.log 2>&1 || { tail -30 $P/quant.log; exit 3; }
tail -1 $P/quant.log
timeout -k 10 300 $T tests/test_gpu_shadow_hints.py > $P/hints.log 2>&1 || { tail -20 $P/hints.log; exit 3; }
tail -1 $P/hints.log
timeout -k 10 900 $T tests/test_gpu_reference_scale.py > $P/scale.log 2>&1 || { tail -30 $P/scale.log; exit 3; }
tail -1 $P/scale.log
timeout -k 10 400 python3 bench.py > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 4; }
tail -c 300 $P/bench.json
MCRT_QUANT_NODES=0 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-roofline-model > $P/bench_q0.json 2> $P/bench_q0.err || { tail -20 $P/bench_q0.err; exit 4; }
python3 tools/bench_summary.py $P/bench.json $P/bench_q0.json
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace -d $Q/tr8 -o t -- python3 tools/scale_emulate.py --ns 8 --ranks 2 --chunks 20 --base-ms 1.375 > $Q/tr8.log 2>&1 || { tail -20 $Q/tr8.log; exit 5; }
python3 tools/prof_timeline.py $(find $Q/tr8 -name "*.db" | head -1) 40 > $Q/tl8.txt 2>&1
find $Q -name "*.db" -size +40M -delete
timeout -k 10 400 python3 bench.py --max-depth 5 > $P/bench_d5.json 2> $P/bench_d5.err || { tail -20 $P/bench_d5.err; exit 4; }
timeout -k 10 400 python3 bench.py --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/bench_d5_rr.err || { tail -20 $P/bench_d5_rr.err; exit 4; }
python3 tools/bench_summary.py $P/bench_d5.json $P/bench_d5_rr.json
echo ALLOK
