export TMPDIR=/tmp
P=gpurun_out/r5a; Q=gpurun_out/r5b; mkdir -p $P $Q
step() { echo "== $1"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_shadow_hints.py -x -v --timeout 200 --timeout-method thread > $P/hints.log 2>&1 || { tail -20 $P/hints.log; exit 3; }
tail -1 $P/hints.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_scale.py -x -v -k "d5" --timeout 580 --timeout-method thread > $P/scale_d5.log 2>&1 || { tail -20 $P/scale_d5.log; exit 3; }
tail -1 $P/scale_d5.log
timeout -k 10 400 python3 bench.py > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 4; }
tail -c 400 $P/bench.json
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace -d $Q/tr8 -o t -- python3 tools/scale_emulate.py --ns 8 --ranks 2 --chunks 20 --base-ms 1.375 > $Q/tr8.log 2>&1 || { tail -20 $Q/tr8.log; exit 5; }
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace -d $Q/tr1 -o t -- python3 tools/scale_emulate.py --ns 1 --chunks 20 > $Q/tr1.log 2>&1 || { tail -20 $Q/tr1.log; exit 5; }
python3 tools/prof_timeline.py $(find $Q/tr8 -name "*.db" | head -1) 40 > $Q/tl8.txt 2>&1
python3 tools/prof_timeline.py $(find $Q/tr1 -name "*.db" | head -1) 40 > $Q/tl1.txt 2>&1
find $Q -name "*.db" -size +40M -delete
timeout -k 10 400 python3 bench.py --max-depth 5 > $P/bench_d5.json 2> $P/bench_d5.err || { tail -20 $P/bench_d5.err; exit 4; }
timeout -k 10 400 python3 bench.py --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/bench_d5_rr.err || { tail -20 $P/bench_d5_rr.err; exit 4; }
echo ALLOK
