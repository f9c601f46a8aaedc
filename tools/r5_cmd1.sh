export TMPDIR=/tmp
P=gpurun_out/r5a; mkdir -p $P
timeout -k 10 300 python -u -m pytest tests/test_gpu_shadow_hints.py -x -v --timeout 200 --timeout-method thread > $P/hints.log 2>&1 && tail -2 $P/hints.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_reference_scale.py -x -v -k "d5" --timeout 580 --timeout-method thread > $P/scale_d5.log 2>&1 && tail -2 $P/scale_d5.log &&
timeout -k 10 400 python3 bench.py > $P/bench.json 2> $P/bench.err && tail -c 600 $P/bench.json &&
timeout -k 10 400 python3 bench.py --max-depth 5 > $P/bench_d5.json 2> $P/bench_d5.err &&
timeout -k 10 400 python3 bench.py --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/bench_d5_rr.err && echo ALLOK
