# the default stop rule (60 steps, <= 8 lanes): whole GPU suite, then the bench line
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcap3}; mkdir -p $P
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline-model > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 6; }
python3 tools/bench_summary.py $P/bench.json
