# radiance in the packed slot order: full GPU suite + smoke, then the bench twice
export TMPDIR=/tmp
P=gpurun_out/${1:-r5radslot}; mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || { tail -40 $P/pytest_gpu.log; exit 3; }
tail -1 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || { tail -20 $P/smoke.log; exit 4; }
tail -1 $P/smoke.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/rs_$r.json 2> $P/rs_$r.err || { tail -20 $P/rs_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/rs_*.json
