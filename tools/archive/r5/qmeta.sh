# compact records with one-shift steps and a stored right-child ref: parity tests, bench twice
export TMPDIR=/tmp
P=gpurun_out/${1:-r5qmeta2}; mkdir -p $P
timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py tests/test_gpu_bdpt.py tests/test_gpu_trace.py tests/test_gpu_shadow_hints.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/qm2_$r.json 2> $P/qm2_$r.err || { tail -20 $P/qm2_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/qm2_*.json
