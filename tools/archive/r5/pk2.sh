# packet walk with VGPR lane state + VALU-only leaf test: parity tests, then the bench twice
export TMPDIR=/tmp
P=gpurun_out/${1:-r5pk2}; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_packets.py tests/test_gpu_shadow_hints.py tests/test_gpu_render.py tests/test_gpu_reference_scale.py tests/test_gpu_trace.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/pk2_$r.json 2> $P/pk2_$r.err || { tail -20 $P/pk2_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/pk2_*.json
