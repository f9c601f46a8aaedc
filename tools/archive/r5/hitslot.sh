# camera-hit records in packed-slot order: parity tests, then the bench twice
export TMPDIR=/tmp
P=gpurun_out/${1:-r5hitslot}; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_reference_scale.py tests/test_gpu_texture_lod.py tests/test_gpu_packets.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  timeout -k 10 300 $B > $P/hs_$r.json 2> $P/hs_$r.err || { tail -20 $P/hs_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/hs_*.json
