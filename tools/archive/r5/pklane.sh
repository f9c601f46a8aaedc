# A/B: wave-packet walk with the lane state in VGPRs (libmcrt_pklane.so, -DMCRT_PK_LANE=1) vs the
# SGPR-mask walk: parity tests on the variant, then the bench twice each
export TMPDIR=/tmp
P=gpurun_out/${1:-r5pklane}; mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_pklane.so
MCRT_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_packets.py tests/test_gpu_shadow_hints.py tests/test_gpu_render.py tests/test_gpu_reference_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$V timeout -k 10 300 $B > $P/pklane_$r.json 2> $P/pklane_$r.err || { tail -20 $P/pklane_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/pklane_*.json
