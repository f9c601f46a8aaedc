# A/B: wave packets with scalar lane masks + per-lane stack bits (libmcrt_pkh.so) vs VGPR lane flags
export TMPDIR=/tmp
P=gpurun_out/${1:-r5pkh}; mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_pkh.so
for L in "" "$V"; do
  MCRT_LIB_PATH=$L timeout -k 10 900 python -u -m pytest tests/test_gpu_packets.py tests/test_gpu_shadow_hints.py tests/test_gpu_render.py tests/test_gpu_reference_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest_$(basename "${L:-base}").log 2>&1 || { tail -40 $P/pytest_$(basename "${L:-base}").log; exit 3; }
  tail -1 $P/pytest_$(basename "${L:-base}").log
done
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$V timeout -k 10 300 $B > $P/pkh_$r.json 2> $P/pkh_$r.err || { tail -20 $P/pkh_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/pkh_*.json
