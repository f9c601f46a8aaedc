# A/B: lane refill of the extension rays (persistent waves; MIN 16 / 32 idle lanes; generic slab or
# octant re-dispatch "o") vs the one-ray-per-lane launch; parity tests on two variants first
export TMPDIR=/tmp
P=gpurun_out/${1:-r5refill}; mkdir -p $P
for v in refill16 refillo16; do
  MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_render.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest_$v.log 2>&1 || { tail -40 $P/pytest_$v.log; exit 3; }
  tail -1 $P/pytest_$v.log
done
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
timeout -k 10 300 $B > $P/base_1.json 2> $P/base_1.err || { tail -20 $P/base_1.err; exit 6; }
for v in refill16 refill32 refillo16 refillo32; do
  MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so timeout -k 10 300 $B > $P/${v}_1.json 2> $P/${v}_1.err || { tail -20 $P/${v}_1.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_1.json $P/refill16_1.json $P/refill32_1.json $P/refillo16_1.json $P/refillo32_1.json
