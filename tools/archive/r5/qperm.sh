# A/B: compact walk with per-lane near/far byte permutation (one instantiation for every octant mix,
# libmcrt_qperm.so) vs the octant dispatch (uniform waves specialised, mixed waves generic)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5qperm}; mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_qperm.so
MCRT_LIB_PATH=$V timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_render.py tests/test_gpu_reference_scale.py tests/test_gpu_bdpt.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$V timeout -k 10 300 $B > $P/qperm_$r.json 2> $P/qperm_$r.err || { tail -20 $P/qperm_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/qperm_*.json
