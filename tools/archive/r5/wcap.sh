# A/B: step limit of the extension rays' compact walks (MCRT_WALK_CAP; suspended walks finished by
# k_walk_resume in dense waves) -- parity at two limits, then the bench over a sweep of limits
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcap}; mkdir -p $P
T="tests/test_gpu_quant_nodes.py tests/test_gpu_render.py tests/test_gpu_reference_scale.py"
MCRT_WALK_CAP=100 timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest_100.log 2>&1 || { tail -40 $P/pytest_100.log; exit 3; }
tail -1 $P/pytest_100.log
MCRT_WALK_CAP=7 timeout -k 10 600 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_render.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest_7.log 2>&1 || { tail -40 $P/pytest_7.log; exit 3; }
tail -1 $P/pytest_7.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  for c in 0 60 80 100 130 170; do
    MCRT_WALK_CAP=$c timeout -k 10 300 $B > $P/cap${c}_$r.json 2> $P/cap${c}_$r.err || { tail -20 $P/cap${c}_$r.err; exit 6; }
  done
done
python3 tools/bench_summary.py $P/cap*_1.json $P/cap*_2.json
