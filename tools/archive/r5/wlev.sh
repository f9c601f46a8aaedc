# A/B: a second stop level in the resume (MCRT_WALK_LEVELS=2) -- parity, then the bench
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wlev}; mkdir -p $P
MCRT_WALK_LEVELS=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2 3; do
  timeout -k 10 300 $B > $P/l1_$r.json 2> $P/l1_$r.err || { tail -20 $P/l1_$r.err; exit 6; }
  MCRT_WALK_LEVELS=2 timeout -k 10 300 $B > $P/l2_$r.json 2> $P/l2_$r.err || { tail -20 $P/l2_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/l1_*.json $P/l2_*.json
