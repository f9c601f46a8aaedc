# A/B: k_walk_resume in XCD-aware block order (MCRT_WALK_XCD=1) -- parity, then the bench
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wxcd}; mkdir -p $P
MCRT_WALK_XCD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2 3; do
  MCRT_WALK_XCD=0 timeout -k 10 300 $B > $P/x0_$r.json 2> $P/x0_$r.err || { tail -20 $P/x0_$r.err; exit 6; }
  MCRT_WALK_XCD=1 timeout -k 10 300 $B > $P/x1_$r.json 2> $P/x1_$r.err || { tail -20 $P/x1_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/x0_*.json $P/x1_*.json
