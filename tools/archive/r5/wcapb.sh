# BDPT closest-hit launches (k_extend, k_extend_pair's light rays) with the stop rule: BDPT parity
# (vertex-exact vs the reference at 1080p, compact vs 64-B records), then bench A/B
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcapb}; mkdir -p $P
timeout -k 10 900 python -u -m pytest tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py tests/test_gpu_rccl.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  for cl in 0:64 60:8 80:12 40:8; do
    c=${cl%:*}; l=${cl#*:}
    MCRT_WALK_CAP=$c MCRT_WALK_LANES=$l timeout -k 10 300 $B > $P/c${c}_l${l}_$r.json 2> $P/c${c}_l${l}_$r.err || { tail -20 $P/c${c}_l${l}_$r.err; exit 6; }
  done
done
python3 tools/bench_summary.py $P/c*_1.json $P/c*_2.json
