# A/B: stop rule of the extension walks -- MCRT_WALK_CAP steps at least, then MCRT_WALK_LANES lanes
# or fewer still walking (64: a fixed step limit); parity with the adaptive rule, then a sweep
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcap2}; mkdir -p $P
MCRT_WALK_LANES=8 MCRT_WALK_CAP=40 timeout -k 10 900 python -u -m pytest tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py -m gpu -x -q --timeout 600 --timeout-method thread > $P/pytest_a.log 2>&1 || { tail -40 $P/pytest_a.log; exit 3; }
tail -1 $P/pytest_a.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  for cl in 0:64 130:64 40:8 60:8 40:16 80:12 100:16 20:4; do
    c=${cl%:*}; l=${cl#*:}
    MCRT_WALK_CAP=$c MCRT_WALK_LANES=$l timeout -k 10 300 $B > $P/c${c}_l${l}_$r.json 2> $P/c${c}_l${l}_$r.err || { tail -20 $P/c${c}_l${l}_$r.err; exit 6; }
  done
done
python3 tools/bench_summary.py $P/c*_1.json $P/c*_2.json
