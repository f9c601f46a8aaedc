# BDPT-only sweep of the stop rule's parameters (bench.py --integrator bdpt)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcapbd}; mkdir -p $P
B="python3 bench.py --integrator bdpt --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  for cl in 0:64 60:8 40:16 100:24 30:32 130:64; do
    c=${cl%:*}; l=${cl#*:}
    MCRT_WALK_CAP=$c MCRT_WALK_LANES=$l timeout -k 10 300 $B > $P/c${c}_l${l}_$r.json 2> $P/c${c}_l${l}_$r.err || { tail -20 $P/c${c}_l${l}_$r.err; exit 6; }
  done
done
python3 tools/bench_summary.py $P/c*_1.json $P/c*_2.json
