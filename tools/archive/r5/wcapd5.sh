# stop rule at depth 5 (with and without Russian roulette): A/B against no stop
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcapd5}; mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt --max-depth 5"
for r in 1 2; do
  for c in 0 60; do
    MCRT_WALK_CAP=$c timeout -k 10 300 $B > $P/d5_c${c}_$r.json 2> $P/d5_c${c}_$r.err || { tail -20 $P/d5_c${c}_$r.err; exit 6; }
    MCRT_WALK_CAP=$c timeout -k 10 300 $B --russian-roulette > $P/rr_c${c}_$r.json 2> $P/rr_c${c}_$r.err || { tail -20 $P/rr_c${c}_$r.err; exit 6; }
  done
done
python3 tools/bench_summary.py $P/d5_*.json $P/rr_*.json
