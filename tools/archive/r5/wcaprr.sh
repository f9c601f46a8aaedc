# stop rule on the first extension launch only (default): depth 5 with Russian roulette vs off
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcaprr}; mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt --max-depth 5 --russian-roulette"
for r in 1 2; do
  MCRT_WALK_CAP=0 timeout -k 10 300 $B > $P/rr_off_$r.json 2> $P/rr_off_$r.err || { tail -20 $P/rr_off_$r.err; exit 6; }
  timeout -k 10 300 $B > $P/rr_b0_$r.json 2> $P/rr_b0_$r.err || { tail -20 $P/rr_b0_$r.err; exit 6; }
  MCRT_WALK_MAXB=1 timeout -k 10 300 $B > $P/rr_b1_$r.json 2> $P/rr_b1_$r.err || { tail -20 $P/rr_b1_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/rr_*.json
