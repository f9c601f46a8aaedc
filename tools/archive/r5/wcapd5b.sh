# stop rule at depth 5 by launch: all bounces vs the first extension launch only vs off
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcapd5b}; mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt --max-depth 5"
for r in 1 2; do
  MCRT_WALK_CAP=0 timeout -k 10 300 $B > $P/d5_off_$r.json 2> $P/d5_off_$r.err || { tail -20 $P/d5_off_$r.err; exit 6; }
  timeout -k 10 300 $B > $P/d5_all_$r.json 2> $P/d5_all_$r.err || { tail -20 $P/d5_all_$r.err; exit 6; }
  MCRT_WALK_MAXB=0 timeout -k 10 300 $B > $P/d5_b0_$r.json 2> $P/d5_b0_$r.err || { tail -20 $P/d5_b0_$r.err; exit 6; }
  MCRT_WALK_MAXB=1 timeout -k 10 300 $B > $P/d5_b1_$r.json 2> $P/d5_b1_$r.err || { tail -20 $P/d5_b1_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/d5_*.json
