# BDPT at depth 5: stop rule off / on every launch / only the launches tracing queue depths <= 1
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wbd5}; mkdir -p $P
B="python3 bench.py --integrator bdpt --max-depth 5 --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  MCRT_WALK_CAP=0 timeout -k 10 300 $B > $P/off_$r.json 2> $P/off_$r.err || { tail -20 $P/off_$r.err; exit 6; }
  timeout -k 10 300 $B > $P/all_$r.json 2> $P/all_$r.err || { tail -20 $P/all_$r.err; exit 6; }
  MCRT_WALK_BDPT_MAXD=1 timeout -k 10 300 $B > $P/d1_$r.json 2> $P/d1_$r.err || { tail -20 $P/d1_$r.err; exit 6; }
  MCRT_WALK_BDPT_MAXD=2 timeout -k 10 300 $B > $P/d2_$r.json 2> $P/d2_$r.err || { tail -20 $P/d2_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/*.json
