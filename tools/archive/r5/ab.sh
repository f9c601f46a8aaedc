# A/B of the compact records: bench (PT + BDPT objects, no CPU legs) with and without, twice
export TMPDIR=/tmp
P=gpurun_out/${1:-r5ab}; mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 400 $B > $P/q1_$r.json 2> $P/q1_$r.err || { tail -20 $P/q1_$r.err; exit 4; }
  MCRT_QUANT_NODES=0 timeout -k 10 400 $B > $P/q0_$r.json 2> $P/q0_$r.err || { tail -20 $P/q0_$r.err; exit 4; }
done
python3 tools/bench_summary.py $P/q1_*.json $P/q0_*.json
