# A/B: closest-hit packet leaves with the OR-ed miss test (scalar masks) vs the select chain
export TMPDIR=/tmp
P=gpurun_out/${1:-r5leafor}; mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_leafor.so
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$V timeout -k 10 300 $B > $P/leafor_$r.json 2> $P/leafor_$r.err || { tail -20 $P/leafor_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/leafor_*.json
