# timing-only A/B: the shading's surfBase[shape] lookup removed (wrong images; the dependent load's cost)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5nosb}; mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_nosb.so
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$V timeout -k 10 300 $B > $P/nosb_$r.json 2> $P/nosb_$r.err || { tail -20 $P/nosb_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/nosb_*.json
