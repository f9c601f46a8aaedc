# N = 1 / 8 per-rank compute (emulated): one 20-frame call vs two staggered 10-frame calls on two slots
export TMPDIR=/tmp
P=gpurun_out/${1:-r5stagger}; mkdir -p $P
E="python3 tools/scale_emulate.py --ns 1,8 --steps 20 --kernels"
timeout -k 10 400 $E --chunks 20 > $P/c20.json 2> $P/c20.err || { tail -20 $P/c20.err; exit 4; }
timeout -k 10 400 $E --chunks 10 --fif 2 > $P/c10_stagger.json 2> $P/c10_stagger.err || { tail -20 $P/c10_stagger.err; exit 4; }
MCRT_STAGGER_CALLS=0 timeout -k 10 400 $E --chunks 10 --fif 2 > $P/c10_nostagger.json 2> $P/c10_nostagger.err || { tail -20 $P/c10_nostagger.err; exit 4; }
timeout -k 10 400 $E --chunks 7,7,6 --fif 2 > $P/c7_stagger.json 2> $P/c7_stagger.err || { tail -20 $P/c7_stagger.err; exit 4; }
python3 - $P <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective")) for k, v in d["per_n"].items()})
PY
