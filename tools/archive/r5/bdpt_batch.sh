# band-split BDPT per rank (emulated) at 8 / 16 / 32 frames per call, N = 1 / 8
export TMPDIR=/tmp
P=gpurun_out/${1:-r5bb}; mkdir -p $P
for b in 8 16 32; do
  timeout -k 10 500 python3 tools/scale_emulate.py --integrator bdpt --ns 1,8 --steps 32 --batch $b > $P/b$b.json 2> $P/b$b.err || { tail -20 $P/b$b.err; exit 4; }
done
python3 - $P <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: (v["max_ms"], v["compute_eff"], v["eff_with_collective"], v["eff_with_collective_serial"]) for k, v in d["per_n"].items()})
PY
