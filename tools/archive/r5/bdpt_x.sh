# band-split BDPT per rank (emulated, 16 frames per call): sparse vs dense splat exchange, N = 1/2/4/8
export TMPDIR=/tmp
P=gpurun_out/${1:-r5bx}; mkdir -p $P
for x in sparse dense; do
  timeout -k 10 600 python3 tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 32 --batch 16 --splat-exchange $x > $P/$x.json 2> $P/$x.err || { tail -20 $P/$x.err; exit 4; }
done
python3 - $P <<'PY'
import json, sys
for x in ("sparse", "dense"):
    d = json.loads(open(sys.argv[1] + "/" + x + ".json").read().strip().splitlines()[-1])
    print(x, {k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective"), v["splat_exchange"].get("bytes_per_rank_per_frame")) for k, v in d["per_n"].items()})
PY
