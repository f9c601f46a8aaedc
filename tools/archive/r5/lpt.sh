# longest-first camera / first-shading tile order (MCRT_LONGEST_FIRST) at N = 1 / 8 (emulated), twice,
# and the launch tails with it on (tools/wave_tail.py)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5lpt}; mkdir -p $P
E="python3 tools/scale_emulate.py --ns 1,8 --steps 20 --chunks 20 --kernels"
for r in 1 2; do
  MCRT_LONGEST_FIRST=0 timeout -k 10 400 $E > $P/off_$r.json 2> $P/off_$r.err || { tail -20 $P/off_$r.err; exit 4; }
  timeout -k 10 400 $E > $P/on_$r.json 2> $P/on_$r.err || { tail -20 $P/on_$r.err; exit 4; }
done
MCRT_WAVE_CLOCK=1 timeout -k 10 400 python3 tools/wave_tail.py --ns 1,8 > $P/wt_on.json 2> $P/wt_on.err || { tail -20 $P/wt_on.err; exit 4; }
python3 - $P <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/o*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: (v["max_ms"], v["compute_eff"], {a: b for a, b in v["rank0_kernel_ms_per_frame"].items() if a in ("k_primary", "k_shade0", "k_shadow_extend")}) for k, v in d["per_n"].items()})
d = json.loads(open(sys.argv[1] + "/wt_on.json").read().strip().splitlines()[-1])
for n, v in d["per_n"].items():
    for k, s in v.items():
        print(n, k, s["span_us"], s["after_99pct_done_us"], s["mean_in_flight_last10pct"])
PY
