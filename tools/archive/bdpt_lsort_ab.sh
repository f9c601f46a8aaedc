mkdir -p gpurun_out/lsort
B="python3 bench.py --integrator bdpt --steps 16 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  for v in ${LSORT_VARIANTS:-0 1 3}; do
    MCRT_BDPT_LIGHT_SORT=$v timeout -k 10 300 $B > gpurun_out/lsort/v${v}_$r.json 2> gpurun_out/lsort/v${v}_$r.err || { tail -20 gpurun_out/lsort/v${v}_$r.err; exit 4; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lsort/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], {k: round(v["ms_per_frame"], 4) for k, v in d.get("kernels", {}).items()})
PY
