#!/bin/bash
# A/B of two in-tree builds of libmcrt on the headline bench (alternating runs):
# tools/r3/gpu_libab.sh <libB path> [runs] [extra bench args]
mkdir -p gpurun_out/libab
B="python bench.py --no-cpu-baseline --no-roofline-model --no-bdpt $3"
R=${2:-2}
for r in $(seq 1 $R); do
  timeout -k 10 300 $B > gpurun_out/libab/A$r.json 2> gpurun_out/libab/A$r.err || { tail -20 gpurun_out/libab/A$r.err; exit 4; }
  MCRT_LIB_PATH=$1 timeout -k 10 300 $B > gpurun_out/libab/B$r.json 2> gpurun_out/libab/B$r.err || { tail -20 gpurun_out/libab/B$r.err; exit 4; }
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/libab/*.json")):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], {k: round(v["avg_ms"], 4) for k, v in d.get("kernels", {}).items()})
PY
