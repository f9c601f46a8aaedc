#!/bin/bash
# A/B of the traversal tree on the headline bench: tools/r3/gpu_ab.sh "<extra bench args A>" "<extra args B>" [runs]
mkdir -p gpurun_out/ab
B="python bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
R=${3:-1}
for r in $(seq 1 $R); do
  for v in A B; do
    args=$1; [ $v = B ] && args=$2
    timeout -k 10 300 $B $args > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.err || { tail -20 gpurun_out/ab/$v$r.err; exit 4; }
  done
done
python - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/ab/*.json")):
    d = json.load(open(f))
    print(f, d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d.get("kernels", {}).items()})
PY
