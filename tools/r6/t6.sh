#!/bin/bash
# round 6: BDPT at maxDepth 5, round-5 library vs this tree (the connect changes)
export TMPDIR=/tmp
P=gpurun_out/r6t6; mkdir -p $P; rm -f $P/*.json
B="python3 bench.py --integrator bdpt --max-depth 5 --steps 32 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_r05.so timeout -k 10 300 $B > $P/r05_$r.json 2> $P/r05_$r.err || { tail -20 $P/r05_$r.err; exit 4; }
  timeout -k 10 300 $B > $P/b_$r.json 2> $P/b_$r.err || { tail -20 $P/b_$r.err; exit 4; }
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
