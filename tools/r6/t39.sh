#!/bin/bash
# round 6: the whole GPU suite + smoke on the exact final tree, then the driver's default bench line and
# the BDPT line at D = 2 and 5
export TMPDIR=/tmp
P=gpurun_out/r6t39; mkdir -p $P
bash tools/gpu_task.sh suite r6t39 || exit $?
bash tools/gpu_task.sh bench r6t39 || exit $?
F="--no-cpu-baseline --no-roofline-model"
timeout -k 10 300 python3 bench.py --integrator bdpt --steps 32 $F > $P/bdpt_d2.json 2> $P/bdpt_d2.err || { tail -20 $P/bdpt_d2.err; exit 4; }
timeout -k 10 300 python3 bench.py --integrator bdpt --max-depth 5 --steps 32 $F > $P/bdpt_d5.json 2> $P/bdpt_d5.err || { tail -20 $P/bdpt_d5.err; exit 4; }
python3 - $P/bdpt_d2.json $P/bdpt_d5.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in d.get("kernels", {}).items()})
PY
