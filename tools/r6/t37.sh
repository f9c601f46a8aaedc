#!/bin/bash
# round 6: GENERAL strategies with a wave per (tile, t) running every s of that t, each strategy fetching the
# camera vertex again from the caches (MCRT_BDPT_GEN_BY_CAMERA=1; 199 VGPRs) against a wave per strategy:
# BDPT tests with the grouping, then a bench A/B at depth 5 and 4
export TMPDIR=/tmp
P=gpurun_out/r6t37; mkdir -p $P; rm -f $P/*.json
MCRT_BDPT_GEN_BY_CAMERA=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py -k "bdpt or BDPT" > $P/tests.log 2>&1 || { tail -30 $P/tests.log; exit 3; }
tail -3 $P/tests.log
for D in 5 4; do
  B="python3 bench.py --integrator bdpt --max-depth $D --steps 32 --no-cpu-baseline --no-roofline-model"
  for r in 1 2; do
    MCRT_BDPT_GEN_BY_CAMERA=0 timeout -k 10 300 $B > $P/off_d${D}_$r.json 2> $P/off_d${D}_$r.err || { tail -20 $P/off_d${D}_$r.err; exit 4; }
    MCRT_BDPT_GEN_BY_CAMERA=1 timeout -k 10 300 $B > $P/on_d${D}_$r.json 2> $P/on_d${D}_$r.err || { tail -20 $P/on_d${D}_$r.err; exit 4; }
  done
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
