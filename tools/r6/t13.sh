#!/bin/bash
# round 6: GENERAL strategies phased (the light vertex's material terms, then the camera vertex's, with the
# MIS pdfs: one material in registers at a time; MCRT_BDPT_GEN_PHASED=1, 138 VGPRs) and phased + capped at
# 4 waves per SIMD (=2, 128 VGPRs + 32 B scratch) against the original order (=0, 153 VGPRs): BDPT tests
# with 1 and 2, then a bench A/B at depth 2 and 5
export TMPDIR=/tmp
P=gpurun_out/r6t13; mkdir -p $P; rm -f $P/*.json
for v in 1 2; do
  MCRT_BDPT_GEN_PHASED=$v timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py -k "bdpt or BDPT" > $P/tests_$v.log 2>&1 || { tail -30 $P/tests_$v.log; exit 3; }
  tail -1 $P/tests_$v.log
done
for D in 2 5; do
  B="python3 bench.py --integrator bdpt --max-depth $D --steps 32 --no-cpu-baseline --no-roofline-model"
  for r in 1 2; do
    for v in 0 1 2; do
      MCRT_BDPT_GEN_PHASED=$v timeout -k 10 300 $B > $P/v${v}_d${D}_$r.json 2> $P/v${v}_d${D}_$r.err || { tail -20 $P/v${v}_d${D}_$r.err; exit 4; }
    done
  done
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
