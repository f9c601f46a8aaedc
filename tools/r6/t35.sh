#!/bin/bash
# round 6: the last-bounce shadow launch and the shadow part of k_shadow_extend as grid-stride launches of at
# most 65536 workgroups instead of capacity-sized grids (k_shadow_extend held at 8 waves per SIMD), against
# libmcrt_base.so: the stop-rule / hint / reference tests, then the PT and BDPT lines, alternating
export TMPDIR=/tmp
P=gpurun_out/r6t35; mkdir -p $P; rm -f $P/*.json
BASE=$PWD/monte-carlo-raytracer_amd/libmcrt_base.so
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py tests/test_gpu_shadow_hints.py tests/test_gpu_render.py tests/test_gpu_packets.py > $P/tests.log 2>&1 || { tail -30 $P/tests.log; exit 3; }
tail -1 $P/tests.log
F="--no-cpu-baseline --no-roofline-model --no-bdpt"
B="python3 bench.py --integrator bdpt --steps 32 --no-cpu-baseline --no-roofline-model"
for r in 1 2 3; do
  MCRT_LIB_PATH=$BASE timeout -k 10 300 python3 bench.py $F > $P/base_pt_$r.json 2> $P/base_pt_$r.err || { tail -20 $P/base_pt_$r.err; exit 4; }
  timeout -k 10 300 python3 bench.py $F > $P/new_pt_$r.json 2> $P/new_pt_$r.err || { tail -20 $P/new_pt_$r.err; exit 4; }
done
for r in 1 2; do
  MCRT_LIB_PATH=$BASE timeout -k 10 300 $B > $P/base_bdpt_$r.json 2> $P/base_bdpt_$r.err || { tail -20 $P/base_bdpt_$r.err; exit 4; }
  timeout -k 10 300 $B > $P/new_bdpt_$r.json 2> $P/new_bdpt_$r.err || { tail -20 $P/new_bdpt_$r.err; exit 4; }
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v.get("ms_per_frame", v) for n, v in k.items()})
PY
