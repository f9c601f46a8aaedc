#!/bin/bash
# round 6: k_bdpt_vertex in 512-thread workgroups (its two queue appends per workgroup: half as many
# atomics on the queue counters) against 256 (libmcrt_base.so): BDPT tests, then the BDPT line at D = 2
# and 5, alternating, 2 runs each
export TMPDIR=/tmp
P=gpurun_out/r6t38; mkdir -p $P; rm -f $P/*.json
BASE=$PWD/monte-carlo-raytracer_amd/libmcrt_base.so
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py tests/test_gpu_reference_scale.py tests/test_gpu_packets.py -k "bdpt or BDPT" > $P/tests.log 2>&1 || { tail -30 $P/tests.log; exit 3; }
tail -1 $P/tests.log
for D in 2 5; do
  B="python3 bench.py --integrator bdpt --max-depth $D --steps 32 --no-cpu-baseline --no-roofline-model"
  for r in 1 2; do
    MCRT_LIB_PATH=$BASE timeout -k 10 300 $B > $P/base_d${D}_$r.json 2> $P/base_d${D}_$r.err || { tail -20 $P/base_d${D}_$r.err; exit 4; }
    timeout -k 10 300 $B > $P/new_d${D}_$r.json 2> $P/new_d${D}_$r.err || { tail -20 $P/new_d${D}_$r.err; exit 4; }
  done
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
