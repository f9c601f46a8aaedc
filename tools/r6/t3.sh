#!/bin/bash
# round 6: BDPT tests, then A/B on the BDPT bench line: the round-5 library (r05) vs this tree with
# MCRT_BDPT_CONNECT = classes | tile
export TMPDIR=/tmp
P=gpurun_out/r6t3; mkdir -p $P; rm -f $P/*.json
for m in classes tile; do
MCRT_BDPT_CONNECT=$m timeout -k 10 600 python -u -m pytest tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py -k "bdpt" -x -v --timeout 300 --timeout-method thread > $P/pytest_$m.log 2>&1 || { tail -30 $P/pytest_$m.log; exit 3; }
tail -1 $P/pytest_$m.log
done
B="python3 bench.py --integrator bdpt --steps 32 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_r05.so timeout -k 10 300 $B > $P/r05_$r.json 2> $P/r05_$r.err || { tail -20 $P/r05_$r.err; exit 4; }
  for m in classes tile; do
    MCRT_BDPT_CONNECT=$m timeout -k 10 300 $B > $P/${m}_$r.json 2> $P/${m}_$r.err || { tail -20 $P/${m}_$r.err; exit 4; }
  done
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
