#!/bin/bash
# round 6: BDPT tests, then the BDPT bench line twice (connect A/B against earlier records)
export TMPDIR=/tmp
P=gpurun_out/r6t4; mkdir -p $P; rm -f $P/*.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_bdpt.py tests/test_gpu_quant_nodes.py -k "bdpt" -x -v --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
B="python3 bench.py --integrator bdpt --steps 32 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  timeout -k 10 300 $B > $P/b_$r.json 2> $P/b_$r.err || { tail -20 $P/b_$r.err; exit 4; }
  for v in "$@"; do   # variant libraries libmcrt_<v>.so (tools/build_variant.sh)
    MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so timeout -k 10 300 $B > $P/${v}_$r.json 2> $P/${v}_$r.err || { tail -20 $P/${v}_$r.err; exit 4; }
  done
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], {n: v["ms_per_frame"] for n, v in k.items()})
PY
