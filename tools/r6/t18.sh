#!/bin/bash
# round 6: camera waves of whole pixels x every frame for a 20-frame call (3 pixels + 4 idle lanes per
# wave instead of 64 consecutive (pixel, frame) paths spanning 4 pixels; MCRT_CAMERA_WHOLE_PIXELS=1)
# against the consecutive packing (=0): packet + full-size reference tests, then the PT line alternating
export TMPDIR=/tmp
P=gpurun_out/r6t18; mkdir -p $P; rm -f $P/*.json
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_packets.py tests/test_gpu_reference_scale.py tests/test_gpu_quant_nodes.py -k "not bdpt and not BDPT" > $P/tests.log 2>&1 || { tail -30 $P/tests.log; exit 3; }
tail -1 $P/tests.log
F="--no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2 3; do
  MCRT_CAMERA_WHOLE_PIXELS=0 timeout -k 10 300 python3 bench.py $F > $P/off_$r.json 2> $P/off_$r.err || { tail -20 $P/off_$r.err; exit 4; }
  MCRT_CAMERA_WHOLE_PIXELS=1 timeout -k 10 300 python3 bench.py $F > $P/on_$r.json 2> $P/on_$r.err || { tail -20 $P/on_$r.err; exit 4; }
done
timeout -k 10 400 python3 bench.py --no-bdpt --no-roofline-model > $P/on_parity.json 2> $P/on_parity.err || { tail -20 $P/on_parity.err; exit 4; }
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("parity_vs_reference", {}).get("pixels_bit_exact"), {n: v.get("ms_per_frame", v) for n, v in k.items()})
PY
