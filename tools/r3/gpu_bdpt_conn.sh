#!/bin/bash
# BDPT per-strategy connect: parity suites touching BDPT, then the bench's BDPT object.
export TMPDIR=/tmp
mkdir -p gpurun_out/bc
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bdpt.py tests/test_gpu_reference_scale.py tests/test_gpu_golden_reference.py tests/test_gpu_two_level.py -k "bdpt or BDPT" > gpurun_out/bc/tests.log 2>&1 || { tail -40 gpurun_out/bc/tests.log; exit 3; }
tail -3 gpurun_out/bc/tests.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-roofline-model > gpurun_out/bc/bench.json 2> gpurun_out/bc/bench.err || { tail -20 gpurun_out/bc/bench.err; exit 4; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bc/bench.json").read().strip().splitlines()[-1])
print("PT", d["value"], d["ms_per_step"])
b = d.get("bdpt", {})
print("BDPT", b.get("value"), b.get("ms_per_step"), json.dumps(b.get("kernels", {}))[:900])
PY
