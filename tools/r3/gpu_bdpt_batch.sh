#!/bin/bash
# batched BDPT: parity suites touching BDPT, then --integrator bdpt at 1 / 2 / 4 / 8 frames per call
export TMPDIR=/tmp
P=gpurun_out/bb
mkdir -p $P
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bdpt.py tests/test_gpu_reference_scale.py tests/test_gpu_golden_reference.py tests/test_gpu_two_level.py -k "bdpt or BDPT" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
tail -2 $P/tests.log
for b in 1 2 4 8; do
  timeout -k 10 300 python3 bench.py --integrator bdpt --steps 16 --warmup 2 --bdpt-batch $b --no-cpu-baseline --no-roofline-model > $P/bench_$b.json 2> $P/bench_$b.err || { tail -20 $P/bench_$b.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$b.json').read().strip().splitlines()[-1])
print('batch $b', d['value'], d['ms_per_step'], {k: v.get('ms_per_frame', round(v['avg_ms'] * v['launches'] / 2, 4)) for k, v in d.get('kernels', {}).items()})"
done
