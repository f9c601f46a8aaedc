#!/bin/bash
# BDPT A/B: the in-tree library (B) vs tools/experiments/build/libmcrt_a.so (A); tests on B first.
export TMPDIR=/tmp
P=gpurun_out/bab
mkdir -p $P
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bdpt.py tests/test_gpu_reference_scale.py tests/test_gpu_golden_reference.py tests/test_gpu_two_level.py -k "bdpt or BDPT" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
tail -2 $P/tests.log
B="python3 bench.py --integrator bdpt --steps 20 --warmup 2 --no-cpu-baseline --no-roofline-model"
for v in B A B A; do
  if [ $v = A ]; then export MCRT_LIB_PATH=$PWD/tools/experiments/build/libmcrt_a.so; else unset MCRT_LIB_PATH; fi
  timeout -k 10 300 $B > $P/bench_$v.json 2> $P/bench_$v.err || { tail -20 $P/bench_$v.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d.get('kernels', {}).items()})"
done
