#!/bin/bash
# leaf-pop prefetch A/B: parity (trace + full-size reference frames) on the new build, then the PT bench
# new (in-tree) vs base (tools/experiments/build/libmcrt_base.so), alternating
export TMPDIR=/tmp
P=gpurun_out/pf
mkdir -p $P
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_trace.py tests/test_gpu_reference_scale.py tests/test_gpu_sah_build.py tests/test_gpu_compact_records.py > $P/tests.log 2>&1 || { tail -30 $P/tests.log; exit 3; }
tail -2 $P/tests.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for v in new base new base; do
  if [ $v = base ]; then export MCRT_LIB_PATH=$PWD/tools/experiments/build/libmcrt_base.so; else unset MCRT_LIB_PATH; fi
  timeout -k 10 400 $B > $P/bench_$v.json 2> $P/bench_$v.err || { tail -20 $P/bench_$v.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d.get('kernels', {}).items()})"
done
