#!/bin/bash
# scalar-cache node loads for wave-uniform steps: parity + A/B bench
cd /root/repo
export TMPDIR=/tmp
L=/root/repo/monte-carlo-raytracer_amd
MCRT_LIB_PATH=$L/libmcrt_sc1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_trace.py tests/test_gpu_render.py tests/test_gpu_reference.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sc_pytest.log 2>&1 || { echo "sc1 parity failed"; tail -30 gpurun_out/sc_pytest.log; exit 3; }
tail -1 gpurun_out/sc_pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 20"
for V in "" _sc1 "" _sc1; do
  if [ -n "$V" ]; then export MCRT_LIB_PATH=$L/libmcrt$V.so; else unset MCRT_LIB_PATH; fi
  timeout -k 10 200 $B > gpurun_out/sc_bench$V.json 2> gpurun_out/sc_bench$V.err || { echo "bench $V failed"; tail -5 gpurun_out/sc_bench$V.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sc_bench$V.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('${V:-base}', d['value'], d['ms_per_step'], {n: k[n]['avg_ms'] for n in ('k_primary','k_shadow_extend','k_shadow')})"
done
