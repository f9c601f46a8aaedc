#!/bin/bash
# round-2 GPU call 19: treelet records (MCRT_TREELET) -- parity with every launch on them, then A/B bench
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
MCRT_TREELET=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_trace.py tests/test_gpu_render.py tests/test_gpu_reference.py \
  tests/test_gpu_golden_reference.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p19_pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/p19_pytest.log; exit 3; }
tail -1 gpurun_out/p19_pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 32"
for V in 1 0 1 0; do
  MCRT_TREELET=$V timeout -k 10 200 $B > gpurun_out/p19_bench$V.json 2> gpurun_out/p19_bench$V.err || { echo "bench $V failed"; tail -5 gpurun_out/p19_bench$V.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/p19_bench$V.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('treelet=$V', d['value'], d['ms_per_step'], {n: k[n]['avg_ms'] for n in ('k_primary','k_shadow_extend','k_shadow','k_shade0','k_shadeN')})"
done
