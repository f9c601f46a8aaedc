#!/bin/bash
# sibling-pair record order (MCRT_BVH_PAIRS=1): parity + A/B bench
cd /root/repo
export TMPDIR=/tmp
MCRT_BVH_PAIRS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_trace.py tests/test_gpu_render.py tests/test_gpu_reference.py tests/test_gpu_golden_reference.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bp_pytest.log 2>&1 || { echo "pairs parity failed"; tail -30 gpurun_out/bp_pytest.log; exit 3; }
tail -1 gpurun_out/bp_pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 32"
for V in 0 1 0 1; do
  MCRT_BVH_PAIRS=$V timeout -k 10 200 $B > gpurun_out/bp_bench$V.json 2> gpurun_out/bp_bench$V.err || { echo "bench $V failed"; tail -5 gpurun_out/bp_bench$V.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bp_bench$V.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('pairs=$V', d['value'], d['ms_per_step'], {n: k[n]['avg_ms'] for n in ('k_primary','k_shadow_extend','k_shadow')})"
done
