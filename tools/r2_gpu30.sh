#!/bin/bash
# round-2 GPU call 30: first shading waves packed like the camera waves (MCRT_SHADE_PACK) -- parity, then A/B bench
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab30
timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_reference.py tests/test_gpu_compact_records.py \
  tests/test_gpu_texture_lod.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab30/pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/ab30/pytest.log; exit 3; }
tail -1 gpurun_out/ab30/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 48"
for V in 1 0 1 0; do
  MCRT_SHADE_PACK=$V timeout -k 10 200 $B > gpurun_out/ab30/b$V.json 2> gpurun_out/ab30/b$V.err || { echo "bench $V failed"; tail -5 gpurun_out/ab30/b$V.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab30/b$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('spack=$V', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in ('k_primary','k_shade0','k_shadow_extend','k_shadeN','k_shadow')})"
done
