#!/bin/bash
# round-2 GPU call 45: wave-uniform compact-record fetches through the scalar cache in the camera-ray launch
# (libmcrt_usl.so = -DMCRT_UNIFORM_SLOAD=1, selected with MCRT_LIB_PATH) -- parity with it, then A/B
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab45
V=$PWD/monte-carlo-raytracer_amd/libmcrt_usl.so
MCRT_LIB_PATH=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_reference.py tests/test_gpu_compact_records.py \
  tests/test_gpu_golden_reference.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab45/pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/ab45/pytest.log; exit 3; }
tail -1 gpurun_out/ab45/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 20"
for R in 1 2; do
  for L in base usl; do
    if [ $L = usl ]; then export MCRT_LIB_PATH=$V; else unset MCRT_LIB_PATH; fi
    timeout -k 10 300 $B > gpurun_out/ab45/${L}_$R.json 2> gpurun_out/ab45/${L}_$R.err || { echo "bench $L failed"; tail -5 gpurun_out/ab45/${L}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab45/${L}_$R.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$L', d['value'], d['ms_per_step'], k['k_primary']['avg_ms'], k['k_shadow_extend']['avg_ms'])"
  done
done
