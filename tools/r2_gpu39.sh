#!/bin/bash
# round-2 GPU call 39: bounce-0 shadow rays on the descent-compact records (MCRT_SHADOW_COMPACT=1; the extension
# rays of the same launch keep the plain records) -- parity with the knob on, then A/B
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab39
MCRT_SHADOW_COMPACT=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_reference.py tests/test_gpu_compact_records.py \
  tests/test_gpu_golden_reference.py tests/test_gpu_trace.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab39/pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/ab39/pytest.log; exit 3; }
tail -1 gpurun_out/ab39/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for R in 1 2; do
  for V in 1 0; do
    for S in 20 96; do
      MCRT_SHADOW_COMPACT=$V timeout -k 10 300 $B --steps $S > gpurun_out/ab39/s${V}_s${S}_$R.json 2> gpurun_out/ab39/s${V}_s${S}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab39/s${V}_s${S}_$R.err; exit 4; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ab39/s${V}_s${S}_$R.json').read().strip().splitlines()[-1]); k=d['kernels']; print('shadow_compact=$V steps=$S', d['value'], d['ms_per_step'], k['k_primary']['avg_ms'], k['k_shadow_extend']['avg_ms'])"
    done
  done
done
