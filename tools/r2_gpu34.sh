#!/bin/bash
# round-2 GPU call 34: batched-frame parity at 4 / 16 / 32 frames per call, then the order of the calls at the
# driver's step count (--steps 20): 16 + 4 (default) vs 4 + 16 vs 8 + 8 + 4 vs 4 x 5
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab34
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/ab34/pytest.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/ab34/pytest.log; exit 3; }
tail -1 gpurun_out/ab34/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing --steps 20 --warmup 5"
for R in 1 2; do
  for V in 16 4,16 8 4; do
    n=$(echo $V | tr , _)
    timeout -k 10 200 $B --chunks $V > gpurun_out/ab34/c${n}_$R.json 2> gpurun_out/ab34/c${n}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab34/c${n}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab34/c${n}_$R.json').read().strip().splitlines()[-1]); print('chunks=$V', d['value'], d['ms_per_step'])"
  done
done
