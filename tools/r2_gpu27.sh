#!/bin/bash
# round-2 GPU call 27: frames per launch 16 / 32 with packed waves
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab27
timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab27/pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/ab27/pytest.log; exit 3; }
tail -1 gpurun_out/ab27/pytest.log
for V in 16 32 16 32; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 96 --batch $V > gpurun_out/ab27/b$V.json 2> gpurun_out/ab27/b$V.err || { echo "bench $V failed"; tail -5 gpurun_out/ab27/b$V.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab27/b$V.json').read().strip().splitlines()[-1]); print('batch=$V', d['value'], d['ms_per_step'])"
done
