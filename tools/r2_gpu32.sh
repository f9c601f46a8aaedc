#!/bin/bash
# round-2 GPU call 32: frames per launch at the driver's step count (--steps 20 --warmup 5): one 20-frame
# sequence (auto 32) vs sequences that leave the second frame slot something to overlap
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab32
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing --steps 20 --warmup 5"
for R in 1 2; do
  for V in 0 10 16 7; do
    timeout -k 10 200 $B --batch $V > gpurun_out/ab32/b${V}_$R.json 2> gpurun_out/ab32/b${V}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab32/b${V}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab32/b${V}_$R.json').read().strip().splitlines()[-1]); print('batch=$V', d['value'], d['ms_per_step'], d['config']['frames_per_launch'])"
  done
done
for V in 0 16; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing --steps 96 --warmup 5 --batch $V > gpurun_out/ab32/s96_b$V.json 2> gpurun_out/ab32/s96_b$V.err || { echo "bench96 $V failed"; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab32/s96_b$V.json').read().strip().splitlines()[-1]); print('steps96 batch=$V', d['value'], d['ms_per_step'])"
done
