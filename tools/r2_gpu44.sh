#!/bin/bash
# round-2 GPU call 44: at 20 steps with packing for any count, one 20-frame call vs two overlapping sequences
# (10 + 10, 12 + 8) on the two frame slots
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab44
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing --steps 20"
for R in 1 2 3; do
  for V in 32 10 12,8; do
    n=$(echo $V | tr , _)
    timeout -k 10 200 $B --chunks $V > gpurun_out/ab44/c${n}_$R.json 2> gpurun_out/ab44/c${n}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab44/c${n}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab44/c${n}_$R.json').read().strip().splitlines()[-1]); print('chunks=$V', d['value'], d['ms_per_step'])"
  done
done
