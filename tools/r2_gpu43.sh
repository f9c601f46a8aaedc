#!/bin/bash
# round-2 GPU call 43: BDPT (config 4) frames in flight 2 (auto) vs 3 vs 4
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab43
B="python3 bench.py --no-cpu-baseline --no-roofline-model --integrator bdpt --steps 24 --no-kernel-timing"
for R in 1 2; do
  for V in 2 3 4; do
    MCRT_FRAMES_IN_FLIGHT=$V timeout -k 10 300 $B > gpurun_out/ab43/f${V}_$R.json 2> gpurun_out/ab43/f${V}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab43/f${V}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab43/f${V}_$R.json').read().strip().splitlines()[-1]); print('bdpt fif=$V', d['value'], d['ms_per_step'])"
  done
done
