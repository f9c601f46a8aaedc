#!/bin/bash
# BDPT frames per call with the current build: 8 (default) vs 16 vs 4, alternating runs
export TMPDIR=/tmp
P=gpurun_out/bb2
mkdir -p $P
B="python3 bench.py --integrator bdpt --steps 16 --warmup 2 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  for b in 8 16 4; do
    timeout -k 10 300 $B --bdpt-batch $b > $P/b${b}_$r.json 2> $P/b${b}_$r.err || { tail -20 $P/b${b}_$r.err; exit 4; }
    python3 -c "
import json
d = json.loads(open('$P/b${b}_$r.json').read().strip().splitlines()[-1])
print('batch $b run $r', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
  done
done
