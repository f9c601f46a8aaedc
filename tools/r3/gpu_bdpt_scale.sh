#!/bin/bash
# band-split BDPT per rank at N = 1 / 8 with 1 / 4 / 8 frames per call (emulated on one GPU)
mkdir -p gpurun_out/scale
for b in 1 4 8; do
  timeout -k 10 400 python tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 16 --batch $b > gpurun_out/scale/bdpt_b$b.json 2> gpurun_out/scale/bdpt_b$b.err || { tail -5 gpurun_out/scale/bdpt_b$b.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/scale/bdpt_b$b.json')); print('batch $b', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
done
