#!/bin/bash
# round-2 GPU call 40: per-rank compute of the tile split at the driver's 20 steps, emulated on one GPU, for the
# call plans 32 (-> 16 + 4, bench.py's default), 8 (-> 8 + 8 + 4) and 4 (-> 4 x 5); 2 frame slots
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab40
for P in 32 8 4; do
  timeout -k 10 400 python3 tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --fif 2 --chunks $P > gpurun_out/ab40/plan$P.json 2> gpurun_out/ab40/plan$P.err || { echo "plan $P failed"; tail -5 gpurun_out/ab40/plan$P.err; exit 4; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab40/plan$P.json')); print('plan $P', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
done
