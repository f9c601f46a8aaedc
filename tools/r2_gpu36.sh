#!/bin/bash
# round-2 GPU call 36: BDPT (config 4) with descent-compact records in every launch (MCRT_COMPACT_TRAV=2) vs the
# default (camera-ray launch of PT only; BDPT traces on the plain records)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab36
B="python3 bench.py --no-cpu-baseline --no-roofline-model --integrator bdpt --steps 16"
for R in 1 2; do
  for V in 1 2; do
    MCRT_COMPACT_TRAV=$V timeout -k 10 300 $B > gpurun_out/ab36/c${V}_$R.json 2> gpurun_out/ab36/c${V}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab36/c${V}_$R.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab36/c${V}_$R.json').read().strip().splitlines()[-1]); k=d['kernels']; print('compact=$V', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in k})"
  done
done
