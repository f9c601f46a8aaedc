#!/bin/bash
# round-2 GPU call 25: BDPT occupancy variants (k_bdpt_connect 228 VGPRs -> 2 waves/SIMD; k_bdpt_vertex 112)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab25
B="python3 bench.py --integrator bdpt --steps 12 --no-cpu-baseline --no-roofline-model"
for V in base cw3 cw4 vw6 base cw3 cw4 vw6; do
  L=""; [ $V != base ] && L="MCRT_LIB_PATH=monte-carlo-raytracer_amd/libmcrt_$V.so"
  env $L timeout -k 10 200 $B > gpurun_out/ab25/$V.json 2> gpurun_out/ab25/$V.err || { echo "$V failed"; tail -5 gpurun_out/ab25/$V.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab25/$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$V', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in ('k_extend','k_bdpt_vertex','k_bdpt_connect','k_bdpt_vis')})"
done
