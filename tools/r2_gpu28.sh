#!/bin/bash
# round-2 GPU call 28: XCD run length (MCRT_XCD_SEG) with the tile-major order
cd /root/repo
mkdir -p gpurun_out/ab28
for V in base seg64 seg256 seg512 base seg64 seg256 seg512; do
  L=""; [ $V != base ] && L="MCRT_LIB_PATH=monte-carlo-raytracer_amd/libmcrt_$V.so"
  env $L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 64 > gpurun_out/ab28/$V.json 2> gpurun_out/ab28/$V.err || { echo "$V failed"; tail -5 gpurun_out/ab28/$V.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab28/$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$V', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in ('k_primary','k_shadow_extend','k_shadow')})"
done
