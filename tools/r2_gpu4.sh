#!/bin/bash
# occupancy probe: traversal kernels with 5 / 4 / 2.5 waves per SIMD (LDS padding)
cd /root/repo
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-roofline-model --steps 40"
for v in base pad4k pad6k pad12k; do
  if [ $v = base ]; then env=""; else env="MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so"; fi
  env $env timeout -k 10 300 $B > gpurun_out/occ_$v.json 2> gpurun_out/occ_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/occ_$v.err; exit 6; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/occ_$v.json')); print('$v', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
