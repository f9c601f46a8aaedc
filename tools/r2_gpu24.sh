#!/bin/bash
# round-2 GPU call 24: compact records in every launch (MCRT_COMPACT_TRAV=2) vs camera rays only (=1) on the
# cache-resident trees (Dragon 111 MB, Sponza 33 MB of records) and the SM proxy
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab24
C="--no-cpu-baseline --no-roofline-model --no-bdpt"
for S in "dragon_proxy --steps 64" "sponza_proxy --steps 64"; do
  for V in 2 1 2 1; do
    n=$(echo $S | cut -d' ' -f1)
    MCRT_COMPACT_TRAV=$V timeout -k 10 300 python3 bench.py $C --scene $S > gpurun_out/ab24/${n}_$V.json 2> gpurun_out/ab24/${n}_$V.err || { echo "$n $V failed"; tail -5 gpurun_out/ab24/${n}_$V.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab24/${n}_$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$n compact=$V', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in ('k_primary','k_shadow_extend','k_shadow')})"
  done
done
