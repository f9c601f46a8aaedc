#!/bin/bash
# round-2 GPU call 38: camera-ray launch on plain (MCRT_COMPACT_TRAV=0) vs descent-compact records (default) now
# that camera waves are packed (2 or 4 pixels x 32 or 16 frames)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab38
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for R in 1 2; do
  for V in 1 0; do
    for S in 20 96; do
      MCRT_COMPACT_TRAV=$V timeout -k 10 300 $B --steps $S > gpurun_out/ab38/c${V}_s${S}_$R.json 2> gpurun_out/ab38/c${V}_s${S}_$R.err || { echo "bench $V failed"; tail -5 gpurun_out/ab38/c${V}_s${S}_$R.err; exit 4; }
      python3 -c "import json; d=json.loads(open('gpurun_out/ab38/c${V}_s${S}_$R.json').read().strip().splitlines()[-1]); k=d['kernels']; print('compact=$V steps=$S', d['value'], d['ms_per_step'], k['k_primary']['avg_ms'], k['k_shadow_extend']['avg_ms'])"
    done
  done
done
