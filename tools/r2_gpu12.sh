#!/bin/bash
# frames-per-launch x frames-in-flight sweep of the PT headline (no profiling in the timed region)
cd /root/repo
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing --steps 48 --warmup 16"
for FIF in 2 3 4; do
  for BT in 2 4 8 16; do
    MCRT_FRAMES_IN_FLIGHT=$FIF timeout -k 10 200 $B --batch $BT > gpurun_out/sw_${FIF}_${BT}.json 2> gpurun_out/sw_${FIF}_${BT}.err || { echo "fif $FIF batch $BT failed"; tail -5 gpurun_out/sw_${FIF}_${BT}.err; exit 4; }
    python3 -c "import json; d=json.loads(open('gpurun_out/sw_${FIF}_${BT}.json').read().strip().splitlines()[-1]); print('fif $FIF batch $BT', d['value'], d['ms_per_step'])"
  done
done
