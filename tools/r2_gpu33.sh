#!/bin/bash
# round-2 GPU call 33: extension-queue order with packed waves -- no sort vs the Morton+octant sort vs a
# stable octant-only sort (MCRT_SORT_KEY=octant); one frame slot everywhere (the sort forces it)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab33
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --steps 64"
run() {   # name, env...
  n=$1; shift
  env "$@" timeout -k 10 240 $B > gpurun_out/ab33/$n.json 2> gpurun_out/ab33/$n.err || { echo "$n failed"; tail -5 gpurun_out/ab33/$n.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab33/$n.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$n', d['value'], d['ms_per_step'], {x: k[x]['avg_ms'] for x in k})"
}
for R in 1 2; do
  run nosort_$R MCRT_FRAMES_IN_FLIGHT=1
  run morton_$R MCRT_SORT_RAYS=1
  run octant_$R MCRT_SORT_RAYS=1 MCRT_SORT_KEY=octant
done
