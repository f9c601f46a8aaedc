#!/bin/bash
# every BASELINE config on one MI355X with this round's build (1 spp per step)
P=gpurun_out/${CFG_DIR:-cfg3}
mkdir -p $P
F="--no-cpu-baseline --no-roofline-model --no-bdpt"
run() { n=$1; shift; timeout -k 10 400 python3 bench.py $F "$@" > $P/$n.json 2> $P/$n.err || { tail -20 $P/$n.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/$n.json').read().strip().splitlines()[-1])
print('$n', d['value'], d['ms_per_step'], d['config'].get('frames_per_launch'))"; }
run dragon_1080p --scene dragon_proxy --tris 871414 --steps 96
run sponza_1080p --scene sponza_proxy --steps 96
run sm_bdpt_1080p --integrator bdpt --steps 32
run sm_sobol_4k --width 3840 --height 2160 --sampler sobol --steps 32
run sm_1080p_96 --steps 96
