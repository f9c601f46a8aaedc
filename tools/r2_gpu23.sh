#!/bin/bash
# round-2 GPU call 23: every BASELINE config on one MI355X with the current build (1 spp per step)
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/configs
C="--no-cpu-baseline --no-roofline-model --no-bdpt"
run() {  # name, args
  timeout -k 10 400 python3 bench.py $C $2 > gpurun_out/configs/$1.json 2> gpurun_out/configs/$1.err || { echo "$1 failed"; tail -10 gpurun_out/configs/$1.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/configs/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['triangles'])"
}
run config2_dragon_1080p_pt "--scene dragon_proxy --steps 64"
run config3_sponza_1080p_pt_1gpu "--scene sponza_proxy --steps 64"
run config5_smproxy_4k_sobol_pt_1gpu "--width 3840 --height 2160 --sampler sobol --steps 16"
run config4_smproxy_1080p_bdpt_1gpu "--integrator bdpt --steps 12"
run headline_smproxy_1080p_pt "--steps 48"
