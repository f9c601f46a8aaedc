#!/bin/bash
# round-2 GPU call 35: every BASELINE config with the current build (packed waves, power-of-two calls), and the
# thread scaling of the CPU baseline (oracle) on the box's CPU share
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/configs
C="--no-cpu-baseline --no-roofline-model --no-bdpt"
run() {  # name, args
  timeout -k 10 400 python3 bench.py $C $2 > gpurun_out/configs/$1.json 2> gpurun_out/configs/$1.err || { echo "$1 failed"; tail -10 gpurun_out/configs/$1.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/configs/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['triangles'], d['config']['frames_per_launch'])"
}
run config2_dragon_1080p_pt "--scene dragon_proxy --steps 64"
run config3_sponza_1080p_pt_1gpu "--scene sponza_proxy --steps 64"
run config5_smproxy_4k_sobol_pt_1gpu "--width 3840 --height 2160 --sampler sobol --steps 32"
run config4_smproxy_1080p_bdpt_1gpu "--integrator bdpt --steps 12"
run headline_smproxy_1080p_pt "--steps 96"
timeout -k 10 400 python3 tools/cpu_scaling.py 96 16 > gpurun_out/configs/cpu_scaling.json 2> gpurun_out/configs/cpu_scaling.err || { echo "cpu scaling failed"; tail -5 gpurun_out/configs/cpu_scaling.err; exit 5; }
cat gpurun_out/configs/cpu_scaling.err
