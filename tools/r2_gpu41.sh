#!/bin/bash
# round-2 GPU call 41: packed waves for ANY frames-per-call count (wave = 64 consecutive (pixel, frame) paths of a
# tile, frames fastest) -- parity, then one 20-frame call vs 16 + 4 at 20 steps, 24 x 4 vs 32 x 3 at 96 steps, and
# the per-rank emulation with one 20-frame call
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/ab41
timeout -k 10 500 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_reference.py tests/test_gpu_compact_records.py \
  tests/test_gpu_texture_lod.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ab41/pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/ab41/pytest.log; exit 3; }
tail -1 gpurun_out/ab41/pytest.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --no-kernel-timing"
run() {  # name, args
  timeout -k 10 300 $B $2 > gpurun_out/ab41/$1.json 2> gpurun_out/ab41/$1.err || { echo "$1 failed"; tail -5 gpurun_out/ab41/$1.err; exit 4; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab41/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
for R in 1 2; do
  run s20_pow2_$R "--steps 20 --pow2-calls"
  run s20_one20_$R "--steps 20"
  run s96_pow2_$R "--steps 96 --pow2-calls"
  run s96_b24_$R "--steps 96 --batch 24"
done
timeout -k 10 400 python3 tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --fif 2 --batch 20 > gpurun_out/ab41/emul_one20.json 2> gpurun_out/ab41/emul_one20.err || { echo "emul failed"; tail -5 gpurun_out/ab41/emul_one20.err; exit 5; }
python3 -c "import json; d=json.load(open('gpurun_out/ab41/emul_one20.json')); print('one 20-frame call', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
