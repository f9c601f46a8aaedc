#!/bin/bash
# Final-state evidence: full GPU suite, smoke, default bench, kernel trace (tools/r3/gpu_full3.sh),
# every BASELINE config (tools/r3/gpu_configs.sh), per-rank scaling emulation (PT, BDPT).
export TMPDIR=/tmp
FULL_DIR=full7 bash tools/r3/gpu_full3.sh || exit $?
CFG_DIR=cfg_final2 bash tools/r3/gpu_configs.sh || exit $?
P=gpurun_out/ev2
mkdir -p $P
timeout -k 10 400 python tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_scale.json 2> $P/pt_scale.err || { tail -5 $P/pt_scale.err; exit 4; }
python -c "import json; d=json.load(open('$P/pt_scale.json')); print('PT', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
timeout -k 10 500 python tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 16 --batch 8 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || { tail -5 $P/bdpt_scale.err; exit 4; }
python -c "import json; d=json.load(open('$P/bdpt_scale.json')); print('BDPT', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
