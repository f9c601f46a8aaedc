#!/bin/bash
# round 6 final: counters + kernel trace of the PT timed call; the per-rank scaling emulation (PT strong and
# weak, BDPT band split, strong); the BDPT counters -- on the final tree
export TMPDIR=/tmp
bash tools/gpu_task.sh evidence r6final_ev || exit $?
P=gpurun_out/r6final_ev
S="python tools/scale_emulate.py --ns 1,2,4,8"
timeout -k 10 400 $S --scaling strong --steps 20 --chunks 20 --kernels > $P/pt_n1248.json 2> $P/pt_strong.err || { tail -20 $P/pt_strong.err; exit 4; }
timeout -k 10 400 $S --scaling weak --steps 20 --chunks 20 --kernels > $P/pt_weak_n1248.json 2> $P/pt_weak.err || { tail -20 $P/pt_weak.err; exit 4; }
timeout -k 10 500 $S --integrator bdpt --scaling strong --steps 32 --batch 16 > $P/bdpt_n1248.json 2> $P/bdpt.err || { tail -20 $P/bdpt.err; exit 4; }
python3 -c "
import json
for n in ('pt_n1248', 'pt_weak_n1248', 'bdpt_n1248'):
    d = json.load(open('$P/' + n + '.json')); print(n, {k: (v['max_ms'], v['compute_eff'], v.get('eff_with_collective')) for k, v in d['per_n'].items()})"
bash tools/gpu_task.sh bdpt-prof r6final_bdptprof || exit $?
