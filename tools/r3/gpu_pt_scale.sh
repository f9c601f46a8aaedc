#!/bin/bash
# per-rank PT compute at N = 1/8 for call plans of the 20 timed steps
mkdir -p gpurun_out/scale
for plan in 20 10 7 5 4; do
  timeout -k 10 300 python tools/scale_emulate.py --ns 1,8 --steps 20 --chunks $plan > gpurun_out/scale/pt_$plan.json 2> gpurun_out/scale/pt_$plan.err || { tail -5 gpurun_out/scale/pt_$plan.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/scale/pt_$plan.json')); print('$plan', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
done
for fif in 3 4; do
  timeout -k 10 300 python tools/scale_emulate.py --ns 1,8 --steps 20 --chunks 10 --fif $fif > gpurun_out/scale/pt_10_f$fif.json 2> gpurun_out/scale/pt_f.err || { tail -5 gpurun_out/scale/pt_f.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/scale/pt_10_f$fif.json')); print('10 fif $fif', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
done
