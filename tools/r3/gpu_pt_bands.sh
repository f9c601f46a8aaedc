#!/bin/bash
# per-rank PT compute at N = 8 vs band height (8-row interleave .. contiguous strips), per-kernel times
mkdir -p gpurun_out/scale
timeout -k 10 300 python tools/scale_emulate.py --ns 1,8 --steps 20 --chunks 20 --kernels > gpurun_out/scale/pt_kern.json 2> gpurun_out/scale/pt_kern.err || { tail -5 gpurun_out/scale/pt_kern.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/scale/pt_kern.json')); [print(n, v['max_ms'], v.get('compute_eff'), v['rank0_kernel_ms_per_frame']) for n, v in d['per_n'].items()]"
for br in 16 32 64 136; do
  timeout -k 10 300 python tools/scale_emulate.py --ns 8 --steps 20 --chunks 20 --band-rows $br --base-ms 0 > gpurun_out/scale/pt_b$br.json 2> gpurun_out/scale/pt_b$br.err || { tail -5 gpurun_out/scale/pt_b$br.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/scale/pt_b$br.json')); print('band rows $br', {n: (v['max_ms'], v.get('rank_ms')) for n, v in d['per_n'].items()})"
done
