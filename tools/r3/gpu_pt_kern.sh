#!/bin/bash
mkdir -p gpurun_out/scale
timeout -k 10 300 python tools/scale_emulate.py --ns 1,8 --steps 20 --chunks 20 --kernels > gpurun_out/scale/pt_kern.json 2> gpurun_out/scale/pt_kern.err || { tail -5 gpurun_out/scale/pt_kern.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/scale/pt_kern.json')); [print(n, v['max_ms'], v['rank0_kernel_ms_per_frame']) for n, v in d['per_n'].items()]"
