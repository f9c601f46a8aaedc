#!/bin/bash
mkdir -p gpurun_out
echo "=== scale_emulate bdpt"
timeout -k 10 600 python tools/scale_emulate.py --integrator bdpt --steps 8 > gpurun_out/scale_bdpt.json 2> gpurun_out/scale_bdpt.err || { tail -5 gpurun_out/scale_bdpt.err; exit 4; }
cat gpurun_out/scale_bdpt.json
echo "=== 2-rank gloo rehearsal, BDPT band split"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --integrator bdpt --dist-backend gloo --steps 4 --warmup 2 --no-cpu-baseline --no-roofline-model \
  > gpurun_out/rehearsal_bdpt2.json 2> gpurun_out/rehearsal_bdpt2.err || { tail -20 gpurun_out/rehearsal_bdpt2.err; exit 5; }
cut -c1-600 gpurun_out/rehearsal_bdpt2.json
