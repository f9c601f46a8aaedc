#!/bin/bash
# round-2 GPU call 46: the driver's command shape (--steps 20 --warmup 5, auto frames per call) as a 2- and 4-rank gloo
# rehearsal on one GPU (ranks share cuda:0): the gathered image must equal the 1-rank image bit for bit
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r46
A="--steps 20 --warmup 5 --no-cpu-baseline --no-roofline-model --no-kernel-timing --no-bdpt"
timeout -k 10 300 python3 bench.py $A --save-image gpurun_out/r46/img1.npy > gpurun_out/r46/g1.json 2> gpurun_out/r46/g1.err || { echo "1-rank failed"; tail -20 gpurun_out/r46/g1.err; exit 3; }
for N in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus $N --dist-backend gloo $A --save-image gpurun_out/r46/img$N.npy > gpurun_out/r46/g$N.json 2> gpurun_out/r46/g$N.err || { echo "$N-rank failed"; tail -20 gpurun_out/r46/g$N.err; exit 4; }
done
python3 -c "
import numpy as np, json
a=np.load('gpurun_out/r46/img1.npy')
for n in (2, 4):
    b=np.load('gpurun_out/r46/img%d.npy'%n); d=json.loads(open('gpurun_out/r46/g%d.json'%n).read().strip().splitlines()[-1])
    print(n, 'ranks: bit-identical to 1 rank:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'frames/call', d['config']['frames_per_launch'], d['config']['parallelism'])
"
rm -f gpurun_out/r46/*.npy
