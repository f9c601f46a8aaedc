#!/bin/bash
# round-2 GPU call 22: the band-gather end collective -- 2-rank gloo rehearsal on one GPU vs the 1-rank image
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--batch 4 --steps 4 --warmup 2 --no-cpu-baseline --no-roofline-model --no-kernel-timing --no-bdpt --tris 2000000"
timeout -k 10 300 python3 bench.py $A --save-image gpurun_out/img1.npy > gpurun_out/g1.json 2> gpurun_out/g1.err || { echo "1-rank failed"; tail -20 gpurun_out/g1.err; exit 3; }
for C in gather reduce; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --dist-backend gloo --end-collective $C $A --save-image gpurun_out/img2_$C.npy > gpurun_out/g2_$C.json 2> gpurun_out/g2_$C.err || { echo "2-rank $C failed"; tail -20 gpurun_out/g2_$C.err; exit 4; }
done
python3 -c "
import numpy as np
a=np.load('gpurun_out/img1.npy'); 
for c in ('gather','reduce'):
    b=np.load('gpurun_out/img2_%s.npy'%c); print(c, 'bit-identical to 1 rank:', np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.shape, float(a[...,:3].mean()), 'max abs diff', float(np.abs(a-b).max()))
"
rm -f gpurun_out/*.npy
tail -1 gpurun_out/g2_gather.json | cut -c1-300
