#!/bin/bash
# 2-rank rehearsal of the driver's multi-GPU command shape on one GPU (gloo, both ranks on cuda:0):
# the gathered PT image must be bit-identical to the 1-rank image (tile split + band gather).
export TMPDIR=/tmp
P=gpurun_out/rehearse
mkdir -p $P
C="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-model --no-kernel-timing --no-bdpt"
timeout -k 10 400 python3 $C --save-image $P/img1.npy > $P/n1.json 2> $P/n1.err || { tail -20 $P/n1.err; exit 3; }
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 $C --gpus 2 --dist-backend gloo --save-image $P/img2.npy > $P/n2.json 2> $P/n2.err || { tail -30 $P/n2.err; exit 4; }
python3 -c "
import json, numpy as np
a = np.load('$P/img1.npy'); b = np.load('$P/img2.npy')
print('images bit-identical:', a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.shape)
for n in ('n1', 'n2'):
    d = json.loads(open('$P/' + n + '.json').read().strip().splitlines()[-1]); print(n, d['value'], d['n_gpus'], d['config'].get('parallelism'))
"
