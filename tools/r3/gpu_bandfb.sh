#!/bin/bash
# End-of-job band gather straight from the frame buffer (gather_bands_fb): product parity tests,
# then the driver's command shape with 2 and 3 ranks on one GPU (gloo) against 1 rank, bit for bit.
export TMPDIR=/tmp
P=gpurun_out/bandfb
mkdir -p $P
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_render.py -k "band or reduce" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
grep -c PASSED $P/tests.log; tail -1 $P/tests.log
C="bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-model --no-kernel-timing --no-bdpt"
timeout -k 10 400 python3 $C --save-image $P/img1.npy > $P/n1.json 2> $P/n1.err || { tail -20 $P/n1.err; exit 4; }
for n in 2 3; do
  timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2951$n $C --gpus $n --dist-backend gloo --save-image $P/img$n.npy > $P/n$n.json 2> $P/n$n.err || { tail -30 $P/n$n.err; exit 5; }
done
python3 -c "
import json, numpy as np
a = np.load('$P/img1.npy')
for n in (2, 3):
    b = np.load('$P/img%d.npy' % n)
    print(n, 'ranks: image bit-identical to 1 rank:', a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.shape)
for n in ('n1', 'n2', 'n3'):
    d = json.loads(open('$P/' + n + '.json').read().strip().splitlines()[-1]); print(n, d['value'], d['n_gpus'], d['config'].get('parallelism'))
"
