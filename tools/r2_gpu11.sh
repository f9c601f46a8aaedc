#!/bin/bash
# band-split BDPT: GPU tests + a 2-rank gloo rehearsal of the bench on one GPU (PT image check is
# the bench's own; here BDPT band vs frame split timing and the N=2 value)
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bdpt.py -x -v --timeout 300 --timeout-method thread > gpurun_out/bdptband.log 2>&1 || { echo "bdpt tests failed"; tail -30 gpurun_out/bdptband.log; exit 3; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/bdptband.log | tail -8
for S in band frame; do
  timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --integrator bdpt --bdpt-split $S --dist-backend gloo --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-model --no-kernel-timing > gpurun_out/bdpt2_$S.json 2> gpurun_out/bdpt2_$S.err || { echo "2-rank bench $S failed"; tail -20 gpurun_out/bdpt2_$S.err; exit 4; }
  tail -1 gpurun_out/bdpt2_$S.json | cut -c1-400
done
