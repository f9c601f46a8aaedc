#!/bin/bash
# round-2 GPU call 21: BDPT first extension launch on the descent-compact records -- BDPT parity + A/B
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bdpt.py tests/test_gpu_golden_reference.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p21_pytest.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/p21_pytest.log; exit 3; }
tail -1 gpurun_out/p21_pytest.log
B="python3 bench.py --integrator bdpt --steps 12 --no-cpu-baseline --no-roofline-model"
for V in 1 0 1 0; do
  MCRT_COMPACT_TRAV=$V timeout -k 10 200 $B > gpurun_out/p21_bench$V.json 2> gpurun_out/p21_bench$V.err || { echo "bench $V failed"; tail -5 gpurun_out/p21_bench$V.err; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/p21_bench$V.json').read().strip().splitlines()[-1]); k=d.get('kernels',{}); print('compact=$V', d['value'], d['ms_per_step'], {n: (k[n]['avg_ms'], k[n]['launches']) for n in k})"
done
