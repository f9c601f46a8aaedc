#!/bin/bash
# Wave-packet camera-ray traversal (variant library libmcrt_pk.so, plain records via
# MCRT_COMPACT_TRAV=0): full-size reference parity, then the bench A/B against the default build.
export TMPDIR=/tmp
P=gpurun_out/pk
mkdir -p $P
export MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_pk.so MCRT_COMPACT_TRAV=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_reference_scale.py -k "sm_pt or sponza or dragon" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
tail -2 $P/tests.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for v in B A B A; do
  if [ $v = A ]; then unset MCRT_LIB_PATH MCRT_COMPACT_TRAV; else export MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_pk.so MCRT_COMPACT_TRAV=0; fi
  timeout -k 10 300 $B > $P/bench_$v.json 2> $P/bench_$v.err || { tail -20 $P/bench_$v.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
done
