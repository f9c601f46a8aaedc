#!/bin/bash
# Wave packets: camera rays (pk) and camera + bounce-0 shadow rays (pks), plain records
# (MCRT_COMPACT_TRAV=0): full-size reference parity of each variant, then PT and BDPT bench A/B.
export TMPDIR=/tmp
P=gpurun_out/pk2
mkdir -p $P
L=$PWD/monte-carlo-raytracer_amd
export MCRT_COMPACT_TRAV=0
MCRT_LIB_PATH=$L/libmcrt_pks.so timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_reference_scale.py -k "sm_pt or sponza or dragon or sm_bdpt" > $P/tests_pks.log 2>&1 || { tail -40 $P/tests_pks.log; exit 3; }
tail -1 $P/tests_pks.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for v in pk pks A pk pks A; do
  if [ $v = A ]; then unset MCRT_LIB_PATH MCRT_COMPACT_TRAV; else export MCRT_LIB_PATH=$L/libmcrt_$v.so MCRT_COMPACT_TRAV=0; fi
  timeout -k 10 300 $B > $P/bench_$v.json 2> $P/bench_$v.err || { tail -20 $P/bench_$v.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
done
BB="python3 bench.py --integrator bdpt --steps 16 --warmup 2 --no-cpu-baseline --no-roofline-model"
for v in pk A; do
  if [ $v = A ]; then unset MCRT_LIB_PATH MCRT_COMPACT_TRAV; else export MCRT_LIB_PATH=$L/libmcrt_$v.so MCRT_COMPACT_TRAV=0; fi
  timeout -k 10 300 $BB > $P/bdpt_$v.json 2> $P/bdpt_$v.err || { tail -20 $P/bdpt_$v.err; exit 5; }
  python3 -c "
import json
d = json.loads(open('$P/bdpt_$v.json').read().strip().splitlines()[-1])
print('bdpt $v', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
done
