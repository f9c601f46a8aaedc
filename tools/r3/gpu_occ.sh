#!/bin/bash
# Occupancy targets of the shading kernels (A/B): variants libmcrt_{sw5,cw4,vw5}.so (tools/build_variant.sh)
# against the in-tree library (base).  Parity subsets on each variant, then alternating bench runs.
export TMPDIR=/tmp
P=gpurun_out/occ
mkdir -p $P
L=$PWD/monte-carlo-raytracer_amd
export MCRT_LIB_PATH=$L/libmcrt_sw5.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "sm_pt_1080p or packets" > $P/t_sw5.log 2>&1 || { tail -30 $P/t_sw5.log; exit 3; }
tail -1 $P/t_sw5.log
for v in cw4 vw5; do
  export MCRT_LIB_PATH=$L/libmcrt_$v.so
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bdpt.py -k "reference or band" > $P/t_$v.log 2>&1 || { tail -30 $P/t_$v.log; exit 3; }
  tail -1 $P/t_$v.log
done
show() { python3 -c "
import json
d = json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"; }
PT="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
BD="python3 bench.py --integrator bdpt --steps 16 --warmup 2 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  for v in base sw5; do
    if [ $v = base ]; then unset MCRT_LIB_PATH; else export MCRT_LIB_PATH=$L/libmcrt_$v.so; fi
    timeout -k 10 300 $PT > $P/pt_$v$r.json 2> $P/pt_$v$r.err || { tail -20 $P/pt_$v$r.err; exit 4; }
    show $P/pt_$v$r.json pt_$v$r
  done
  for v in base cw4 vw5; do
    if [ $v = base ]; then unset MCRT_LIB_PATH; else export MCRT_LIB_PATH=$L/libmcrt_$v.so; fi
    timeout -k 10 300 $BD > $P/bd_$v$r.json 2> $P/bd_$v$r.err || { tail -20 $P/bd_$v$r.err; exit 5; }
    show $P/bd_$v$r.json bd_$v$r
  done
done
