#!/bin/bash
# Shading workgroup size A/B (larger octant groups for the extension queue): variants
# libmcrt_sb512 / libmcrt_sb1024 (tools/build_variant.sh -DSHADE_BLOCK=...) vs the in-tree library.
export TMPDIR=/tmp
P=gpurun_out/sb2
mkdir -p $P
L=$PWD/monte-carlo-raytracer_amd
for v in s0512 s01024; do
  export MCRT_LIB_PATH=$L/libmcrt_$v.so
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu -k "sm_pt_1080p or packets or render" > $P/t_$v.log 2>&1 || { tail -30 $P/t_$v.log; exit 3; }
  tail -1 $P/t_$v.log
done
show() { python3 -c "
import json
d = json.loads(open('$1').read().strip().splitlines()[-1])
print('$2', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"; }
PT="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2; do
  for v in base s0512 s01024; do
    if [ $v = base ]; then unset MCRT_LIB_PATH; else export MCRT_LIB_PATH=$L/libmcrt_$v.so; fi
    timeout -k 10 300 $PT > $P/pt_$v$r.json 2> $P/pt_$v$r.err || { tail -20 $P/pt_$v$r.err; exit 4; }
    show $P/pt_$v$r.json pt_$v$r
  done
done
