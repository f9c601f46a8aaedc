#!/bin/bash
# (1) packet stack written by every lane (variant libmcrt_pkaw.so): parity + A/B;
# (2) call plans 20 vs 10 + 10 at N = 1 and per-rank N = 8.
export TMPDIR=/tmp
P=gpurun_out/combo1
mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/libmcrt_pkaw.so
MCRT_LIB_PATH=$V timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/ -m gpu -k "packets or sm_pt_1080p" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
tail -1 $P/tests.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2; do
  for v in aw base c10; do
    unset MCRT_LIB_PATH; X=""
    [ $v = aw ] && export MCRT_LIB_PATH=$V
    [ $v = c10 ] && X="--chunks 10"
    timeout -k 10 300 $B $X > $P/${v}_$r.json 2> $P/${v}_$r.err || { tail -20 $P/${v}_$r.err; exit 4; }
    python3 -c "
import json
d = json.loads(open('$P/${v}_$r.json').read().strip().splitlines()[-1])
print('$v $r', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
  done
done
unset MCRT_LIB_PATH
timeout -k 10 400 python tools/scale_emulate.py --ns 8 --steps 20 --chunks 10 --base-ms 1.4901 > $P/scale_c10.json 2> $P/scale_c10.err || { tail -5 $P/scale_c10.err; exit 5; }
python -c "import json; d=json.load(open('$P/scale_c10.json')); print('scale chunks 10', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
