#!/bin/bash
# A/B of an environment switch on the headline bench (alternating runs), optional parity tests first:
# tools/r3/gpu_envab.sh "VAR=value" [runs] ["pytest -k expression"]
export TMPDIR=/tmp
P=gpurun_out/envab
mkdir -p $P
if [ -n "$3" ]; then
  env $1 timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/ -m gpu -k "$3" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
  tail -1 $P/tests.log
fi
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for r in $(seq 1 ${2:-2}); do
  for v in B A; do
    if [ $v = B ]; then E="$1"; else E="MCRT_AB_BASE=1"; fi
    env $E timeout -k 10 300 $B > $P/$v$r.json 2> $P/$v$r.err || { tail -20 $P/$v$r.err; exit 4; }
    python3 -c "
import json
d = json.loads(open('$P/$v$r.json').read().strip().splitlines()[-1])
print('$v$r', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
  done
done
