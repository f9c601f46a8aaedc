#!/bin/bash
# Call plans for the 20 timed steps: one 20-frame call (default) against 10 + 10 and 5 x 4 on the
# two frame slots (does the SALU-bound packet camera launch of one call overlap the TA-bound
# traversal of the other?)
export TMPDIR=/tmp
P=gpurun_out/chunks
mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2; do
  for c in 20 10 5 12,8; do
    timeout -k 10 300 $B --chunks $c > $P/c${c}_$r.json 2> $P/c${c}_$r.err || { tail -20 $P/c${c}_$r.err; exit 4; }
    python3 -c "
import json
d = json.loads(open('$P/c${c}_$r.json').read().strip().splitlines()[-1])
print('chunks $c run $r', d['value'], d['ms_per_step'])"
  done
done
for c in 20 10; do
  timeout -k 10 400 python tools/scale_emulate.py --ns 1,8 --steps 20 --chunks $c > $P/scale_c$c.json 2> $P/scale_c$c.err || { tail -5 $P/scale_c$c.err; exit 5; }
  python -c "import json; d=json.load(open('$P/scale_c$c.json')); print('scale chunks $c', {n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
done
