#!/bin/bash
# round 6: strong scaling with each rank's 20 frames in 2 or 4 calls (two frame slots in flight, so one
# call's launch tails overlap the next call's launches) against one 20-frame call: per-rank emulation N = 1, 8
export TMPDIR=/tmp
P=gpurun_out/r6t20; mkdir -p $P; rm -f $P/*.json
for c in 20 10 5; do
  timeout -k 10 400 python tools/scale_emulate.py --ns 1,8 --scaling strong --steps 20 --chunks $c --kernels > $P/strong_c$c.json 2> $P/strong_c$c.err || { tail -20 $P/strong_c$c.err; exit 4; }
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d.get('fif'), {k: (v['max_ms'], v['compute_eff'], v.get('eff_with_collective'), v.get('frames_per_call')) for k, v in d['per_n'].items()})
PY
