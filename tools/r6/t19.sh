#!/bin/bash
# round 6: strong scaling (a step = one frame split over the ranks) with the stopped walks engaged at a
# rank's share: the per-rank emulation at N = 1 and 8 with MCRT_WALK_MIN_PATHS 16 M (default), 4 M, 1 M
export TMPDIR=/tmp
P=gpurun_out/r6t19; mkdir -p $P; rm -f $P/*.json
S="python tools/scale_emulate.py --ns 1,8 --scaling strong --steps 20 --chunks 20 --kernels"
for m in 16000000 4000000 1000000; do
  MCRT_WALK_MIN_PATHS=$m timeout -k 10 400 $S > $P/strong_min$m.json 2> $P/strong_min$m.err || { tail -20 $P/strong_min$m.err; exit 4; }
done
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: (v['max_ms'], v['compute_eff'], v.get('eff_with_collective'), v['rank0_kernel_ms_per_frame']) for k, v in d['per_n'].items()})
PY
