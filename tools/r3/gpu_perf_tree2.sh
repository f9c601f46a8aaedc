#!/bin/bash
# perf tree bins sweep (3-axis SAH, host build): 64 / 128 / 256 bins, PT bench timed call
P=gpurun_out/pt3b
mkdir -p $P
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt --perf-tree"
for b in 256 128 64 256; do
  timeout -k 10 400 $B --bvh-bins $b > $P/bench_$b.json 2> $P/bench_$b.err || { tail -20 $P/bench_$b.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$b.json').read().strip().splitlines()[-1])
print('bins $b', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d.get('kernels', {}).items()}, d['config'].get('bvh_build_ms'))"
done
