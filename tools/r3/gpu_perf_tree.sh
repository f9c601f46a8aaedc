#!/bin/bash
# perf tree A/B: parity at 1080p against the Bvh2 frames, then the PT bench (timed call) alternating
P=gpurun_out/pt3
mkdir -p $P
timeout -k 10 400 python3 tools/r3/perf_tree_parity.py > $P/parity.json 2> $P/parity.err || { tail -20 $P/parity.err; exit 3; }
cat $P/parity.json
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for v in base perf base perf; do
  F=""; [ $v = perf ] && F="--perf-tree"
  timeout -k 10 400 $B $F > $P/bench_$v.json 2> $P/bench_$v.err || { tail -20 $P/bench_$v.err; exit 4; }
  python3 -c "
import json
d = json.loads(open('$P/bench_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d.get('kernels', {}).items()}, d['config'].get('bvh_build_ms'))"
done
