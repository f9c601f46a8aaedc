#!/bin/bash
# the driver's default bench command on the current tree
export TMPDIR=/tmp
P=gpurun_out/${B1_DIR:-bench1}
mkdir -p $P
timeout -k 10 600 python3 bench.py > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 3; }
python3 -c "
import json
d = json.loads(open('$P/bench.json').read().strip().splitlines()[-1])
r = d.get('roofline', {})
print('PT', d['value'], d['ms_per_step'], 'frac', r.get('frac'), 'cpu', d.get('cpu_baseline', {}).get('value'), 'BDPT', d.get('bdpt', {}).get('value'))"
