#!/bin/bash
# round-3 checkpoint: full GPU suite, smoke, default bench, kernel trace of the default bench
export TMPDIR=/tmp
P=gpurun_out/${FULL_DIR:-full3}
mkdir -p $P
timeout -k 10 1500 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || { tail -30 $P/pytest_gpu.log; exit 3; }
tail -3 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || { tail -20 $P/smoke.log; exit 4; }
tail -2 $P/smoke.log
timeout -k 10 600 python3 bench.py > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 5; }
python3 -c "
import json
d = json.loads(open('$P/bench.json').read().strip().splitlines()[-1])
r = d.get('roofline', {})
print('PT', d['value'], d['ms_per_step'], 'frac', r.get('frac'), 'traffic/alg', r.get('traffic_over_alg'), 'cpu', d.get('cpu_baseline', {}).get('value'))
print('BDPT', d.get('bdpt', {}).get('value'), d.get('bdpt', {}).get('ms_per_step'))"
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $P/trace -o k -- python3 bench.py --no-cpu-baseline > $P/trace.log 2>&1 || { tail -5 $P/trace.log; exit 6; }
echo "trace done"
