#!/bin/bash
# round 6 final: the driver command under rocprofv3 --kernel-trace --stats on the final tree (after the BDPT
# vertex-launch changes), with the kernel statistics
export TMPDIR=/tmp
P=gpurun_out/r6final3; mkdir -p $P
timeout -s KILL 900 rocprofv3 --kernel-trace --stats -d $P/prof -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 3; }
python3 tools/rocpd_stats.py $(find $P/prof -name "*.db" | head -1) > $P/kernel_stats.csv || exit 5
rm -rf $P/prof
python3 - $P/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["bdpt"]["value"], d.get("parity_vs_reference", {}).get("pixels_bit_exact"))
PY
