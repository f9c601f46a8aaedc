#!/bin/bash
# round 6 final: the driver command under rocprofv3 --kernel-trace --stats (with the tree's counters in
# profiles/), every BASELINE config at 1 spp per step, the depth-5 lines -- on the final tree
export TMPDIR=/tmp
P=gpurun_out/r6final2; mkdir -p $P
timeout -s KILL 900 rocprofv3 --kernel-trace --stats -d $P/prof -o b -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 3; }
python3 tools/rocpd_stats.py $(find $P/prof -name "*.db" | head -1) > $P/kernel_stats.csv || exit 5
rm -rf $P/prof
bash tools/gpu_task.sh summary 2>/dev/null; python3 - $P/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["bdpt"]["value"], d.get("parity_vs_reference", {}).get("pixels_bit_exact"))
PY
bash tools/gpu_task.sh configs r6final_configs || exit $?
F="--no-cpu-baseline --no-roofline-model"
timeout -k 10 400 python3 bench.py $F --max-depth 5 > $P/bench_d5.json 2> $P/d5.err || { tail -20 $P/d5.err; exit 4; }
timeout -k 10 400 python3 bench.py $F --max-depth 5 --russian-roulette --no-bdpt > $P/bench_d5_rr.json 2> $P/d5rr.err || { tail -20 $P/d5rr.err; exit 4; }
