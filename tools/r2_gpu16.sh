#!/bin/bash
# round-2 GPU call 16: cooperative 4-lane record fetch vs per-lane fetch (tools/probe/chase_probe.hip)
cd /root/repo
mkdir -p gpurun_out
P=tools/probe/chase_probe
timeout -k 5 30 $P ttest 1 1 || { echo "transpose test failed"; exit 3; }
: > gpurun_out/chase16.jsonl
for n in 8192 32768 2000000 20000000; do
  for m in lane4 coop4 lane1 quad; do
    timeout -k 5 60 $P $m $n 256 >> gpurun_out/chase16.jsonl 2>> gpurun_out/chase16.err || { echo "probe $m $n failed"; cat gpurun_out/chase16.err; exit 4; }
  done
done
timeout -k 5 60 $P coop4 2000000 256 16 >> gpurun_out/chase16.jsonl
timeout -k 5 60 $P coop4 32768 256 16 >> gpurun_out/chase16.jsonl
python3 -c "
import json
for l in open('gpurun_out/chase16.jsonl'):
    d=json.loads(l); print(f\"{d['mode']:6s} {d['array_mb']:8.1f} MB w{d['waves_per_cu']:2d} {d['gsteps_per_s']:7.1f} Gsteps/s {d['ns_per_step_per_chain']:7.1f} ns/step\")
"
