#!/bin/bash
# Gather cost per load width and per active-lane fraction (tools/probe/chase_probe.hip):
# lane4 / lane3 / lane3d / lane2 / lane1 and act2 / act4 at L2, Infinity-Cache and HBM residency.
mkdir -p gpurun_out/chase2
O=gpurun_out/chase2/chase.jsonl
: > $O
for n in 32768 2000000 20000000; do
  for m in lane4 lane3 lane3d lane3q lane2 lane1 act2 act4; do
    timeout -k 5 30 tools/probe/chase_probe $m $n 256 32 3 >> $O || { echo "fail $m $n"; exit 3; }
  done
done
cat $O
