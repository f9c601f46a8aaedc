#!/bin/bash
# N = 8 per-rank emulation, 10 + 10 frames on two slots vs one 20-frame call: kernel trace, overlap
export TMPDIR=/tmp
P=gpurun_out/ovl
mkdir -p $P
for ch in 10 20; do
  timeout -s KILL 300 rocprofv3 --kernel-trace -d $P/c$ch -o k -- python3 tools/scale_emulate.py --ns 8 --chunks $ch --steps 20 > $P/c$ch.log 2>&1 || { tail -5 $P/c$ch.log; exit 3; }
  tail -1 $P/c$ch.log | cut -c1-400
  python3 tools/kernel_overlap.py $(find $P/c$ch -name "*.db" | head -1) --last 80 > $P/c$ch.txt
  tail -1 $P/c$ch.txt
done
