#!/bin/bash
# round 6: light-table entries (and their shapes) read with one scalar fetch per distinct index of the wave
# (tableEntryFew, lights <= 8) against libmcrt_base.so (the tree before, scene tables already scalar):
# PT and BDPT bench lines, alternating, 2 runs each; the default line carries parity_vs_reference
export TMPDIR=/tmp
P=gpurun_out/r6t15; mkdir -p $P; rm -f $P/*.json
BASE=$PWD/monte-carlo-raytracer_amd/libmcrt_base.so
F="--no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2; do
  MCRT_LIB_PATH=$BASE timeout -k 10 300 python3 bench.py $F > $P/base_pt_$r.json 2> $P/base_pt_$r.err || { tail -20 $P/base_pt_$r.err; exit 4; }
  timeout -k 10 300 python3 bench.py $F > $P/new_pt_$r.json 2> $P/new_pt_$r.err || { tail -20 $P/new_pt_$r.err; exit 4; }
done
B="python3 bench.py --integrator bdpt --steps 32 --no-cpu-baseline --no-roofline-model"
for r in 1 2; do
  MCRT_LIB_PATH=$BASE timeout -k 10 300 $B > $P/base_bdpt_$r.json 2> $P/base_bdpt_$r.err || { tail -20 $P/base_bdpt_$r.err; exit 4; }
  timeout -k 10 300 $B > $P/new_bdpt_$r.json 2> $P/new_bdpt_$r.err || { tail -20 $P/new_bdpt_$r.err; exit 4; }
done
timeout -k 10 400 python3 bench.py --no-bdpt --no-roofline-model > $P/new_parity.json 2> $P/new_parity.err || { tail -20 $P/new_parity.err; exit 4; }
python3 - $P/*.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    k = d.get("kernels", {})
    print(f.split("/")[-1], d["value"], d["ms_per_step"], d.get("parity_vs_reference", {}).get("pixels_bit_exact"), {n: v.get("ms_per_frame", v) for n, v in k.items()})
PY
