#!/bin/bash
# Packet child-record prefetch (variant libmcrt_pkpf.so): parity, bench A/B, SQ counters of the
# camera launch for both builds.
export TMPDIR=/tmp
P=gpurun_out/pkpf
mkdir -p $P
V=$PWD/monte-carlo-raytracer_amd/${VLIB:-libmcrt_pkpf.so}
MCRT_LIB_PATH=$V timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/ -m gpu -k "packets or sm_pt_1080p" > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
tail -1 $P/tests.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
for r in 1 2; do
  for v in B A; do
    if [ $v = B ]; then export MCRT_LIB_PATH=$V; else unset MCRT_LIB_PATH; fi
    timeout -k 10 300 $B > $P/$v$r.json 2> $P/$v$r.err || { tail -20 $P/$v$r.err; exit 4; }
    python3 -c "
import json
d = json.loads(open('$P/$v$r.json').read().strip().splitlines()[-1])
print('$v$r', d['value'], d['ms_per_step'], {k: round(v['ms_per_frame'], 4) for k, v in d.get('kernels', {}).items()})"
  done
done
unset MCRT_LIB_PATH
C="python3 bench.py --no-kernel-timing --no-bdpt --no-cpu-baseline --no-roofline-model"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY -d $P/sqA -o s -- $C > $P/sqA.log 2>&1 || { tail -5 $P/sqA.log; exit 5; }
python3 tools/pmc_summary.py $(find $P/sqA -name "*.db" | head -1) k_primary_pk | tail -2
