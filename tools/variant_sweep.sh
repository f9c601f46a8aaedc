#!/bin/bash
# Profiles bench.py once per alternative in-tree build monte-carlo-raytracer_amd/libmcrt_<V>.so (GPU box).
# usage: tools/variant_sweep.sh V1 V2 ...   -> gpurun_out/sweep_<V>/ rocprofv3 databases
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  MCRT_LIB_PATH="$GRAFT_REPO_ROOT/monte-carlo-raytracer_amd/libmcrt_$v.so" timeout -k 10 300 \
    rocprofv3 --kernel-trace -d gpurun_out/sweep_$v -o b -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/sweep_$v.log | head -1)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
