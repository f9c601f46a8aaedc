#!/bin/bash
# the rest of gpu_full.sh after a fixed test: the GPU suite from the count-query test on
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests/ -m gpu -x -q --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_accumulate.py > gpurun_out/gpu_full.log 2>&1; rc=$?
tail -6 gpurun_out/gpu_full.log
[ $rc -ne 0 ] && exit $rc
sed -n '/=== scale_emulate bdpt/,$p' tools/r3/gpu_full.sh > /tmp/rest.sh
bash -c "step() { echo \"=== \$1\"; }; $(sed -n '/step "scale_emulate bdpt"/,$p' tools/r3/gpu_full.sh)"
