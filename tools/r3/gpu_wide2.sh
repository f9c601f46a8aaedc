#!/bin/bash
# wide tree: its GPU tests + the full-size comparison with the reference, then A/B x2
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_wide.py "tests/test_gpu_reference_scale.py::test_wide_tree_full_size_vs_reference" -x -v -s --timeout 800 --timeout-method thread \
  > gpurun_out/wide_tests2.log 2>&1; rc=$?
grep -E "PASS|FAIL|bit-exact|ties resolved|passed|failed" gpurun_out/wide_tests2.log | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/r3/gpu_ab.sh "--tree wide" "" 2
