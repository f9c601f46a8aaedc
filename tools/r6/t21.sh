#!/bin/bash
# round 6: the full-size reference tests with EVERY pixel's vertices compared in the 960x540 depth-5 BDPT
# case too (clref_job.FULL_VERTEX_CASES)
export TMPDIR=/tmp
P=gpurun_out/r6t21; mkdir -p $P
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_reference_scale.py > $P/pytest_scale.log 2>&1 || { tail -30 $P/pytest_scale.log; exit 3; }
tail -15 $P/pytest_scale.log
