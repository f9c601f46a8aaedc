#!/bin/bash
# one pytest selection on the GPU: $1 = pytest args
export TMPDIR=/tmp
P=gpurun_out/quick
mkdir -p $P
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $1 > $P/tests.log 2>&1 || { tail -40 $P/tests.log; exit 3; }
grep -E "PASSED|FAILED" $P/tests.log | tail -12; tail -1 $P/tests.log
