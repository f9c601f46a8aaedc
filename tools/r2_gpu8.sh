#!/bin/bash
# full GPU suite after the device SAH build became the default + the C++ OBJ path
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest_full.log | tail -5
grep -E "FAILED|Error" gpurun_out/pytest_full.log | head -10
exit $rc
