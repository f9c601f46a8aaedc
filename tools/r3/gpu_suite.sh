#!/bin/bash
# full GPU suite + smoke on the current tree
export TMPDIR=/tmp
P=gpurun_out/${SUITE_DIR:-suite}
mkdir -p $P
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || { tail -30 $P/pytest_gpu.log; exit 3; }
tail -1 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || { tail -20 $P/smoke.log; exit 4; }
tail -2 $P/smoke.log
