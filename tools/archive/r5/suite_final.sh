# the GPU suite and smoke on the final tree
export TMPDIR=/tmp
P=gpurun_out/r5suite_final; mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || { tail -40 $P/pytest_gpu.log; exit 3; }
tail -1 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || { tail -20 $P/smoke.log; exit 4; }
tail -1 $P/smoke.log
