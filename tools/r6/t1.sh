#!/bin/bash
# round 6, first GPU pass: compact-walk tests (incl. the far-from-origin scene), the sparse splat
# exchange with two frames in flight, then bench A/B: round-5 library (A) vs this tree (B)
export TMPDIR=/tmp
P=gpurun_out/r6t1; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant_nodes.py "tests/test_gpu_bdpt.py::test_sparse_exchange_two_frames_in_flight" -x -v --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -3 $P/pytest.log
bash tools/gpu_task.sh ab $PWD/monte-carlo-raytracer_amd/libmcrt_r05.so 2
