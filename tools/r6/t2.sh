#!/bin/bash
# round 6: the sparse-exchange in-flight test, then bench A/B (round-5 library A vs this tree B)
export TMPDIR=/tmp
P=gpurun_out/r6t2; mkdir -p $P
timeout -k 10 300 python -u -m pytest "tests/test_gpu_bdpt.py::test_sparse_exchange_two_frames_in_flight" "tests/test_gpu_bdpt.py::test_bdpt_band_split_sparse_exchange" -x -v --timeout 200 --timeout-method thread > $P/pytest.log 2>&1 || { tail -30 $P/pytest.log; exit 3; }
tail -3 $P/pytest.log
bash tools/gpu_task.sh ab $PWD/monte-carlo-raytracer_amd/libmcrt_r05.so 2
