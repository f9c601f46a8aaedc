#!/bin/bash
# Round 3: full-size pinning of the timed call + BDPT 1080p, then the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_scale.py -x -v --timeout 800 --timeout-method thread \
  > gpurun_out/pin.log 2>&1 || { tail -40 gpurun_out/pin.log; exit 3; }
tail -15 gpurun_out/pin.log
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
