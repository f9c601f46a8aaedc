#!/bin/bash
# Round 3: wide tree first GPU run -- its tests, A/B bench, then the full GPU suite.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/wide_tests.log 2>&1; rc=$?
tail -25 gpurun_out/wide_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
B="python bench.py --no-cpu-baseline --no-roofline-model --no-bdpt"
timeout -k 10 300 $B --tree wide > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err || { tail -20 gpurun_out/bench_wide.err; exit 4; }
timeout -k 10 300 $B > gpurun_out/bench_bvh2.json 2> gpurun_out/bench_bvh2.err || { tail -20 gpurun_out/bench_bvh2.err; exit 4; }
python - <<'PY'
import json
for n in ("wide", "bvh2"):
    d = json.load(open(f"gpurun_out/bench_{n}.json"))
    print(n, d["value"], d["ms_per_step"], {k: v["avg_ms"] for k, v in d.get("kernels", {}).items()})
PY
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_full.log
exit $rc
