#!/bin/bash
# device SAH build: identity tests (default lib) + build-time sweep over the LDS request size
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sah_build.py -x -q -s --timeout 240 --timeout-method thread > gpurun_out/sah2.log 2>&1 || { echo "sah tests failed"; tail -30 gpurun_out/sah2.log; exit 3; }
grep -E "passed|failed|device SAH build" gpurun_out/sah2.log
for V in "" _s1024 _s256; do
  if [ -n "$V" ]; then export MCRT_LIB_PATH=/root/repo/monte-carlo-raytracer_amd/libmcrt$V.so; else unset MCRT_LIB_PATH; fi
  echo "variant ${V:-default(512)}"
  timeout -k 10 120 python3 -u tools/prof_build.py 10000000 3 2>&1 | grep builder || exit 4
done
unset MCRT_LIB_PATH
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profb2 -o b -- python3 tools/prof_build.py 10000000 2 > gpurun_out/profb2.log 2>&1 || { echo "rocprof failed"; exit 5; }
