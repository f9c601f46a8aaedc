#!/bin/bash
# round-2 GPU call 3: C++ consumer, scene updates, accumulate pins; packed-slab and ray-sort A/B
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_capi_consumer.py tests/test_gpu_scene_updates.py tests/test_gpu_accumulate.py \
  -v --timeout 300 --timeout-method thread > gpurun_out/pytest3.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest3.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_pk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_golden_reference.py tests/test_gpu_trace.py -q --timeout 200 --timeout-method thread > gpurun_out/pytest3_pk.log 2>&1
echo "pk parity rc=$?"; tail -3 gpurun_out/pytest3_pk.log
B="python3 bench.py --no-cpu-baseline --no-roofline-model --steps 40"
for v in base pk sort; do
  case $v in
    base) env="";;
    pk) env="MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_pk.so";;
    sort) env="MCRT_SORT_RAYS=1";;
  esac
  env $env timeout -k 10 300 $B > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 6; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernels'].items()})"
done
