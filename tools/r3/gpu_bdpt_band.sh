#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bdpt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bdpt_tests.log 2>&1; rc=$?
tail -3 gpurun_out/bdpt_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/scale_emulate.py --integrator bdpt --steps 8 > gpurun_out/scale_bdpt.json 2> gpurun_out/scale_bdpt.err || { tail -5 gpurun_out/scale_bdpt.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/scale_bdpt.json')); print({n: (v['max_ms'], v['compute_eff']) for n, v in d['per_n'].items()})"
