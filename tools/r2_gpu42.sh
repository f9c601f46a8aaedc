#!/bin/bash
# round-2 GPU call 42: final state -- full GPU suite, smoke(), default bench, kernel-trace profile of it
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/r42
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r42/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r42/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/r42/pytest.log | head -20; exit 3; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r42/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r42/smoke.log; exit 4; }
tail -1 gpurun_out/r42/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/r42/bench_default.json 2> gpurun_out/r42/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/r42/bench_default.err; exit 5; }
python3 -c "import json; d=json.loads(open('gpurun_out/r42/bench_default.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['traffic'], r['gather_ceiling']['frac_of_l2_resident'], d['bdpt']['value'])"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r42/trace -o t -- python3 bench.py > gpurun_out/r42/trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/r42/trace.log; exit 6; }
echo trace done
