# full GPU suite + smoke, then the per-rank scaling emulation (PT and band-split BDPT, N = 1 / 2 / 4 / 8)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5suite}; mkdir -p $P
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 600 --timeout-method thread > $P/pytest_gpu.log 2>&1 || { tail -40 $P/pytest_gpu.log; exit 3; }
tail -1 $P/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || { tail -20 $P/smoke.log; exit 4; }
tail -2 $P/smoke.log
timeout -k 10 500 python3 tools/scale_emulate.py --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_scale.json 2> $P/pt_scale.err || { tail -20 $P/pt_scale.err; exit 4; }
timeout -k 10 600 python3 tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 32 --batch 16 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || { tail -20 $P/bdpt_scale.err; exit 4; }
python3 - $P <<'PY'
import json, sys
for n in ("pt", "bdpt"):
    d = json.loads(open(sys.argv[1] + "/" + n + "_scale.json").read().strip().splitlines()[-1])
    print(n, {k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective")) for k, v in d["per_n"].items()})
PY
