# stop rule limited to calls of >= 16 M paths: the new tests, then the scaling emulation (weak, strong, BDPT)
export TMPDIR=/tmp
P=gpurun_out/${1:-r5wcapsc}; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_quant_nodes.py -m gpu -x -q --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
timeout -k 10 600 python3 tools/scale_emulate.py --scaling weak --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_weak.json 2> $P/pt_weak.err || { tail -20 $P/pt_weak.err; exit 4; }
timeout -k 10 500 python3 tools/scale_emulate.py --scaling strong --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_strong.json 2> $P/pt_strong.err || { tail -20 $P/pt_strong.err; exit 4; }
timeout -k 10 600 python3 tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 32 --batch 16 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || { tail -20 $P/bdpt_scale.err; exit 4; }
python3 - $P <<'PY'
import json, sys
for n in ("pt_weak", "pt_strong", "bdpt_scale"):
    d = json.loads(open(sys.argv[1] + "/" + n + ".json").read().strip().splitlines()[-1])
    print(n, {k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective")) for k, v in d["per_n"].items()})
PY
