# weak scaling (bench.py default): the batched-frame and bench-launcher tests, then the per-rank
# emulation with N x 20 band-frames per rank (PT), and one default 1-GPU bench line
export TMPDIR=/tmp
P=gpurun_out/${1:-r5weak}; mkdir -p $P
timeout -k 10 600 python -u -m pytest tests/test_gpu_render.py tests/test_gpu_rccl.py -m gpu -x -v --timeout 300 --timeout-method thread > $P/pytest.log 2>&1 || { tail -40 $P/pytest.log; exit 3; }
tail -1 $P/pytest.log
timeout -k 10 600 python3 tools/scale_emulate.py --scaling weak --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_weak.json 2> $P/pt_weak.err || { tail -20 $P/pt_weak.err; exit 4; }
python3 - $P <<'PY'
import json, sys
d = json.loads(open(sys.argv[1] + "/pt_weak.json").read().strip().splitlines()[-1])
print({k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective")) for k, v in d["per_n"].items()})
PY
timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-reference-parity > $P/bench.json 2> $P/bench.err || { tail -20 $P/bench.err; exit 5; }
python3 tools/bench_summary.py $P/bench.json || tail -c 600 $P/bench.json
# A/B: the near-tie repeat's cost (variant without it: not bit-exact, timing only)
B="python3 bench.py --no-cpu-baseline --no-roofline-model --no-reference-parity --no-bdpt"
for r in 1 2; do
  timeout -k 10 300 $B > $P/base_$r.json 2> $P/base_$r.err || { tail -20 $P/base_$r.err; exit 6; }
  MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_noretr.so timeout -k 10 300 $B > $P/noretr_$r.json 2> $P/noretr_$r.err || { tail -20 $P/noretr_$r.err; exit 6; }
done
python3 tools/bench_summary.py $P/base_*.json $P/noretr_*.json
