# Round-5 final tree, part B: counters of the PT timed call and of the BDPT calls, the per-rank scaling
# emulation (weak and strong PT, band-split BDPT) and every BASELINE config.  Outputs under gpurun_out/r5fin.
export TMPDIR=/tmp
P=gpurun_out/r5fin; mkdir -p $P
fail() { echo "FAILED: $1"; [ -f "$2" ] && tail -30 "$2"; exit "${3:-3}"; }
bash tools/gpu_task.sh evidence r5fin/evidence > $P/evidence.log 2>&1 || fail evidence $P/evidence.log 5
bash tools/gpu_task.sh bdpt-prof r5fin/bdpt_prof > $P/bdpt_prof.log 2>&1 || fail bdpt_prof $P/bdpt_prof.log 5
find $P/evidence $P/bdpt_prof -name "*.db" -delete
timeout -k 10 600 python3 tools/scale_emulate.py --scaling weak --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_weak.json 2> $P/pt_weak.err || fail pt_weak $P/pt_weak.err 4
timeout -k 10 500 python3 tools/scale_emulate.py --scaling strong --ns 1,2,4,8 --steps 20 --chunks 20 --kernels > $P/pt_strong.json 2> $P/pt_strong.err || fail pt_strong $P/pt_strong.err 4
timeout -k 10 600 python3 tools/scale_emulate.py --integrator bdpt --ns 1,2,4,8 --steps 32 --batch 16 > $P/bdpt_scale.json 2> $P/bdpt_scale.err || fail bdpt_scale $P/bdpt_scale.err 4
python3 - $P <<'PY'
import json, sys
for n in ("pt_weak", "pt_strong", "bdpt_scale"):
    d = json.loads(open(sys.argv[1] + "/" + n + ".json").read().strip().splitlines()[-1])
    print(n, {k: (v["max_ms"], v["compute_eff"], v.get("eff_with_collective")) for k, v in d["per_n"].items()})
PY
bash tools/gpu_task.sh configs r5fin/configs > $P/configs.log 2>&1 || fail configs $P/configs.log 5
tail -6 $P/configs.log
echo ALLOK
