# k_shadow with 32 rays per wave below a launch size (MCRT_THIN_BELOW), N = 1 / 8 emulated
export TMPDIR=/tmp
P=gpurun_out/${1:-r5thin}; mkdir -p $P
E="python3 tools/scale_emulate.py --ns 1,8 --steps 20 --chunks 20 --kernels"
timeout -k 10 400 $E > $P/off.json 2> $P/off.err || { tail -20 $P/off.err; exit 4; }
MCRT_THIN_BELOW=3000000 timeout -k 10 400 $E > $P/t3m.json 2> $P/t3m.err || { tail -20 $P/t3m.err; exit 4; }
MCRT_THIN_BELOW=100000000 timeout -k 10 400 $E > $P/tall.json 2> $P/tall.err || { tail -20 $P/tall.err; exit 4; }
python3 - $P <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: (v["max_ms"], v["compute_eff"], v["rank0_kernel_ms_per_frame"]["k_shadow"]) for k, v in d["per_n"].items()})
PY
