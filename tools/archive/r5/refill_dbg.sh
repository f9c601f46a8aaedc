export TMPDIR=/tmp
P=gpurun_out/r5rdbg; mkdir -p $P
for D in 2 3 4; do
  timeout -k 10 120 python3 tools/archive/r5/dbg/refill_dbg.py $P/base_$D.npy $D || exit 3
  for v in refill16 refill64; do
    MCRT_LIB_PATH=$PWD/monte-carlo-raytracer_amd/libmcrt_$v.so timeout -k 10 120 python3 tools/archive/r5/dbg/refill_dbg.py $P/${v}_$D.npy $D || exit 3
  done
done
python3 - $P <<'PY'
import numpy as np, sys
P = sys.argv[1]
for D in (2, 3, 4):
    a = np.load(f"{P}/base_{D}.npy")
    for v in ("refill16", "refill64"):
        b = np.load(f"{P}/{v}_{D}.npy")
        d = (a.view(np.uint32) != b.view(np.uint32)).any(-1)
        idx = np.argwhere(d)[:5].tolist()
        print(D, v, int(d.sum()), idx, [(a[tuple(i)][:3].tolist(), b[tuple(i)][:3].tolist()) for i in idx[:2]])
PY
rm -f $P/*.npy
