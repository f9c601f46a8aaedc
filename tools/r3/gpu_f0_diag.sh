#!/bin/bash
mkdir -p gpurun_out/f0
timeout -k 10 200 python3 tools/r3/bdpt_f0_diag.py gpurun_out/f0/cur.npz 0 && \
timeout -k 10 200 python3 tools/r3/bdpt_f0_diag.py gpurun_out/f0/cur2.npz 0 && \
MCRT_LIB_PATH=$PWD/tools/experiments/build/libmcrt_a.so timeout -k 10 200 python3 tools/r3/bdpt_f0_diag.py gpurun_out/f0/old.npz 0 && \
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/f0/cur.npz"); b = np.load("gpurun_out/f0/cur2.npz"); c = np.load("gpurun_out/f0/old.npz")
for k in a.files:
    x, y, z = a[k].view(np.uint8), b[k].view(np.uint8), c[k].view(np.uint8)
    print(k, x.size, "cur-vs-cur2 bytes differ", int((x != y).sum()) if x.size == y.size else "size", "cur-vs-old", int((x != z).sum()) if x.size == z.size else ("size", x.size, z.size))
PY
