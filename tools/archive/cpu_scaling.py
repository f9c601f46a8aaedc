"""Thread scaling of bench.py's cpu_baseline (the oracle, oracle/mcrt_oracle.c) on the host cores of the
GPU box: the same San-Miguel proxy, camera and frame, a fixed sample of evenly spaced rows rendered at
1, 2, 4, ... threads.  Prints one JSON line.  CPU only (no GPU needed).

  python tools/cpu_scaling.py [rows] [max_threads]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)

from mcrt import scenes  # noqa: E402
from mcrt.camera import scene_camera  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def main():
    nrows = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    top = int(sys.argv[2]) if len(sys.argv) > 2 else min(len(os.sched_getaffinity(0)), 64)
    W, H, D = 1920, 1080, 2
    sc = scenes.san_miguel_proxy()
    cam = scene_camera("san_miguel_proxy", W, H, frame=0, jitter=True)
    o = po.OracleScene(sc)
    t0 = time.perf_counter()
    o.build()
    build_s = time.perf_counter() - t0
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(np.int32))
    o.render_rows(cam, rows[:4], frame=0, max_depth=D, threads=4)   # page in the tree
    out = []
    n = 1
    ref = None
    while n <= top:
        t0 = time.perf_counter()
        rad, _ = o.render_rows(cam, rows, frame=0, max_depth=D, threads=n)
        el = time.perf_counter() - t0
        if ref is None:
            ref = rad
        same = bool(np.array_equal(rad.view(np.uint32), ref.view(np.uint32)))   # thread count changes nothing
        mps = len(rows) * W / el / 1e6
        out.append({"threads": n, "seconds": round(el, 3), "mpaths_s": round(mps, 4), "bit_identical": same})
        print(f"threads {n}: {el:.2f} s, {mps:.4f} Mpaths/s", file=sys.stderr, flush=True)
        n *= 2
    base = out[0]["mpaths_s"]
    for r in out:
        r["speedup"] = round(r["mpaths_s"] / base, 2)
        r["efficiency"] = round(r["mpaths_s"] / base / r["threads"], 3)
    print(json.dumps({"what": "oracle cpu_baseline thread scaling", "scene": sc.name, "triangles": sc.num_triangles,
                      "sample": f"{len(rows)} of {H} evenly spaced rows of frame 0, {W} px each, D={D}",
                      "cpus_visible": len(os.sched_getaffinity(0)), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                      "bvh_build_s": round(build_s, 1), "runs": out}))


if __name__ == "__main__":
    main()
