"""CHECKER (test infrastructure, oracle/): renders frames of bench.py's workload with the
REFERENCE's own kernels -- PathTracing.cl + the RadeonRays intersect_bvh2_lds.cl kernels compiled
for gfx950 from /root/reference by oracle/refbuild/Makefile and run through the ROCm OpenCL
runtime by clref_runner.so (oracle/_ref) -- in a process of its own, so the OpenCL runtime stays
out of the HIP process that is measured.  bench.py calls it after its timed region, on rank 0, as
part of its cpu_baseline leg, and compares the product's frame with these bit for bit
(`parity_vs_reference` in the bench line).  Never on the product path.

usage: python oracle/clref_frame.py OUT.npz SCENE TRIS W H MAX_DEPTH FRAME [FRAME ...]
Cameras are bench.py's: camera of frame f = the TAA-jittered camera of f % 64 (bench.py cam_of).
"""
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


def bench_scene(name, tris):
    """bench.py's scene selection (same generators, same arguments)."""
    if name == "san_miguel_proxy":
        return scenes.san_miguel_proxy(tris=tris)
    if name == "sponza_proxy":
        return scenes.sponza_proxy()
    if name == "dragon_proxy":
        return scenes.dragon_proxy(tris=min(tris, 871_414))
    raise KeyError(f"no reference parity for scene {name}")


def main():
    out, name, tris, W, H, D = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), \
        int(sys.argv[6])
    frames = [int(a) for a in sys.argv[7:]]
    t0 = time.perf_counter()
    sc = bench_scene(name, tris)
    cs = po.CLRefScene(sc, "ieee")   # Bvh2 nodes: the oracle's restatement, byte-identical to RR's builder
    setup_s = time.perf_counter() - t0
    res = {}
    t0 = time.perf_counter()
    for f in frames:
        res[f"f{f}"] = cs.render(scene_camera(name, W, H, frame=f % 64, jitter=True), frame=f, max_depth=D)
    res["device"] = np.array(po.clref("ieee").clref_device().decode())
    np.savez(out, **res)
    print(f"clref_frame: {name} {W}x{H} D={D} frames {frames}: setup {setup_s:.1f}s, render "
          f"{time.perf_counter() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
