"""BASELINE.json config 1 on the CPU: the Stanford-Dragon proxy at 512x512, 4 spp, unidirectional
PT (the reference's plumbing case on an OpenCL CPU device; PathTracingApp.cpp:348-407 sets the
scene up).  The oracle (C restatement of PathTracing.cl + RadeonRays' Bvh2/LDS traversal, test
infrastructure) renders the four frames and accumulates them with the box filter
(ReconstructionPass); its frames are checked against the REFERENCE's own kernels run live on an
MI355X (tests/clref_job.py ... config1 -> tests/golden/config1_dragon512.npz: rows
clref_job.CONFIG1_ROWS of frames 0..3) at the oracle's usual tolerance, and the CPU time of the
whole 4-spp job is reported (BASELINE.md section 4's CPU number)."""
import os
import time

import numpy as np

from clref_job import CONFIG1, scale_scene
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "config1_dragon512.npz")


def frac_within(a, b, rtol=1e-4):
    d = np.abs(a[..., :3].astype(np.float64) - b[..., :3])
    return (d <= rtol * np.maximum(1.0, np.abs(b[..., :3]))).all(-1).mean()


def test_config1_dragon_512_4spp():
    key, name, W, H, _, frames, D = CONFIG1
    z = np.load(GOLD, allow_pickle=False)
    rows = z["rows"]
    o = po.OracleScene(scale_scene(name))
    t0 = time.perf_counter()
    o.build()
    build_s = time.perf_counter() - t0
    cam = scene_camera(name, W, H)
    threads = min(len(os.sched_getaffinity(0)), 16)
    box = T.make_filter(T.BOX)
    wsum = wts = None
    t0 = time.perf_counter()
    for f in frames:
        rad, _ = o.render(cam, frame=f, max_depth=D, threads=threads)
        wsum, wts, img = po.accumulate(np.ascontiguousarray(rad, np.float32), f, box, wsum, wts)
        ok = frac_within(rad[rows], z[f"f{f}"])
        assert ok >= 0.995, (f, ok)
    el = time.perf_counter() - t0
    assert np.isfinite(img).all() and img[..., :3].mean() > 0
    assert (wts == len(frames)).all()   # box filter: weight 1 per frame
    print(f"config 1 on the CPU: {W}x{H} x {len(frames)} spp in {el:.2f} s ({W * H * len(frames) / el / 1e6:.3f} Mpaths/s, "
          f"{threads} threads; BVH build {build_s:.2f} s)")
