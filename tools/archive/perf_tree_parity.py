"""Perf tree (mcrt_accel_opts.device_build 4, host 3-axis SAH) against the reference's Bvh2 on the
San-Miguel proxy at 1080p: the PT frames of both trees (the Bvh2 frames are bit-exact with the
reference's kernels, tests/test_gpu_reference_scale.py) compared at SURVEY App. A's tolerance
(|dL| <= 1e-4 max(1, |L|) per pixel), plus build time and node count.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd")]


def main():
    import torch
    torch.cuda.init()
    from mcrt import lib, scenes
    from mcrt.camera import scene_camera
    W, H = 1920, 1080
    scene = scenes.san_miguel_proxy()
    ctx = lib.Context(0)
    out = {}
    frames = {}
    for name, mode in (("bvh2", 2), ("perf3", 4)):
        t0 = time.perf_counter()
        ds = lib.DeviceScene(ctx, scene, device_build=mode)
        info = ds.info()
        out[name] = {"build_s": round(time.perf_counter() - t0, 2), "nodes": info["nodes"], "depth": info.get("depth")}
        fb = lib.FrameBuffer(ctx, W, H)
        imgs = []
        for f in range(2):
            fb.render(ds, scene_camera("san_miguel_proxy", W, H, frame=f, jitter=True), frame=f, max_depth=2)
            imgs.append(fb.read(0)[..., :3].copy())
        frames[name] = imgs
        fb.close()
        ds.close()
    for f in range(2):
        a, b = frames["perf3"][f], frames["bvh2"][f]
        ok = (np.abs(a - b) <= 1e-4 * np.maximum(1.0, np.abs(b))).all(-1)
        ex = (a.view(np.uint32) == b.view(np.uint32)).all(-1)
        out[f"frame{f}"] = {"within_1e-4": round(float(ok.mean()), 5), "bit_exact": round(float(ex.mean()), 5),
                            "mean_perf3": float(a.mean()), "mean_bvh2": float(b.mean())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
