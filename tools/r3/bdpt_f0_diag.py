"""Diagnostic: SM-proxy 1080p BDPT frame 0 (fresh frame buffer) -> npz of radiance and state arrays.
usage: MCRT_LIB_PATH=... python tools/r3/bdpt_f0_diag.py out.npz [frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd")]


def main():
    import torch
    torch.cuda.init()
    from mcrt import lib, scenes, types as T
    from mcrt.camera import scene_camera
    W, H = 1920, 1080
    frames = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, scenes.san_miguel_proxy())
    fb = lib.FrameBuffer(ctx, W, H)
    cam = scene_camera("san_miguel_proxy", W, H)
    out = {}
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=2, integrator=T.INTEGRATOR_BDPT)
        out[f"rad{f}"] = fb.read(0)
        for k in ("camera_vertices", "light_vertices", "camera_counts", "light_counts", "slots", "splat",
                  "sampled_light"):
            out[f"{k}{f}"] = fb.read_bdpt(k)
    np.savez(sys.argv[1], **out)
    print("stats", fb.stats())


if __name__ == "__main__":
    main()
