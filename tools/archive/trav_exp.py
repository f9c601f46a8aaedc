"""Traversal experiment (GPU box): the product's AoS query kernel variants and the reference's
RadeonRays intersect_main on identical primary / extension / shadow rays of the bench scene.
Run under rocprofv3 --kernel-trace to compare kernel durations.
usage: python tools/trav_exp.py [variants=0,1,2,3] [reps=3]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)


def aos(o, d, tmax):
    from mcrt import types as T
    r = np.zeros(len(o), T.RAY_DTYPE)
    r["o"][:, :3] = o[:, :3]
    r["o"][:, 3] = tmax
    r["d"][:, :3] = d[:, :3]
    r["extra"] = -1
    return r


def main():
    import torch
    from mcrt import lib, scenes
    from mcrt.camera import scene_camera
    from oracle import pyoracle as po
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    W, H = 1920, 1080
    sc = scenes.san_miguel_proxy()
    cam = scene_camera("san_miguel_proxy", W, H)
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, sc)
    fb = lib.FrameBuffer(ctx, W, H)
    fb.render(ds, cam, frame=0, max_depth=2)
    eo, ed, _ = fb.read_queue(1)
    so, sd, _ = fb.read_queue(0)
    # primary rays (float32 numpy restatement of GeneratePerspectiveRays; timing only)
    c = cam[0]
    y, x = np.mgrid[0:H, 0:W].astype(np.float32)
    u = (x * np.float32(1.0 / W))[..., None]
    v = (y * np.float32(1.0 / H))[..., None]
    r00, r10, r01, r11 = (np.asarray(c[k][:3], np.float32) for k in ("r00", "r10", "r01", "r11"))
    d = (r00 + (r10 - r00) * u) * (1 - v) + (r01 + (r11 - r01) * u) * v
    d = (d / np.linalg.norm(d, axis=-1, keepdims=True)).reshape(-1, 3).astype(np.float32)
    o = np.broadcast_to(np.asarray(c["pos"][:3], np.float32), d.shape)
    sets = {"primary": aos(o, d, 1000.0), "extension": aos(eo, ed, 1000.0), "shadow": aos(so, sd, so[:, 3])}
    sets["shadow"]["o"][:, 3] = so[:, 3]
    print({k: len(v) for k, v in sets.items()})
    res = {}
    for name, rays in sets.items():
        n = len(rays)
        rt = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
        anyhit = name == "shadow"
        out = torch.zeros(n * (4 if anyhit else 32), dtype=torch.uint8, device="cuda")
        for v in variants:
            os.environ["MCRT_TRACE_VARIANT"] = str(v)
            for _ in range(reps):
                (ds.trace_any if anyhit else ds.trace_closest)(rt.data_ptr(), n, out.data_ptr())
            ctx.sync()
            res[f"{name}_v{v}"] = out.cpu().numpy().copy()
    os.environ["MCRT_TRACE_VARIANT"] = "0"
    ref = {}
    try:
        cs = po.CLRefScene(sc, "ieee")
        for name, rays in sets.items():
            for _ in range(reps):
                ref[name] = cs.trace(rays, any_hit=(name == "shadow"))
    except Exception as e:   # noqa: BLE001
        print("reference skipped:", e)
    # agreement between variants (same tree, same arithmetic => identical results)
    for name in sets:
        base = res[f"{name}_v{variants[0]}"]
        for v in variants[1:]:
            print(name, f"v{v} identical to v{variants[0]}:", bool((res[f'{name}_v{v}'] == base).all()))


if __name__ == "__main__":
    main()
