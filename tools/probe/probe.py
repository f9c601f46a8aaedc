"""Stage-by-stage bit comparison of the product's shading functions with the reference's
(GPU box).  Child: reference OpenCL (primary rays/hits from its own pipeline, then
oracle/refbuild/clprobe.cl).  Parent: tools/probe/libshade_probe.so on the same inputs.
usage: python tools/probe/probe.py OUT_DIR"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from clref_job import build_scene  # noqa: E402

CASES = [("cornell", 64, 64), ("mixed", 96, 64), ("dragon_small", 80, 64), ("sm_small", 192, 112)]


def scene_of(name):
    if name == "sm_small":
        from mcrt import scenes
        return scenes.san_miguel_proxy(tris=1_000_000)
    return build_scene(name)
SLOTS = ["p|off", "gn", "sn", "sdpdu", "sdpdv", "uv", "sn_nm", "sdpdu_nm", "sdpdv_nm", "Li|pdf", "wi|light",
         "bsdf", "bsdf*cos|pdf*choice", "L", "fs|pdf", "wn|type", "Kd|eta", "Ks|ax", "op|ay", "Kt"]


def cam_of(name, W, H):
    from mcrt.camera import scene_camera
    return scene_camera({"dragon_small": "dragon_proxy", "sm_small": "san_miguel_proxy"}.get(name, name), W, H)


def child(out_dir):
    from oracle import pyoracle as po
    L = po.clref("ieee")
    L.clref_probe.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for name, W, H in CASES:
        cs = po.CLRefScene(scene_of(name), "ieee")
        cs.render(cam_of(name, W, H), frame=0, max_depth=1)
        rays = cs.read("rays", W, H)
        isect = cs.read("isect", W, H)
        from mcrt import types as T
        dirs = np.ascontiguousarray(rays.view(T.RAY_DTYPE)["d"])
        out = np.zeros((W * H, 20, 4), np.float32)
        st = L.clref_probe(cs.h, os.path.join(ROOT, "oracle", "_ref", "clref_probe.hsaco").encode(),
                           isect.ctypes.data, dirs.ctypes.data, W, H, 0, out.ctypes.data)
        if st != 0:
            raise RuntimeError(f"clref_probe {st}: {L.clref_error().decode()}")
        np.savez(os.path.join(out_dir, f"probe_ref_{name}.npz"), isect=isect, dirs=dirs, out=out)


def parent(out_dir):
    r = subprocess.run([sys.executable, __file__, out_dir, "child"], timeout=300)
    if r.returncode != 0:
        sys.exit(r.returncode)
    lib = ctypes.CDLL(os.path.join(HERE, "libshade_probe.so"))
    lib.probe_shade.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    for name, W, H in CASES:
        z = np.load(os.path.join(out_dir, f"probe_ref_{name}.npz"))
        sc = scene_of(name)
        desc = sc.desc()
        isect, dirs = np.ascontiguousarray(z["isect"]), np.ascontiguousarray(z["dirs"])
        out = np.zeros((W * H, 20, 4), np.float32)
        st = lib.probe_shade(ctypes.byref(desc), isect.ctypes.data, dirs.ctypes.data, W, H, 0, 1, out.ctypes.data)
        if st != 0:
            raise RuntimeError("probe_shade failed")
        np.save(os.path.join(out_dir, f"probe_prod_{name}.npy"), out)
        ref = z["out"]
        hit = isect.view(np.int32).reshape(-1, 8)[:, 0] >= 0
        print(f"[{name}] {hit.sum()} hit pixels; bit-exact fraction per stage:")
        for k, nm in enumerate(SLOTS):
            eq = (out[hit, k].view(np.uint32) == ref[hit, k].view(np.uint32)).all(-1)
            print(f"   {k:2d} {nm:22s} {eq.mean():.5f}")


if __name__ == "__main__":
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    if len(sys.argv) > 2:
        child(out)
    else:
        parent(out)
