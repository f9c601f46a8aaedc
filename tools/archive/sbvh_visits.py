"""Spatial splits as a perf tree, modelled first (analysis tool, CPU; VERDICT r3 item 3, third A/B).

Builds the San-Miguel proxy's reference Bvh2 with the oracle (test infrastructure), takes its
triangle leaves, and rebuilds them with tools/sbvh_model.c: 3-axis binned SAH without spatial
splits (control) and with them at several overlap thresholds.  The same rays as
tools/trav_sim.py (camera rays in 8x8 tile order, one diffuse bounce from their hits, shadow
rays to the sun) are replayed over every tree with tools/trav_sim.c; reported per query class:
node visits per ray, leaf visits, the mean over waves of the wave's longest lane (64-lane
lockstep), and the fraction of rays whose closest-hit t differs from the reference tree's.
usage: python tools/sbvh_visits.py [tris] [W] [H] [variant,variant...]"""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd"), os.path.join(ROOT, "tools")]
import trav_sim as ts  # noqa: E402
from mcrt import scenes  # noqa: E402
from mcrt.camera import scene_camera  # noqa: E402
from oracle import pyoracle as po  # noqa: E402


def sbvh_lib():
    so = "/tmp/sbvh_model.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", os.path.join(ROOT, "tools", "sbvh_model.c"), "-o", so, "-lm"],
                   check=True)
    L = ctypes.CDLL(so)
    L.sbvh_build.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_float,
                             ctypes.c_int, ctypes.c_float]
    L.sbvh_build.restype = ctypes.c_int
    L.sbvh_extra_refs.restype = ctypes.c_long
    return L


def replay(L, nodes, rays0, sun, rng_seed=1):
    rng = np.random.default_rng(rng_seed)
    res, hits = {}, {}
    rays = rays0
    for q, any_ in (("camera", 0), ("bounce", 0), ("shadow", 1)):
        out = np.zeros((len(rays), 3 + ts.KMAX), np.int32)
        ht = np.zeros(len(rays), np.float32)
        hn = np.zeros(len(rays), np.int32)
        L.set_order(0)
        L.sim(nodes.ctypes.data, rays.ctypes.data, len(rays), any_, out.ctypes.data, ht.ctypes.data, hn.ctypes.data)
        act = rays["extra"][:, 1] != 0
        n = (len(out) // 64) * 64
        waves = out[:n, 0].reshape(-1, 64).max(1)
        res[q] = {"rays": int(act.sum()), "visits": round(float(out[act, 0].mean()), 3),
                  "leaf_visits": round(float(out[act, 1].mean()), 3), "wave_max": round(float(waves.mean()), 2)}
        hits[q] = ht.copy()
        if q == "camera":
            cam_t, cam_n, cam_rays = ht, hn, rays
            rays = ts.bounce_rays(nodes, rays, ht, hn, rng)
        elif q == "bounce":
            rays = ts.bounce_rays(nodes, cam_rays, cam_t, cam_n, rng)
            rays["d"][:, :3] = sun
            rays["o"][:, 3] = 1000.0
    return res, hits


def main():
    tris = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 272
    t0 = time.time()
    sc = scenes.san_miguel_proxy(tris=tris)
    o = po.OracleScene(sc)
    o.build()
    ref = o.nodes()
    leaves = np.ascontiguousarray(ref[ref["addr_left"] == 0xffffffff])
    print(f"scene {sc.num_triangles} tris, reference {len(ref)} nodes, {time.time() - t0:.1f}s", flush=True)
    T = ts.lib()
    S = sbvh_lib()
    cam = scene_camera("san_miguel_proxy", W, H)
    rays = ts.camera_rays(cam, W, H)
    sun = -np.asarray(sc.lights["d"][0, :3], np.float32)
    sun /= np.linalg.norm(sun)
    out = {"triangles": int(len(leaves)), "resolution": [W, H]}
    base, base_hits = replay(T, ref, rays, sun)
    out["reference_bvh2"] = {"nodes": int(len(ref)), **base}
    print("reference_bvh2", out["reference_bvh2"], flush=True)
    variants = [("sah3_no_splits", -1.0, 0, 0.0), ("sbvh_a1e-5", 1e-5, 64, 1.0), ("sbvh_a1e-4", 1e-4, 64, 1.0),
                ("sbvh_rr_defaults", 0.05, 10, 0.5)]
    if len(sys.argv) > 4:
        variants = [v for v in variants if v[0] in sys.argv[4].split(",")]
    for name, alpha, depth, budget in variants:
        t1 = time.time()
        cap = int(2 * len(leaves) * (1 + budget)) + 16
        nodes = np.zeros(cap, ref.dtype)
        n = S.sbvh_build(leaves.ctypes.data, len(leaves), nodes.ctypes.data, cap, alpha, depth, budget)
        assert n > 0, name
        nodes = nodes[:n]
        bt = time.time() - t1
        r, hits = replay(T, nodes, rays, sun)
        diff = {q: round(float((hits[q] != base_hits[q]).mean()), 6) for q in hits}
        out[name] = {"nodes": int(n), "extra_refs": int(S.sbvh_extra_refs()), "build_s": round(bt, 1), **r,
                     "hit_t_differs": diff}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
