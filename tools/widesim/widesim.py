"""Bvh2 vs 4-wide quantized tree on the San-Miguel proxy (analysis tool, CPU).

Builds the product's Bvh2 records on the host (mcrt.lib.build_host_records, the RR-identical
tree), collapses them with the experiment's wide builder (tools/widesim/wide.cpp), and
replays camera rays, one diffuse bounce and sun shadow rays through both trees: steps per query
(internal / triangle) and whether the closest hits agree (same triangle, or the same t).
usage: python tools/widesim/widesim.py [tris] [W] [H]
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd"), os.path.join(ROOT, "tools")]
from mcrt import lib as mlib, scenes, types as T  # noqa: E402
from mcrt.camera import scene_camera  # noqa: E402
from trav_sim import camera_rays  # noqa: E402


def load():
    so = "/tmp/widesim.so"
    src = [os.path.join(ROOT, "tools", "widesim", "widesim.cpp"),
           os.path.join(ROOT, "tools", "widesim", "wide.cpp")]
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-pthread", *src, "-o", so],
                   check=True)
    L = ctypes.CDLL(so)
    L.ws_build.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                           ctypes.c_size_t, ctypes.c_void_p]
    L.ws_set_leafbox.argtypes = [ctypes.c_int]
    L.ws_set_sort.argtypes = [ctypes.c_int]
    L.ws_trace.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    L.ws_tris.restype = ctypes.c_void_p
    L.ws_build_alt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.ws_use_tree.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    L.ws_alt_ptr.restype = ctypes.c_void_p
    L.ws_alt_n.restype = ctypes.c_size_t
    return L


def world_triangles(sc):
    """(n, 9) float32 world-space triangles in shape order and the shapes' first triangle, with
    the host build's arithmetic (mcrt_capi.cpp xformPoint: separately rounded float32 ops)."""
    f32 = np.float32
    tris, first, acc = [], [], 0
    for s in sc.shapes:
        first.append(acc)
        n = int(s["numTriangles"])
        acc += n
        idx = sc.indices[int(s["startIdx"]):int(s["startIdx"]) + 3 * n].astype(np.int64) + int(s["startVertex"])
        p = sc.positions[idx, :3].astype(f32)
        M = s["toWorldTransform"].astype(f32).reshape(4, 4)
        out = np.empty_like(p)
        for i in range(3):
            a = np.zeros(len(p), f32)
            a = a + M[i, 0] * p[:, 0]
            a = a + M[i, 1] * p[:, 1]
            a = a + M[i, 2] * p[:, 2]
            a = a + M[i, 3] * f32(0)
            out[:, i] = a + M[i, 3]
        tris.append(out.reshape(-1, 9))
    return np.ascontiguousarray(np.concatenate(tris)), np.array(first, np.uint32)


def trace(L, rays, any_, mode, threads=8):
    n = len(rays)
    st = np.zeros((n, 2), np.int32)
    t = np.zeros(n, np.float32)
    h = np.zeros(n, np.int32)
    L.ws_trace(rays.ctypes.data, n, any_, mode, st.ctypes.data, t.ctypes.data, h.ctypes.data, threads)
    return st, t, h


def bounce(rec, rays, t, h, rng):
    ok = h >= 0
    out = np.zeros(len(rays), T.RAY_DTYPE)
    r = rec[np.maximum(h, 0)]
    e1, e2 = r[:, 4:7], r[:, 8:11]
    n = np.cross(e1, e2)
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-20)
    d = rays["d"][:, :3]
    n = np.where((n * d).sum(1, keepdims=True) > 0, -n, n)
    a = np.where(np.abs(n[:, :1]) > 0.9, np.array([[0, 1, 0]], np.float32), np.array([[1, 0, 0]], np.float32))
    t1 = np.cross(a, n)
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(n, t1)
    u1, u2 = rng.random(len(rays)), rng.random(len(rays))
    rr, ph = np.sqrt(u1), 2 * np.pi * u2
    w = t1 * (rr * np.cos(ph))[:, None] + t2 * (rr * np.sin(ph))[:, None] + n * np.sqrt(1 - u1)[:, None]
    p = rays["o"][:, :3] + t[:, None] * d + n * 1e-5
    out["o"][:, :3] = p
    out["o"][:, 3] = 1000.0
    out["d"][:, :3] = w
    out["extra"][:, 0] = -1
    out["extra"][:, 1] = ok.astype(np.int32)
    return out


def main():
    tris = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 480
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 272
    t0 = time.time()
    sc = scenes.san_miguel_proxy(tris=tris)
    rec, _ = mlib.build_host_records(sc)
    print(f"scene {sc.num_triangles} tris, Bvh2 {len(rec)} records, {time.time() - t0:.1f}s", flush=True)
    L = load()
    info = np.zeros(3, np.int64)
    t0 = time.time()
    tri9, first = world_triangles(sc)
    assert L.ws_build(rec.ctypes.data, len(rec), tri9.ctypes.data, first.ctypes.data, len(first), len(tri9),
                      info.ctypes.data) == 0
    L.ws_set_leafbox(int(os.environ.get("WS_LEAFBOX", "1")))
    L.ws_set_sort(int(os.environ.get("WS_SORT", "1")))
    print(f"wide: {info[0]} nodes ({info[0] * 64 / 1e6:.0f} MB) + {info[1]} triangle records, depth {info[2]}, "
          f"{time.time() - t0:.1f}s (Bvh2 {len(rec) * 64 / 1e6:.0f} MB)", flush=True)
    wtri = np.ctypeslib.as_array(ctypes.cast(L.ws_tris(), ctypes.POINTER(ctypes.c_float)), (int(info[1]) * 16,))
    wtri = wtri.reshape(-1, 16)
    cam = scene_camera("san_miguel_proxy", W, H)
    rng = np.random.default_rng(1)
    cam_rays = camera_rays(cam, W, H)
    sets = [("camera", cam_rays, 0)]
    s2, t2, h2 = trace(L, cam_rays, 0, 0)
    b = bounce(rec, cam_rays, t2, h2, rng)
    sets.append(("bounce", b, 0))
    ld = -np.asarray(sc.lights["d"][0, :3], np.float32)
    ld /= np.linalg.norm(ld)
    sh = bounce(rec, cam_rays, t2, h2, np.random.default_rng(2))
    sh["d"][:, :3] = ld
    sets.append(("shadow", sh, 1))
    if os.environ.get("WS_ALT"):
        # the RR Bvh2 against a 3-axis binned SAH Bvh2 over the same leaf records
        t0 = time.time()
        L.ws_build_alt(rec.ctypes.data, len(rec), int(os.environ["WS_ALT"]))
        alt_p, alt_n = L.ws_alt_ptr(), L.ws_alt_n()
        alt = np.ctypeslib.as_array(ctypes.cast(alt_p, ctypes.POINTER(ctypes.c_float)), (alt_n * 16,)).reshape(-1, 16)
        print(f"3-axis SAH Bvh2 ({os.environ['WS_ALT']} bins) built in {time.time() - t0:.1f}s", flush=True)
        for name, rays, any_ in sets:
            act = rays["extra"][:, 1] != 0
            L.ws_use_tree(rec.ctypes.data, len(rec))
            sA, tA, hA = trace(L, rays, any_, 0)
            L.ws_use_tree(alt_p, alt_n)
            sB, tB, hB = trace(L, rays, any_, 0)
            vA, vB = sA[act].sum(1).mean(), sB[act].sum(1).mean()
            ra = np.where(hA[:, None] >= 0, rec[np.maximum(hA, 0)][:, [3, 7]], -1)
            rb = np.where(hB[:, None] >= 0, alt[np.maximum(hB, 0)][:, [3, 7]], -1)
            diff = act & ~(ra.view(np.uint32) == rb.view(np.uint32)).all(1)
            print(f"{name:7s} RR Bvh2 {vA:6.2f} visits | 3-axis SAH {vB:6.2f} ({vB / vA:.3f}x) | "
                  f"results differ {int(diff.sum())}", flush=True)
        return
    for name, rays, any_ in sets:
        act = rays["extra"][:, 1] != 0
        sA, tA, hA = trace(L, rays, any_, 0)
        sB, tB, hB = trace(L, rays, any_, 1)
        iA, lA = sA[act, 0].mean(), sA[act, 1].mean()
        iB, lB = sB[act, 0].mean(), sB[act, 1].mean()
        line = (f"{name:7s} rays {act.sum():7d} | Bvh2 internal {iA:6.2f} tri {lA:6.2f} total {iA + lA:6.2f} | "
                f"wide internal {iB:6.2f} tri {lB:6.2f} total {iB + lB:6.2f} ({(iB + lB) / (iA + lA):.3f}x)")
        if any_:
            line += f" | occlusion differs {int(((hA >= 0) != (hB >= 0))[act].sum())}"
        else:
            # same triangle: compare the Bvh2 leaf record's (shape, prim) with the wide record's
            ra = np.where(hA[:, None] >= 0, rec[np.maximum(hA, 0)][:, [3, 7]], -1)
            rb = np.where(hB[:, None] >= 0, wtri[np.maximum(hB, 0)][:, [3, 7]], -1)
            same = (ra.view(np.uint32) == rb.view(np.uint32)).all(1)
            diff = act & ~same
            tie = diff & (tA.view(np.uint32) == tB.view(np.uint32))
            line += f" | hits differ {int(diff.sum())} (equal t {int(tie.sum())}, max rel dt " \
                    f"{float(np.max(np.abs(tA[diff] - tB[diff]) / np.maximum(tA[diff], 1e-30))) if diff.any() else 0:.2e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
