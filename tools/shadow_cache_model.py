"""Occluder-cache model for any-hit shadow rays (analysis tool, CPU).

Question: how many node visits would an exact occluder hint save?  A shadow ray first tests
ONE candidate leaf (its box from the parent record, then its triangle, with the traversal's
own arithmetic); if that reports a hit the ray is occluded -- the leaf's box test passing
implies every ancestor's does (monotone rounding of superset boxes), so the reference's
any-hit walk would reach that leaf or an earlier occluder -- and the walk is skipped.
Otherwise the normal walk runs.  Candidates modelled:
  pixel : the occluder the same pixel's bounce-0 shadow ray found in the previous frame
          (TAA-jittered camera);
  cell  : the last occluder found by any shadow ray whose origin fell in the same cell of a
          G^3 grid over the scene bounds (hash of the cell; bounce-0 and bounce-1 rays).
Frames A (fills the caches) and B (uses them) differ in jitter and bounce samples.
Usage: python tools/shadow_cache_model.py [tris] [W] [H]
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import trav_sim as TS  # noqa: E402
from trav_sim import scenes, po, T, scene_camera  # noqa: E402


def jittered_camera_rays(cam, W, H, jx, jy):
    rays = TS.camera_rays(cam, W, H)
    r00, r10, r11, r01 = (cam[k][0, :3].astype(np.float32) for k in ("r00", "r10", "r11", "r01"))
    ys, xs = np.mgrid[0:H, 0:W]
    tx, ty = xs // 8, ys // 8
    key = (ty * (W // 8) + tx) * 64 + (ys % 8) * 8 + (xs % 8)
    order = np.argsort(key.ravel(), kind="stable")
    u = ((xs.ravel()[order] + jx) / W).astype(np.float32)[:, None]
    v = ((ys.ravel()[order] + jy) / H).astype(np.float32)[:, None]
    d = (r00 * (1 - u) + r10 * u) * (1 - v) + (r01 * (1 - u) + r11 * u) * v
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays["d"][:, :3] = d
    return rays


def tri_hits(nodes, rays, cand):
    """Vectorised triangle test of each ray against its candidate leaf (-1 = none)."""
    ok = cand >= 0
    nd = nodes[np.maximum(cand, 0)]
    v0 = nd["lmin_v0"].astype(np.float64)
    e1 = nd["lmax_v1"] - v0
    e2 = nd["rmin_v2"] - v0
    d = rays["d"][:, :3].astype(np.float64)
    o = rays["o"][:, :3].astype(np.float64)
    s1 = np.cross(d, e2)
    den = (s1 * e1).sum(1)
    den = np.where(den == 0, 1e-30, den)
    dd = o - v0
    b1 = (dd * s1).sum(1) / den
    s2 = np.cross(dd, e1)
    b2 = (d * s2).sum(1) / den
    t = (e2 * s2).sum(1) / den
    hit = (b1 >= 0) & (b1 <= 1) & (b2 >= 0) & (b1 + b2 <= 1) & (t >= 0) & (t < rays["o"][:, 3])
    return ok & hit


def shadow_rays_from(nodes, rays, hit_t, hit_node, ld, rng):
    s = TS.bounce_rays(nodes, rays, hit_t, hit_node, rng)
    s["d"][:, :3] = ld
    s["o"][:, 3] = 1000.0
    return s


def cell_keys(p, lo, hi, G):
    c = np.clip(((p - lo) / (hi - lo) * G).astype(np.int64), 0, G - 1)
    return (c[:, 0] * G + c[:, 1]) * G + c[:, 2]


def main():
    tris = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 960
    H = int(sys.argv[3]) if len(sys.argv) > 3 else 544
    t0 = time.time()
    sc = scenes.san_miguel_proxy(tris=tris)
    o = po.OracleScene(sc)
    o.build()
    nodes = o.nodes()
    print(f"scene {sc.num_triangles} tris, {len(nodes)} nodes, {time.time() - t0:.1f}s", flush=True)
    L = TS.lib()
    L.sim_union.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 2
    cam = scene_camera("san_miguel_proxy", W, H)
    ld = -np.asarray(sc.lights["d"][0, :3], np.float32)
    ld /= np.linalg.norm(ld)
    r = nodes[0]
    lo = np.minimum(r["lmin_v0"], r["rmin_v2"]).astype(np.float32)
    hi = np.maximum(r["lmax_v1"], r["rmax"]).astype(np.float32)

    def trace(rays, any_):
        out = np.zeros((len(rays), 3 + TS.KMAX), np.int32)
        ht = np.zeros(len(rays), np.float32)
        hn = np.zeros(len(rays), np.int32)
        L.set_order(0)
        L.sim(nodes.ctypes.data, rays.ctypes.data, len(rays), any_, out.ctypes.data, ht.ctypes.data, hn.ctypes.data)
        return out[:, 0], ht, hn

    frames = []
    for f, (jx, jy) in enumerate(((0.13, 0.71), (0.62, 0.27))):
        rng = np.random.default_rng(10 + f)
        cr = jittered_camera_rays(cam, W, H, jx, jy)
        _, ct, cn = trace(cr, 0)
        s0 = shadow_rays_from(nodes, cr, ct, cn, ld, rng)             # bounce-0 shadow rays
        s0["extra"][:, 1] = cn >= 0
        v0, _, o0 = trace(s0, 1)
        br = TS.bounce_rays(nodes, cr, ct, cn, rng)                   # diffuse bounce
        _, bt, bn = trace(br, 0)
        s1 = shadow_rays_from(nodes, br, bt, bn, ld, rng)             # bounce-1 shadow rays
        s1["extra"][:, 1] = (bn >= 0) & (br["extra"][:, 1] != 0)
        v1, _, o1 = trace(s1, 1)
        frames.append(dict(s0=s0, v0=v0, o0=o0, s1=s1, v1=v1, o1=o1))
        print(f"frame {f}: traced ({time.time() - t0:.0f}s)", flush=True)

    A, B = frames
    for name, rk, vk, ok_ in (("bounce-0", "s0", "v0", "o0"), ("bounce-1", "s1", "v1", "o1")):
        act = B[rk]["extra"][:, 1] != 0
        occ = B[ok_] >= 0
        base = B[vk][act].sum()
        line = f"{name}: rays {act.sum()} occluded {occ[act].mean():.3f} visits/ray {B[vk][act].mean():.1f}" \
               f" (occluded {B[vk][act & occ].mean():.1f}, clear {B[vk][act & ~occ].mean():.1f})"
        print(line, flush=True)
        cands = {}
        if rk == "s0":
            cands["pixel"] = A[ok_]
        for G in (256, 512):
            # last writer per cell from frame A's rays of BOTH bounces (one shared table)
            table = {}
            for kk, oo in (("s0", "o0"), ("s1", "o1")):
                pa = A[kk]["o"][:, :3]
                keys = cell_keys(pa, lo, hi, G)
                m = A[oo] >= 0
                for k_, n_ in zip(keys[m], A[oo][m]):
                    table[int(k_)] = int(n_)
            kb = cell_keys(B[rk]["o"][:, :3], lo, hi, G)
            cands[f"cell{G}"] = np.array([table.get(int(k_), -1) for k_ in kb], np.int32)
        for cname, cand in cands.items():
            h = tri_hits(nodes, B[rk], cand) & act
            if rk == "s0":   # bounce-0 shadow rays are traced as 8x8-tile wave packets
                nw = (len(h) + 63) // 64
                u0 = np.zeros(nw, np.int32)
                u1 = np.zeros(nw, np.int32)
                L.sim_union(nodes.ctypes.data, B[rk].ctypes.data, len(h), 1, np.zeros(len(h), np.uint8).ctypes.data,
                            u0.ctypes.data)
                L.sim_union(nodes.ctypes.data, B[rk].ctypes.data, len(h), 1, h.astype(np.uint8).ctypes.data,
                            u1.ctypes.data)
                print(f"   {cname:8s} packet union per wave {u0.mean():.1f} -> {u1.mean():.1f} "
                      f"(x{u1.sum() / u0.sum():.3f}; all lanes done in {(u1 == 0).mean():.3f} of waves)", flush=True)
            # cost model: a hint hit = 2 record fetches (parent for the box, the leaf);
            # a hint miss = 2 extra fetches on top of the walk; no hint = the walk
            has = (cand >= 0) & act
            cost = np.where(h, 2, B[vk] + np.where(has, 2, 0))[act].sum()
            print(f"   {cname:8s} hint present {has[act].mean():.3f} hint occludes {h[act].mean():.3f} "
                  f"(of occluded {h[act & occ].sum() / max(1, (act & occ).sum()):.3f})  visits x{cost / base:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
