"""Where the C oracle's headline frame diverges from the product (the pixels
outside the 1e-4 band "must be explained by lobe- or hit-boundary proximity logs").

GPU box job.  The product is bit-exact with the reference's own PathTracing.cl + RR
intersect_bvh2_lds.cl run live (tests/test_gpu_reference_scale.py), so the reference pipeline's
per-bounce buffers (clref_read) stand in for the product's: this renders the bench's headline frame
(San-Miguel proxy, 1920x1080, D = 2, random sampler, the bench's TAA-jittered camera of frame F)
with the reference (D = 1 for bounce-0 buffers, D = 2 for bounce-1 buffers) and with the oracle
under its path log (oracle/mcrt_oracle.h ORC_PATHLOG_FLOATS), then walks every pixel outside the
band to the FIRST discrete event that differs:

  primary_hit      camera ray hits another triangle (shape/prim)
  shadow0          bounce-0 shadow ray: occluded on one side only
  lobe             BSDF lobe chosen at bounce 0 differs
  termination      extension ray alive on one side only
  extension_hit    bounce-1 ray hits another triangle
  shadow1          bounce-1 shadow ray: occluded on one side only
  continuous       same discrete path; radiance differs by float rounding alone

and, per hit-type event, the proximity that explains it, evaluated in float64 on the oracle's
ray: the hit triangle's minimum barycentric (distance to its nearest edge) and the relative gap
between the two triangles' hit distances; per shadow event, the smallest barycentric of the
occluder either side found, and per continuous event the relative error.

usage: python tools/oracle_divergence.py OUT.json [frame] [scene W H]   (default: the headline)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

D = 2


def tri_index(scene):
    """(shapeid, primid) -> row of scene.world_triangles()"""
    off = np.concatenate([[0], np.cumsum(scene.shapes["numTriangles"].astype(np.int64))])
    return lambda s, p: off[s] + p


def ray_tri(o, d, P):
    """float64 Moller-Trumbore of rays (n,3) against triangles (n,3,3): t, u, v, w (= 1-u-v)."""
    o, d, P = o.astype(np.float64), d.astype(np.float64), P.astype(np.float64)
    e1, e2 = P[:, 1] - P[:, 0], P[:, 2] - P[:, 0]
    pv = np.cross(d, e2)
    det = (e1 * pv).sum(1)
    det = np.where(np.abs(det) < 1e-300, 1e-300, det)
    tv = o - P[:, 0]
    u = (tv * pv).sum(1) / det
    qv = np.cross(tv, e1)
    v = (d * qv).sum(1) / det
    t = (e2 * qv).sum(1) / det
    return t, u, v, 1.0 - u - v


def bary_margin(o, d, P):
    t, u, v, w = ray_tri(o, d, P)
    return np.minimum(np.minimum(u, v), w), t


def pct(a, qs=(50, 90, 99)):
    a = np.asarray(a, np.float64)
    if a.size == 0:
        return None
    return {f"p{q}": float(np.percentile(a, q)) for q in qs} | {"max": float(a.max()), "n": int(a.size)}


def main():
    from mcrt import types as T
    from mcrt.camera import scene_camera
    from oracle import pyoracle as po
    from clref_job import scale_scene

    out_path = sys.argv[1]
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    name = sys.argv[3] if len(sys.argv) > 3 else "san_miguel_proxy"
    W, H = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (1920, 1080)
    t0 = time.time()
    sc = scale_scene(name)
    cam = scene_camera(name, W, H, frame=frame, jitter=True)
    o = po.OracleScene(sc)
    o.build()
    cs = po.CLRefScene(sc, "ieee", nodes=o.nodes())   # the oracle's Bvh2 = RR's, node for node
    print(f"scene + builds {time.time() - t0:.1f}s", flush=True)

    # reference, bounce 0: D = 1 leaves the primary rays/hits and bounce-0 shadow buffers
    cs.render(cam, frame=frame, max_depth=1)
    r_ray0 = cs.read("rays", W, H).view(T.RAY_DTYPE)
    r_hit0 = cs.read("isect", W, H).view(T.ISECT_DTYPE)
    r_occ0 = cs.read("occlusion", W, H).view(np.int32).copy()
    # reference, bounce 1
    ref = cs.render(cam, frame=frame, max_depth=D).reshape(-1, 4)
    r_ray1 = cs.read("rays", W, H).view(T.RAY_DTYPE)
    r_hit1 = cs.read("isect", W, H).view(T.ISECT_DTYPE)
    r_occ1 = cs.read("occlusion", W, H).view(np.int32).copy()
    r_thr = cs.read("throughput", W, H).view(np.int32).reshape(-1, 8)   # prevBsdfFlags at [4]
    print(f"reference frames {time.time() - t0:.1f}s", flush=True)

    log = o.path_log(W, H, D)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    orc, _ = o.render(cam, frame=frame, max_depth=D, threads=threads)
    orc = orc.reshape(-1, 4)
    o.path_log(None)
    print(f"oracle frame {time.time() - t0:.1f}s", flush=True)

    iv = log.view(np.int32)
    d3 = np.abs(orc[:, :3].astype(np.float64) - ref[:, :3])
    bad = ~(d3 <= 1e-4 * np.maximum(1.0, np.abs(ref[:, :3]))).all(1)
    n = len(ref)

    # discrete events, oracle vs reference
    o_hit0 = (iv[:, 0, 0], iv[:, 0, 1])
    prim_diff = (o_hit0[0] != r_hit0["shapeid"]) | ((o_hit0[0] != -1) & (o_hit0[1] != r_hit0["primid"]))
    o_occl0 = iv[:, 0, 7]
    has_sh0 = o_occl0 != -2
    sh0_diff = has_sh0 & ((o_occl0 != -1) != (r_occ0 != -1))
    o_type = iv[:, 0, 5]
    lobe_diff = (o_type != -1) & (o_type != r_thr[:, 4])
    o_alive = log[:, 0, 21] > 0
    # the D = 2 frame rewrote a pixel's ray at bounce 0 iff its path went on (its active flag is
    # cleared again at bounce 1 when the extension ray misses, so compare the rays themselves)
    r_alive = ((r_ray1["o"][:, :3] != r_ray0["o"][:, :3]) | (r_ray1["d"][:, :3] != r_ray0["d"][:, :3])).any(1)
    term_diff = o_alive != r_alive
    o_hit1 = (iv[:, 1, 0], iv[:, 1, 1])
    ext_diff = o_alive & r_alive & ((o_hit1[0] != r_hit1["shapeid"]) |
                                    ((o_hit1[0] != -1) & (o_hit1[1] != r_hit1["primid"])))
    o_occl1 = iv[:, 1, 7]
    sh1_diff = (o_occl1 != -2) & ((o_occl1 != -1) != (r_occ1 != -1))

    order = [("primary_hit", prim_diff), ("shadow0", sh0_diff), ("lobe", lobe_diff), ("termination", term_diff),
             ("extension_hit", ext_diff), ("shadow1", sh1_diff)]
    cat = np.full(n, -1, np.int32)
    for k, (_, m) in enumerate(order):
        cat[(cat == -1) & m] = k
    cats = {name: int(((cat == k) & bad).sum()) for k, (name, _) in enumerate(order)}
    cats["continuous"] = int(((cat == -1) & bad).sum())

    wt = sc.world_triangles()
    ti = tri_index(sc)
    res = {"what": "first differing discrete event of each pixel outside the 1e-4 band, oracle vs the "
                   "reference pipeline (= product, bit-exact), headline frame",
           "scene": f"{name} ({sc.num_triangles} tris)", "size": [W, H], "max_depth": D, "frame": frame,
           "pixels": n, "within_1e-4": float(1 - bad.mean()), "outside": int(bad.sum()),
           "categories": cats,
           "categories_frac_of_all_pixels": {k: v / n for k, v in cats.items()},
           "event_rates_all_pixels": {name: float(m.mean()) for name, m in order}}

    def hit_proximity(mask, log_b, r_hit, o_shape, o_prim):
        sel = np.nonzero(mask & bad)[0]
        if len(sel) == 0:
            return None
        ro = log[sel, log_b, 24:27]
        rd = log[sel, log_b, 27:30]
        both = (o_shape[sel] >= 0) & (r_hit["shapeid"][sel] >= 0)
        rep = {"n": int(len(sel)), "one_side_missed": int((~both).sum())}
        s2 = sel[both]
        if len(s2):
            Po = wt[ti(o_shape[s2], o_prim[s2])]
            Pr = wt[ti(r_hit["shapeid"][s2], r_hit["primid"][s2])]
            mo, to = bary_margin(ro[both], rd[both], Po)
            mr, tr = bary_margin(ro[both], rd[both], Pr)
            gap = np.abs(to - tr) / np.maximum(np.abs(to), 1e-30)
            # edge proximity: the closer of the two triangles' barycentric margins (0 = on an edge)
            edge = np.minimum(np.abs(mo), np.abs(mr))
            rep.update({"edge_margin": pct(edge), "t_rel_gap": pct(gap),
                        "explained_edge_1e-5": float((edge < 1e-5).mean()),
                        "explained_tgap_1e-5": float((gap < 1e-5).mean()),
                        "explained_either": float(((edge < 1e-5) | (gap < 1e-5)).mean())})
        return rep

    res["primary_hit"] = hit_proximity(cat == 0, 0, r_hit0, o_hit0[0], o_hit0[1])
    res["extension_hit"] = hit_proximity(cat == 4, 1, r_hit1, o_hit1[0], o_hit1[1])
    # primary rays: how far apart are the two camera rays (oracle restatement vs reference)
    sel = np.nonzero((cat == 0) & bad)[0]
    if len(sel):
        dd = np.abs(log[sel, 0, 27:30].astype(np.float64) - r_ray0["d"][sel, :3]).max(1)
        res["primary_hit"]["ray_dir_absdiff"] = pct(dd)

    def shadow_proximity(mask, b, r_occ):
        sel = np.nonzero(mask & bad)[0]
        if len(sel) == 0:
            return None
        occ_o = iv[sel, b, 7]
        occ = np.where(occ_o != -1, occ_o, r_occ[sel])   # the side that found an occluder
        rep = {"n": int(len(sel)), "oracle_occluded": int((occ_o != -1).sum())}
        # RR occluded_main reports the hit shape id only: distance of the ray to the occluder shape's
        # silhouette is not recoverable without the prim, so report the shadow-ray length instead
        rep["shadow_tmax"] = pct(log[sel, b, 14])
        rep["occluder_is_light_shape"] = int(np.isin(occ, sc.lights["shapeId"]).sum()) if "shapeId" in \
            sc.lights.dtype.names else None
        return rep

    res["shadow0"] = shadow_proximity(cat == 1, 0, r_occ0)
    res["shadow1"] = shadow_proximity(cat == 5, 1, r_occ1)
    sel = np.nonzero((cat == -1) & bad)[0]
    if len(sel):
        rel = (d3[sel] / np.maximum(1.0, np.abs(ref[sel, :3]))).max(1)
        res["continuous"] = {"n": int(len(sel)), "rel_err": pct(rel),
                             "bounce0_lobe": {str(int(k)): int(v) for k, v in
                                              zip(*np.unique(o_type[sel], return_counts=True))}}
    res["note"] = ("categories are exclusive and ordered by path position (the first difference explains "
                   "the rest of the path). edge_margin = min barycentric of the nearer of the two triangles "
                   "for the oracle's ray (float64); t_rel_gap = |t_oracle_tri - t_ref_tri| / t. A difference "
                   "is 'explained' when the ray passes within 1e-5 (barycentric) of an edge or the two "
                   "surfaces are within 1e-5 relative distance (coplanar / touching geometry).")
    res["elapsed_s"] = round(time.time() - t0, 1)
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("within_1e-4", "outside", "categories")}), flush=True)


if __name__ == "__main__":
    main()
