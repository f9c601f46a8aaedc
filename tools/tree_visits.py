"""Node visits per query of the product's flat trees (analysis tool, CPU): the host-built records
(mcrt_accel_build_host_records: device_build 3 = the reference's Bvh2, 4 = the 3-axis SAH perf
tree) converted to tools/trav_sim.c's node format and replayed with the traversal's visit order
(nearer child first, strict t < closest) over camera rays in 8x8 tile order, one diffuse bounce
from their hits and shadow rays toward the scene's first light.
usage: python tools/r3/tree_visits.py [W H]"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd"), os.path.join(ROOT, "tools")]
import trav_sim as ts  # noqa: E402
from mcrt import lib, scenes  # noqa: E402
from mcrt.camera import scene_camera  # noqa: E402

NODE = np.dtype([("lmin_v0", np.float32, 3), ("left", np.uint32), ("lmax_v1", np.float32, 3), ("mesh", np.uint32),
                 ("rmin_v2", np.float32, 3), ("right", np.uint32), ("rmax", np.float32, 3), ("prim", np.uint32)])


def to_nodes(rec):
    n = np.zeros(len(rec), NODE)
    ints = rec.view(np.int32)
    leaf = ints[:, 12] < 0
    i = ~leaf
    n["lmin_v0"][i] = np.stack([rec[i, 0], rec[i, 2], rec[i, 8]], 1)
    n["lmax_v1"][i] = np.stack([rec[i, 1], rec[i, 3], rec[i, 9]], 1)
    n["rmin_v2"][i] = np.stack([rec[i, 4], rec[i, 6], rec[i, 10]], 1)
    n["rmax"][i] = np.stack([rec[i, 5], rec[i, 7], rec[i, 11]], 1)
    n["left"][i] = ints[i, 12]
    n["right"][i] = ints[i, 13]
    v0 = rec[leaf, 0:3]
    n["lmin_v0"][leaf] = v0
    n["lmax_v1"][leaf] = v0 + rec[leaf, 4:7]
    n["rmin_v2"][leaf] = v0 + rec[leaf, 8:11]
    n["left"][leaf] = 0xffffffff
    n["right"][leaf] = 0xffffffff
    return n


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 480
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 272
    sc = scenes.san_miguel_proxy()
    L = ts.lib()
    cam = scene_camera("san_miguel_proxy", W, H)
    res = {"resolution": [W, H]}
    for name, mode in (("bvh2_reference", 3), ("perf_3axis", 4)):
        rec, info = lib.build_host_records(sc, device_build=mode)
        nodes = to_nodes(rec)
        rng = np.random.default_rng(1)
        rays = ts.camera_rays(cam, W, H)
        r = {}
        for q, any_ in (("camera", 0), ("bounce", 0)):
            out = np.zeros((len(rays), 3 + ts.KMAX), np.int32)
            ht = np.zeros(len(rays), np.float32)
            hn = np.zeros(len(rays), np.int32)
            L.set_order(0)
            L.sim(nodes.ctypes.data, rays.ctypes.data, len(rays), any_, out.ctypes.data, ht.ctypes.data, hn.ctypes.data)
            act = rays["extra"][:, 1] != 0
            r[q] = {"rays": int(act.sum()), "visits": round(float(out[act, 0].mean()), 2),
                    "leaf_visits": round(float(out[act, 1].mean()), 2)}
            if q == "camera":
                rays = ts.bounce_rays(nodes, rays, ht, hn, rng)
        res[name] = r
        print(name, r, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
