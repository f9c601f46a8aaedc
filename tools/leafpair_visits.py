"""Leaf-pair schemes for the Bvh2 traversal (analysis tool, CPU): loop
iterations per query now, with both leaves of a leaf-pair parent tested in one iteration when the
ray hits both boxes (P1), and with the parent's record carrying both triangles (P2), per ray and as
64-lane lockstep waves (a wave runs as long as its longest lane) over camera rays in 8x8 tile order
and one diffuse bounce from their hits, on the San-Miguel proxy's reference tree
(tools/trav_sim.c sim_pairs).  usage: python tools/leafpair_visits.py"""
import ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd"), os.path.join(ROOT, "tools")]
import trav_sim as ts
from tree_visits import to_nodes
from mcrt import lib, scenes
from mcrt.camera import scene_camera
W, H = 480, 272
sc = scenes.san_miguel_proxy()
L = ts.lib()
L.sim_pairs.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
cam = scene_camera("san_miguel_proxy", W, H)
t0 = time.time()
rec, info = lib.build_host_records(sc, device_build=3)
print("build", time.time() - t0, flush=True)
nodes = to_nodes(rec)
rng = np.random.default_rng(1)
rays = ts.camera_rays(cam, W, H)
for q in ("camera", "bounce"):
    out = np.zeros((len(rays), 3 + ts.KMAX), np.int32)
    ht = np.zeros(len(rays), np.float32); hn = np.zeros(len(rays), np.int32)
    L.set_order(0)
    L.sim(nodes.ctypes.data, rays.ctypes.data, len(rays), 0, out.ctypes.data, ht.ctypes.data, hn.ctypes.data)
    o2 = np.zeros((len(rays), 5), np.int32)
    L.sim_pairs(nodes.ctypes.data, rays.ctypes.data, len(rays), 0, o2.ctypes.data)
    act = rays["extra"][:, 1] != 0
    n = len(rays) // 64 * 64
    wv = lambda c: o2[:n, c].reshape(-1, 64).max(1).sum()
    print(q, "visits", o2[act, 0].mean(), "(sim", out[act, 0].mean(), ") iter P1", o2[act, 1].mean(), "P2", o2[act, 2].mean(),
          "pair parents", o2[act, 3].mean(), "both", o2[act, 4].mean(),
          "| wave iters base", wv(0), "P1", wv(1) / wv(0), "P2", wv(2) / wv(0), flush=True)
    if q == "camera":
        rays = ts.bounce_rays(nodes, rays, ht, hn, rng)
