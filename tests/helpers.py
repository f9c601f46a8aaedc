"""Shared test helpers (scene fixtures, ray generators, comparisons)."""
import os

import numpy as np

from mcrt import types as T
from mcrt.scenes import SceneBuilder

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def rr_cornell_scene():
    """RadeonRays conformance fixture (Resources/CornellBox/orig.objm) + its golden rays/hits."""
    z = np.load(os.path.join(GOLDEN, "rr_cornell.npz"), allow_pickle=False)
    b = SceneBuilder("rr_cornell")
    m = b.add_material()
    for i in range(int(z["nshapes"])):
        P = z[f"P{i}"]
        b.add_mesh(P, np.tile([0, 1, 0], (len(P), 1)), np.zeros((len(P), 2)), z[f"T{i}"], m)
    return b.build(), z


def bunny_scene():
    z = np.load(os.path.join(GOLDEN, "bunny.npz"), allow_pickle=False)
    b = SceneBuilder("bunny")
    m = b.add_material()
    P = z["P"]
    b.add_mesh(P, np.tile([0, 1, 0], (len(P), 1)), np.zeros((len(P), 2)), z["T"], m)
    return b.build()


def sobol():
    from mcrt import sobol_matrices
    return sobol_matrices()


def random_rays(scene, n, seed, tmax=1000.0, inside=True):
    """Rays from points inside the scene bbox towards random directions (conformance style)."""
    rng = np.random.default_rng(seed)
    lo, hi = scene.bbox()
    rays = np.zeros(n, T.RAY_DTYPE)
    o = rng.uniform(lo, hi, size=(n, 3)) if inside else rng.uniform(lo - 1, hi + 1, size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays["o"][:, :3] = o
    rays["o"][:, 3] = tmax
    rays["d"][:, :3] = d
    rays["extra"][:, 0] = -1
    rays["extra"][:, 1] = 1
    return rays


def closest_agreement(a, b, tol_dt2=1e-5):
    """RadeonRays conformance criterion (radeon_rays_conformance_test_cl.h:532-542):
    shapeid equal and (dt)^2 <= 1e-5 where hit.  Returns (fraction shapeid equal, max dt^2)."""
    eq = a["shapeid"] == b["shapeid"]
    hit = (a["shapeid"] >= 0) & eq
    dt2 = ((a["uvwt"][hit, 3].astype(np.float64) - b["uvwt"][hit, 3]) ** 2)
    return eq.mean(), (dt2.max() if dt2.size else 0.0)


def path_rays(oscene, cam, frame=0, max_depth=2, threads=8):
    """The camera rays (bounce 0) and extension rays (bounce 1 ..) the oracle's PT traces for one
    frame of `cam` (its path log: o, d, tmax of the ray traced for each bounce's hit), as RAY_DTYPE
    arrays with mask -1 (PT rays, mcrt_kernels.hip), one per bounce."""
    W, H = int(cam["width"][0]), int(cam["height"][0])
    log = oscene.path_log(W, H, max_depth)
    try:
        oscene.render(cam, frame=frame, max_depth=max_depth, threads=threads)
        log = log.copy()
    finally:
        oscene.path_log(None)
    out = []
    for b in range(max_depth):
        rec = log[:, b]
        live = rec[:, 0].view(np.int32) != -2
        r = np.zeros(int(live.sum()), T.RAY_DTYPE)
        r["o"][:, :3] = rec[live, 24:27]
        r["o"][:, 3] = rec[live, 30]
        r["d"][:, :3] = rec[live, 27:30]
        r["extra"][:, 0] = -1
        r["extra"][:, 1] = 1
        out.append(r)
    return out
