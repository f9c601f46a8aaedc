"""CPU tests: the oracle against outputs of the REFERENCE's own OpenCL kernels
(assets/kernels/PathTracing.cl + RadeonRays intersect_bvh2_lds.cl compiled for gfx950 and run
through the ROCm OpenCL runtime on an MI355X by tests/clref_job.py; fixtures
tests/golden/clref_{ieee,fast}.npz, 'fast' = the reference's -cl-fast-relaxed-math build).

Tolerance: per pixel |dL| <= 1e-4 * max(1, |L|) on >= 99.5 % of pixels per 1-spp frame; the rest
are path divergences from fp32 differences (GPU libm vs host libm, FMA contraction).
"""
import os

import numpy as np
import pytest

from clref_job import CASES, build_scene
from helpers import bunny_scene, closest_agreement, rr_cornell_scene
from mcrt import scenes
from mcrt.camera import scene_camera
from oracle import pyoracle as po

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def frac_within(a, b, rtol=1e-4):
    d = np.abs(a[..., :3].astype(np.float64) - b[..., :3])
    return (d <= rtol * np.maximum(1.0, np.abs(b[..., :3]))).all(-1).mean()


@pytest.fixture(scope="module")
def oracles():
    return {}


@pytest.mark.parametrize("variant", ["ieee", "fast"])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}_d{c[4]}" for c in CASES])
def test_frames_match_reference_opencl(oracles, variant, case):
    name, W, H, frames, D = case
    z = np.load(os.path.join(GOLD, f"clref_{variant}.npz"), allow_pickle=False)
    if name not in oracles:
        o = po.OracleScene(build_scene(name))
        o.build()
        oracles[name] = o
    o = oracles[name]
    cam = scene_camera("dragon_proxy" if name == "dragon_small" else name, W, H)
    for f in frames:
        ref = z[f"{name}_{W}x{H}_d{D}_f{f}"]
        mine, _ = o.render(cam, frame=f, max_depth=D)
        assert frac_within(mine, ref) >= 0.995, (name, D, f)


def test_rr_queries_match_reference_opencl():
    z = np.load(os.path.join(GOLD, "clref_ieee.npz"), allow_pickle=False)
    sc, g = rr_cornell_scene()
    o = po.OracleScene(sc)
    o.build()
    h = o.closest(g["rays_closest"])
    ref = z["rr_cornell_closest"]
    np.testing.assert_array_equal(h["shapeid"], ref["shapeid"])
    np.testing.assert_array_equal(h["primid"], ref["primid"])
    np.testing.assert_array_equal(o.any(g["rays_any"]), z["rr_cornell_any"])
    for nm, s in (("bunny", bunny_scene()), ("mixed", scenes.test_scene())):
        o = po.OracleScene(s)
        o.build()
        h = o.closest(z[f"{nm}_rays"])
        eq, dt2 = closest_agreement(h, z[f"{nm}_closest"])
        assert eq > 0.9995 and dt2 <= 1e-5, (nm, eq, dt2)
