"""The premise of the compact walk's exactness for closest hits (mcrt_traverse.h qwalk; DESIGN.md
§5b; VERDICT r5 "what's weak" 1).  The compact walk visits nodes in another order than the
reference (intersect_bvh2_lds.cl:107-178: its 8-bit outward child boxes change the nearer-first
choice), and repeats a walk on the exact records when its final distance has a near tie (two hits
within alpha = 2^-18).  That gives the reference's answer only if the reference's own answer does
not depend on its visit order beyond that margin.  It can: the reference culls a leaf at its parent
when the leaf box's entry e (fast_intersect_bbox2, :54-63) exceeds the closest distance so far,
but accepts a triangle by its Moller-Trumbore t (common.cl:177-218), computed differently; for a
triangle X with t_X < e_X, a hit Y with t_X < t_Y < e_X found first culls X.  The slab error grows
with |o / d| rather than with t, so it is largest for short hits far from the world origin.

orc_tie_premise (oracle/mcrt_oracle.c) enumerates, per ray, every triangle hit up to twice the
reference's distance (padded boxes, no culling) with the product's arithmetic and finds every such
order-dependent pair among the hits that can decide the answer.  The compact walk sends a walk to
the exact records when its final hit is such a triangle X or when it met X at its leaf and X's box
test failed (mcrt_traverse.h qwalk); only an X whose whole subtree it culls above the leaf escapes
that rule, so the premise asserted here is that order-dependent pairs beyond the near-tie margin
do not occur on the headline scene (the San-Miguel proxy, 10 M triangles, the bench camera; camera
and bounce-1 extension rays of one frame) and are rare on the same scene moved 1000 units from the
origin (where they do occur: rays leaving a surface nearly parallel to it).  The GPU tests compare
both scenes' frames with the exact walk bit for bit (test_gpu_quant_nodes.py).
tools/tie_premise.py runs the full 1920 x 1080 frames (profiles/r06/tie_premise.json).
"""
import numpy as np
import pytest

from helpers import path_rays
from mcrt import scenes
from mcrt.camera import scene_camera, scene_camera_at

ALPHA = 2.0 ** -18   # QTIE_HI / QTIE_LO (mcrt_traverse.h)
W, H = 320, 180       # the bench camera at 1/6 of 1080p per axis (29 k pixels x 2 bounces)


def premise(sc, cam):
    from oracle import pyoracle as po
    o = po.OracleScene(sc)
    o.build()
    rays = np.concatenate(path_rays(o, cam, frame=0, max_depth=2))
    return rays, o.tie_premise(rays, ALPHA)


@pytest.fixture(scope="module")
def sm():
    return scenes.san_miguel_proxy()


@pytest.mark.parametrize("offset", [0.0, 1000.0])
def test_order_dependent_pairs_within_tie_margin(sm, offset):
    sc = sm if offset == 0.0 else scenes.translated(sm, (offset, offset, offset))
    cam = scene_camera_at("san_miguel_proxy", W, H, (offset,) * 3, jitter=True)
    rays, p = premise(sc, cam)
    hit = np.isfinite(p[:, 0])
    assert hit.mean() > 0.5 and len(rays) > W * H
    assert p[:, 5].sum() <= 1e-3 * len(rays), f"{int(p[:, 5].sum())} rays incompletely checked"
    gaps = p[:, 1]
    bad = gaps > ALPHA
    # triangles whose box entry and distance disagree are common (an axis-aligned triangle's box
    # entry and its t are one plane computed two ways) ...
    assert (p[:, 4] > 0).any()
    # ... but pairs that make the reference's answer order-dependent beyond the margin are absent at
    # the origin and rare far from it
    lim = 0 if offset == 0.0 else max(2, len(rays) // 10_000)
    assert bad.sum() <= lim, (f"{int(bad.sum())} of {len(rays)} rays have an order-dependent pair beyond 2^-18: "
                              f"worst gap {gaps.max():.3e}, t {p[bad, 0][:5]}")
