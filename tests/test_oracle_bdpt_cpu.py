"""CPU tests: the oracle's BDPT restatement (oracle/mcrt_oracle.c, KRN/BDPT.cl in RTBDPTPass order)
against the REFERENCE's own BDPT.cl kernels run on an MI355X (committed fixtures
tests/golden/clref_bdpt_ieee.npz, tests/clref_job.py ... bdpt): frames rendered in sequence from
fresh (zero-filled) state, so the s = 1 strategy's previous-frame sampled light vertex
(BDPT.cl:585-586) is reproduced too.

Tolerance (as the PT oracle): per pixel |dL| <= 1e-4 * max(1, |L|) on >= 99.5 % of
pixels per 1-spp frame, the rest are path divergences (host libm and IEEE division vs the GPU's,
no contraction) -- in BDPT a diverged light subpath also moves its light-tracing splats; subpath
vertex counts equal on >= 99.5 % of pixels."""
import os

import numpy as np
import pytest

from clref_job import BDPT_CASES, bdpt_key, build_scene
from mcrt.camera import scene_camera
from oracle import pyoracle as po

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("case", BDPT_CASES, ids=[bdpt_key(c) for c in BDPT_CASES])
def test_bdpt_oracle_matches_reference(case):
    name, W, H, frames, D = case
    key = bdpt_key(case)
    z = np.load(os.path.join(GOLD, "clref_bdpt_ieee.npz"), allow_pickle=False)
    o = po.OracleScene(build_scene(name))
    o.build()
    b = po.OracleBDPT(o, W, H, D)
    cam = scene_camera(name, W, H)
    for f in frames:
        rad, cc, lc, st = b.render(cam, frame=f)
        ref = z[f"{key}_f{f}"][..., :3].astype(np.float64)
        d = np.abs(rad[..., :3] - ref)
        ok = (d <= 1e-4 * np.maximum(1.0, np.abs(ref))).all(-1).mean()
        assert ok >= 0.995, (key, f, ok)
        assert st[0] > 0 and st[2] > 0
    assert (cc == z[f"{key}_camera_counts"].view(np.int32)).mean() >= 0.995
    assert (lc == z[f"{key}_light_counts"].view(np.int32)).mean() >= 0.995


def test_bdpt_oracle_rows_and_no_lights():
    """Row-subset rendering (the bench's CPU baseline sample) fills only those rows' own
    strategies; a scene without lights renders black (RTBDPTPass.cpp:69)."""
    sc = build_scene("mixed")
    o = po.OracleScene(sc)
    o.build()
    W, H = 48, 32
    cam = scene_camera("mixed", W, H)
    full, _, _, _ = po.OracleBDPT(o, W, H, 2).render(cam, frame=0)
    rows = np.array([3, 17, 30], np.int32)
    part, cc, _, st = po.OracleBDPT(o, W, H, 2).render(cam, frame=0, rows=rows)
    assert (cc.reshape(H, W)[rows] >= 1).all() and (cc.reshape(H, W)[[0, 1, 2]] == 0).all()
    assert st[0] > 0 and np.abs(part).sum() > 0
    sc.lights = sc.lights[:0]
    o2 = po.OracleScene(sc)
    o2.build()
    rad, _, _, _ = po.OracleBDPT(o2, W, H, 2).render(cam, frame=0)
    assert not rad.any()
    assert full[..., :3].max() > 0
