"""Compact records (mcrt_traverse.h traverseQOct; TraceCtx::qnodes): the per-ray walks of the
extension, shadow and BDPT launches fetch 32-B internal records with outward-rounded 8-bit child
boxes and 48-B leaves instead of the 64-B records.  The answers must be the 64-B walk's -- the
reference's (intersect_bvh2_lds.cl) -- bit for bit: every frame is compared with the same frame
rendered with MCRT_QUANT_NODES=0, ray queries (closest: shape, primitive, barycentrics, distance;
any: hit or not) with the 64-B records' answers, and near-tie repeats are counted.  The full-size
reference tests (test_gpu_reference_scale.py) run with the compact records on, as the bench."""
import os

import numpy as np
import pytest

from helpers import random_rays
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera, scene_camera_at

pytestmark = pytest.mark.gpu


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def sm_small():
    return scenes.san_miguel_proxy(tris=1_000_000)


FAR = (1000.0, 1000.0, 1000.0)   # the proxy moved away from the world origin (tests/test_tie_premise_cpu.py)


def _frames(hip_ctx, sc, name, W, H, D, integrator=T.INTEGRATOR_PT, calls=2, batch=4, counts=False, offset=None):
    from mcrt import lib
    ds = lib.DeviceScene(hip_ctx, sc)
    info = ds.info()
    fb = lib.FrameBuffer(hip_ctx, W, H)
    out, retr, rays = [], 0, 0
    for c in range(calls):
        cams = [scene_camera(name, W, H, frame=c * batch + k, jitter=True) if offset is None else
                scene_camera_at(name, W, H, offset, frame=c * batch + k, jitter=True) for k in range(batch)]
        if counts:
            hip_ctx.set_profiling(2)
        fb.render_frames(ds, cams, frame=c * batch, max_depth=D, integrator=integrator)
        hip_ctx.sync()
        if counts:
            hip_ctx.set_profiling(False)
            retr += sum(fb.retrace_counts(D))
            rays += sum(fb.queue_counts(D)[1][:D - 1])
        out.append(np.stack([fb.read_frame(k) for k in range(batch)]))
    fb.close()
    ds.close()
    return np.stack(out), info, retr, rays


CASES = [("mixed", 96, 64, 3), ("mixed", 64, 48, 5), ("sm", 256, 144, 2), ("sm", 256, 144, 4)]


@pytest.mark.parametrize("name,W,H,D", CASES + [("sm_far", 256, 144, 2), ("sm_far", 480, 270, 3)])
def test_pt_frames_identical_to_64b_records(hip_ctx, sm_small, name, W, H, D):
    """sm_far: the proxy 1000 units from the origin, where slab tests carry errors of |o / d| ulp and
    the reference's closest hit can depend on its visit order (mcrt_traverse.h, compact records)."""
    off = FAR if name == "sm_far" else None
    sc, cam = ((scenes.test_scene(), "mixed") if name == "mixed" else
               (sm_small if off is None else scenes.translated(sm_small, off), "san_miguel_proxy"))
    q, info_q, retr, rays = _with_env({"MCRT_QUANT_NODES": "1"},
                                      lambda: _frames(hip_ctx, sc, cam, W, H, D, counts=True, offset=off))
    p, info_p, _, _ = _with_env({"MCRT_QUANT_NODES": "0"}, lambda: _frames(hip_ctx, sc, cam, W, H, D, offset=off))
    assert info_q["bytes"] > info_p["bytes"], "compact records not built"
    assert np.isfinite(q).all() and q[..., :3].max() > 0
    diff = q.view(np.uint32) != p.view(np.uint32)
    assert not diff.any(), f"{int(diff.any(-1).sum())} pixels differ"
    # repeats (near ties: two hits within 2^-18 of the distance, crossing or overlapping surfaces;
    # order-dependent candidates) are rare at the origin: 0.18 % of the 1 M-triangle proxy's
    # extension rays; far from it, where flat boxes' entries carry large slab errors, more
    lim = rays // 100 if off is None else rays // 3
    assert rays > 0 and retr <= max(8, lim), (retr, rays)


@pytest.mark.parametrize("cap,lanes", [("1", "64"), ("17", "64"), ("60", "8"), ("8", "48")])
@pytest.mark.parametrize("name,W,H,D", [CASES[1], CASES[3]])
def test_capped_walks_identical(hip_ctx, sm_small, name, W, H, D, cap, lanes):
    """MCRT_WALK_CAP / MCRT_WALK_LANES: k_shadow_extend stops a wave's extension walks once it has
    taken `cap` steps and at most `lanes` lanes still walk; k_walk_resume finishes the unfinished
    ones from their saved state (next record, hit so far, stack).  The visits are those of one
    uncut walk, so the frames are bit-identical to walks that never stop; cap 1 with 64 lanes
    suspends nearly every walk.  (60, 8) is the default; here on every extension launch and at any
    call size (the defaults: the first launch of calls of >= 16 M paths)."""
    sc, cam = (scenes.test_scene(), "mixed") if name == "mixed" else (sm_small, "san_miguel_proxy")
    a, _, _, _ = _with_env({"MCRT_WALK_CAP": cap, "MCRT_WALK_LANES": lanes, "MCRT_WALK_MIN_PATHS": "0",
                            "MCRT_WALK_MAXB": "8"}, lambda: _frames(hip_ctx, sc, cam, W, H, D))
    b, _, _, _ = _with_env({"MCRT_WALK_CAP": "0"}, lambda: _frames(hip_ctx, sc, cam, W, H, D))
    assert np.isfinite(a).all() and a[..., :3].max() > 0
    diff = a.view(np.uint32) != b.view(np.uint32)
    assert not diff.any(), f"{int(diff.any(-1).sum())} pixels differ"


def test_bdpt_frames_match_64b_records(hip_ctx, sm_small):
    """BDPT: the subpath and connection rays over the compact records; equal up to the order of the
    light-tracing splats' float atomics (tests/test_gpu_bdpt.py's 4e-6)."""
    args = (hip_ctx, sm_small, "san_miguel_proxy", 256, 144, 2, T.INTEGRATOR_BDPT)
    q = _with_env({"MCRT_QUANT_NODES": "1"}, lambda: _frames(*args))[0]
    p = _with_env({"MCRT_QUANT_NODES": "0"}, lambda: _frames(*args))[0]
    assert np.isfinite(q).all() and q[..., :3].max() > 0
    np.testing.assert_allclose(q[..., :3], p[..., :3], rtol=4e-6, atol=4e-6)


@pytest.mark.parametrize("cap,lanes", [("1", "64"), ("60", "8")])
def test_bdpt_capped_walks_match(hip_ctx, sm_small, cap, lanes):
    """BDPT's closest-hit launches (k_extend, the light rays of k_extend_pair) with the stop rule on
    (at any call size; cap 1 suspends nearly every walk): the same hits, so the frames equal those
    without it up to the order of the light-tracing splats' float atomics."""
    args = (hip_ctx, sm_small, "san_miguel_proxy", 256, 144, 2, T.INTEGRATOR_BDPT)
    a = _with_env({"MCRT_WALK_CAP": cap, "MCRT_WALK_LANES": lanes, "MCRT_WALK_MIN_PATHS": "0"}, lambda: _frames(*args))[0]
    b = _with_env({"MCRT_WALK_CAP": "0"}, lambda: _frames(*args))[0]
    assert np.isfinite(a).all() and a[..., :3].max() > 0
    np.testing.assert_allclose(a[..., :3], b[..., :3], rtol=4e-6, atol=4e-6)


@pytest.mark.parametrize("name", ["mixed", "sm", "sm_far"])
def test_queries_identical_to_64b_records(hip_ctx, sm_small, name):
    """mcrt_trace_closest / mcrt_trace_any over random rays (RadeonRays' query API) with and without
    the compact records: the same hit records bit for bit (sm_far: the proxy 1000 units from the
    origin)."""
    import torch
    from mcrt import lib
    sc = scenes.test_scene() if name == "mixed" else sm_small if name == "sm" else scenes.translated(sm_small, FAR)
    rays = random_rays(sc, 50_000, seed=5)
    n = len(rays)

    def run():
        ds = lib.DeviceScene(hip_ctx, sc)
        r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
        hits = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        occ = torch.zeros(n, dtype=torch.int32, device="cuda")
        ds.trace_closest(r.data_ptr(), n, hits.data_ptr())
        ds.trace_any(r.data_ptr(), n, occ.data_ptr())
        hip_ctx.sync()
        out = hits.cpu().numpy().copy(), occ.cpu().numpy().copy()
        ds.close()
        return out

    hq, oq = _with_env({"MCRT_QUANT_NODES": "1"}, run)
    hp, op = _with_env({"MCRT_QUANT_NODES": "0"}, run)
    assert (oq == 1).any() and (hq.view(np.int32).reshape(n, 8)[:, 0] >= 0).any()
    assert np.array_equal(oq, op), int((oq != op).sum())
    assert np.array_equal(hq, hp), int((hq.reshape(n, 32) != hp.reshape(n, 32)).any(-1).sum())


def test_lbvh_keeps_64b_records(hip_ctx, sm_small):
    """The compact walk takes the next record as the left child: the LBVH's numbering is not
    depth-first, so that tree keeps the 64-B walk (same answers, no compact records)."""
    from mcrt import lib
    ds = lib.DeviceScene(hip_ctx, scenes.test_scene(), device_build=1)
    info = ds.info()
    ds.close()
    assert info["bytes"] == 64 * info["nodes"]
