"""GPU parity of the HIP traversal (mcrt_trace_closest / mcrt_trace_any, the drop-in for
RadeonRays QueryIntersection / QueryOcclusion) against the reference's golden brute force
(RR conformance criterion: shapeid equal, dt^2 <= 1e-5) and against the oracle's restatement
of intersect_bvh2_lds.cl (same BVH topology: hit shape/prim equal except exact ties)."""
import numpy as np
import pytest

from helpers import bunny_scene, closest_agreement, random_rays, rr_cornell_scene
from mcrt import scenes
from mcrt import types as T
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def _gpu_trace(ctx, scene, rays, any_hit=False, init=-7):
    import torch
    from mcrt import lib
    ds = lib.DeviceScene(ctx, scene)
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    if any_hit:
        out = torch.full((len(rays),), init, dtype=torch.int32, device="cuda")
        ds.trace_any(r.data_ptr(), len(rays), out.data_ptr())
    else:
        h0 = np.zeros(len(rays), T.ISECT_DTYPE)
        h0["shapeid"] = init
        h0["primid"] = init
        out = torch.from_numpy(h0.view(np.uint8).copy()).cuda()
        ds.trace_closest(r.data_ptr(), len(rays), out.data_ptr())
    ctx.sync()
    res = out.cpu().numpy()
    ds.close()
    return res if any_hit else res.view(T.ISECT_DTYPE)


def test_rr_conformance_closest(hip_ctx):
    sc, z = rr_cornell_scene()
    h = _gpu_trace(hip_ctx, sc, z["rays_closest"])
    eq, dt2 = closest_agreement(h, z["golden_closest"])
    assert eq == 1.0, eq
    assert dt2 <= 1e-5


def test_rr_conformance_any(hip_ctx):
    sc, z = rr_cornell_scene()
    np.testing.assert_array_equal(_gpu_trace(hip_ctx, sc, z["rays_any"], any_hit=True), z["golden_any"])


@pytest.mark.parametrize("which", ["bunny", "mixed"])
def test_closest_vs_oracle(hip_ctx, which):
    sc = bunny_scene() if which == "bunny" else scenes.test_scene()
    rays = random_rays(sc, 20000, seed=11)
    o = po.OracleScene(sc)
    o.build()
    ho = o.closest(rays)
    hg = _gpu_trace(hip_ctx, sc, rays)
    same = (ho["shapeid"] == hg["shapeid"]) & (ho["primid"] == hg["primid"])
    assert same.mean() > 0.999, same.mean()
    hit = same & (ho["shapeid"] >= 0)
    np.testing.assert_allclose(hg["uvwt"][hit, 3], ho["uvwt"][hit, 3], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(hg["uvwt"][hit, :2], ho["uvwt"][hit, :2], atol=2e-3)
    # mismatches must be near-ties (same distance within tolerance)
    diff = ~same & (ho["shapeid"] >= 0) & (hg["shapeid"] >= 0)
    if diff.any():
        np.testing.assert_allclose(hg["uvwt"][diff, 3], ho["uvwt"][diff, 3], rtol=1e-3)


def test_any_vs_oracle(hip_ctx):
    sc = scenes.test_scene()
    rays = random_rays(sc, 20000, seed=12, tmax=3.0)
    o = po.OracleScene(sc)
    o.build()
    a = o.any(rays)
    g = _gpu_trace(hip_ctx, sc, rays, any_hit=True)
    assert (a == g).mean() > 0.999


def test_inactive_untouched_and_mask(hip_ctx):
    sc, z = rr_cornell_scene()
    rays = z["rays_closest"][:512].copy()
    rays["extra"][::2, 1] = 0
    h = _gpu_trace(hip_ctx, sc, rays)
    assert (h["shapeid"][::2] == -7).all() and (h["primid"][::2] == -7).all()
    full = _gpu_trace(hip_ctx, sc, z["rays_closest"][:512])
    masked = z["rays_closest"][:512].copy()
    masked["extra"][:, 0] = np.where(full["shapeid"] >= 0, full["shapeid"], -1)
    hm = _gpu_trace(hip_ctx, sc, masked)
    assert not np.any((full["shapeid"] >= 0) & (hm["shapeid"] == full["shapeid"]))


def test_single_triangle_known_answer(hip_ctx):
    # RR UnitTest Intersection_1Ray (radeon_rays_apitest_cl.h:203-247): triangle (-1,-1,0),(0,1,0),(1,-1,0)
    b = scenes.SceneBuilder()
    m = b.add_material()
    b.add_mesh([(-1, -1, 0), (0, 1, 0), (1, -1, 0)], [(0, 0, 1)] * 3, [(0, 0)] * 3, [(0, 1, 2)], m)
    sc = b.build()
    rays = np.zeros(3, T.RAY_DTYPE)
    rays["o"] = [(0, 0, -10, 10000), (0, 0, 10, 10000), (5, 5, -10, 10000)]
    rays["d"] = [(0, 0, 1, 0), (0, 0, -1, 0), (0, 0, 1, 0)]
    rays["extra"] = (-1, 1)
    h = _gpu_trace(hip_ctx, sc, rays)
    assert list(h["shapeid"]) == [0, 0, -1]   # no backface culling (RR_BACKFACE_CULL OFF)
    np.testing.assert_allclose(h["uvwt"][:2, 3], [10.0, 10.0], rtol=1e-6)
    assert list(_gpu_trace(hip_ctx, sc, rays, any_hit=True)) == [1, 1, -1]


def test_empty_query_and_errors(hip_ctx):
    from mcrt import lib
    sc, _ = rr_cornell_scene()
    ds = lib.DeviceScene(hip_ctx, sc, build=False)
    with pytest.raises(lib.MCRTError):
        ds.trace_closest(0, 1, 0)        # not built
    ds.build()
    ds.trace_closest(0, 0, 0)            # n = 0 is a no-op
    ds.close()


def _stacked_quads(n):
    """n parallel unit quads at z = 0..n-1: a ray along +z through the centre intersects every
    internal node's both children, so a closest-hit traversal keeps ~log2(2n) entries on its
    stack (more than the 16-entry LDS stack for n = 2^16)."""
    b = scenes.SceneBuilder("stacked")
    m = b.add_material()
    z = np.arange(n, dtype=np.float32)
    P = np.zeros((4 * n, 3), np.float32)
    P[0::4] = np.stack([-np.ones(n), -np.ones(n), z], -1)
    P[1::4] = np.stack([np.ones(n), -np.ones(n), z], -1)
    P[2::4] = np.stack([np.ones(n), np.ones(n), z], -1)
    P[3::4] = np.stack([-np.ones(n), np.ones(n), z], -1)
    k = 4 * np.arange(n)[:, None]
    T_ = np.concatenate([k + [0, 1, 2], k + [0, 2, 3]], 1).reshape(-1, 3)
    b.add_mesh(P, np.tile([0, 0, 1], (len(P), 1)), np.zeros((len(P), 2)), T_, m)
    return b.build()


def test_traversal_stack_overflow_is_reported(hip_ctx, monkeypatch):
    """A traversal that needs more stack entries than its spill column holds drops entries
    (mcrt_traverse.h); the next synchronisation must report it (MCRT_ERROR_DEVICE), not return
    silently.  The spill columns are capped at 0 entries by the MCRT_TEST_SPILL_CAP test hook, so
    the deep stack of a ray along a column of 65536 quads overflows the 16-entry LDS stack."""
    import torch
    from mcrt import lib
    sc = _stacked_quads(1 << 16)
    rays = np.zeros(64, T.RAY_DTYPE)
    rays["o"] = (0.1, 0.2, -10.0, 1e6)
    rays["d"] = (0.0, 0.0, 1.0, 0.0)
    rays["extra"] = (-1, 1)
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    h = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    # the default spill capacity covers the tree: correct hit, no error
    ok = lib.DeviceScene(hip_ctx, sc)
    assert ok.layout()["depth"] > 16
    ok.trace_closest(r.data_ptr(), 64, h.data_ptr())
    hip_ctx.sync()
    hits = h.cpu().numpy().view(T.ISECT_DTYPE)
    assert (hits["shapeid"] == 0).all()
    np.testing.assert_allclose(hits["uvwt"][:, 3], 10.0, rtol=1e-6)
    ok.close()
    monkeypatch.setenv("MCRT_TEST_SPILL_CAP", "0")
    bad = lib.DeviceScene(hip_ctx, sc)
    monkeypatch.delenv("MCRT_TEST_SPILL_CAP")
    bad.trace_closest(r.data_ptr(), 64, h.data_ptr())
    with pytest.raises(lib.MCRTError, match="overflow"):
        hip_ctx.sync()
    hip_ctx.sync()   # the flag is cleared once reported
    bad.close()


def test_device_count_queries_with_events(hip_ctx):
    """RR's QueryIntersection / QueryOcclusion with the ray count in device memory and events
    (radeon_rays.h:272-277): min(*count, maxrays) rays are traced -- bit-identical to the
    host-count call on those rays -- the rest of the output is untouched; a count above maxrays
    is clamped; the second query waits on the first's event."""
    import torch
    from mcrt import lib
    sc = scenes.test_scene()
    n = 5000
    rays = random_rays(sc, n, seed=3)
    ds = lib.DeviceScene(hip_ctx, sc)
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    ref_h = torch.full((n * 32,), 0xAB, dtype=torch.uint8, device="cuda")   # a miss leaves uvwt untouched
    ref_o = torch.zeros(n, dtype=torch.int32, device="cuda")
    ds.trace_closest(r.data_ptr(), n, ref_h.data_ptr())
    ds.trace_any(r.data_ptr(), n, ref_o.data_ptr())
    hip_ctx.sync()
    for k in (0, 1, 1234, n, n + 999):
        cnt = torch.tensor([k], dtype=torch.int32, device="cuda")
        h = torch.full((n * 32,), 0xAB, dtype=torch.uint8, device="cuda")
        o = torch.full((n,), -5, dtype=torch.int32, device="cuda")
        e1 = ds.trace_count(False, r.data_ptr(), cnt.data_ptr(), n, h.data_ptr(), want_event=True)
        e2 = ds.trace_count(True, r.data_ptr(), cnt.data_ptr(), n, o.data_ptr(), wait_event=e1, want_event=True)
        lib.event_wait(e2)
        m = min(k, n)
        hh, rh = h.cpu().numpy().reshape(n, 32), ref_h.cpu().numpy().reshape(n, 32)
        np.testing.assert_array_equal(hh[:m], rh[:m])
        assert (hh[m:] == 0xAB).all()
        oo, ro = o.cpu().numpy(), ref_o.cpu().numpy()
        np.testing.assert_array_equal(oo[:m], ro[:m])
        assert (oo[m:] == -5).all()
        lib.event_destroy(e1)
        lib.event_destroy(e2)
    with pytest.raises(lib.MCRTError):
        ds.trace_count(False, r.data_ptr(), None, n, ref_h.data_ptr())
    ds.close()
