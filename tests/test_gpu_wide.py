"""The 4-wide quantized tree (mcrt_accel_opts.traversal_tree = MCRT_TREE_WIDE; mcrt_wide.h,
mcrt_widebuild.hip, mcrt_traverse.h traverseWide) on the GPU:

  * the device build equals the host restatement (mcrt_wide.cpp) record for record;
  * any-hit answers equal the Bvh2's (the RadeonRays-identical tree) on every ray;
  * closest hits equal the Bvh2's -- same triangle, bit-identical (u, v, t) -- except where two
    triangles lie at the same distance up to the slab test's rounding (a relative |dt| <= 1e-6),
    which the two trees visit in different orders;
  * frames (PT and BDPT, batched) agree with the Bvh2 frames on >= 99.9 % of pixels bit for bit;
  * the traversal-stack overflow of a too-deep tree is reported, as for the Bvh2.
The full-size comparison against the reference's own kernels is in test_gpu_reference_scale.py.
"""
import numpy as np
import pytest

from helpers import bunny_scene, random_rays, rr_cornell_scene
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _scene(name):
    return {"cornell": lambda: rr_cornell_scene()[0], "bunny": bunny_scene, "mixed": scenes.test_scene,
            "dragon_200k": lambda: scenes.dragon_proxy(tris=200_000),
            "sm_1m": lambda: scenes.san_miguel_proxy(tris=1_000_000)}[name]()


@pytest.mark.parametrize("name", ["cornell", "bunny", "mixed", "dragon_200k", "sm_1m"])
def test_device_wide_records_identical_to_host(hip_ctx, name):
    from mcrt import lib
    sc = _scene(name)
    ds = lib.DeviceScene(hip_ctx, sc, tree=T.TREE_WIDE)
    assert ds.tree() == T.TREE_WIDE
    dn, dt = ds.read_wide()
    hn, ht = lib.build_host_wide(sc)
    assert dn.shape == hn.shape and dt.shape == ht.shape
    bad = np.nonzero((dn != hn).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} node records differ, first {bad[:8]}"
    assert (dt.view(np.uint32) == ht.view(np.uint32)).all()
    ds.close()


def _trace(ctx, ds, rays):
    import torch
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    h = torch.zeros(len(rays) * 32, dtype=torch.uint8, device="cuda")
    h.view(torch.int32)[:] = -9   # untouched records stay -9
    o = torch.full((len(rays),), -7, dtype=torch.int32, device="cuda")
    ds.trace_closest(r.data_ptr(), len(rays), h.data_ptr())
    ds.trace_any(r.data_ptr(), len(rays), o.data_ptr())
    ctx.sync()
    return h.cpu().numpy().view(T.ISECT_DTYPE), o.cpu().numpy()


def _camera_rays(name, W, H):
    cam = scene_camera(name, W, H)
    r00, r10, r11, r01 = (cam[k][0, :3].astype(np.float64) for k in ("r00", "r10", "r11", "r01"))
    ys, xs = np.mgrid[0:H, 0:W]
    u, v = (xs / W).ravel()[:, None], (ys / H).ravel()[:, None]
    d = (r00 * (1 - u) + r10 * u) * (1 - v) + (r01 * (1 - u) + r11 * u) * v
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.zeros(len(d), T.RAY_DTYPE)
    rays["o"][:, :3] = cam["pos"][0, :3]
    rays["o"][:, 3] = 1000.0
    rays["d"][:, :3] = d
    rays["extra"] = (-1, 1)
    return rays


@pytest.mark.parametrize("name", ["mixed", "dragon_200k", "sm_1m"])
def test_wide_queries_match_bvh2(hip_ctx, name):
    from mcrt import lib
    sc = _scene(name)
    rays = random_rays(sc, 60000, seed=21)
    rays[::7]["extra"][:, 0] = 0    # masked (RR_RAY_MASK, shape 0)
    rays[::11]["extra"][:, 1] = 0   # inactive: records untouched
    cam_name = {"mixed": "mixed", "dragon_200k": "dragon_proxy", "sm_1m": "san_miguel_proxy"}[name]
    rays = np.concatenate([rays, _camera_rays(cam_name, 256, 144)])
    a = lib.DeviceScene(hip_ctx, sc)
    w = lib.DeviceScene(hip_ctx, sc, tree=T.TREE_WIDE)
    ha, oa = _trace(hip_ctx, a, rays)
    hw, ow = _trace(hip_ctx, w, rays)
    a.close()
    w.close()
    np.testing.assert_array_equal(ow, oa)   # any hit: identical answers, inactive untouched
    same = (ha.view(np.uint32).reshape(len(rays), -1) == hw.view(np.uint32).reshape(len(rays), -1)).all(1)
    diff = ~same
    # a differing closest hit must be a (near-)tie: both hits, same t up to the slab rounding
    both = (ha["shapeid"] >= 0) & (hw["shapeid"] >= 0)
    assert both[diff].all(), "a ray hit in one tree and missed in the other"
    ta, tw = ha["uvwt"][:, 3].astype(np.float64), hw["uvwt"][:, 3].astype(np.float64)
    rel = np.abs(ta - tw) / np.maximum(np.abs(ta), 1e-30)
    assert (rel[diff] <= 1e-6).all(), rel[diff].max()
    assert diff.mean() <= 1e-4, (int(diff.sum()), len(rays))
    print(f"{name}: {int(diff.sum())} of {len(rays)} closest hits are ties resolved differently")


def _render(ctx, sc, cam_name, W, H, tree, n=3, D=3, bdpt=False):
    from mcrt import lib
    ds = lib.DeviceScene(ctx, sc, tree=tree)
    fb = lib.FrameBuffer(ctx, W, H)
    rad = []
    if bdpt:
        for f in range(n):
            fb.render(ds, scene_camera(cam_name, W, H), frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
            rad.append(fb.read(0))
    else:
        cams = [scene_camera(cam_name, W, H, frame=f, jitter=True) for f in range(n)]
        fb.render_frames(ds, cams, frame=0, max_depth=D)
        rad = [fb.read_frame(k) for k in range(n)]
    fb.accumulate(T.make_filter(T.BOX), 0)
    img = fb.read(2)
    fb.close()
    ds.close()
    return rad, img


@pytest.mark.parametrize("name,bdpt", [("mixed", False), ("sm_1m", False), ("mixed", True)])
def test_wide_frames_match_bvh2(hip_ctx, name, bdpt):
    sc = _scene(name)
    cam_name = "mixed" if name == "mixed" else "san_miguel_proxy"
    W, H = (96, 72) if name == "mixed" else (320, 180)
    ra, _ = _render(hip_ctx, sc, cam_name, W, H, T.TREE_BVH2, bdpt=bdpt)
    rw, _ = _render(hip_ctx, sc, cam_name, W, H, T.TREE_WIDE, bdpt=bdpt)
    for k, (a, w) in enumerate(zip(ra, rw)):
        assert np.isfinite(w).all()
        ex = (a.view(np.uint32) == w.view(np.uint32)).all(-1)
        if bdpt:   # splat order: the reference's own CAS atomics leave it open (test_gpu_bdpt.py)
            ex |= (np.abs(a - w) <= 4e-6 * (np.abs(a) + np.abs(w)) + 1e-30).all(-1)
        assert ex.mean() >= 0.999, (k, float(ex.mean()))


def _stacked_quads(n):
    from mcrt.scenes import SceneBuilder
    b = SceneBuilder("stack")
    m = b.add_material()
    z = np.arange(n, dtype=np.float64)[:, None] * 1e-3 + 10.0
    quad = np.array([[-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0]], np.float64)
    P = (quad[None, :, :] + np.concatenate([np.zeros((n, 2)), z], 1)[:, None, :]).reshape(-1, 3)
    k = 4 * np.arange(n)[:, None]
    T_ = np.concatenate([k + [0, 1, 2], k + [0, 2, 3]], 1).reshape(-1, 3)
    b.add_mesh(P, np.tile([0, 0, 1], (len(P), 1)), np.zeros((len(P), 2)), T_, m)
    return b.build()


def test_wide_stack_overflow_is_reported(hip_ctx, monkeypatch):
    """As test_gpu_trace.py::test_traversal_stack_overflow_is_reported for the wide tree: with
    the spill columns capped at 0 entries (MCRT_TEST_SPILL_CAP) a ray down a column of 65536
    stacked quads needs more than the 16 LDS entries; the default capacity traces it correctly."""
    import torch
    from mcrt import lib
    sc = _stacked_quads(1 << 16)
    rays = np.zeros(64, T.RAY_DTYPE)
    rays["o"] = (0.1, 0.2, -10.0, 1e6)
    rays["d"] = (0.0, 0.0, 1.0, 0.0)
    rays["extra"] = (-1, 1)
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    h = torch.zeros(64 * 32, dtype=torch.uint8, device="cuda")
    ok = lib.DeviceScene(hip_ctx, sc, tree=T.TREE_WIDE)
    assert ok.tree() == T.TREE_WIDE
    ok.trace_closest(r.data_ptr(), 64, h.data_ptr())
    hip_ctx.sync()
    hits = h.cpu().numpy().view(T.ISECT_DTYPE)
    assert (hits["shapeid"] == 0).all()
    np.testing.assert_allclose(hits["uvwt"][:, 3], 20.0, rtol=1e-6)   # origin z = -10, first quad at z = 10
    ok.close()
    monkeypatch.setenv("MCRT_TEST_SPILL_CAP", "0")
    bad = lib.DeviceScene(hip_ctx, sc, tree=T.TREE_WIDE)
    monkeypatch.delenv("MCRT_TEST_SPILL_CAP")
    bad.trace_closest(r.data_ptr(), 64, h.data_ptr())
    with pytest.raises(lib.MCRTError, match="overflow"):
        hip_ctx.sync()
    hip_ctx.sync()
    bad.close()


def test_wide_request_on_instanced_scene_keeps_two_level(hip_ctx):
    from mcrt import lib
    ds = lib.DeviceScene(hip_ctx, scenes.instances_test_scene(), tree=T.TREE_WIDE)
    assert ds.layout()["two_level"] == 1 and ds.tree() == T.TREE_BVH2
    ds.close()
