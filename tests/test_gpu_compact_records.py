"""Descent-compact traversal records (mcrt_traverse.h traverseOct2, mcrt_kernels.hip
k_pack_compact): the camera-ray launch walks them by default; MCRT_COMPACT_TRAV=2 makes every
launch walk them and MCRT_COMPACT_TRAV=0 none.  They store each child box only once (the other
child's value of each slot is the node's own box, carried from the previous step), so every slab
test must see the same floats as with the plain records: closest hits, occlusion answers and
whole frames are compared bit for bit between the three settings."""
import numpy as np
import pytest

from helpers import random_rays
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _traces(ctx, sc, rays):
    import torch
    from mcrt import lib
    ds = lib.DeviceScene(ctx, sc)
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    h = torch.zeros(len(rays) * 32, dtype=torch.uint8, device="cuda")
    o = torch.full((len(rays),), -7, dtype=torch.int32, device="cuda")
    ds.trace_closest(r.data_ptr(), len(rays), h.data_ptr())
    ds.trace_any(r.data_ptr(), len(rays), o.data_ptr())
    ctx.sync()
    out = h.cpu().numpy().view(T.ISECT_DTYPE), o.cpu().numpy()
    info = ds.accel_info() if hasattr(ds, "accel_info") else None
    ds.close()
    return out, info


def _frames(ctx, sc, cam_name, W, H, n=2, D=3):
    from mcrt import lib
    ds = lib.DeviceScene(ctx, sc)
    fb = lib.FrameBuffer(ctx, W, H)
    rad = []
    for f in range(n):
        fb.render(ds, scene_camera(cam_name, W, H, frame=f, jitter=True), frame=f, max_depth=D)
        rad.append(fb.read(0))
        fb.accumulate(T.make_filter(T.BOX), f)
    img = fb.read(2)
    fb.close()
    ds.close()
    return rad, img


@pytest.mark.parametrize("which", ["mixed", "sm_small"])
def test_compact_records_queries_bit_exact(hip_ctx, monkeypatch, which):
    sc = scenes.test_scene() if which == "mixed" else scenes.san_miguel_proxy(tris=300_000)
    rays = random_rays(sc, 40000, seed=5)
    # some rays start outside the scene and some are masked / inactive (RR_RAY_MASK, Q12)
    rays[::7]["extra"][:, 0] = 0
    rays[::11]["extra"][:, 1] = 0
    res = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("MCRT_COMPACT_TRAV", mode)
        res[mode], _ = _traces(hip_ctx, sc, rays)
    (h0, o0), (h2, o2) = res["0"], res["2"]
    np.testing.assert_array_equal(h2.view(np.uint8), h0.view(np.uint8))
    np.testing.assert_array_equal(o2, o0)
    assert (h0["shapeid"] >= 0).mean() > 0.3 and (o0 == 1).mean() > 0.1


@pytest.mark.parametrize("which,W,H", [("mixed", 96, 64), ("san_miguel_proxy", 160, 96)])
def test_compact_records_frames_bit_exact(hip_ctx, monkeypatch, which, W, H):
    sc = scenes.test_scene() if which == "mixed" else scenes.san_miguel_proxy(tris=1_000_000)
    out = {}
    for mode in ("0", "1", "2"):
        monkeypatch.setenv("MCRT_COMPACT_TRAV", mode)
        out[mode] = _frames(hip_ctx, sc, which, W, H)
    for mode in ("1", "2"):
        for a, b in zip(out[mode][0], out["0"][0]):
            np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
        np.testing.assert_array_equal(out[mode][1].view(np.uint32), out["0"][1].view(np.uint32))
    assert out["0"][1][..., :3].max() > 0


def test_compact_records_single_triangle(hip_ctx, monkeypatch):
    """A one-triangle tree: the root is a leaf (TraceCtx.rootWord carries the leaf bit)."""
    b = scenes.SceneBuilder("tri")
    m = b.add_material()
    P = np.array([[-1, 0, -1], [1, 0, -1], [0, 0, 1]], np.float32)
    N = np.tile(np.array([[0, 1, 0]], np.float32), (3, 1))
    UV = np.zeros((3, 2), np.float32)
    b.add_mesh(P, N, UV, np.array([[0, 1, 2]], np.uint32), m)
    b.add_directional_light((0.0, -1.0, 0.0), 10.0)
    sc = b.build()
    rays = np.zeros(4, T.RAY_DTYPE)
    rays["o"][:, :3] = [[0, 1, 0], [0, 1, 0], [5, 1, 5], [0, -1, 0]]
    rays["o"][:, 3] = 1000.0
    rays["d"][:, :3] = [[0, -1, 0], [0, 1, 0], [0, -1, 0], [0, 1, 0]]
    rays["extra"][:, 0] = -1
    rays["extra"][:, 1] = 1
    res = {}
    for mode in ("0", "2"):
        monkeypatch.setenv("MCRT_COMPACT_TRAV", mode)
        res[mode], _ = _traces(hip_ctx, sc, rays)
    np.testing.assert_array_equal(res["2"][0].view(np.uint8), res["0"][0].view(np.uint8))
    np.testing.assert_array_equal(res["2"][1], res["0"][1])
    assert list(res["0"][1]) == [1, -1, -1, 1]
