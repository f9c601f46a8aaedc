"""GPU tests of the on-device BVH build (mcrt_accel_opts.device_build = 1, mcrt_gpubuild.hip).

The device build writes a different tree (linear BVH) over bit-identical triangle data, so
closest hits must agree with the host build (whose tree is RadeonRays' own, pinned bit-exact by
tests/test_gpu_reference.py) except where two triangles tie at the same t (then the visit order
decides, `t < closest_t` is strict): same shape/primitive on >= 99.99 % of rays, bit-identical t
and barycentrics wherever the primitive agrees, identical any-hit answers, and frames that are
bit-identical to the host build's on >= 99.9 % of pixels (a tie changes the whole path)."""
import time

import numpy as np
import pytest

from helpers import bunny_scene, random_rays, rr_cornell_scene
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _trace(ds, rays, any_hit=False):
    import torch
    r = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    if any_hit:
        out = torch.full((len(rays),), -7, dtype=torch.int32, device="cuda")
        ds.trace_any(r.data_ptr(), len(rays), out.data_ptr())
    else:
        h0 = np.zeros(len(rays), T.ISECT_DTYPE)
        h0["shapeid"] = -7
        out = torch.from_numpy(h0.view(np.uint8).copy()).cuda()
        ds.trace_closest(r.data_ptr(), len(rays), out.data_ptr())
    ds.ctx.sync()
    res = out.cpu().numpy()
    return res if any_hit else res.view(T.ISECT_DTYPE)


@pytest.mark.parametrize("which", ["cornell", "bunny", "mixed", "dragon"])
def test_device_build_queries_match_host_build(hip_ctx, which):
    from mcrt import lib
    if which == "cornell":
        sc = rr_cornell_scene()[0]
    elif which == "bunny":
        sc = bunny_scene()
    elif which == "mixed":
        sc = scenes.test_scene()
    else:
        sc = scenes.dragon_proxy(tris=200_000)
    rays = random_rays(sc, 50000, seed=5)
    host = lib.DeviceScene(hip_ctx, sc)
    dev = lib.DeviceScene(hip_ctx, sc, device_build=True)
    info = dev.info()
    assert info["nodes"] == 2 * sc.num_triangles - 1 and info["triangles"] == sc.num_triangles
    hh, hd = _trace(host, rays), _trace(dev, rays)
    same = (hh["shapeid"] == hd["shapeid"]) & (hh["primid"] == hd["primid"])
    assert same.mean() >= 0.9999, same.mean()
    hit = same & (hh["shapeid"] >= 0)
    np.testing.assert_array_equal(hh["uvwt"][hit].view(np.uint32), hd["uvwt"][hit].view(np.uint32))
    ah, ad = _trace(host, rays, True), _trace(dev, rays, True)
    np.testing.assert_array_equal(ah, ad)
    host.close()
    dev.close()


def test_device_build_frames_match_host_build(hip_ctx):
    from mcrt import lib
    sc = scenes.test_scene()
    W, H = 128, 96
    cam = scene_camera("mixed", W, H)
    out = []
    for device in (False, True):
        ds = lib.DeviceScene(hip_ctx, sc, device_build=device)
        fb = lib.FrameBuffer(hip_ctx, W, H)
        imgs = []
        for f in range(2):
            fb.render(ds, cam, frame=f, max_depth=3)
            imgs.append(fb.read(0))
        out.append(np.stack(imgs))
        fb.close()
        ds.close()
    eq = (out[0].view(np.uint32) == out[1].view(np.uint32)).all(-1)
    assert eq.mean() >= 0.999, eq.mean()


def test_device_build_large_scene_speed(hip_ctx):
    """2M-triangle San-Miguel proxy: the device build is much faster than the host build and its
    tree traces the same primitives on (almost) every camera ray."""
    from mcrt import lib
    sc = scenes.san_miguel_proxy(tris=2_000_000)
    t0 = time.perf_counter()
    dev = lib.DeviceScene(hip_ctx, sc, device_build=True)
    hip_ctx.sync()
    t_dev = time.perf_counter() - t0
    t0 = time.perf_counter()
    host = lib.DeviceScene(hip_ctx, sc, device_build=3)   # the RR-identical tree built on the host
    t_host = time.perf_counter() - t0
    print(f"2M tris: device build {dev.info()['build_ms']:.1f} ms ({t_dev:.2f} s with upload), "
          f"host build {host.info()['build_ms']:.1f} ms ({t_host:.2f} s)")
    assert dev.info()["build_ms"] < host.info()["build_ms"]
    W, H = 160, 90
    cam = scene_camera("san_miguel_proxy", W, H)
    imgs = []
    for ds in (host, dev):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.render(ds, cam, frame=0, max_depth=2)
        imgs.append(fb.read(0))
        fb.close()
    eq = (imgs[0].view(np.uint32) == imgs[1].view(np.uint32)).all(-1)
    assert eq.mean() >= 0.999, eq.mean()
    host.close()
    dev.close()


@pytest.mark.parametrize("which", ["mixed", "dragon"])
def test_perf_tree_frames_within_reference_tolerance(hip_ctx, which):
    """The perf tree (device_build 4: host binned SAH over all three axes, an A/B option) against
    the reference's Bvh2 (device_build 2, bit-exact with the reference's kernels): the same
    triangles in another tree, so only equal-t hit ties may resolve differently -- frames at
    SURVEY App. A's tolerance (|dL| <= 1e-4 max(1, |L|) on >= 99.5 % of pixels), closest hits on
    random rays identical in distance."""
    from mcrt import lib
    sc = scenes.test_scene() if which == "mixed" else scenes.dragon_proxy(tris=200_000)
    W, H = 160, 120
    cam = scene_camera("mixed" if which == "mixed" else "dragon_proxy", W, H)
    rays = random_rays(sc, 20000, seed=7)
    out, hits = [], []
    for mode in (2, 4):
        ds = lib.DeviceScene(hip_ctx, sc, device_build=mode)
        if mode == 4:
            assert ds.builder() == 4
        fb = lib.FrameBuffer(hip_ctx, W, H)
        imgs = []
        for f in range(2):
            fb.render(ds, cam, frame=f, max_depth=3)
            imgs.append(fb.read(0)[..., :3].copy())
        out.append(np.stack(imgs))
        hits.append(_trace(ds, rays))
        fb.close()
        ds.close()
    ok = (np.abs(out[1] - out[0]) <= 1e-4 * np.maximum(1.0, np.abs(out[0]))).all(-1)
    assert ok.mean() >= 0.995, ok.mean()
    t0, t1 = hits[0]["uvwt"][:, 3], hits[1]["uvwt"][:, 3]
    miss0, miss1 = hits[0]["shapeid"] < 0, hits[1]["shapeid"] < 0
    np.testing.assert_array_equal(miss0, miss1)
    np.testing.assert_array_equal(t0[~miss0], t1[~miss1])
