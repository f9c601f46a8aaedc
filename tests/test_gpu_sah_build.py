"""GPU tests of the on-device SAH build (mcrt_accel_opts.device_build = 2, mcrt_sahbuild.hip).

It restates RadeonRays' Bvh2 build (bvh2.cpp:144-712) for the GPU, so its records must be
byte-identical to the host build's (mcrt_bvh.cpp, pinned node for node to the reference's own
builder by tests/test_bvh2l_cpu.py / test_gpu_reference.py).  The only freedom is the sign of a
zero bound (min/max reductions instead of the reference's sequential _mm_min_ps), which no slab
test distinguishes: +0 and -0 compare equal here.  Frames then follow bit for bit."""
import time

import numpy as np
import pytest

from helpers import bunny_scene, rr_cornell_scene
from mcrt import scenes
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _soup(kind, n, seed):
    """Synthetic stress cases: 'grid' (many equal centroid coordinates -> median fallbacks,
    ties in the bins), 'clusters' (identical triangles: zero centroid extent), 'coplanar'."""
    rng = np.random.default_rng(seed)
    b = scenes.SceneBuilder(kind)
    m = b.add_material(kd=(0.5, 0.5, 0.5))
    k = np.arange(n)
    if kind == "grid":
        c = np.stack([k % 97, (k // 97) % 13 * 0.5, np.zeros(n)], 1)
    elif kind == "clusters":
        c = np.where((k % 7 < 3)[:, None], np.stack([k % 7, np.ones(n), 2 * np.ones(n)], 1),
                     rng.uniform(-10, 10, (n, 3)))
    else:
        c = np.stack([rng.uniform(-10, 10, n), rng.uniform(-10, 10, n), np.zeros(n)], 1)
    off = rng.uniform(-0.05, 0.05, (n, 3, 3))
    if kind == "coplanar":
        off[..., 2] = 0.0
    if kind == "clusters":
        off[k % 7 < 3] = 0.01 * np.eye(3)
    P = (c[:, None, :] + off).reshape(-1, 3)
    tris = np.arange(3 * n).reshape(-1, 3)
    b.add_mesh(P, np.tile([0.0, 0.0, 1.0], (3 * n, 1)), np.zeros((3 * n, 2)), tris, m)
    b.add_point_light((0, 0, 20), (10, 10, 10))
    return b.build()


def _same_records(a, b):
    """byte equality with +0 == -0 in float fields"""
    if a.shape != b.shape:
        return False
    ai, bi = a.view(np.uint32), b.view(np.uint32)
    eq = (ai == bi) | ((ai & 0x7fffffff) == 0) & ((bi & 0x7fffffff) == 0)
    return bool(eq.all())


CASES = ["cornell", "bunny", "mixed", "dragon_200k", "grid_50k", "clusters_30k", "coplanar_20k", "tiny_2",
         "tiny_9", "single"]


def _scene(name):
    if name == "cornell":
        return rr_cornell_scene()[0]
    if name == "bunny":
        return bunny_scene()
    if name == "mixed":
        return scenes.test_scene()
    if name == "dragon_200k":
        return scenes.dragon_proxy(tris=200_000)
    if name.startswith(("grid", "clusters", "coplanar")):
        kind, n = name.split("_")
        return _soup(kind, int(n[:-1]) * 1000, 3)
    n = {"tiny_2": 2, "tiny_9": 9, "single": 1}[name]
    return _soup("coplanar", n, 5)


@pytest.mark.parametrize("name", CASES)
def test_device_sah_records_identical_to_host_build(hip_ctx, name):
    from mcrt import lib
    sc = _scene(name)
    host = lib.DeviceScene(hip_ctx, sc, device_build=3)
    dev = lib.DeviceScene(hip_ctx, sc, device_build=2)
    assert dev.builder() == 2 and host.builder() == 0
    default = lib.DeviceScene(hip_ctx, sc)
    assert default.builder() == 2   # the default build is the device one
    default.close()
    assert dev.layout()["depth"] == host.layout()["depth"]
    a, b = host.records(), dev.records()
    assert _same_records(a, b), np.nonzero((a.view(np.uint32) != b.view(np.uint32)).any(1))[0][:10]
    host.close()
    dev.close()


def test_device_sah_san_miguel_identical_and_fast(hip_ctx):
    """The headline scene (10 M triangles): identical records; build time recorded (target
    < 200 ms; the host build takes ~2 s)."""
    from mcrt import lib
    sc = scenes.san_miguel_proxy()
    host = lib.DeviceScene(hip_ctx, sc, device_build=3)
    a = host.records()
    host.close()
    dev = lib.DeviceScene(hip_ctx, sc, build=False)
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        dev.build(device_build=2)
        hip_ctx.sync()
        times.append((time.perf_counter() - t0) * 1e3)
    assert dev.builder() == 2
    print(f"device SAH build of {sc.num_triangles} triangles: {min(times):.1f} ms (runs {times})")
    assert _same_records(a, dev.records())
    assert min(times) < 1000.0
    dev.close()


def test_device_sah_frames_bit_identical(hip_ctx):
    from mcrt import lib
    sc = scenes.test_scene()
    W, H = 96, 64
    cam = scene_camera("mixed", W, H)
    out = []
    for device in (3, 2):
        ds = lib.DeviceScene(hip_ctx, sc, device_build=device)
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.render(ds, cam, frame=1, max_depth=3)
        out.append(fb.read(0))
        fb.close()
        ds.close()
    np.testing.assert_array_equal(out[0], out[1])
