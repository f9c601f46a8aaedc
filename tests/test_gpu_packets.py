"""Wave-packet traversal of the coherent launches (mcrt_traverse.h traversePacket): the camera rays
of PT (k_primary_pk) and BDPT (k_extend_pair's camera half) and PT's bounce-0 shadow rays
(k_shadow_extend) walk the tree one node per wave.  A lane that hits both children still visits
them nearer-first (the wave revisits the first child for the lanes that preferred the second), so
every lane tests the nodes of the per-ray traversal in the per-ray order: results must be BIT-
IDENTICAL to MCRT_CAMERA_PACKETS=0 (every launch per ray), ties included.  Compared here: single
frames, batched TAA calls (packed waves), band splits, BDPT vertices, a one-triangle tree (the root
is a leaf) and the camera AOV pass; the full-size reference tests run with packets on."""
import numpy as np
import pytest

from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _with_packets(monkeypatch, on):
    if on:
        monkeypatch.delenv("MCRT_CAMERA_PACKETS", raising=False)
    else:
        monkeypatch.setenv("MCRT_CAMERA_PACKETS", "0")


def _pt(ctx, sc, cam_name, W, H, D, batch, band=None):
    from mcrt import lib
    band = band or {}
    ds = lib.DeviceScene(ctx, sc)
    fb = lib.FrameBuffer(ctx, W, H)
    cams = [scene_camera(cam_name, W, H, frame=f, jitter=True) for f in range(2 * batch)]
    rad = []
    if batch == 1:
        for f in range(2):
            fb.render(ds, cams[f], frame=f, max_depth=D, **band)
            rad.append(fb.read(0))
            fb.accumulate(T.make_filter(T.BOX), f)
    else:
        for f0 in (0, batch):
            fb.render_frames(ds, cams[f0:f0 + batch], frame=f0, max_depth=D, **band)
            rad.append(fb.read(0))
            fb.accumulate_frames([T.make_filter(T.BOX)], f0)
    out = rad + [fb.read(1), fb.read(2)]
    fb.close()
    ds.close()
    return out


def _same(a, b, what):
    for k, (x, y) in enumerate(zip(a, b)):
        np.testing.assert_array_equal(x.view(np.uint32), y.view(np.uint32), err_msg=f"{what} output {k}")


@pytest.mark.parametrize("which,W,H,D,batch", [
    ("mixed", 96, 64, 3, 1),
    ("mixed", 96, 64, 5, 8),
    ("san_miguel_proxy", 160, 96, 2, 1),
    ("san_miguel_proxy", 160, 96, 2, 20),   # the bench's call shape: 20 TAA frames, packed waves
])
def test_packets_pt_bit_exact(hip_ctx, monkeypatch, which, W, H, D, batch):
    sc = scenes.test_scene() if which == "mixed" else scenes.san_miguel_proxy(tris=1_000_000)
    out = {}
    for on in (False, True):
        _with_packets(monkeypatch, on)
        out[on] = _pt(hip_ctx, sc, which, W, H, D, batch)
    _same(out[True], out[False], f"{which} D={D} batch={batch}")
    assert out[False][-1][..., :3].max() > 0


def test_packets_band_split_bit_exact(hip_ctx, monkeypatch):
    """A rank's share (8-row bands dealt to 3 ranks): partial tiles and short launches."""
    sc = scenes.test_scene()
    for r in range(3):
        band = dict(band_rows=8, num_bands=3, band_index=r)
        out = {}
        for on in (False, True):
            _with_packets(monkeypatch, on)
            out[on] = _pt(hip_ctx, sc, "mixed", 100, 70, 2, 4, band)
        _same(out[True], out[False], f"band {r}")


def test_packets_bdpt_vertices_bit_exact(hip_ctx, monkeypatch):
    """BDPT's first camera rays as packets: the camera vertices, counts and own-strategy
    contributions of the per-ray build (radiance may differ in the last bits where light-tracing
    splats land: their float atomics are unordered in the reference too)."""
    from mcrt import lib
    sc = scenes.test_scene()
    W, H, D = 96, 64, 3
    out = {}
    for on in (False, True):
        _with_packets(monkeypatch, on)
        ds = lib.DeviceScene(hip_ctx, sc)
        fb = lib.FrameBuffer(hip_ctx, W, H)
        cams = [scene_camera("mixed", W, H, frame=f, jitter=True) for f in range(4)]
        fb.render_frames(ds, cams, frame=0, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        out[on] = {k: fb.read_bdpt(k) for k in ("camera_vertices", "camera_counts", "light_counts")}
        out[on]["radiance"] = fb.read(0)
        fb.close()
        ds.close()
    for k in ("camera_vertices", "camera_counts", "light_counts"):
        np.testing.assert_array_equal(out[True][k], out[False][k], err_msg=k)
    np.testing.assert_allclose(out[True]["radiance"], out[False]["radiance"], rtol=4e-6, atol=1e-7)
    assert (out[False]["camera_counts"].view(np.int32) > 1).mean() > 0.3


def test_packets_single_triangle_and_aov(hip_ctx, monkeypatch):
    """A one-triangle tree (the root record is a leaf) and the camera-ray AOV pass."""
    from mcrt import lib
    b = scenes.SceneBuilder("tri")
    m = b.add_material()
    P = np.array([[-1, 0, -1], [1, 0, -1], [0, 0, 1]], np.float32)
    N = np.tile(np.array([[0, 1, 0]], np.float32), (3, 1))
    UV = np.zeros((3, 2), np.float32)
    b.add_mesh(P, N, UV, np.array([[0, 1, 2]], np.uint32), m)
    b.add_directional_light((0.0, -1.0, 0.0), 10.0)
    sc = b.build()
    fwd = np.array([0.0, -3.0, 3.0], np.float32) / np.float32(np.sqrt(18.0))
    cam = lib.make_pinhole_camera((0.0, 3.0, -3.0), fwd, (0, 1, 0), 60.0, 0.1, 100.0, 64, 48)
    out = {}
    for on in (False, True):
        _with_packets(monkeypatch, on)
        ds = lib.DeviceScene(hip_ctx, sc)
        fb = lib.FrameBuffer(hip_ctx, 64, 48)
        fb.render(ds, cam, frame=0, max_depth=2)
        out[on] = (fb.read(0), fb.render_aov(ds, cam, T.AOV_ALBEDO))
        fb.close()
        ds.close()
    _same(out[True], out[False], "one triangle")
    assert (out[False][0][..., :3] > 0).any()
