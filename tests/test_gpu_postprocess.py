"""GPU post-process passes (mcrt_postprocess) against the oracle's restatements of the
reference's BilateralDenoise (KRN/Denoise.cl:6-47) and ReinhardToneMapping
(KRN/ToneMapping.cl:42-63).  The reference kernels read and write image2d_t objects, which the
MI355X OpenCL runtime does not support, so they cannot run here; the oracle (IEEE C) is the
pin, at a tolerance that covers exp/division rounding (device: 2.5-ulp OpenCL division and the
device-library exp, as the reference's own build) -- rtol 2e-5."""
import numpy as np
import pytest

from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rendered(hip_ctx):
    from mcrt import lib
    W, H = 80, 56
    ds = lib.DeviceScene(hip_ctx, scenes.test_scene())
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("mixed", W, H)
    for f in range(4):
        fb.render(ds, cam, frame=f, max_depth=2)
        fb.accumulate(T.make_filter(T.BOX), f)
    yield fb, fb.read(2)
    fb.close()
    ds.close()


@pytest.mark.parametrize("radius,ss,sr", [(1, 1.0, 0.1), (3, 2.0, 0.5), (10, 4.0, 2.0)])
def test_denoise_matches_oracle(rendered, radius, ss, sr):
    fb, img = rendered
    fb.postprocess(denoise=True, radius=radius, sigma_spatial=ss, sigma_range=sr)
    got = fb.read(3)
    ref = po.denoise(img, radius, ss, sr)
    np.testing.assert_allclose(got, ref, rtol=2e-5, atol=1e-7)


def test_tonemap_matches_oracle(rendered):
    fb, img = rendered
    fb.postprocess(tonemap=True, min_luminance=2.0)
    got = fb.read(3)
    ref = po.tonemap(img, 2.0)
    ok = np.isfinite(ref)
    np.testing.assert_array_equal(np.isfinite(got), ok)   # L = 0 -> 0/0, as the reference
    np.testing.assert_allclose(got[ok], ref[ok], rtol=2e-5, atol=1e-7)


def test_denoise_then_tonemap_and_passthrough(rendered):
    fb, img = rendered
    fb.postprocess(denoise=True, radius=2, sigma_spatial=1.5, sigma_range=0.3, tonemap=True, min_luminance=4.0)
    got = fb.read(3)
    ref = po.tonemap(po.denoise(img, 2, 1.5, 0.3), 4.0)
    ok = np.isfinite(ref)
    np.testing.assert_allclose(got[ok], ref[ok], rtol=4e-5, atol=1e-7)
    fb.postprocess()   # both passes off: the display image is the accumulated image
    np.testing.assert_array_equal(fb.read(3), img)
    # radius 0 with denoise on: Denoise.cl:18-19 writes nothing -> the previous denoised image stays
    fb.postprocess(denoise=True, radius=2, sigma_spatial=1.5, sigma_range=0.3)
    prev = fb.read(3)
    fb.postprocess(denoise=True, radius=0)
    np.testing.assert_array_equal(fb.read(3), prev)
