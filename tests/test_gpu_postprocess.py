"""GPU post-process passes (mcrt_postprocess) against the reference and the oracle.

* ReinhardToneMapping (KRN/ToneMapping.cl:42-63): its two functions, computeLuminanceFromRGB
  (colors.cl:19-22) and toneMapControlled (ToneMapping.cl:37-40), run live from the reference
  sources through oracle/refbuild/clprobe_tonemap.cl; k_tonemap must match them BIT FOR BIT.
* BilateralDenoise (KRN/Denoise.cl:6-47) reads its window through image2d_t inline (no function to
  call), and the MI355X OpenCL runtime has no image support, so it cannot run here: the oracle's
  IEEE C restatement is the pin (parity unpinned against reference code), at a tolerance that
  covers exp/division rounding (device: 2.5-ulp OpenCL division and the device-library exp, as the
  reference's own build) -- rtol 2e-5."""
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


def _tonemap_product(hip_ctx, img, Lwhite):
    """k_tonemap over an arbitrary float4 image: installed as the accumulation with unit weights
    (image = sum / 1, exact), then mcrt_postprocess."""
    import torch
    from mcrt import lib
    H, W = img.shape[:2]
    fb = lib.FrameBuffer(hip_ctx, W, H)
    s = torch.from_numpy(np.ascontiguousarray(img, np.float32).reshape(-1)).cuda()
    w = torch.ones(H * W, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    fb.set_accumulation(s.data_ptr(), w.data_ptr())
    hip_ctx.sync()
    np.testing.assert_array_equal(fb.read(2), img)   # the installed image is the input, bit for bit
    fb.postprocess(tonemap=True, min_luminance=Lwhite)
    out = fb.read(3)
    fb.close()
    return out


@pytest.mark.parametrize("Lwhite", [2.0, 0.37, 11.5])
def test_tonemap_bit_exact_vs_reference_functions(hip_ctx, rendered, Lwhite):
    """k_tonemap == the reference's computeLuminanceFromRGB + toneMapControlled run live, on the
    rendered image and on HDR values over 12 decades (zeros, single-channel, huge, tiny)."""
    _, img = rendered
    rng = np.random.default_rng(7)
    hdr = (10.0 ** rng.uniform(-6, 6, size=(48, 64, 4))).astype(np.float32)
    hdr[rng.random((48, 64)) < 0.05] = 0.0                      # L = 0: 0/0 as the reference
    hdr[..., 0][rng.random((48, 64)) < 0.1] = 0.0                # one channel off
    hdr[..., 3] = rng.uniform(0, 1, size=(48, 64)).astype(np.float32)   # alpha passes through
    for src in (img, hdr):
        got = _tonemap_product(hip_ctx, src, Lwhite)
        ref = po.clref_tonemap(src, Lwhite)
        np.testing.assert_array_equal(got.view(np.uint32)[np.isfinite(ref)], ref.view(np.uint32)[np.isfinite(ref)])
        np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))


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
