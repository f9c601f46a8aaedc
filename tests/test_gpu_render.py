"""GPU parity of the fused wavefront integrator (mcrt_render_frame / mcrt_accumulate)
against the oracle (CPU restatement of PathTracing.cl + ShadowPass + ReconstructionPass).

Tolerance (fp32, stated per SURVEY.md App. A): per pixel |dL| <= 1e-4 * max(1, |L|) for at
least 99.5 % of pixels at 1 spp; the remainder are path divergences (lobe / hit boundary),
bounded by the image-level check: mean relative error of the 1-spp frame and of the
accumulated image <= 1e-3 and per-channel means within 1e-3 relative."""
import numpy as np
import pytest

from helpers import sobol
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu


def pixel_agreement(a, b, rtol=1e-4):
    d = np.abs(a[..., :3].astype(np.float64) - b[..., :3])
    ok = (d <= rtol * np.maximum(1.0, np.abs(b[..., :3]))).all(-1)
    return ok.mean()


@pytest.fixture(scope="module")
def mixed():
    sc = scenes.test_scene()
    sc.sobol = sobol()
    o = po.OracleScene(sc)
    o.build()
    return sc, o


@pytest.mark.parametrize("max_depth", [1, 2, 5])
@pytest.mark.parametrize("sampler", [T.SAMPLER_RANDOM, T.SAMPLER_SOBOL])
def test_frame_parity(hip_ctx, mixed, max_depth, sampler):
    from mcrt import lib
    sc, o = mixed
    W, H = 96, 64
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    for frame in (0, 3):
        cam = scene_camera("mixed", W, H)
        fb.render(ds, cam, frame=frame, max_depth=max_depth, sampler=sampler)
        g = fb.read(0)
        r, _ = o.render(cam, frame=frame, max_depth=max_depth, sampler=sampler)
        assert np.isfinite(g).all()
        frac = pixel_agreement(g, r)
        assert frac >= 0.995, (frame, frac)
        mean_g, mean_r = g[..., :3].mean((0, 1)), r[..., :3].mean((0, 1))
        np.testing.assert_allclose(mean_g, mean_r, rtol=2e-2)
    fb.close()
    ds.close()


def test_accumulated_image_parity(hip_ctx, mixed):
    from mcrt import lib
    sc, o = mixed
    W, H = 64, 48
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    filt = T.make_filter(T.BOX)
    wsum = wts = None
    for frame in range(8):
        cam = scene_camera("mixed", W, H)
        fb.render(ds, cam, frame=frame, max_depth=2)
        fb.accumulate(filt, frame)
        r, _ = o.render(cam, frame=frame, max_depth=2)
        wsum, wts, img_o = po.accumulate(r, frame, filt, wsum, wts)
    img_g = fb.read(2)
    m = np.abs(img_o[..., :3]) > 1e-3
    rel = np.abs(img_g[..., :3] - img_o[..., :3])[m] / np.abs(img_o[..., :3])[m]
    assert rel.mean() <= 1e-3, rel.mean()
    np.testing.assert_allclose(img_g[..., :3].mean((0, 1)), img_o[..., :3].mean((0, 1)), rtol=1e-3)
    fb.close()
    ds.close()


def test_band_split_reproduces_full_frame(hip_ctx, mixed):
    """Tile split across ranks (8-row bands dealt round-robin) gives the same pixels as one GPU."""
    from mcrt import lib
    sc, _ = mixed
    W, H = 64, 80
    ds = lib.DeviceScene(hip_ctx, sc)
    cam = scene_camera("mixed", W, H)
    full = lib.FrameBuffer(hip_ctx, W, H)
    full.render(ds, cam, frame=2)
    ref = full.read(0)
    acc = np.zeros_like(ref)
    for rank in range(3):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.render(ds, cam, frame=2, band_rows=8, num_bands=3, band_index=rank)
        part = fb.read(0)
        rows = np.array([(y // 8) % 3 == rank for y in range(H)])
        acc[rows] = part[rows]
        fb.close()
    np.testing.assert_array_equal(acc, ref)
    full.close()
    ds.close()


def test_cornell_box_frame(hip_ctx, golden):
    from mcrt import lib
    sc = scenes.cornell_box(f"{golden}/cornell_original.npz")
    o = po.OracleScene(sc)
    o.build()
    W, H = 64, 64
    cam = scene_camera("cornell", W, H)
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    fb.render(ds, cam, frame=1, max_depth=2)
    g = fb.read(0)
    r, _ = o.render(cam, frame=1, max_depth=2)
    assert pixel_agreement(g, r) >= 0.995
    fb.close()
    ds.close()


def test_frame_stats_and_no_lights(hip_ctx, mixed):
    from mcrt import lib
    sc, _ = mixed
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, 32, 32)
    cam = scene_camera("mixed", 32, 32)
    fb.render(ds, cam, frame=0, max_depth=2)
    st = fb.stats()
    assert st["closest_rays"] >= 32 * 32 and st["any_rays"] > 0
    ds.update_lights(np.zeros(0, T.LIGHT_DTYPE))
    fb.render(ds, cam, frame=0, max_depth=2)
    assert not fb.read(0).any()
    fb.close()
    ds.close()


@pytest.mark.parametrize("num_bands,band_index", [(1, 0), (3, 1)])
def test_frames_in_flight_accumulate_bit_exact(hip_ctx, mixed, num_bands, band_index):
    """mcrt_framebuffer_set_frames_in_flight: frames rendered in 2..4 overlapping slots and
    accumulated in call order give the one-slot accumulators and last radiance bit for bit."""
    from mcrt import lib
    sc, _ = mixed
    W, H = 96, 72
    ds = lib.DeviceScene(hip_ctx, sc)
    cam = scene_camera("mixed", W, H)
    filt = T.make_filter(T.BOX)
    out = {}
    for fif in (1, 2, 4):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.set_frames_in_flight(fif)
        for frame in range(9):
            fb.render(ds, cam, frame=frame, max_depth=3, band_rows=8, num_bands=num_bands, band_index=band_index)
            fb.accumulate(filt, frame)
        out[fif] = (fb.read(0), fb.read(1), fb.read(2), fb.stats())
        fb.close()
    for fif in (2, 4):
        for k in range(3):
            np.testing.assert_array_equal(out[fif][k].view(np.uint32), out[1][k].view(np.uint32))
        assert out[fif][3] == out[1][3]
    assert out[1][2][..., :3].max() > 0
    with pytest.raises(lib.MCRTError):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        try:
            fb.set_frames_in_flight(5)
        finally:
            fb.close()
    ds.close()


def test_russian_roulette_off_below_start_depth(hip_ctx, mixed):
    """RR is opt-in (the reference has none): with rr_start_depth >= maxDepth
    no extension ray is tested, so the frame is the parity-mode frame bit for bit."""
    from mcrt import lib
    sc, _ = mixed
    W, H = 64, 48
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("mixed", W, H)
    fb.render(ds, cam, frame=2, max_depth=3)
    a = fb.read(0)
    fb.render(ds, cam, frame=2, max_depth=3, rr=True, rr_start=3)
    b = fb.read(0)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    fb.close()
    ds.close()


def test_russian_roulette_unbiased(hip_ctx, mixed):
    """RR perf mode (extension rays survive with p = min(0.95, max(throughput)) and carry
    throughput / p).  Its coin is a separate hash, so the reference's per-(pixel, frame, bounce)
    sample streams are untouched and each RR path is the parity path, cut short or rescaled.
    Unbiasedness: over pixels x frames the mean of (RR - parity) radiance is zero within 4
    standard errors; RR must trace fewer closest-hit rays."""
    from mcrt import lib
    sc, _ = mixed
    W, H, D, F = 64, 48, 5, 24
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("mixed", W, H)
    diffs, base, rays = [], [], [0, 0]
    for frame in range(F):
        fb.render(ds, cam, frame=frame, max_depth=D)
        a = fb.read(0)[..., :3].astype(np.float64)
        rays[0] += fb.stats()["closest_rays"]
        fb.render(ds, cam, frame=frame, max_depth=D, rr=True, rr_start=1)
        b = fb.read(0)[..., :3].astype(np.float64)
        rays[1] += fb.stats()["closest_rays"]
        assert np.isfinite(b).all()
        diffs.append((b - a).sum(-1).ravel())
        base.append(a.sum(-1).ravel())
    d = np.concatenate(diffs)
    se = d.std() / np.sqrt(d.size)
    assert abs(d.mean()) <= 4 * se + 1e-7, (d.mean(), se)
    assert (d != 0).any()                               # RR did act
    assert abs(d.mean()) <= 0.02 * np.concatenate(base).mean()
    assert rays[1] < rays[0], rays
    fb.close()
    ds.close()


@pytest.mark.parametrize("num_bands,band_index,count", [(1, 0, 2), (1, 0, 4), (1, 0, 5), (4, 3, 8), (2, 1, 16), (1, 0, 32),
                                                       (1, 0, 64), (8, 5, 160)])
def test_batched_frames_bit_exact(hip_ctx, mixed, num_bands, band_index, count):
    """mcrt_render_frames + mcrt_accumulate_frames over `count` frames (per-frame jittered
    cameras, per-frame filter weights) give the accumulators of `count` single-frame renders
    and accumulations bit for bit, and the batch's first-frame radiance.  160 frames of one band
    of 8: a rank's call in bench.py's weak scaling at N = 8 (20 steps x 8 frames)."""
    from mcrt import lib
    sc, _ = mixed
    W, H, D = 96, 72, 3
    ds = lib.DeviceScene(hip_ctx, sc)
    band = dict(band_rows=8, num_bands=num_bands, band_index=band_index)
    cams = [scene_camera("mixed", W, H, frame=f, jitter=True) for f in range(2 * count)]
    filts = [T.make_filter(T.GAUSSIAN, pixel_offset=(0.1 * (f % 5) - 0.2, 0.05 * f - 0.3)) for f in range(2 * count)]
    ref = lib.FrameBuffer(hip_ctx, W, H)
    rad0 = {}
    for f in range(2 * count):
        ref.render(ds, cams[f], frame=f, max_depth=D, **band)
        if f % count == 0:
            rad0[f] = ref.read(0)
        ref.accumulate(filts[f], f)
    want = (ref.read(1), ref.read(2))
    fb = lib.FrameBuffer(hip_ctx, W, H)
    for f0 in (0, count):
        fb.render_frames(ds, cams[f0:f0 + count], frame=f0, max_depth=D, **band)
        np.testing.assert_array_equal(fb.read(0).view(np.uint32), rad0[f0].view(np.uint32))
        fb.accumulate_frames(filts[f0:f0 + count], f0)
    np.testing.assert_array_equal(fb.read(1).view(np.uint32), want[0].view(np.uint32))
    np.testing.assert_array_equal(fb.read(2).view(np.uint32), want[1].view(np.uint32))
    assert want[1][..., :3].max() > 0
    st = fb.stats()
    assert st["closest_rays"] > 0
    with pytest.raises(lib.MCRTError):
        fb.accumulate_frames(filts[:2] if count != 2 else filts[:3], 0)   # neither 1 nor count filters
    with pytest.raises(lib.MCRTError):   # MCRT_MAX_BATCH_FRAMES
        fb.render_frames(ds, [cams[0]] * 257, frame=0, max_depth=D)
    with pytest.raises(lib.MCRTError):   # BDPT: MCRT_MAX_BDPT_BATCH_FRAMES (whole-frame arrays per frame)
        fb.render_frames(ds, [cams[0]] * 33, frame=0, max_depth=D, integrator=T.INTEGRATOR_BDPT)
    fb.close()
    ref.close()
    ds.close()


def test_batched_no_lights_after_lit_batch(hip_ctx, mixed):
    """A batch rendered after the lights are removed accumulates zeros for EVERY frame of the
    batch (not stale radiance of the slot's previous batch), exactly as single frames do."""
    from mcrt import lib
    sc, _ = mixed
    W, H, D, count = 64, 48, 2, 4
    cams = [scene_camera("mixed", W, H, frame=f, jitter=True) for f in range(2 * count)]
    filt = T.make_filter(T.BOX)
    ds = lib.DeviceScene(hip_ctx, sc)
    single = lib.FrameBuffer(hip_ctx, W, H)
    batch = lib.FrameBuffer(hip_ctx, W, H)
    for f in range(count):
        single.render(ds, cams[f], frame=f, max_depth=D)
        single.accumulate(filt, f)
    batch.render_frames(ds, cams[:count], frame=0, max_depth=D)
    batch.accumulate(filt, 0)
    lit = batch.read(1)
    assert lit[..., :3].max() > 0
    ds.update_lights(np.zeros(0, T.LIGHT_DTYPE))
    for f in range(count, 2 * count):
        single.render(ds, cams[f], frame=f, max_depth=D)
        single.accumulate(filt, f)
    batch.render_frames(ds, cams[count:], frame=count, max_depth=D)
    batch.accumulate(filt, count)
    for which in (1, 2):
        np.testing.assert_array_equal(batch.read(which).view(np.uint32), single.read(which).view(np.uint32))
    np.testing.assert_array_equal(batch.read(1)[..., :3], lit[..., :3])   # + 4 x zero radiance
    single.close()
    batch.close()
    ds.close()


@pytest.mark.parametrize("ranks,W,H,BR", [(1, 64, 40, 8), (2, 96, 80, 8), (3, 96, 84, 8), (3, 96, 84, 16),
                                         (8, 64, 140, 8)])
def test_band_pack_unpack_through_product(hip_ctx, mixed, ranks, W, H, BR):
    """bench.py's end of job (mcrt.dist.gather_bands_fb), every rank emulated by its own frame
    buffer on this GPU: each renders and accumulates its 8-row bands, packs its own rows straight
    from the frame buffer (mcrt_framebuffer_bands_pack) into its chunk of the gather buffer, and
    rank 0 unpacks the other chunks into its accumulators (mcrt_framebuffer_bands_unpack, image
    recomputed).  Accumulators and image must equal one frame buffer rendering the whole image,
    bit for bit (H = 84, 140: a partial last 8-row block)."""
    import torch
    from mcrt import dist as mdist
    from mcrt import lib
    sc, _ = mixed
    D, frames, batch = 2, 4, 2
    cams = [scene_camera("mixed", W, H, frame=f, jitter=True) for f in range(frames)]
    filt = T.make_filter(T.BOX)
    ds = lib.DeviceScene(hip_ctx, sc)
    full = lib.FrameBuffer(hip_ctx, W, H)
    for f0 in range(0, frames, batch):
        full.render_frames(ds, cams[f0:f0 + batch], frame=f0, max_depth=D)
        full.accumulate(filt, f0)
    wsum = torch.empty(W * H * 4, dtype=torch.float32, device="cuda")
    wts = torch.empty(W * H, dtype=torch.float32, device="cuda")
    full.copy_device(1, wsum.data_ptr())
    full.copy_device(3, wts.data_ptr())
    hip_ctx.sync()
    want = (full.read(1), full.read(2), wts.cpu().numpy())
    send, recv = mdist.band_buffers(H, W, BR, ranks, "cuda")
    maxr = mdist.splat_chunk_rows(H, BR, ranks)
    n = maxr * 5 * W
    recv.fill_(float("nan"))   # rows a chunk does not hold are never read
    fbs = []
    for r in range(ranks):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        if r == 0:
            with pytest.raises(RuntimeError):   # nothing rendered yet
                fb.bands_pack(send.data_ptr())
        for f0 in range(0, frames, batch):
            fb.render_frames(ds, cams[f0:f0 + batch], frame=f0, max_depth=D, band_rows=BR, num_bands=ranks,
                             band_index=r)
            fb.accumulate(filt, f0)
        # the chunk geometry a C++ host reads (mcrt_framebuffer_band_layout) = mcrt.dist's
        assert fb.band_layout() == (maxr, ranks, r)
        fb.bands_pack(recv[r * n:].data_ptr())   # rank r's chunk of the gather
        hip_ctx.sync()
        fbs.append(fb)
    if ranks > 1:
        with pytest.raises(RuntimeError):
            fbs[0].bands_unpack(recv.data_ptr(), maxr - 8)   # chunk too small for the largest share
    fbs[0].bands_unpack(recv.data_ptr(), maxr)
    fbs[0].copy_device(3, wts.data_ptr())
    hip_ctx.sync()
    np.testing.assert_array_equal(fbs[0].read(1).view(np.uint32), want[0].view(np.uint32))
    np.testing.assert_array_equal(fbs[0].read(2).view(np.uint32), want[1].view(np.uint32))
    np.testing.assert_array_equal(wts.cpu().numpy().view(np.uint32), want[2].view(np.uint32))
    assert want[1][..., :3].max() > 0
    for fb in fbs:
        fb.close()
    full.close()
    ds.close()


@pytest.mark.parametrize("ranks", [2, 3])
def test_multi_gpu_reduce_through_product(hip_ctx, mixed, ranks):
    """The multi-GPU path of bench.py, every rank emulated by its own frame buffer on this GPU:
    each renders its 8-row band share of batched frames and accumulates them; the accumulators
    leave through mcrt_framebuffer_copy_device into torch buffers (the RCCL reduce's input),
    are summed as the reduce does (bands are disjoint, so every pixel is x + 0 + ... = x) and
    installed with mcrt_framebuffer_set_accumulation on rank 0.  The accumulators and the image
    must equal one frame buffer rendering the whole image, bit for bit."""
    import torch
    from mcrt import dist as mdist
    from mcrt import lib
    sc, _ = mixed
    W, H, D, frames, batch = 96, 80, 3, 8, 4
    cams = [scene_camera("mixed", W, H, frame=f, jitter=True) for f in range(frames)]
    filt = T.make_filter(T.BOX)
    ds = lib.DeviceScene(hip_ctx, sc)
    full = lib.FrameBuffer(hip_ctx, W, H)
    for f0 in range(0, frames, batch):
        full.render_frames(ds, cams[f0:f0 + batch], frame=f0, max_depth=D)
        full.accumulate(filt, f0)
    want = (full.read(1), full.read(2))
    bufs, fbs = [], []
    for r in range(ranks):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        for f0 in range(0, frames, batch):
            fb.render_frames(ds, cams[f0:f0 + batch], frame=f0, max_depth=D, band_rows=8, num_bands=ranks,
                             band_index=r)
            fb.accumulate(filt, f0)
        buf, s, w = mdist.packed_accumulators(W * H, "cuda")
        fb.copy_device(1, s.data_ptr())
        fb.copy_device(3, w.data_ptr())
        hip_ctx.sync()
        bufs.append(buf)
        fbs.append(fb)
    total = bufs[0].clone()
    for b in bufs[1:]:
        total += b
    torch.cuda.synchronize()
    _, s0, w0 = mdist.packed_accumulators(W * H, "cuda", base=total)
    fbs[0].set_accumulation(s0.data_ptr(), w0.data_ptr())
    np.testing.assert_array_equal(fbs[0].read(1).view(np.uint32), want[0].view(np.uint32))
    np.testing.assert_array_equal(fbs[0].read(2).view(np.uint32), want[1].view(np.uint32))
    assert want[1][..., :3].max() > 0
    for fb in fbs:
        fb.close()
    full.close()
    ds.close()
