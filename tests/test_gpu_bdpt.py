"""GPU parity of the BDPT integrator (mcrt_bdpt.hip) against the REFERENCE's own BDPT.cl kernels
run live on this MI355X through RTBDPTPass's launch sequence (tests/clref_job.py ... bdpt, in a
child process).

What is compared, per case (frames rendered in order from fresh buffers on both sides, since
the reference's s = 1 strategy reads the previous frame's sampled light vertex, BDPT.cl:585):
  * vertex counts of both subpaths: bit-exact;
  * every defined field of every camera / light subpath vertex (position, normals, directions,
    uv, throughput, pdfFwd, pdfRev, type, flags, light, material): bit-exact;
  * the frame radiance: the reference sums each pixel's strategies with float atomics whose
    order depends on thread scheduling (light-tracing splats from other pixels interleave,
    BDPT.cl:888-907), so the image is compared with a relative tolerance of 4e-6 (a few ulp of
    a sum of <= ~30 non-negative terms) and the bit-exact fraction is reported."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import BDPT_CASES, bdpt_key, build_scene
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
REL_TOL = 4e-6


@pytest.fixture(scope="module")
def clref_bdpt(tmp_path_factory):
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = str(tmp_path_factory.mktemp("clref") / "clref_bdpt.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee", "bdpt"],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail("reference BDPT job failed:\n" + r.stdout + r.stderr)
    return np.load(out, allow_pickle=False)


def our_planes(raw, depths, N):
    """(depths, planes, N, 4) float32 view of the product's vertex planes (planes 0-7 = the vertex)."""
    f = raw.view(np.float32)
    return f.reshape(depths, f.size // (depths * N * 4), N, 4)


def compare_vertices(ours, ref, counts, depths, N, label):
    """Bit-exact comparison of the defined vertex fields; returns a list of mismatch messages."""
    bad = []
    f32 = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)   # noqa: E731
    for d in range(depths):
        live = counts > d
        if not live.any():
            continue
        o = ours[d]                         # (8, N, 4)
        r = ref[:, d]                       # (N,) structured
        typ = r["type"]
        fields = {
            "p": (o[0, :, :3], r["p"][:, :3]), "throughput": (o[6, :, :3], r["throughput"][:, :3]),
            "pdfFwd": (o[1, :, 3], r["pdfFwd"]), "pdfRev": (o[2, :, 3], r["pdfRev"]),
            "type": (o[7, :, 0].view(np.int32), typ), "flags": (o[7, :, 1].view(np.int32), r["flags"]),
            "lightIdx": (o[7, :, 2].view(np.int32), r["lightIdx"]),
        }
        surf = {
            "gn": (o[1, :, :3], r["gn"][:, :3]), "sn": (o[2, :, :3], r["sn"][:, :3]),
            "wo": (o[3, :, :3], r["wo"][:, :3]), "sdpdu": (o[4, :, :3], r["sdpdu"][:, :3]),
            "sdpdv": (o[5, :, :3], r["sdpdv"][:, :3]), "uv": (np.stack([o[4, :, 3], o[5, :, 3]], -1), r["uv"]),
            "traceErrorOffset": (o[0, :, 3], r["traceErrorOffset"]),
            "materialIdx": (o[7, :, 3].view(np.int32), r["materialIdx"]),
        }
        light = {"gn": (o[1, :, :3], r["gn"][:, :3]), "pdfPos": (o[3, :, 3], r["pdfPos"])}
        for group, sel in ((fields, live), (surf, live & (typ == 2)), (light, live & (typ == 1))):
            for name, (a, b) in group.items():
                a, b = np.asarray(a)[sel], np.asarray(b)[sel]
                if a.dtype == np.float32:
                    ne = f32(a) != f32(b)
                    ne &= ~(np.isnan(a) & np.isnan(b))
                else:
                    ne = a != b
                if ne.ndim > 1:
                    ne = ne.any(-1)
                if ne.any():
                    bad.append(f"{label} depth {d} {name}: {int(ne.sum())}/{int(sel.sum())} differ")
    return bad


@pytest.mark.parametrize("case", BDPT_CASES, ids=[bdpt_key(c) for c in BDPT_CASES])
def test_bdpt_matches_reference(hip_ctx, clref_bdpt, case):
    from mcrt import lib
    name, W, H, frames, D = case
    key = bdpt_key(case)
    N = W * H
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera(name, W, H)
    report = []
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=D, sampler=T.SAMPLER_RANDOM, integrator=T.INTEGRATOR_BDPT)
        g = fb.read(0)[..., :3]
        ref = clref_bdpt[f"{key}_f{f}"][..., :3]
        exact = (g.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(g) & np.isnan(ref))
        close = np.abs(g - ref) <= REL_TOL * (np.abs(g) + np.abs(ref)) + 1e-30
        close |= exact
        # pixels no light-tracing splat landed on: the reference's sum order is the own (t, s)
        # order there, so they must be bit-exact
        nosplat = (fb.read_bdpt("splat").view(np.float32).reshape(H, W, 4)[..., :3] == 0).all(-1)
        ex_ns = exact.all(-1)[nosplat]
        report.append(f"frame {f}: bit-exact {exact.mean():.5f} (no-splat pixels {ex_ns.mean():.5f} of "
                      f"{int(nosplat.sum())}), within {REL_TOL:g} {close.mean():.5f}, mean {g.mean():.6f} vs {ref.mean():.6f}")
        if not ex_ns.all():
            report.append(f"frame {f}: {int((~ex_ns).sum())} no-splat pixels outside bit-exactness")
        if not close.all():
            report.append(f"frame {f}: {int((~close).sum())} pixels outside tolerance")
    # state of the last frame: counts and vertices
    cc = fb.read_bdpt("camera_counts").view(np.int32)
    lc = fb.read_bdpt("light_counts").view(np.int32)
    rcc = clref_bdpt[f"{key}_camera_counts"].view(np.int32)
    rlc = clref_bdpt[f"{key}_light_counts"].view(np.int32)
    bad = [r for r in report if "outside" in r]
    if (cc != rcc).any():
        bad.append(f"camera counts differ at {int((cc != rcc).sum())} pixels")
    if (lc != rlc).any():
        bad.append(f"light counts differ at {int((lc != rlc).sum())} pixels")
    bad += compare_vertices(our_planes(fb.read_bdpt("camera_vertices"), D + 2, N),
                           clref_bdpt[f"{key}_camera_vertices"].view(po.REF_VERTEX_DTYPE).reshape(N, D + 2),
                           cc, D + 2, N, "camera")
    bad += compare_vertices(our_planes(fb.read_bdpt("light_vertices"), D + 1, N),
                            clref_bdpt[f"{key}_light_vertices"].view(po.REF_VERTEX_DTYPE).reshape(N, D + 1),
                            lc, D + 1, N, "light")
    print(key, report)
    fb.close()
    ds.close()
    assert not bad, (bad, report)


def test_bdpt_frames_in_flight(hip_ctx):
    """BDPT frames overlapping in 2 and 4 frame slots (per-slot BDPT sets; the shared
    sampled-light-vertex planes, which the s = 1 strategy reads from the PREVIOUS frame,
    BDPT.cl:585-586, are kept in frame order by an event between the connect launches), with only
    mcrt_accumulate between the frames and one read-back at the end, against one slot:
      * the sampled-light planes after the last frame, both subpaths' vertex counts and the
        camera vertices: bit-exact (no atomics involved);
      * the last radiance and the accumulated image: within the splat tolerance (light-tracing
        splats are float atomics, so their order varies from run to run even with one slot)."""
    from mcrt import lib
    name, W, H, D, frames = "mixed", 96, 64, 2, 7
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    cam = scene_camera(name, W, H)
    filt = T.make_filter(T.BOX)
    out = {}
    for fif in (1, 2, 4):
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.set_frames_in_flight(fif)
        for f in range(frames):
            fb.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
            fb.accumulate(filt, f)
        out[fif] = {"rad": fb.read(0), "img": fb.read(2), "wts": fb.read(1),
                    **{k: fb.read_bdpt(k) for k in ("sampled_light", "camera_counts", "light_counts",
                                                    "camera_vertices")}}
        fb.close()
    ds.close()
    ref = out[1]
    assert ref["img"][..., :3].max() > 0
    N = W * H
    live = ref["camera_counts"].view(np.int32)[None, :] > np.arange(D + 2)[:, None]   # (depth, N)
    for fif in (2, 4):
        o = out[fif]
        for k in ("sampled_light", "camera_counts", "light_counts"):
            np.testing.assert_array_equal(o[k], ref[k], err_msg=f"fif={fif} {k}")
        # vertices of the last frame (depths past a path's end keep older frames' data in each set)
        a = our_planes(o["camera_vertices"], D + 2, N).view(np.uint32)[:, :8]
        b = our_planes(ref["camera_vertices"], D + 2, N).view(np.uint32)[:, :8]
        ne = (a != b).any(-1).any(1)   # (depth, N)
        assert not (ne & live).any(), (fif, int((ne & live).sum()))
        for k in ("rad", "img"):
            a, b = o[k][..., :3], ref[k][..., :3]
            close = np.abs(a - b) <= REL_TOL * (np.abs(a) + np.abs(b)) + 1e-30
            assert close.all(), (fif, k, int((~close).sum()))


@pytest.mark.parametrize("D", [2, 4])
def test_light_strategies_in_vertex_launch(hip_ctx, monkeypatch, D):
    """The light-tracing strategies (t = 1) evaluated by the vertex launches that create their light
    vertices (the default) against the connection launch that re-reads them
    (MCRT_BDPT_LIGHT_IN_VERTEX=0), over a batched call: the vertex fields, counts, own-strategy slots and
    sampled-light planes bit-exact (t = 1 strategies write none of them); the splat plane and the
    radiance within the splat tolerance (the placement changes the queue order of the splats' float
    atomics only)."""
    from mcrt import lib
    name, W, H = "mixed", 96, 64
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    cams = [scene_camera(name, W, H, frame=f, jitter=True) for f in range(4)]
    out = {}
    for on in ("0", "1"):
        monkeypatch.setenv("MCRT_BDPT_LIGHT_IN_VERTEX", on)
        fb = lib.FrameBuffer(hip_ctx, W, H)
        fb.render_frames(ds, cams, frame=0, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        out[on] = {"rad": fb.read(0), **{k: fb.read_bdpt(k) for k in lib.FrameBuffer.BDPT_READ}}
        fb.close()
    ds.close()
    a, b = out["1"], out["0"]
    N = W * H * len(cams)
    for k, depths in (("camera_vertices", D + 2), ("light_vertices", D + 1)):
        # the vertex fields (planes 0-7); the material planes of a light vertex of depth D are read only
        # by the connection launch's light-tracing class, so the default placement leaves them unwritten
        np.testing.assert_array_equal(our_planes(a[k], depths, N)[:, :8], our_planes(b[k], depths, N)[:, :8], err_msg=k)
    for k in ("camera_counts", "light_counts", "slots", "sampled_light"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    sa, sb = a["splat"].view(np.float32), b["splat"].view(np.float32)
    assert (sb != 0).mean() > 0.01   # light-tracing splats landed
    for x, y, k in ((sa, sb, "splat"), (a["rad"][..., :3], b["rad"][..., :3], "rad")):
        close = np.abs(x - y) <= REL_TOL * (np.abs(x) + np.abs(y)) + 1e-30
        assert close.all(), (k, int((~close).sum()))


@pytest.mark.parametrize("ranks", [2, 3])
def test_bdpt_band_split_matches_whole_frames(hip_ctx, ranks):
    """Band-split BDPT (multi-GPU, emulated on one GPU with one framebuffer per rank): rank r
    renders the camera and light subpaths of its 8-row bands; the ranks' rank-major splat buffers
    are summed (mcrt.dist.exchange_splats' reduce-scatter, in rank order here) and every rank
    completes its bands with ITS chunk of the sum (mcrt_bdpt_gather); the accumulators are summed
    at the end.  Against whole frames in
    one framebuffer, over 5 frames (the sampled-light state, BDPT.cl:585-586, persists on the
    pixel's owner):
      * camera / light vertex counts and the sampled-light planes of every pixel: bit-exact;
      * each frame's radiance and the reduced accumulation: within the splat tolerance (sums of
        the same splats in another order)."""
    import torch
    from mcrt import lib
    from mcrt import dist as mdist
    name, W, H, D, frames = "mixed", 96, 64, 2, 5
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    cam = scene_camera(name, W, H)
    filt = T.make_filter(T.BOX)
    full = lib.FrameBuffer(hip_ctx, W, H)
    fbs = [lib.FrameBuffer(hip_ctx, W, H) for _ in range(ranks)]
    rows = [mdist.band_rows_of(H, 8, ranks, r) for r in range(ranks)]
    cr = mdist.splat_chunk_rows(H, 8, ranks)
    C = mdist.SPLAT_CHANNELS
    bufs = [torch.zeros(C * W * cr * ranks, dtype=torch.float32, device="cuda") for _ in range(ranks)]
    N = W * H
    for f in range(frames):
        full.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        full.accumulate(filt, f)
        for r, fb in enumerate(fbs):
            fb.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT, band_rows=8, num_bands=ranks,
                      band_index=r)
            with pytest.raises(lib.MCRTError):   # the frame is not complete before the exchange
                fb.accumulate(filt, f)
            assert fb.bdpt_splat_layout() == (cr * W, ranks)
            fb.bdpt_splats_copy(bufs[r].data_ptr())   # enqueued on the frame's stream
        torch.cuda.synchronize()
        total = bufs[0].clone()
        for r in range(1, ranks):
            total += bufs[r]
        if f == 0:   # the rank-major layout: chunk r = rank r's rows of the summed splat image
            img = np.zeros((H, W, 4), np.float32)
            for fb in fbs:
                img += fb.read_bdpt("splat").view(np.float32).reshape(H, W, 4)
            np.testing.assert_allclose(total.cpu().numpy().reshape(ranks, cr, W, C),
                                       mdist.rank_major_pack(img[..., :C], 8, ranks), rtol=1e-6, atol=1e-30)
        chunks = [total[r * C * W * cr:(r + 1) * C * W * cr].clone() for r in range(ranks)]
        torch.cuda.synchronize()
        for r, fb in enumerate(fbs):
            fb.bdpt_gather(chunks[r].data_ptr())
            fb.accumulate(filt, f)
        ref = full.read(0)
        for r, fb in enumerate(fbs):
            a, b = fb.read(0)[rows[r], :, :3], ref[rows[r], :, :3]
            close = np.abs(a - b) <= REL_TOL * (np.abs(a) + np.abs(b)) + 1e-30
            assert close.all(), (ranks, f, r, int((~close).sum()))
        want = {k: full.read_bdpt(k) for k in ("camera_counts", "light_counts", "sampled_light")}
        for k, w in want.items():
            got = np.zeros_like(w)
            per = w.size // N   # bytes per pixel in this array (planes x pixel layout for sampled_light)
            for r, fb in enumerate(fbs):
                pix = (rows[r][:, None] * W + np.arange(W)[None, :]).ravel()
                g = fb.read_bdpt(k)
                if k == "sampled_light":   # D planes of float4 x N
                    gv, wv = g.view(np.uint32).reshape(D, N, 4), got.view(np.uint32).reshape(D, N, 4)
                    wv[:, pix] = gv[:, pix]
                else:
                    got.view(np.int32)[pix] = g.view(np.int32)[pix]
            assert per > 0
            np.testing.assert_array_equal(got, w, err_msg=f"frame {f} {k}")
    # end of job: ONE sum of the per-rank accumulators (zero outside each rank's bands)
    acc = sum(fb.read(1).astype(np.float64) for fb in fbs)
    ref_acc = full.read(1)
    close = np.abs(acc - ref_acc) <= 2 * REL_TOL * np.abs(ref_acc) + 1e-30
    assert close.all(), int((~close).sum())
    for fb in fbs + [full]:
        fb.close()
    ds.close()


def _frame_planes(raw, depths, frames, N):
    """(depths, planes, frames, N, 4) view of a batched call's vertex planes (stride N x frames)."""
    f = raw.view(np.float32)
    return f.reshape(depths, f.size // (depths * frames * N * 4), frames, N, 4)


@pytest.mark.parametrize("calls", [(3, 4), (1, 2, 4)])
def test_bdpt_batched_frames_match_single_calls(hip_ctx, calls):
    """mcrt_render_frames with the BDPT integrator (frame k of a call = path k*N + pixel in every
    plane; the s = 1 strategies walk the call's frames in order, BDPT.cl:585-586) against one
    mcrt_render_frame per frame, on the TAA-jittered mixed scene:
      * per frame: both subpaths' vertex counts and every live vertex's 8 planes, and the own-strategy
        slots -- bit-exact (no atomics involved);
      * the sampled-light planes after each call: bit-exact;
      * per frame radiance (mcrt_framebuffer_read_frame): bit-exact wherever no splat landed, within
        the splat tolerance elsewhere; the accumulated image within the tolerance."""
    from mcrt import lib
    name, W, H, D = "mixed", 96, 64, 2
    N = W * H
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    total = sum(calls)
    cams = [scene_camera(name, W, H, frame=f, jitter=True) for f in range(total)]
    filt = T.make_filter(T.BOX)
    one = lib.FrameBuffer(hip_ctx, W, H)
    single = []
    for f in range(total):
        one.render(ds, cams[f], frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        one.accumulate(filt, f)
        single.append({"rad": one.read(0), "splat": one.read_bdpt("splat"),
                       **{k: one.read_bdpt(k) for k in ("camera_vertices", "light_vertices", "camera_counts",
                                                        "light_counts", "slots", "sampled_light")}})
    img_one = one.read(2)
    one.close()
    fb = lib.FrameBuffer(hip_ctx, W, H)
    f0 = 0
    for B in calls:
        fb.render_frames(ds, cams[f0:f0 + B], frame=f0, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        fb.accumulate_frames([filt] * B, f0)
        cv = _frame_planes(fb.read_bdpt("camera_vertices"), D + 2, B, N)
        lv = _frame_planes(fb.read_bdpt("light_vertices"), D + 1, B, N)
        cc = fb.read_bdpt("camera_counts").view(np.int32).reshape(B, N)
        lc = fb.read_bdpt("light_counts").view(np.int32).reshape(B, N)
        slots = fb.read_bdpt("slots").view(np.uint32).reshape(-1, B, N, 4)
        splat = fb.read_bdpt("splat").view(np.float32).reshape(B, H, W, 4)
        for k in range(B):
            s = single[f0 + k]
            np.testing.assert_array_equal(cc[k], s["camera_counts"].view(np.int32), err_msg=f"f{f0 + k} camera counts")
            np.testing.assert_array_equal(lc[k], s["light_counts"].view(np.int32), err_msg=f"f{f0 + k} light counts")
            for got, ref, cnt, depths in ((cv, s["camera_vertices"], cc[k], D + 2), (lv, s["light_vertices"], lc[k], D + 1)):
                a = got[:, :8, k].view(np.uint32)
                b = our_planes(ref, depths, N)[:, :8].view(np.uint32)
                live = cnt[None, :] > np.arange(depths)[:, None]
                ne = (a != b).any(-1).any(1)
                assert not (ne & live).any(), (f0 + k, depths, int((ne & live).sum()))
            np.testing.assert_array_equal(slots[:, k], s["slots"].view(np.uint32).reshape(-1, N, 4),
                                          err_msg=f"f{f0 + k} own-strategy slots")
            g, r = fb.read_frame(k)[..., :3], s["rad"][..., :3]
            nosplat = (splat[k][..., :3] == 0).all(-1) & (s["splat"].view(np.float32).reshape(H, W, 4)[..., :3] == 0).all(-1)
            assert (g[nosplat].view(np.uint32) == r[nosplat].view(np.uint32)).all(), f0 + k
            close = np.abs(g - r) <= REL_TOL * (np.abs(g) + np.abs(r)) + 1e-30
            assert close.all(), (f0 + k, int((~close).sum()))
        np.testing.assert_array_equal(fb.read_bdpt("sampled_light"), single[f0 + B - 1]["sampled_light"],
                                      err_msg=f"sampled-light planes after frames {f0}..{f0 + B - 1}")
        f0 += B
    img = fb.read(2)[..., :3]
    close = np.abs(img - img_one[..., :3]) <= 2 * REL_TOL * np.abs(img_one[..., :3]) + 1e-30
    assert close.all(), int((~close).sum())
    assert img.max() > 0
    fb.close()
    ds.close()


def test_bdpt_batched_band_split(hip_ctx):
    """Batched band-split BDPT (2 ranks emulated on one GPU, 3 frames per call): the rank-major
    splat chunk of a rank holds the call's frames (mcrt_bdpt_splat_layout), one sum of the ranks'
    buffers completes every frame; each rank's rows of every frame match whole single frames
    within the splat tolerance."""
    import torch
    from mcrt import lib
    from mcrt import dist as mdist
    name, W, H, D, B, ranks = "mixed", 96, 64, 2, 3, 2
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    cams = [scene_camera(name, W, H, frame=f, jitter=True) for f in range(B)]
    one = lib.FrameBuffer(hip_ctx, W, H)
    ref = []
    for f in range(B):
        one.render(ds, cams[f], frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        ref.append(one.read(0))
    one.close()
    cr = mdist.splat_chunk_rows(H, 8, ranks)
    rows = [mdist.band_rows_of(H, 8, ranks, r) for r in range(ranks)]
    fbs = [lib.FrameBuffer(hip_ctx, W, H) for _ in range(ranks)]
    bufs = []
    for r, fb in enumerate(fbs):
        fb.render_frames(ds, cams, frame=0, max_depth=D, integrator=T.INTEGRATOR_BDPT, band_rows=8,
                         num_bands=ranks, band_index=r)
        assert fb.bdpt_splat_layout() == (cr * W * B, ranks)
        bufs.append(torch.zeros(mdist.SPLAT_CHANNELS * W * cr * B * ranks, dtype=torch.float32, device="cuda"))
        fb.bdpt_splats_copy(bufs[r].data_ptr())
    torch.cuda.synchronize()
    total = bufs[0] + bufs[1]
    per = mdist.SPLAT_CHANNELS * W * cr * B
    for r, fb in enumerate(fbs):
        chunk = total[r * per:(r + 1) * per].clone()
        torch.cuda.synchronize()
        fb.bdpt_gather(chunk.data_ptr())
        for k in range(B):
            a, b = fb.read_frame(k)[rows[r], :, :3], ref[k][rows[r], :, :3]
            close = np.abs(a - b) <= REL_TOL * (np.abs(a) + np.abs(b)) + 1e-30
            assert close.all(), (r, k, int((~close).sum()))
    for fb in fbs:
        fb.close()
    ds.close()


@pytest.mark.parametrize("ranks", [2, 3])
def test_bdpt_band_split_sparse_exchange(hip_ctx, ranks):
    """The sparse splat exchange (mcrt_framebuffer_set_splat_exchange, mcrt.dist.exchange_splats_sparse)
    emulated on one GPU: rank r lists the splats landing in other ranks' rows, the lists are routed
    to the rows' owners as an all-to-all would (here in Python), and every rank adds what it receives
    (mcrt_bdpt_gather_sparse).  Every frame's radiance within the splat tolerance of whole frames;
    the records are few (the dense exchange moves every pixel), each lands in its receiver's rows."""
    import torch
    from mcrt import lib
    from mcrt import dist as mdist
    name, W, H, D, frames = "mixed", 96, 64, 2, 4
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    cam = scene_camera(name, W, H)
    filt = T.make_filter(T.BOX)
    full = lib.FrameBuffer(hip_ctx, W, H)
    fbs = [lib.FrameBuffer(hip_ctx, W, H) for _ in range(ranks)]
    for fb in fbs:
        fb.set_splat_exchange(True)
    rows = [mdist.band_rows_of(H, 8, ranks, r) for r in range(ranks)]
    owner = np.zeros(H, np.int64)
    for r in range(ranks):
        owner[rows[r]] = r
    sent_total = 0
    for f in range(frames):
        full.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        full.accumulate(filt, f)
        lists = []
        for r, fb in enumerate(fbs):
            fb.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT, band_rows=8, num_bands=ranks,
                      band_index=r)
            with pytest.raises(lib.MCRTError):   # the dense calls refuse a sparse frame
                fb.bdpt_gather(None)
            counts = fb.bdpt_splats_sparse()   # sizes only
            buf = torch.zeros(4 * max(int(counts.sum()), 1), dtype=torch.float32, device="cuda")
            again = fb.bdpt_splats_sparse(buf.data_ptr(), buf.numel() // 4)
            np.testing.assert_array_equal(again, counts)
            assert counts[r] == 0
            torch.cuda.synchronize()
            hip_ctx.sync()
            rec = buf.cpu().numpy()[:4 * int(counts.sum())].reshape(-1, 4)
            seg = np.repeat(np.arange(ranks), counts)   # grouped by receiving rank, in rank order
            tgt = rec[:, 0].view(np.int32)
            assert (owner[tgt // W] == seg).all()
            lists.append((rec, seg))
            sent_total += int(counts.sum())
        for q, fb in enumerate(fbs):
            mine = np.concatenate([rec[seg == q] for rec, seg in lists])
            recv = torch.from_numpy(np.ascontiguousarray(mine, np.float32).ravel() if len(mine) else
                                    np.zeros(4, np.float32)).cuda()
            torch.cuda.synchronize()
            fb.bdpt_gather_sparse(recv.data_ptr(), len(mine))
            fb.accumulate(filt, f)
        ref = full.read(0)
        for r, fb in enumerate(fbs):
            a, b = fb.read(0)[rows[r], :, :3], ref[rows[r], :, :3]
            close = np.abs(a - b) <= REL_TOL * (np.abs(a) + np.abs(b)) + 1e-30
            assert close.all(), (ranks, f, r, int((~close).sum()))
    assert 0 < sent_total < frames * W * H   # few records against a dense exchange of every pixel
    for fb in fbs + [full]:
        fb.close()
    ds.close()


def test_sparse_exchange_two_frames_in_flight(hip_ctx):
    """The sparse splat exchange with two frames in flight and no host synchronisation between calls
    (ADVICE r5): two band frame buffers (2 ranks emulated on one GPU) exchange their records through
    growable mcrt.dist.SparseSplatBuffers with device copies ordered on the frame streams, as the
    RCCL all-to-all runs (mcrt.dist.exchange_splats_sparse).  Each call's grouping must wait for the
    other slot's call (mcrt_bdpt_splats_sparse), and a grown buffer must outlive its last use; the
    accumulated images equal a run that synchronises the device after every step, within the splat
    tolerance."""
    import torch
    from mcrt import lib
    from mcrt import dist as mdist
    name, W, H, D, B, calls, ranks = "mixed", 96, 64, 2, 2, 6, 2
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    filt = T.make_filter(T.BOX)
    rows = [mdist.band_rows_of(H, 8, ranks, r) for r in range(ranks)]

    def run(sync):
        fbs = [lib.FrameBuffer(hip_ctx, W, H) for _ in range(ranks)]
        bufs = [mdist.SparseSplatBuffers("cuda") for _ in range(ranks)]
        for fb in fbs:
            fb.set_splat_exchange(True)
        for c in range(calls):
            cams = [scene_camera(name, W, H, frame=c * B + k, jitter=True) for k in range(B)]
            sends, counts, done = [], [], []
            for r, fb in enumerate(fbs):
                fb.render_frames(ds, cams, frame=c * B, max_depth=D, integrator=T.INTEGRATOR_BDPT, band_rows=8,
                                 num_bands=ranks, band_index=r)
                # the first call sizes the buffer at its minimum; later calls grow it (retired buffers)
                send = bufs[r].get("send", 1 if c == 0 else 256 * c)
                n = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
                if int(n.sum()) > send.numel() // 4:
                    send = bufs[r].get("send", int(n.sum()))
                    n = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.ExternalStream(fb.stream()))
                sends.append(send)
                counts.append(np.asarray(n, np.int64))
                done.append(ev)
                if sync:
                    torch.cuda.synchronize()
            for q, fb in enumerate(fbs):   # rank q's receive side of the all-to-all
                total = int(sum(cnt[q] for cnt in counts))
                recv = bufs[q].get("recv", total)
                s = torch.cuda.ExternalStream(fb.stream())
                at = 0
                for r in range(ranks):
                    s.wait_event(done[r])
                    off = int(counts[r][:q].sum())
                    k = int(counts[r][q])
                    if k:
                        with torch.cuda.stream(s):
                            recv[4 * at:4 * (at + k)].copy_(sends[r][4 * off:4 * (off + k)])
                    at += k
                if sync:
                    torch.cuda.synchronize()
                fb.bdpt_gather_sparse(recv.data_ptr(), total)
                fb.accumulate_frames([filt] * B, c * B)
        hip_ctx.sync()
        torch.cuda.synchronize()
        out = [fb.read(2) for fb in fbs]   # the accumulated image of the 12 frames
        for fb in fbs:
            fb.close()
        return out, sum(len(b.retired) for b in bufs)

    a, retired = run(False)
    b, _ = run(True)
    assert retired > 0   # buffers grew while earlier calls could still use them
    for r in range(ranks):
        x, y = a[r][rows[r], :, :3], b[r][rows[r], :, :3]
        fin = np.isfinite(x)
        # (a BDPT pixel can be NaN in the reference too: the same pixels in both runs)
        assert np.array_equal(fin, np.isfinite(y)) and fin.mean() > 0.99 and x[fin].max() > 0
        close = np.abs(x[fin] - y[fin]) <= REL_TOL * (np.abs(x[fin]) + np.abs(y[fin])) + 1e-30
        assert close.all(), (r, int((~close).sum()))
    ds.close()
