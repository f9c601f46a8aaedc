"""BASELINE.json configs at FULL size against the REFERENCE's own kernels run live on this MI355X
(tests/clref_job.py ... scale, one child process per sampler build):

  * headline + config 4's scene: San-Miguel proxy (9,984,786 triangles) 1920x1080, PT, D = 2,
    frames 0 and 1 -- every radiance value BIT-EXACT (PathTracing.cl + intersect_bvh2_lds.cl);
  * the exact call bench.py times: ONE mcrt_render_frames call of 20 TAA-jittered frames
    (129 .. 148) on that scene -- frames 1, 7 and 19 of the batch bit-exact against the reference
    run live with the same cameras, and the accumulators and image after the call bit-identical
    to 20 x (mcrt_render_frame + mcrt_accumulate);
  * config 1: Dragon proxy 512x512, 4 spp: the four frames bit-exact, and the accumulated image
    (4 x mcrt_render_frame + mcrt_accumulate, box filter) bit-identical to the oracle's
    ReconstructionPass restatement over the REFERENCE's four frames (the reference's own
    ReconstructionPass writes an image2d_t, which this GPU's OpenCL cannot run);
  * config 3: Sponza proxy (16 x 1024^2 mip-mapped textures) 1920x1080, PT -- bit-exact;
  * config 4: San-Miguel proxy BDPT at 1920x1080 (the bench's BDPT object), frames 0 and 1 in sequence from fresh buffers
    (BDPT.cl) -- vertex counts bit-exact, every defined field of the vertices of EVERY pixel
    bit-exact (the job writes the reference's full vertex arrays beside its npz, for the 960x540
    depth-5 case too; other BDPT cases compare every 17th pixel plus three full rows and a 64 x 64
    block, clref_job.bdpt_vertex_sel), radiance within 4e-6 relative (splat atomics, tests/test_gpu_bdpt.py) and
    bit-exact where no light-tracing splat landed;
  * SURVEY §8(d)'s depth-5 sensitivity run on the headline scene: PT at 1920x1080 (frames 0 and 1
    bit-exact) and BDPT at 960x540 (as config 4 above), maxDepth 5;
  * config 5: San-Miguel proxy 3840x2160 with the Sobol sampler (the reference rebuilt with
    RT_SAMPLER_SOBOL, samplers.cl:18), frames 0 and 600 -- frame 600's sample index
    pix + 600 x W x H exceeds 2^32 and wraps -- bit-exact; plus the mixed
    scene at depth 5 and Sobol BDPT on the mixed scene."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import (FULL_VERTEX_CASES, SCALE_CASES, TIMED_F0, TIMED_STEPS, bdpt_vertex_sel, full_vertex_path,
                       scale_scene, taa_camera)
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po
from test_gpu_bdpt import REL_TOL, compare_vertices, our_planes

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [(v, c) for v in SCALE_CASES for c in SCALE_CASES[v]]


@pytest.fixture(scope="module")
def clref_scale(tmp_path_factory):
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = {}
    for variant in SCALE_CASES:
        path = str(tmp_path_factory.mktemp("clref") / f"scale_{variant}.npz")
        r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), path, variant, "scale"],
                           capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            pytest.fail(f"reference scale job ({variant}) failed:\n" + r.stdout + r.stderr)
        print(r.stdout)
        out[variant] = np.load(path, allow_pickle=False)
        _JOB_PATHS[variant] = path
    return out


_JOB_PATHS = {}


_scenes = {}


def device_scene(ctx, name):
    from mcrt import lib
    if name not in _scenes:
        for k in list(_scenes):
            _scenes.pop(k).close()
        _scenes[name] = lib.DeviceScene(ctx, scale_scene(name))
    return _scenes[name]


@pytest.mark.parametrize("variant,case", CASES, ids=[c[0] for _, c in CASES])
def test_full_size_config_matches_reference(hip_ctx, clref_scale, variant, case):
    from mcrt import lib
    key, name, W, H, integ, frames, D = case
    ref = clref_scale[variant]
    sampler = T.SAMPLER_SOBOL if variant.startswith("sobol") else T.SAMPLER_RANDOM
    ds = device_scene(hip_ctx, name)
    if integ == "pt_taa":
        return timed_call_matches(hip_ctx, ds, ref, key, name, W, H, frames, D)
    if integ == "pt_acc":
        return accumulated_matches(hip_ctx, ds, ref, key, name, W, H, frames, D)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera(name, W, H)
    bad = []
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=D, sampler=sampler,
                  integrator=T.INTEGRATOR_BDPT if integ == "bdpt" else T.INTEGRATOR_PT)
        g = fb.read(0)[..., :3]
        r = ref[f"{key}_f{f}"][..., :3]
        exact = (g.view(np.uint32) == r.view(np.uint32)) | (np.isnan(g) & np.isnan(r))
        assert r.max() > 0, (key, f, "empty reference frame")
        if integ == "pt":
            if not exact.all():
                bad.append(f"frame {f}: {int((~exact.all(-1)).sum())} of {W * H} pixels differ")
            continue
        close = exact | (np.abs(g - r) <= REL_TOL * (np.abs(g) + np.abs(r)) + 1e-30)
        nosplat = (fb.read_bdpt("splat").view(np.float32).reshape(H, W, 4)[..., :3] == 0).all(-1)
        if not close.all():
            bad.append(f"frame {f}: {int((~close.all(-1)).sum())} pixels outside {REL_TOL}")
        if not exact.all(-1)[nosplat].all():
            bad.append(f"frame {f}: {int((~exact.all(-1)[nosplat]).sum())} no-splat pixels not bit-exact")
    if integ == "bdpt":
        N = W * H
        sel = bdpt_vertex_sel(W, H)
        cc = fb.read_bdpt("camera_counts").view(np.int32)
        lc = fb.read_bdpt("light_counts").view(np.int32)
        for nm, a, b in (("camera", cc, ref[f"{key}_camera_counts"]), ("light", lc, ref[f"{key}_light_counts"])):
            if (a != b).any():
                bad.append(f"{nm} counts differ at {int((a != b).sum())} pixels")
        for which, depths, counts in (("camera_vertices", D + 2, cc), ("light_vertices", D + 1, lc)):
            full = full_vertex_path(_JOB_PATHS.get(variant, ""), key, which)
            if key in FULL_VERTEX_CASES:   # every pixel's vertices (the job wrote the full arrays)
                assert os.path.exists(full), f"{key}: the reference job wrote no full {which} array"
                theirs = np.load(full, mmap_mode="r").view(po.REF_VERTEX_DTYPE).reshape(N, depths)
                bad += compare_vertices(our_planes(fb.read_bdpt(which), depths, N), theirs, counts, depths, N, which)
                continue
            ours = our_planes(fb.read_bdpt(which), depths, N)[:, :, sel]
            theirs = ref[f"{key}_{which}"].view(po.REF_VERTEX_DTYPE).reshape(len(sel), depths)
            bad += compare_vertices(ours, theirs, counts[sel], depths, len(sel), which)
    fb.close()
    assert not bad, (key, bad)


def _exact(g, r):
    return (g.view(np.uint32) == r.view(np.uint32)) | (np.isnan(g) & np.isnan(r))


def timed_call_matches(ctx, ds, ref, key, name, W, H, frames, D):
    """bench.py's timed region: one 20-frame mcrt_render_frames call (packed camera / shading
    waves, tile-major order, XCD remap) + one mcrt_accumulate, against the reference frame by frame
    and against 20 single frames + accumulates (tools: bench.py step / run)."""
    from mcrt import lib
    box = T.make_filter(T.BOX)
    cams = [taa_camera(name, W, H, f) for f in range(TIMED_F0, TIMED_F0 + TIMED_STEPS)]
    bad = []
    fa = lib.FrameBuffer(ctx, W, H)
    fa.render_frames(ds, cams, frame=TIMED_F0, max_depth=D)
    fa.accumulate(box, 0)   # 0: the batch's first frame overwrites, the others add (bench.py step)
    batched = {f: fa.read_frame(f - TIMED_F0) for f in frames}
    acc_a, img_a = fa.read(1), fa.read(2)
    fa.close()
    for f in frames:
        g, r = batched[f][..., :3], ref[f"{key}_f{f}"][..., :3]
        assert r.max() > 0, (key, f, "empty reference frame")
        ex = _exact(g, r)
        if not ex.all():
            bad.append(f"batch frame {f - TIMED_F0} (frame {f}) vs reference: {int((~ex.all(-1)).sum())} pixels differ")
    fb = lib.FrameBuffer(ctx, W, H)
    for k in range(TIMED_STEPS):
        fb.render(ds, cams[k], frame=TIMED_F0 + k, max_depth=D)
        if TIMED_F0 + k in batched:
            ex = _exact(fb.read(0), batched[TIMED_F0 + k])
            if not ex.all():
                bad.append(f"frame {TIMED_F0 + k}: batched vs single radiance differ at {int((~ex.all(-1)).sum())} px")
        fb.accumulate(box, 0 if k == 0 else TIMED_F0 + k)
    for nm, a, b in (("weighted sum", acc_a, fb.read(1)), ("image", img_a, fb.read(2))):
        ex = _exact(a, b)
        if not ex.all():
            bad.append(f"{nm} after the batched call differs from 20 single frames at {int((~ex.all(-1)).sum())} px")
    fb.close()
    assert not bad, (key, bad)


def accumulated_matches(ctx, ds, ref, key, name, W, H, frames, D):
    """Config 1: frames bit-exact against the reference, and the product's accumulation of them
    bit-identical to the oracle's accumulation (orc_accumulate) of the reference's frames."""
    from mcrt import lib
    box = T.make_filter(T.BOX)
    cam = scene_camera(name, W, H)
    fb = lib.FrameBuffer(ctx, W, H)
    bad = []
    wsum = wts = None
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=D)
        fb.accumulate(box, f)
        r = ref[f"{key}_f{f}"]
        assert r[..., :3].max() > 0, (key, f, "empty reference frame")
        ex = _exact(fb.read(0)[..., :3], r[..., :3])
        if not ex.all():
            bad.append(f"frame {f}: {int((~ex.all(-1)).sum())} of {W * H} pixels differ")
        wsum, wts, img = po.accumulate(np.ascontiguousarray(r, np.float32), f, box, wsum, wts)
    for nm, a, b in (("weighted sum", fb.read(1), wsum), ("image", fb.read(2), img)):
        ex = _exact(a, b)
        if not ex.all():
            bad.append(f"{nm} after {len(frames)} spp differs from the oracle's accumulation of the reference "
                       f"frames at {int((~ex.all(-1)).sum())} px")
    fb.close()
    assert not bad, (key, bad)


def test_perf_tree_full_size_vs_reference(hip_ctx, clref_scale):
    """The perf-mode tree (mcrt_accel_opts.device_build 4: the host 3-axis binned SAH, a different
    tree from the reference's Bvh2) on the headline scene at 1080p against the reference's kernels
    run live (frames 0 and 1 of sm_pt_1080p).  Another tree visits leaves in another order, so only
    triangles at exactly equal t could resolve differently: the frames must be bit-exact on >= 99.99 %
    of pixels and within SURVEY App. A's tolerance (|dL| <= 1e-4 max(1, |L|)) on >= 99.5 %."""
    from mcrt import lib
    key, name, W, H, integ, frames, D = next(c for c in SCALE_CASES["ieee"] if c[0] == "sm_pt_1080p")
    ref = clref_scale["ieee"]
    for k in list(_scenes):   # one 10 M-triangle scene on the device at a time
        _scenes.pop(k).close()
    ds = lib.DeviceScene(hip_ctx, scale_scene(name), device_build=4)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera(name, W, H)
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=D)
        g = fb.read(0)[..., :3]
        r = ref[f"{key}_f{f}"][..., :3]
        exact = _exact(g, r).all(-1)
        d = np.abs(g.astype(np.float64) - r)
        close = (d <= 1e-4 * np.maximum(1.0, np.abs(r))).all(-1)
        assert exact.mean() >= 0.9999 and close.mean() >= 0.995, (f, float(exact.mean()), float(close.mean()))
    fb.close()
    ds.close()
