"""GPU parity of the product against the REFERENCE's own OpenCL kernels run live on this
MI355X (tests/clref_job.py in a child process, so the OpenCL runtime stays out of the HIP
test process).  Radiance must match the OpenCL-default-fp build BIT FOR BIT (see
tests/test_gpu_golden_reference.py); ray queries as RadeonRays' conformance protocol."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import CASES, build_scene
from helpers import bunny_scene, closest_agreement, rr_cornell_scene
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def clref(tmp_path_factory):
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = str(tmp_path_factory.mktemp("clref") / "clref_ieee.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee"], capture_output=True,
                       text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail("reference OpenCL job failed:\n" + r.stdout + r.stderr)
    return np.load(out, allow_pickle=False)


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}_d{c[4]}" for c in CASES])
def test_product_frames_match_reference(hip_ctx, clref, case):
    from mcrt import lib
    name, W, H, frames, D = case
    sc = build_scene(name)
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("dragon_proxy" if name == "dragon_small" else name, W, H)
    for f in frames:
        fb.render(ds, cam, frame=f, max_depth=D, sampler=T.SAMPLER_RANDOM)
        g = fb.read(0)
        ref = clref[f"{name}_{W}x{H}_d{D}_f{f}"]
        diff = (g[..., :3].view(np.uint32) != ref[..., :3].view(np.uint32)).any(-1)
        assert not diff.any(), (name, D, f, int(diff.sum()))
    fb.close()
    ds.close()


def test_product_queries_match_reference(hip_ctx, clref):
    import torch
    from mcrt import lib
    sc, z = rr_cornell_scene()
    for nm, s, rays, ref in (("rr_cornell", sc, z["rays_closest"], clref["rr_cornell_closest"]),
                             ("bunny", bunny_scene(), clref["bunny_rays"], clref["bunny_closest"]),
                             ("mixed", scenes.test_scene(), clref["mixed_rays"], clref["mixed_closest"])):
        ds = lib.DeviceScene(hip_ctx, s)
        r = torch.from_numpy(np.ascontiguousarray(rays).view(np.uint8).copy()).cuda()
        h = torch.zeros(len(rays) * 32, dtype=torch.uint8, device="cuda")
        ds.trace_closest(r.data_ptr(), len(rays), h.data_ptr())
        hip_ctx.sync()
        hits = h.cpu().numpy().view(T.ISECT_DTYPE)
        eq, dt2 = closest_agreement(hits, ref)
        assert eq > 0.999 and dt2 <= 1e-5, (nm, eq, dt2)
        ds.close()


def test_san_miguel_proxy_bit_exact_vs_reference(hip_ctx, tmp_path):
    """A 2M-triangle San-Miguel proxy at 960x544, depth 2, two frames: every pixel equal."""
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    from mcrt import lib
    W, H, tris = 960, 544, 2_000_000
    out = str(tmp_path / "sm_ref.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee", "sm", str(W), str(H), str(tris)],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail("reference OpenCL job failed:\n" + r.stdout + r.stderr)
    ref = np.load(out, allow_pickle=False)
    sc = scenes.san_miguel_proxy(tris=tris)
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("san_miguel_proxy", W, H)
    for f in (0, 1):
        fb.render(ds, cam, frame=f, max_depth=2)
        g = fb.read(0)
        diff = (g[..., :3].view(np.uint32) != ref[f"f{f}"][..., :3].view(np.uint32)).any(-1)
        assert not diff.any(), (f, int(diff.sum()))
    fb.close()
    ds.close()
