"""GPU parity of the product against the REFERENCE's own OpenCL kernels run live on this
MI355X (tests/clref_job.py in a child process, so the OpenCL runtime stays out of the HIP
test process).  Same tolerance as tests/test_gpu_render.py."""
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
        d = np.abs(g[..., :3].astype(np.float64) - ref[..., :3])
        frac = (d <= 1e-4 * np.maximum(1.0, np.abs(ref[..., :3]))).all(-1).mean()
        assert frac >= 0.995, (name, D, f, frac)
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
