"""k_accumulate (ReconstructionPass, KRN/reconstruction.cl:6-60) in isolation, and its filter
weights (KRN/filters.cl:12-69) against the reference's own filter functions run live.

  * filter weights: the product evaluates the weight of each frame's filter on the device, like
    the reference; for 144 filter records (every filter type at the reference's defaults,
    PathTracingSettings.h:55-66, and variations; TAA offsets of frames 0..11 and edge offsets)
    the weight k_accumulate applies must equal the weight the reference's filters.cl computes on
    this GPU (oracle/refbuild/clprobe_filters.cl, device-layout struct) BIT FOR BIT;
  * accumulation: the product's own per-frame radiance, accumulated by the product and by the
    oracle's ReconstructionPass restatement with the reference's weights: the weighted sums and
    the weight sums must be bit-exact; the image (sum / weight) within 3 ulp (the reference's
    OpenCL-default 2.5-ulp division vs the oracle's IEEE one)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import filter_table
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ref_weights(tmp_path_factory):
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = str(tmp_path_factory.mktemp("clref") / "filters.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee", "filters"],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        pytest.fail("reference filter probe failed:\n" + r.stdout + r.stderr)
    z = np.load(out, allow_pickle=False)
    tab = filter_table()   # same records (field by field: np.save does not keep the struct's gap bytes)
    for name in tab.dtype.names:
        assert np.array_equal(z["filters"][name].view(np.uint32), tab[name].view(np.uint32)), name
    return z["weights"]


def _ulp_diff(a, b):
    ia = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(ia - ib)


def test_filter_weights_match_reference(hip_ctx, ref_weights):
    import torch
    from mcrt import lib
    table = filter_table()
    sc = scenes.test_scene()
    ds = lib.DeviceScene(hip_ctx, sc)
    W, H = 8, 8
    fb = lib.FrameBuffer(hip_ctx, W, H)
    cam = scene_camera("mixed", W, H)
    wts = torch.zeros(W * H, dtype=torch.float32, device="cuda")
    got = np.zeros(len(table), np.float32)
    for i in range(len(table)):
        fb.render(ds, cam, frame=0, max_depth=1)
        fb.accumulate(table[i:i + 1], 0)    # frame 0: the weight sum IS this frame's weight
        fb.copy_device(3, wts.data_ptr())
        hip_ctx.sync()
        w = wts.cpu().numpy()
        assert (w == w[0]).all()
        got[i] = w[0]
    fb.close()
    ds.close()
    assert np.isfinite(ref_weights).all() and (ref_weights > 0).any()
    diff = got.view(np.uint32) != ref_weights.view(np.uint32)
    assert not diff.any(), [(int(i), int(table[i]["filterType"]), got[i], ref_weights[i]) for i in np.nonzero(diff)[0][:8]]


@pytest.mark.parametrize("kind", [T.BOX, T.TRIANGLE, T.GAUSSIAN, T.MITCHELL, T.LANCZOS])
def test_accumulate_isolated_vs_oracle(hip_ctx, ref_weights, kind):
    from mcrt import lib
    table = filter_table()
    rows = np.nonzero(table["filterType"] == kind)[0][:12]   # default settings, TAA offsets of frames 0..11
    sc = scenes.test_scene()
    ds = lib.DeviceScene(hip_ctx, sc)
    W, H = 64, 48
    fb = lib.FrameBuffer(hip_ctx, W, H)
    wsum = wts = None
    for f, row in enumerate(rows[:8]):
        cam = scene_camera("mixed", W, H, frame=f, jitter=True)
        fb.render(ds, cam, frame=f, max_depth=3)
        rad = fb.read(0)
        fb.accumulate(table[row:row + 1], f)
        wsum, wts, img = po.accumulate_w(rad, f, ref_weights[row], wsum, wts)
    g_wsum = fb.read(1)
    g_img = fb.read(2)
    assert g_wsum[..., :3].max() > 0
    np.testing.assert_array_equal(g_wsum.view(np.uint32), wsum.view(np.uint32))
    import torch
    t = torch.zeros(W * H, dtype=torch.float32, device="cuda")
    fb.copy_device(3, t.data_ptr())
    hip_ctx.sync()
    np.testing.assert_array_equal(t.cpu().numpy().view(np.uint32), wts.reshape(-1).view(np.uint32))
    fin = np.isfinite(img)
    assert (np.isfinite(g_img) == fin).all()
    assert _ulp_diff(g_img[fin], img[fin]).max() <= 3
    fb.close()
    ds.close()
