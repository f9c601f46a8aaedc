"""The multi-GPU path through RCCL and through the driver's command.

* A 1-rank `nccl` (= RCCL) process group in this process runs the end-of-job band gather
  (mcrt.dist.gather_bands_fb: pack -> dist.gather -> unpack) and the BDPT splat exchange
  (mcrt.dist.exchange_splats: splats_copy -> reduce_scatter_tensor on the frame's stream ->
  bdpt_gather) on real RCCL kernels; the result must be the no-collective frame: PT bit for bit,
  BDPT up to the order of its float-atomic light-tracing splats (rtol 4e-6, tests/test_gpu_bdpt.py).
* `python bench.py --gpus 2 --dist-backend gloo` with NO launcher starts its own 2 ranks
  (torch.distributed.run as a child process) and reports n_gpus 2; its image equals the
  1-rank image bit for bit (RCCL refuses two ranks on one GPU, so the 2-rank rehearsal uses gloo;
  the nccl path is the 8-GPU driver run).
The reference is single-device (PlatformManager.cpp:59-79): multi-GPU is the north star's addition.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def nccl_one_rank(tmp_path):
    import torch
    import torch.distributed as dist
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist
    dist.destroy_process_group()


def test_rccl_band_gather_and_splat_exchange(hip_ctx, nccl_one_rank):
    import torch
    from mcrt import dist as mdist
    from mcrt import lib
    dist = nccl_one_rank
    sc = scenes.test_scene()
    W, H, D, frames = 80, 56, 2, 3
    cam = scene_camera("mixed", W, H)
    ds = lib.DeviceScene(hip_ctx, sc)
    filt = T.make_filter(T.BOX)
    for integ in (T.INTEGRATOR_PT, T.INTEGRATOR_BDPT):
        plain = lib.FrameBuffer(hip_ctx, W, H)
        fb = lib.FrameBuffer(hip_ctx, W, H)
        band = dict(band_rows=8, num_bands=1, band_index=0)
        full = own = None
        for f in range(frames):
            plain.render(ds, cam, frame=f, max_depth=D, integrator=integ)
            plain.accumulate(filt, f)
            fb.render(ds, cam, frame=f, max_depth=D, integrator=integ, **band)
            if integ == T.INTEGRATOR_BDPT:   # the per-frame splat exchange, RCCL on the frame's stream
                if full is None:
                    full, own = mdist.splat_buffers(fb)
                mdist.exchange_splats(fb, full, own)
            fb.accumulate(filt, f)
        hip_ctx.sync()
        send, recv = mdist.band_buffers(H, W, 8, 1, "cuda")
        mdist.gather_bands_fb(hip_ctx, fb, H, W, 8, send, recv, dst=0)   # dist.gather over RCCL
        hip_ctx.sync()
        torch.cuda.synchronize()
        if integ == T.INTEGRATOR_PT:   # the same paths, the same sums: bit for bit
            np.testing.assert_array_equal(fb.read(2).view(np.uint32), plain.read(2).view(np.uint32))
            np.testing.assert_array_equal(fb.read(1).view(np.uint32), plain.read(1).view(np.uint32))
        else:   # light-tracing splats are float atomics: two renders differ by their order only
            np.testing.assert_allclose(fb.read(2), plain.read(2), rtol=4e-6, atol=1e-30)
            np.testing.assert_allclose(fb.read(1), plain.read(1), rtol=4e-6, atol=1e-30)
        plain.close()
        fb.close()
    # the sparse splat exchange's two all-to-alls over RCCL (counts, then records on the frame's stream)
    plain = lib.FrameBuffer(hip_ctx, W, H)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    fb.set_splat_exchange(True)
    sbufs = mdist.SparseSplatBuffers("cuda")
    for f in range(frames):
        plain.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT)
        plain.accumulate(filt, f)
        fb.render(ds, cam, frame=f, max_depth=D, integrator=T.INTEGRATOR_BDPT, band_rows=8, num_bands=1, band_index=0)
        mdist.exchange_splats_sparse(fb, sbufs)
        fb.accumulate(filt, f)
    hip_ctx.sync()
    np.testing.assert_allclose(fb.read(2), plain.read(2), rtol=4e-6, atol=1e-30)
    plain.close()
    fb.close()
    # one more collective on the same group: the timing reduction bench.py ends with
    t = torch.tensor([1.5], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 1.5
    ds.close()


def _bench(tmp_path, gpus, tag, extra=()):
    img = str(tmp_path / f"{tag}.npy")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--scene", "dragon_proxy",
           "--tris", "200000", "--width", "256", "--height", "200", "--steps", "6", "--warmup", "2",
           "--batch", "4", "--no-cpu-baseline", "--no-bdpt", "--no-kernel-timing", "--save-image", img, *extra]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), np.load(img)


@pytest.mark.timeout(600)
def test_bench_gpus_flag_launches_ranks(tmp_path):
    """Strong scaling: the 2-rank job (one frame per step split over the ranks) saves the 1-rank image."""
    one, img1 = _bench(tmp_path, 1, "n1", ("--scaling", "strong"))
    two, img2 = _bench(tmp_path, 2, "n2", ("--dist-backend", "gloo", "--scaling", "strong"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2, (one, two)
    assert "x 2" in two["config"]["parallelism"] and two["scaling"] == "strong"
    np.testing.assert_array_equal(img2.view(np.uint32), img1.view(np.uint32))


@pytest.mark.timeout(600)
def test_bench_weak_scaling_two_ranks(tmp_path):
    """Weak scaling (the default): 2 ranks x 6 steps = 12 frames, each tile-split over the ranks in
    calls of 2 x 4 band-frames, save the image of ONE rank rendering 12 frames in calls of 8 (the
    same frame sequence, warmup included), bit for bit; value counts 2 frames per step."""
    one, img1 = _bench(tmp_path, 1, "w1", ("--steps", "12", "--batch", "8"))
    two, img2 = _bench(tmp_path, 2, "w2", ("--dist-backend", "gloo"))
    assert one["scaling"] == two["scaling"] == "weak"
    assert two["config"]["global_batch"] == 2 and two["config"]["max_frames_per_call"] == 8, two["config"]
    assert two["config"]["frames_per_launch"] == 8 and "2 frames per step" in two["config"]["parallelism"]
    np.testing.assert_array_equal(img2.view(np.uint32), img1.view(np.uint32))
    # value = whole-job paths / time: 256 x 200 x 6 steps x 2 frames per step
    assert abs(two["value"] - 256 * 200 * 12 / (two["ms_per_step"] * 6 * 1e-3) / 1e6) < 1e-2 * two["value"]


@pytest.mark.timeout(600)
def test_bench_bdpt_sparse_exchange_two_ranks(tmp_path):
    """`bench.py --integrator bdpt --gpus 2 --dist-backend gloo`: the band split with the sparse splat
    exchange (mcrt.dist.exchange_splats_sparse through gloo all-to-alls) against one rank: the same
    accumulated image up to the order of the splat sums."""
    extra = ("--integrator", "bdpt", "--bdpt-batch", "4", "--scaling", "strong", "--splat-exchange", "sparse")
    one, img1 = _bench(tmp_path, 1, "b1", extra)
    two, img2 = _bench(tmp_path, 2, "b2", extra + ("--dist-backend", "gloo"))
    assert two["n_gpus"] == 2 and "sparse" in two["config"]["parallelism"], two["config"]
    np.testing.assert_allclose(img2, img1, rtol=2e-5, atol=1e-30)


def test_bench_nccl_needs_one_gpu_per_rank(tmp_path):
    """Asking for more nccl ranks than visible GPUs fails loudly instead of running fewer ranks."""
    import torch
    n = torch.cuda.device_count() + 1
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       capture_output=True, text=True, timeout=280, env=env)
    assert r.returncode != 0
    assert "need" in r.stderr and "GPUs" in r.stderr, r.stderr[-2000:]
