"""Multi-rank logic on CPU (gloo, world_size 2): the band partition covers every row exactly
once, and the per-rank accumulators reduced to rank 0 reproduce the single-process
accumulation of the oracle exactly (the GPU path uses the same functions over
RCCL in bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mcrt import dist as mdist
from mcrt import scenes
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

W, H, FRAMES, BAND_ROWS = 40, 36, 3, 8


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("band_rows", [8, 16, 24])
def test_bands_partition_rows(n, band_rows):
    for height in (1, 7, 8, 36, 1080):
        rows = np.concatenate([mdist.band_rows_of(height, band_rows, n, r) for r in range(n)])
        assert np.array_equal(np.sort(rows), np.arange(height)), (n, band_rows, height)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _accumulate_band(rank, world):
    sc = scenes.test_scene(n_sphere=12)
    o = po.OracleScene(sc)
    o.build()
    cam = scene_camera("mixed", W, H)
    rows = mdist.band_rows_of(H, BAND_ROWS, world, rank)
    mask = np.zeros((H, W), bool)
    mask[rows] = True
    filt = T.make_filter(T.BOX)
    wsum = np.zeros((H, W, 4), np.float32)
    wts = np.zeros((H, W), np.float32)
    for f in range(FRAMES):
        rad, _ = o.render_rows(cam, rows.astype(np.int32), frame=f, max_depth=2, threads=2)
        s, w, _ = po.accumulate(rad, f, filt, wsum.copy(), wts.copy())
        wsum = np.where(mask[..., None], s, wsum)   # a rank only touches its own pixels
        wts = np.where(mask, w, wts)
    return wsum, wts


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wsum, wts = _accumulate_band(rank, world)
    # the bench's path: both accumulators in one packed buffer, ONE reduce
    buf, ts, tw = mdist.packed_accumulators(H * W, "cpu")
    ts.copy_(torch.from_numpy(wsum).reshape(-1))
    tw.copy_(torch.from_numpy(wts).reshape(-1))
    mdist.reduce_packed(buf, dst=0)
    if rank == 0:
        np.savez(out_path, wsum=ts.numpy().reshape(H, W, 4), wts=tw.numpy().reshape(H, W))
    dist.barrier()
    dist.destroy_process_group()


def _gather_worker(rank, world, port, out_path, height, width, band_rows):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # synthetic accumulators, zero outside the rank's rows (as every rank's framebuffer is)
    rng = np.random.default_rng(7)
    full_s = rng.random((height, width, 4), dtype=np.float32) * 3.0
    full_w = rng.random((height, width), dtype=np.float32) + 0.5
    rows = mdist.band_rows_of(height, band_rows, world, rank)
    s = np.zeros_like(full_s)
    w = np.zeros_like(full_w)
    s[rows], w[rows] = full_s[rows], full_w[rows]
    ts = torch.from_numpy(s.reshape(-1).copy())
    tw = torch.from_numpy(w.reshape(-1).copy())
    mdist.gather_bands(ts, tw, height, width, band_rows, dst=0)
    buf, rs, rw = mdist.packed_accumulators(height * width, "cpu")
    rs.copy_(torch.from_numpy(s.reshape(-1)))
    rw.copy_(torch.from_numpy(w.reshape(-1)))
    mdist.reduce_packed(buf, dst=0)
    if rank == 0:
        np.savez(out_path, gs=ts.numpy(), gw=tw.numpy(), rs=rs.numpy(), rw=rw.numpy(),
                 fs=full_s.reshape(-1), fw=full_w.reshape(-1))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height,band_rows", [(2, 36, 8), (3, 1080 // 8, 16), (4, 40, 8)])
def test_band_gather_equals_reduce(tmp_path, world, height, band_rows):
    """bench.py's end-of-job collective: gathering each rank's own band rows to rank 0 gives the
    sum-reduce of the full-frame accumulators bit for bit (and the whole image)."""
    out = str(tmp_path / "g.npz")
    mp.start_processes(_gather_worker, args=(world, _free_port(), out, height, 24, band_rows), nprocs=world,
                       join=True, start_method="spawn")
    z = np.load(out)
    assert np.array_equal(z["gs"].view(np.uint32), z["rs"].view(np.uint32))
    assert np.array_equal(z["gw"].view(np.uint32), z["rw"].view(np.uint32))
    assert np.array_equal(z["gs"], z["fs"]) and np.array_equal(z["gw"], z["fw"])


class _FakeBandsFB:
    """Host model of mcrt_framebuffer_bands_pack / _unpack (the kernels' row layout: a rank's
    local 8-row block tb at rows 8 tb .. 8 tb + 7, i.e. band_rows_of order; 5 W floats a row)
    over torch CPU tensors, so gather_bands_fb's orchestration runs under gloo without a GPU.
    The kernels themselves are checked against a whole-image render in
    tests/test_gpu_render.py::test_band_pack_unpack_through_product."""

    def __init__(self, s, w, height, width, band_rows, world, rank):
        self.s, self.w = s, w   # (H, W, 4), (H, W) float32 numpy, zero outside the rank's rows
        self.H, self.W, self.br, self.world, self.rank = height, width, band_rows, world, rank

    def _rows(self, r):
        return mdist.band_rows_of(self.H, self.br, self.world, r)

    def bands_pack(self, ptr):
        rows = self._rows(self.rank)
        dst = _BUFS[ptr]
        v = dst[:len(rows) * 5 * self.W].view(len(rows), 5 * self.W)
        v[:, :4 * self.W] = torch.from_numpy(self.s[rows].reshape(len(rows), -1))
        v[:, 4 * self.W:] = torch.from_numpy(self.w[rows])

    def bands_unpack(self, ptr, maxr):
        src = _BUFS[ptr].view(self.world, maxr, 5 * self.W)
        for r in range(self.world):
            if r == self.rank:
                continue
            rows = self._rows(r)
            self.s[rows] = src[r, :len(rows), :4 * self.W].numpy().reshape(len(rows), self.W, 4)
            self.w[rows] = src[r, :len(rows), 4 * self.W:].numpy()


_BUFS = {}


class _NoCtx:
    def sync(self):
        pass


def _gather_fb_worker(rank, world, port, out_path, height, width, band_rows):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(11)
    full_s = rng.random((height, width, 4), dtype=np.float32) * 3.0
    full_w = rng.random((height, width), dtype=np.float32) + 0.5
    rows = mdist.band_rows_of(height, band_rows, world, rank)
    s = np.zeros_like(full_s)
    w = np.zeros_like(full_w)
    s[rows], w[rows] = full_s[rows], full_w[rows]
    fb = _FakeBandsFB(s, w, height, width, band_rows, world, rank)
    send, recv = mdist.band_buffers(height, width, band_rows, world, "cpu")
    send.fill_(float("nan"))   # rows past the rank's last row are never read
    _BUFS[send.data_ptr()], _BUFS[recv.data_ptr()] = send, recv
    mdist.gather_bands_fb(_NoCtx(), fb, height, width, band_rows, send, recv, dst=0)
    if rank == 0:
        np.savez(out_path, s=fb.s, w=fb.w, fs=full_s, fw=full_w)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height,band_rows", [(2, 36, 8), (3, 1080 // 8, 16), (4, 43, 8)])
def test_band_gather_fb_whole_image(tmp_path, world, height, band_rows):
    """bench.py's end-of-job path (gather_bands_fb): packed own rows, ONE gather, unpack on rank
    0 -> rank 0 holds the whole image's accumulators bit for bit."""
    out = str(tmp_path / "gfb.npz")
    mp.start_processes(_gather_fb_worker, args=(world, _free_port(), out, height, 24, band_rows), nprocs=world,
                       join=True, start_method="spawn")
    z = np.load(out)
    assert np.array_equal(z["s"].view(np.uint32), z["fs"].view(np.uint32))
    assert np.array_equal(z["w"].view(np.uint32), z["fw"].view(np.uint32))


def test_two_rank_reduce_matches_single_process(tmp_path):
    out = str(tmp_path / "reduced.npz")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    z = np.load(out)
    ref_s, ref_w = _accumulate_band(0, 1)
    assert np.array_equal(z["wts"], ref_w)
    assert np.array_equal(z["wsum"].view(np.uint32), ref_s.view(np.uint32))
    img = mdist.resolve(z["wsum"], z["wts"])
    assert np.isfinite(img).all()


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_frame_split_partitions_frames(n):
    for frames in (1, 5, 16, 4096):
        got = np.concatenate([mdist.frame_split(frames, n, r) for r in range(n)])
        assert np.array_equal(np.sort(got), np.arange(frames))


def _accumulate_frames(rank, world):
    """Frame split: every rank accumulates whole frames (first accumulation overwrites)."""
    sc = scenes.test_scene(n_sphere=12)
    o = po.OracleScene(sc)
    o.build()
    cam = scene_camera("mixed", W, H)
    filt = T.make_filter(T.BOX)
    wsum = np.zeros((H, W, 4), np.float32)
    wts = np.zeros((H, W), np.float32)
    for i, f in enumerate(mdist.frame_split(4, world, rank)):
        rad, _ = o.render(cam, frame=int(f), max_depth=2, threads=2)
        wsum, wts, _ = po.accumulate(rad, 0 if i == 0 else int(f), filt, wsum, wts)
    return wsum, wts


def _frame_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wsum, wts = _accumulate_frames(rank, world)
    ts, tw = torch.from_numpy(wsum), torch.from_numpy(wts)
    mdist.reduce_accumulators(ts, tw, dst=0)
    if rank == 0:
        np.savez(out_path, wsum=ts.numpy(), wts=tw.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_frame_split_matches_single_process(tmp_path):
    """bench.py --integrator bdpt: the reduced frame-split accumulators equal the single-process
    accumulation up to the order of the per-pixel sums (rank sums added last)."""
    out = str(tmp_path / "reduced_frames.npz")
    mp.start_processes(_frame_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    z = np.load(out)
    ref_s, ref_w = _accumulate_frames(0, 1)
    np.testing.assert_array_equal(z["wts"], ref_w)
    np.testing.assert_allclose(z["wsum"], ref_s, rtol=1e-6, atol=1e-7)


def _bdpt_band_worker(rank, world, port, out_path):
    """Band-split BDPT with the oracle's BDPT: rank r renders the subpaths of its bands (its
    splats land anywhere), the ranks' radiance buffers are laid out rank-major and summed with ONE
    reduce-scatter per frame (mcrt.dist.reduce_scatter_chunks; own strategies are non-zero only on
    the owner's rows), and the per-rank sampled-light state persists across frames on the owner."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = scenes.test_scene(n_sphere=12)
    o = po.OracleScene(sc)
    o.build()
    cam = scene_camera("mixed", W, H)
    b = po.OracleBDPT(o, W, H, 2)
    rows = mdist.band_rows_of(H, BAND_ROWS, world, rank).astype(np.int32)
    out = {}
    for f in range(FRAMES):
        rad, cc, _, _ = b.render(cam, frame=f, rows=rows, threads=2)
        # the product's exchange: rank-major chunks, ONE reduce-scatter -> this rank's rows
        full = torch.from_numpy(mdist.rank_major_pack(rad, BAND_ROWS, world).reshape(-1).copy())
        chunk = torch.zeros(full.numel() // world, dtype=torch.float32)
        mdist.reduce_scatter_chunks(full, chunk)
        own = chunk.numpy().reshape(-1, W, 4)[:len(rows)]
        img = np.zeros((H, W, 4), np.float32)
        img[rows] = own
        t = torch.from_numpy(img.reshape(-1).copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)   # (test only: assemble the image on every rank)
        cct = torch.from_numpy(cc.copy())
        dist.all_reduce(cct, op=dist.ReduceOp.SUM)   # counts are zero off the owner's rows
        out[f"rad{f}"] = t.numpy().reshape(H, W, 4)
        out[f"cc{f}"] = cct.numpy()
    if rank == 0:
        np.savez(out_path, **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bdpt_band_split_matches_whole_frames(tmp_path, world):
    out = str(tmp_path / "bdpt.npz")
    mp.start_processes(_bdpt_band_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    z = np.load(out)
    sc = scenes.test_scene(n_sphere=12)
    o = po.OracleScene(sc)
    o.build()
    cam = scene_camera("mixed", W, H)
    b = po.OracleBDPT(o, W, H, 2)
    for f in range(FRAMES):
        rad, cc, _, _ = b.render(cam, frame=f, threads=2)
        np.testing.assert_array_equal(z[f"cc{f}"], cc)   # every subpath, on exactly one rank
        d = np.abs(z[f"rad{f}"][..., :3].astype(np.float64) - rad[..., :3])
        assert (d <= 1e-5 * np.maximum(1.0, np.abs(rad[..., :3]))).all(), f   # splat sum order only


@pytest.mark.parametrize("height,band_rows,world", [(36, 8, 2), (64, 8, 3), (1080, 8, 8), (1080, 16, 3), (100, 24, 4)])
def test_rank_major_splat_layout(height, band_rows, world):
    """The rank-major splat layout of the BDPT band split (k_bdpt_splat_pack): chunk r holds exactly
    rank r's rows (band_rows_of order) then zeros; every row of the image lands in one chunk."""
    W = 5
    img = np.arange(height * W * 2, dtype=np.float32).reshape(height, W, 2) + 1
    packed = mdist.rank_major_pack(img, band_rows, world)
    cr = mdist.splat_chunk_rows(height, band_rows, world)
    assert packed.shape == (world, cr, W, 2)
    seen = np.zeros(height, int)
    for r in range(world):
        rows = mdist.band_rows_of(height, band_rows, world, r)
        np.testing.assert_array_equal(packed[r, :len(rows)], img[rows])
        assert (packed[r, len(rows):] == 0).all()
        seen[rows] += 1
    assert (seen == 1).all()


class _FakeSparseFB:
    """The splat-list side of a band-split BDPT frame (mcrt_bdpt_splats_sparse / gather_sparse) on
    the CPU: random splat records of this rank, each owned by the rank whose 8-row bands hold its
    target row; gather_sparse keeps what arrives."""

    def __init__(self, height, width, world, rank, n, seed):
        rng = np.random.default_rng(seed + rank)
        self.H, self.W, self.world, self.rank = height, width, world, rank
        owner = np.zeros(height, np.int64)
        for r in range(world):
            owner[mdist.band_rows_of(height, 8, world, r)] = r
        tgt = rng.integers(0, height * width, n).astype(np.int32)
        keep = owner[tgt // width] != rank   # the rank's own splats stay in place (not listed)
        self.rec = np.zeros((int(keep.sum()), 4), np.float32)
        self.rec[:, 0] = tgt[keep].view(np.float32)
        self.rec[:, 1:] = rng.random((int(keep.sum()), 3), dtype=np.float32)
        self.owner = owner
        self.got = None

    def bdpt_splats_sparse(self, dst_ptr=None, capacity=0):
        dest = self.owner[self.rec[:, 0].view(np.int32) // self.W]
        order = np.argsort(dest, kind="stable")
        counts = np.bincount(dest, minlength=self.world).astype(np.int64)
        if dst_ptr is not None and capacity >= counts.sum():
            _BUFS[dst_ptr][:4 * len(order)] = torch.from_numpy(self.rec[order].ravel())
        return counts

    def stream(self):
        return 0

    def bdpt_gather_sparse(self, recv_ptr, records):
        self.got = _BUFS[recv_ptr][:4 * records].numpy().reshape(-1, 4).copy()


class _CpuSparseBuffers(mdist.SparseSplatBuffers):
    def get(self, name, records):
        b = super().get(name, records)
        _BUFS[b.data_ptr()] = b
        return b


def _sparse_worker(rank, world, port, out_path, height, width, n):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fb = _FakeSparseFB(height, width, world, rank, n, seed=5)
    sent, got = mdist.exchange_splats_sparse(fb, _CpuSparseBuffers("cpu"))
    np.savez(out_path + f".{rank}.npz", got=fb.got, sent=sent, recvd=got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,height", [(2, 40), (3, 64), (4, 1080 // 8)])
def test_sparse_splat_exchange_routes_records(tmp_path, world, height):
    """mcrt.dist.exchange_splats_sparse (the band split's sparse splat exchange) over gloo: one
    all-to-all of the counts, one of the records; every record arrives exactly once, at the rank
    whose bands hold its target row."""
    width, n = 24, 300
    out = str(tmp_path / "sp")
    mp.start_processes(_sparse_worker, args=(world, _free_port(), out, height, width, n), nprocs=world, join=True,
                       start_method="spawn")
    fbs = [_FakeSparseFB(height, width, world, r, n, seed=5) for r in range(world)]
    got = [np.load(out + f".{r}.npz") for r in range(world)]
    for q in range(world):
        want = np.concatenate([fb.rec[fb.owner[fb.rec[:, 0].view(np.int32) // width] == q] for fb in fbs])
        g = got[q]["got"]
        assert int(got[q]["recvd"]) == len(want) == len(g)
        key = lambda a: a[np.lexsort(a.view(np.int32).T[::-1])]   # noqa: E731
        assert np.array_equal(key(g).view(np.uint32), key(want).view(np.uint32))
    assert sum(int(z["sent"]) for z in got) == sum(len(fb.rec) for fb in fbs)


def _timed_region_worker(rank, world, port, out_path, height, width, band_rows):
    """bench.timed_region with the PT path's end_of_job (gather_bands_fb) over gloo on the host
    model of the frame buffer: the trace of events and rank 0's final accumulators."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    warm_s = rng.random((height, width, 4), dtype=np.float32)   # the warm-up frames' sums
    warm_w = rng.random((height, width), dtype=np.float32) + 0.5
    timed_s = rng.random((height, width, 4), dtype=np.float32)  # what the timed frames add
    timed_w = rng.random((height, width), dtype=np.float32)
    rows = mdist.band_rows_of(height, band_rows, world, rank)
    s = np.zeros_like(warm_s)
    w = np.zeros_like(warm_w)
    s[rows], w[rows] = warm_s[rows], warm_w[rows]
    fb = _FakeBandsFB(s, w, height, width, band_rows, world, rank)
    send, recv = mdist.band_buffers(height, width, band_rows, world, "cpu")
    _BUFS[send.data_ptr()], _BUFS[recv.data_ptr()] = send, recv
    trace, calls = [], []

    def render():   # the timed frames accumulate into the rank's own rows
        fb.s[rows] += timed_s[rows]
        fb.w[rows] += timed_w[rows]

    def end_of_job(warm):
        calls.append(warm)
        mdist.gather_bands_fb(_NoCtx(), fb, height, width, band_rows, send, recv, dst=0, apply=not warm)

    el = bench.timed_region(render, end_of_job, world, lambda: None, device="cpu", trace=trace)
    if rank == 0:
        np.savez(out_path, s=fb.s, w=fb.w, fs=warm_s + timed_s, fw=warm_w + timed_w, el=el,
                 trace=np.array(trace), calls=np.array(calls))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_warms_end_collective_before_timing(tmp_path, world):
    """RCCL sets up point-to-point connections on first use, and the PT job's gather was
    its first send/recv, inside the timed region.  bench.timed_region (used by bench.py's PT and BDPT
    paths) issues the end collective once untimed before t_start -- without applying it -- and once
    timed; rank 0's accumulators are still exactly the whole image's."""
    out = str(tmp_path / "tr.npz")
    mp.start_processes(_timed_region_worker, args=(world, _free_port(), out, 40, 16, 8), nprocs=world, join=True,
                       start_method="spawn")
    z = np.load(out)
    assert list(z["trace"]) == ["end_collective:warm", "t_start", "render", "end_collective:timed", "t_end"]
    assert list(z["calls"]) == [True, False]
    assert np.array_equal(z["s"].view(np.uint32), z["fs"].view(np.uint32))
    assert np.array_equal(z["w"].view(np.uint32), z["fw"].view(np.uint32))
    assert float(z["el"]) > 0
