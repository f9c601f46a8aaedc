"""Multi-GPU image partition and reduction, one process per GPU.

Tile split: the image is cut into 8-row blocks; bands of `band_rows` rows (a multiple of 8)
are dealt round-robin to the ranks (interleaved for balance against sky/foliage skew).  The
kernels enumerate a rank's pixels with the same formula (mcrt_kernels.hip tilePixel), every
rank keeps full-frame accumulators that are zero outside its rows, and ONE collective ends the
job -- paths are independent and the RNG is keyed by the global pixel index, so the combined
image equals the single-GPU image bit for bit (each pixel has exactly one non-zero contribution).
The collective is a gather of each rank's own rows to rank 0 (gather_bands: each xGMI link
carries one rank's 1/N share once, in parallel) rather than a sum-reduce of the full frames
(reduce_packed: a ring moves ~2x the whole frame through every link); both give the same bits.
"""
import numpy as np


def band_blocks(height, band_rows, num_bands, band_index):
    """Global 8-row block indices owned by `band_index` (tilePixel's gb for tb = 0, 1, ...)."""
    if band_rows % 8 or band_rows <= 0:
        raise ValueError("band_rows must be a positive multiple of 8")
    if not 0 <= band_index < num_bands:
        raise ValueError("band_index out of range")
    bpb = band_rows // 8
    nblocks = (height + 7) // 8
    out = []
    tb = 0
    while True:
        gb = (tb // bpb) * bpb * num_bands + band_index * bpb + (tb % bpb)
        if gb >= nblocks:
            # later local blocks can only map further down the image
            if tb % bpb == 0:
                break
            tb += 1
            continue
        out.append(gb)
        tb += 1
    return np.asarray(out, np.int64)


def band_rows_of(height, band_rows, num_bands, band_index):
    """Image rows owned by `band_index`."""
    rows = (band_blocks(height, band_rows, num_bands, band_index)[:, None] * 8 + np.arange(8)[None, :]).ravel()
    return rows[rows < height]


# floats per pixel of the exchanged splats (MCRT_SPLAT_CHANNELS: r, g, b as the reference's splat
# buffer, BDPT.cl:654-669)
SPLAT_CHANNELS = 3


def splat_chunk_rows(height, band_rows, num_bands):
    """Rows of one chunk of the rank-major splat layout (mcrt_bdpt_splat_layout): the largest
    rank's 8-row block count x 8."""
    return max(len(band_blocks(height, band_rows, num_bands, r)) for r in range(num_bands)) * 8


def rank_major_pack(img, band_rows, num_bands):
    """(H, W, C) -> (num_bands, chunk_rows, W, C): chunk r = rank r's rows in its tile order
    (band_rows_of), zero past its last row -- the layout k_bdpt_splat_pack writes."""
    H = img.shape[0]
    cr = splat_chunk_rows(H, band_rows, num_bands)
    out = np.zeros((num_bands, cr) + img.shape[1:], img.dtype)
    for r in range(num_bands):
        rows = band_rows_of(H, band_rows, num_bands, r)
        out[r, :len(rows)] = img[rows]
    return out


def reduce_scatter_chunks(full, chunk, group=None):
    """chunk <- sum over ranks of chunk `rank` of `full` (ONE reduce-scatter: every xGMI link
    carries 1/N of the frame; float32 tensors, full = N x chunk).  gloo has no reduce-scatter:
    an all-reduce of a host copy, then the rank's slice (the CPU tests and the one-GPU rehearsal)."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    n = chunk.numel()
    if full.numel() != world * n:
        raise ValueError("full buffer must hold world x chunk elements")
    if dist.get_backend(group) == "gloo":
        h = full.cpu() if full.is_cuda else full.clone()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        chunk.copy_(h[rank * n:(rank + 1) * n])
    else:
        dist.reduce_scatter_tensor(chunk, full, op=dist.ReduceOp.SUM, group=group)


def splat_buffers(fb, device="cuda"):
    """The two device buffers of exchange_splats for frame buffer fb after a band-split frame:
    (full rank-major buffer, own chunk), float32.  Left uninitialised: mcrt_bdpt_splats_copy
    zeroes `full` on the frame's stream and the collective writes all of `chunk` (a zero-fill on
    torch's stream would race with that pack, which runs on another stream)."""
    import torch
    cp, chunks = fb.bdpt_splat_layout()
    c = SPLAT_CHANNELS
    return (torch.empty(c * cp * chunks, dtype=torch.float32, device=device),
            torch.empty(c * cp, dtype=torch.float32, device=device))


def exchange_splats(fb, full, chunk, group=None):
    """Band-split BDPT (mcrt_frame_params.num_bands > 1): the frame's light-tracing strategies
    splat into any pixel of the image, so after each rank rendered its bands the ranks' splats are
    exchanged once: each rank writes its splats rank-major (mcrt_bdpt_splats_copy: chunk r = the
    rows of rank r's bands), ONE reduce-scatter hands every rank the sums of its own rows, and the
    rank completes its bands with them (mcrt_bdpt_gather).  Each pixel's camera subpath, light
    subpath and persistent sampled-light vertex (BDPT.cl:585-586) stay on the rank that owns the
    pixel, so the N-rank frame equals the 1-GPU frame up to the order of the splat sums (which the
    reference's own CAS atomics leave open).  A batched call (mcrt_render_frames) exchanges all its
    frames at once: a rank's chunk holds them frame after frame.  full, chunk: from splat_buffers,
    or larger (the leading chunks x chunk_pixels of the current layout are used)."""
    import torch
    import torch.distributed as dist
    cp, chunks = fb.bdpt_splat_layout()
    c = SPLAT_CHANNELS
    if full.numel() < c * cp * chunks or chunk.numel() < c * cp:
        raise ValueError("splat buffers smaller than the frame's layout (mcrt.dist.splat_buffers)")
    full, chunk = full[:c * cp * chunks], chunk[:c * cp]
    fb.bdpt_splats_copy(full.data_ptr())   # enqueued on the frame's stream
    if full.is_cuda and dist.get_backend(group) != "gloo":
        # RCCL: the collective is ordered after the pack on the frame's own stream, and the gather
        # (the same stream) after the collective -- no host synchronisation in the exchange
        s = torch.cuda.ExternalStream(fb.stream(), device=full.device)
        with torch.cuda.stream(s):
            reduce_scatter_chunks(full, chunk, group)
    else:   # gloo rehearsal / CPU: through the host
        if full.is_cuda:
            torch.cuda.synchronize(full.device)
        reduce_scatter_chunks(full, chunk, group)
        if chunk.is_cuda:   # the copy into chunk ran on torch's stream; the gather reads it on the frame's
            torch.cuda.current_stream(chunk.device).synchronize()
    fb.bdpt_gather(chunk.data_ptr())


class SparseSplatBuffers:
    """Growable device buffers of exchange_splats_sparse (send and receive records, 4 floats each).
    A buffer that grows is not freed: an earlier call's all-to-all or unpack on another frame slot's
    stream may still use it, and torch's caching allocator would hand its memory out again at once
    (it only tracks torch's own streams).  The retired buffers are kept until release(), which the
    caller may invoke after a device synchronisation (growth is geometric, so they are few)."""

    def __init__(self, device="cuda"):
        self.device = device
        self.bufs = {}
        self.retired = []

    def get(self, name, records):
        import torch
        b = self.bufs.get(name)
        if b is None or b.numel() < 4 * records:
            if b is not None:
                self.retired.append(b)
            b = torch.empty(4 * max(records + records // 4, 1024), dtype=torch.float32, device=self.device)
            self.bufs[name] = b
        return b

    def release(self):
        """Drops the retired buffers; only after every stream that used them has completed."""
        self.retired.clear()


def exchange_splats_sparse(fb, bufs, group=None):
    """Band-split BDPT with the sparse splat exchange (mcrt_framebuffer_set_splat_exchange): each rank
    lists the few light-tracing splats that land in other ranks' rows (~2.6 % of its paths on the
    San-Miguel proxy, against a dense exchange of every pixel), ONE all-to-all of the per-rank counts
    and ONE all-to-all of the records (RCCL on the frame's stream) deliver them to the rows' owners,
    and mcrt_bdpt_gather_sparse adds them and completes the rank's bands.  The same frame as the
    dense exchange up to the order of the splat sums.  The counts are host data (the all-to-all's split
    sizes), so this waits for the frame's visibility pass."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    send = bufs.get("send", 0)
    counts = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
    total = int(counts.sum())
    if total > send.numel() // 4:   # grow and group again
        send = bufs.get("send", total)
        counts = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
    if len(counts) != world:
        raise ValueError("the frame's band count differs from the group's size")
    nccl = send.is_cuda and dist.get_backend(group) != "gloo"
    sc = torch.as_tensor(counts, dtype=torch.int64, device=send.device if nccl else "cpu")
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    rcounts = rc.cpu().tolist()
    rtotal = int(sum(rcounts))
    recv = bufs.get("recv", rtotal)
    ins, outs = [4 * int(c) for c in counts], [4 * int(c) for c in rcounts]
    if nccl:
        s = torch.cuda.ExternalStream(fb.stream(), device=send.device)
        with torch.cuda.stream(s):
            dist.all_to_all_single(recv[:4 * rtotal], send[:4 * total], output_split_sizes=outs, input_split_sizes=ins,
                                   group=group)
    else:   # gloo (CPU tests, one-GPU rehearsal): through the host
        if send.is_cuda:
            torch.cuda.synchronize(send.device)
        hs = send[:4 * total].cpu()
        hr = torch.empty(4 * rtotal, dtype=torch.float32)
        dist.all_to_all_single(hr, hs, output_split_sizes=outs, input_split_sizes=ins, group=group)
        recv[:4 * rtotal].copy_(hr)
        if recv.is_cuda:
            torch.cuda.current_stream(recv.device).synchronize()
    fb.bdpt_gather_sparse(recv.data_ptr(), rtotal)
    return total, rtotal


def frame_split(num_frames, world, rank):
    """Frame split (BDPT, whose light-tracing splats land anywhere in the image): rank r renders
    whole frames r, r + N, r + 2N, ... of the sequence 0 .. num_frames-1."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return np.arange(rank, num_frames, world, dtype=np.int64)


def packed_accumulators(num_pixels, device, base=None):
    """One contiguous float32 buffer holding sum(w*L) (4 per pixel) then sum(w) (1 per pixel), so
    the end-of-job reduction is a single collective; returns (buf, wsum view, wts view).
    base: an existing packed buffer to view instead of a new one (e.g. the reduced sum)."""
    import torch
    buf = torch.empty(num_pixels * 5, dtype=torch.float32, device=device) if base is None else base
    if buf.numel() != num_pixels * 5:
        raise ValueError("packed accumulator buffer has the wrong size")
    return buf, buf[:num_pixels * 4], buf[num_pixels * 4:]


def reduce_packed(buf, dst=0, group=None):
    """ONE sum-reduce of a packed accumulator buffer into rank `dst` (in place on dst)."""
    import torch.distributed as dist
    if buf.is_cuda and dist.get_backend(group) == "gloo":   # gloo rehearsal: reduce via a host copy
        h = buf.cpu()
        dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM, group=group)
        buf.copy_(h)
        return
    dist.reduce(buf, dst=dst, op=dist.ReduceOp.SUM, group=group)


def gather_bands(wsum, wts, height, width, band_rows, dst=0, group=None):
    """The end-of-job collective of the tile split: every rank sends only its own rows of the
    accumulators (sum(w*L) float4 and sum(w) per pixel, packed into one row-major buffer padded
    to the largest share) and rank `dst` writes them into its full-frame accumulators in place.
    Bit-identical to reduce_packed (the other ranks' accumulators are zero in those rows) with
    1/N of the frame per link instead of a ring's ~2 frames.  wsum: float32 (H*W*4,), wts:
    (H*W,), contiguous, on the GPU (RCCL) or the CPU (gloo; a GPU tensor under gloo goes via
    the host)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    rows_all = [band_rows_of(height, band_rows, world, r) for r in range(world)]
    maxr = max(len(r) for r in rows_all)
    host = wsum.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if host else wsum.device
    s = (wsum.cpu() if host else wsum).view(height, width * 4)
    w = (wts.cpu() if host else wts).view(height, width)
    own = torch.as_tensor(rows_all[rank], device=dev)
    send = torch.zeros(maxr, width * 5, dtype=torch.float32, device=dev)
    send[:len(own), :width * 4] = s[own]
    send[:len(own), width * 4:] = w[own]
    recv = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send, recv, dst=dst, group=group)
    if rank == dst:
        for r, rows in enumerate(rows_all):
            if r == rank or len(rows) == 0:
                continue
            idx = torch.as_tensor(rows, device=dev)
            s[idx] = recv[r][:len(rows), :width * 4]
            w[idx] = recv[r][:len(rows), width * 4:]
        if host:
            wsum.copy_(s.reshape(-1))
            wts.copy_(w.reshape(-1))


def band_buffers(height, width, band_rows, world, device):
    """(send, recv) for gather_bands_fb: one rank's packed rows (largest share) and world of them."""
    import torch
    maxr = splat_chunk_rows(height, band_rows, world)
    return (torch.empty(maxr * 5 * width, dtype=torch.float32, device=device),
            torch.empty(world * maxr * 5 * width, dtype=torch.float32, device=device))


def gather_bands_fb(ctx, fb, height, width, band_rows, send, recv, dst=0, group=None, apply=True):
    """gather_bands without the full-frame copies: the rank's own rows are packed straight from
    its frame buffer (mcrt_framebuffer_bands_pack, on the context stream after the last
    accumulate: ONE kernel instead of two full-frame copies plus row gathers), ONE gather brings
    every rank's rows to `dst`, and dst writes the others' rows into its accumulators in place and
    recomputes the image (mcrt_framebuffer_bands_unpack: one kernel instead of a scatter per rank
    and a copy back).  The collective runs on torch's current stream between two host
    synchronisations, as gather_bands.  send / recv: band_buffers (recv is only used on dst).
    Same bits as gather_bands and as one GPU rendering the whole image.  apply=False: the same pack
    and collective on the same buffers without the unpack (bench.py runs it once before timing, so
    the collective's first-use setup -- RCCL's peer connections -- stays out of the timed region and
    the accumulators are untouched)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    maxr = splat_chunk_rows(height, band_rows, world)
    n = maxr * 5 * width
    if send.numel() < n or (rank == dst and recv.numel() < world * n):
        raise ValueError("band buffers smaller than the band layout (mcrt.dist.band_buffers)")
    send = send[:n]
    fb.bands_pack(send.data_ptr())
    ctx.sync()
    if send.is_cuda and dist.get_backend(group) == "gloo":   # gloo rehearsal: through the host
        h = send.cpu()
        parts = [torch.empty_like(h) for _ in range(world)] if rank == dst else None
        dist.gather(h, parts, dst=dst, group=group)
        if rank == dst:
            recv[:world * n].copy_(torch.cat(parts))
    else:
        dist.gather(send, list(recv[:world * n].view(world, n).unbind(0)) if rank == dst else None,
                    dst=dst, group=group)
    if rank == dst:
        if recv.is_cuda:
            torch.cuda.synchronize(recv.device)
        if apply:
            fb.bands_unpack(recv.data_ptr(), maxr)


def reduce_accumulators(wsum, wts, dst=0, group=None):
    """Sum separate per-rank accumulator tensors into rank `dst` (two collectives; the bench
    packs both into one buffer with packed_accumulators and calls reduce_packed once)."""
    reduce_packed(wsum, dst, group)
    reduce_packed(wts, dst, group)


def resolve(wsum, wts):
    """image = sum(w * L) / sum(w) (k_resolve); numpy or torch."""
    return wsum / wts[..., None]
