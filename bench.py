"""Benchmark: Mpaths/s of the MI355X path tracer on the San-Miguel proxy at 1920x1080
(BASELINE.json metric), PT with maxDepth 2 (the reference default), random sampler.
`--integrator bdpt` measures the BDPT integrator instead: one path =
one camera + one light subpath with all their connections.

One step = one 1-spp frame of the whole image per GPU (mcrt_render_frames + mcrt_accumulate_frames).
N GPUs: one process per GPU (torch.distributed.run).  The image is tile-split into 8-row bands
dealt round-robin to the ranks (north star); each rank accumulates its bands, and one RCCL
collective ends the job (inside the timed region): a gather of every rank's own band rows to
rank 0 (--end-collective reduce: the full-frame sum-reduce instead; the same bits).
  --scaling weak (default): a step is N frames (global batch N, 1 frame per GPU), each frame
      tile-split over the ranks, so a rank's launches hold as many paths as one GPU's (20 steps
      at N = 8: 160 band-frames in one call) -- the shape of the BASELINE configs' 1024-8192 spp
      jobs; the image equals one GPU rendering the N x steps frames, bit for bit.  BDPT: whole
      frames per rank (its per-frame arrays are whole-frame sized, so its band-split calls cannot
      widen), one reduce of the accumulators at the end.
  --scaling strong: a step is one frame split over the ranks (a rank's launches hold 1/N of the
      paths; their tails weigh N times more); BDPT band split with one splat
      reduce-scatter per call.

Also reported (one JSON line on rank 0):
  roofline      dominant kernel (k_shadow_extend): compulsory bytes per launch (ray I/O + 64 B per
                DISTINCT BVH node the launch visits, counted by the oracle) over its average HIP-event
                duration in an untimed one-slot pass, vs the 8 TB/s HBM peak; traffic = rocprofv3
                memory-side bytes per launch from the committed counter summary (profiles/)
  cpu_baseline  the oracle (C restatement of the reference kernels) on a bounded sample of rows of
                the same frames, all host cores (rank 0, N = 1 only)
  bdpt          SURVEY config 4's integrator (BDPT) on the same scene: Mpaths/s (band split over
                the ranks), per-kernel times, roofline of its dominant kernel (k_extend) and a CPU
                baseline of the oracle's BDPT restatement
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)

METRIC = "Mpaths/sec + achieved HBM GB/s, San-Miguel 1920x1080 at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(scene, cam_of, W, H, D, target_s=15.0):
    """Times the oracle (C restatement of the reference kernels, oracle/mcrt_oracle.c) on a bounded,
    evenly spread sample of rows of the bench's own frames (per-frame jittered cameras)."""
    from oracle import pyoracle as po
    # the box exposes all host CPUs but one GPU job owns a share of them (OMP_NUM_THREADS there)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    o = po.OracleScene(scene)
    t0 = time.perf_counter()
    o.build()
    build_s = time.perf_counter() - t0
    f0 = 0
    # calibrate on 8 rows, then size the sample to ~target_s
    cal_rows = np.linspace(0, H - 1, 8).astype(np.int32)
    t0 = time.perf_counter()
    o.render_rows(cam_of(f0), cal_rows, frame=f0, max_depth=D, threads=threads)
    dt = max(time.perf_counter() - t0, 1e-3)
    nrows = int(np.clip(8 * target_s / dt, 8, H))
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(np.int32))
    t0 = time.perf_counter()
    rad, st = o.render_rows(cam_of(f0), rows, frame=f0, max_depth=D, threads=threads)
    el = time.perf_counter() - t0
    paths0 = paths = len(rows) * W
    frames = 1
    # a whole frame can take well under target_s: render further frames (1, 2, ...) of the same
    # rows until the sample is ~target_s of CPU work
    while len(rows) == H and el + el / frames <= target_s:
        t0 = time.perf_counter()
        o.render_rows(cam_of(f0 + frames), rows, frame=f0 + frames, max_depth=D, threads=threads)
        el += time.perf_counter() - t0
        paths += paths0
        frames += 1
    return {
        "value": paths / el / 1e6, "unit": "Mpaths/s", "cores": threads, "kind": "port",
        "sample": f"{len(rows)} of {H} rows (evenly spaced) of frames {f0}..{f0 + frames - 1} (TAA-jittered cameras), "
                  f"{paths} paths, D={D}, random sampler; oracle = C restatement of PathTracing.cl + RR Bvh2/LDS "
                  f"traversal, {threads} threads, {el:.1f}s (BVH build {build_s:.1f}s not timed)",
        "_rows": rows, "_radiance": rad, "_stats": st, "_paths": paths0, "_frame0": f0, "_oracle": o,
        "_threads": threads,
    }


def reference_parity(scene_name, tris, fb, ds, cam_of, W, H, D, frame, band):
    """CHECKER, part of the cpu_baseline leg (after the timed region, rank 0, N = 1): the reference's
    own kernels (PathTracing.cl + RadeonRays intersect_bvh2_lds.cl compiled for gfx950 from
    /root/reference, run through ROCm OpenCL by oracle/_ref/clref_runner.so) render the first timed
    frame with its TAA camera in a child process (oracle/clref_frame.py); the product renders the
    same frame again (mcrt_render_frame, bit-identical to the batched call: tests/
    test_gpu_reference_scale.py) and the share of bit-identical pixels is reported."""
    import subprocess
    import tempfile
    from oracle import pyoracle as po
    if not po.clref_available():
        return {"skipped": "oracle/_ref/clref_runner.so not built (make -C oracle/refbuild)"}
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "clref_frame.npz")
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "clref_frame.py"), path, scene_name,
                            str(tris), str(W), str(H), str(D), str(frame)], capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            return {"error": (r.stdout + r.stderr)[-800:]}
        z = np.load(path, allow_pickle=False)
        ref, device = z[f"f{frame}"], str(z["device"])
        el = time.perf_counter() - t0
    fb.render(ds, cam_of(frame), frame=frame, max_depth=D, **band)
    g = fb.read(0)
    exact = ((g.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(g) & np.isnan(ref)))[..., :3].all(-1)
    d = np.abs(g[..., :3].astype(np.float64) - ref[..., :3])
    close = (d <= 1e-4 * np.maximum(1.0, np.abs(ref[..., :3]))).all(-1)
    return {"pixels_bit_exact": round(float(exact.mean()), 6), "pixels_within_1e-4": round(float(close.mean()), 6),
            "frame": int(frame), "pixels": int(W * H), "reference_nonzero": bool(ref[..., :3].max() > 0),
            "checker": ("the reference's PathTracing.cl + RadeonRays intersect_bvh2_lds.cl, compiled for gfx950 from "
                        f"the reference sources (OpenCL default fp), run live on {device} (oracle/clref_frame.py)"),
            "checker_s": round(el, 1)}


def roofline_shadow_extend(scene, cam_of, W, H, D, batch, avg_ms, qcounts, ctx, oracle=None, quant=False):
    """HBM roofline of k_shadow_extend (the dominant kernel): the shadow rays of bounce 0 and the
    extension rays for bounce 1 of `batch` frames in one launch.

    ALGORITHMIC bytes = the launch's compulsory traffic, which no cache can avoid:
      extension ray: read (o, d) 32 B + write its hit record 16 B        = 48 B
      shadow ray:    read (o, d, L) 48 B + radiance read-modify-write 32 B = 80 B
      BVH:           64 B x the DISTINCT node records the launch's queries visit (each must come
                     from HBM at least once per launch; re-reads of a node are cache traffic).
    The distinct nodes are counted by the oracle (the reference's Bvh2 + LDS traversal, same tree,
    same visit order) marking every node the queries of `batch` full frames visit.  The ray
    counts are the product's own queue sizes.  traffic = the L2-to-memory bytes per launch from
    rocprofv3 counters (profiles/, tools/pmc_json.py), for comparison: traffic / alg = the re-read
    factor of the launch's node fetches."""
    from oracle import pyoracle as po
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    o = oracle
    if o is None:
        o = po.OracleScene(scene)
        o.build()
    touched = o.track_touched(True)
    t0 = time.perf_counter()
    for f in range(batch):
        o.render(cam_of(f), frame=f, max_depth=D, threads=threads)
    el = time.perf_counter() - t0
    o.track_touched(False)
    n_nodes = int(((touched[1] | touched[2]) != 0).sum())
    n_ext, n_sh = qcounts[1][0], qcounts[0][0]   # extension rays for bounce 1, shadow rays of bounce 0
    if quant:
        # the extension rays walk the compact records (32 B per internal node, 48 B per leaf), the
        # bounce-0 shadow rays the 64-B records (wave packets): each distinct record once per format
        leaf = o.nodes()["addr_left"] == 0xFFFFFFFF   # RR Bvh2 leaf (intersect_bvh2_lds.cl)
        ext = touched[1] != 0
        node_bytes = 32 * int((ext & ~leaf).sum()) + 48 * int((ext & leaf).sum()) + 64 * int((touched[2] != 0).sum())
    else:
        node_bytes = 64 * n_nodes
    alg = batch * (n_ext * 48 + n_sh * 80) + node_bytes
    achieved = alg / (avg_ms * 1e-3) / 1e9
    tr = pmc_traffic("k_shadow_extend")
    rs = pmc_traffic("k_walk_resume")   # the stopped walks' second launch (mcrt_kernels.hip k_walk_resume)
    if tr is not None and rs is not None:
        tr["fetch_raw"] += rs["fetch_raw"]
        tr["write"] += rs["write"]
    traffic = None
    if tr is not None:   # streamed reads: ray (o, d) 32 B, shadow ray 48 B + radiance 16 B
        traffic = calibrated_traffic(tr["fetch_raw"], tr["write"], batch * (n_ext * 32 + n_sh * 64))
    out = {"bound": "hbm", "kernel": "k_shadow_extend" + (" + k_walk_resume" if rs is not None else ""),
           "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
           "traffic": None if traffic is None else round(traffic),
           "alg_bytes_per_launch": int(alg), "avg_launch_ms": round(avg_ms, 4),
           "model": ("compulsory bytes per launch: 48 B per extension ray + 80 B per shadow ray + each DISTINCT "
                     "BVH record the launch visits once (oracle-counted over the launch's frames): " +
                     ("32 B per internal / 48 B per leaf compact record for the extension rays, 64 B per record "
                      "for the bounce-0 shadow packets" if quant else "64 B per record")),
           "node_bytes_per_launch": int(node_bytes),
           "distinct_nodes_per_launch": n_nodes, "nodes_total": int(o.num_nodes), "frames_per_launch": batch,
           "rays_per_launch": {"extension": int(batch * n_ext), "shadow": int(batch * n_sh)},
           "node_count_pass_s": round(el, 1)}
    if tr is not None:
        out["traffic_source"] = tr["source"]
        out["traffic_rule"] = ("FETCH_SIZE x 1024 (exact for 64-B node gathers, calibrated) + half the launch's "
                               "streamed ray-record reads (reported at half) + WRITE_SIZE x 1024; with "
                               "k_walk_resume's FETCH_SIZE / WRITE_SIZE added (the HIP-event time covers both)")
        out["traffic_rate_gbs"] = round(traffic / (avg_ms * 1e-3) / 1e9, 1)
        out["traffic_over_alg"] = round(traffic / alg, 2)
        if "limiter" in tr:
            out["limiter"] = tr["limiter"]
    try:   # attainable HBM bandwidth of an in-repo stream copy
        att = ctx.stream_copy_gbps(2 << 30, 5)
        out["attainable"] = round(att, 1)
        out["frac_of_attainable"] = round(achieved / att, 4)
    except Exception as e:   # noqa: BLE001 -- reported, not fatal
        log(f"[bench] stream copy failed: {e}")
    return out


def gather_ceiling(ctx, rl, vq, avg_ms, hint_frac=0.0, leaf_frac=None):
    """The latency roofline of the traversal launch: its node-visit rate (the launch's rays x the
    oracle's visits per query, over its HIP-event time) against the rate of a pure dependent-gather
    probe with the same access pattern, 32 waves per CU, with its records resident in L2, in the
    Infinity Cache, or (the tree's own size) in HBM.  The launch's extension rays walk the compact
    records (mcrt_traverse.h qwalk: 32-B internal nodes, 48-B leaves fetched in one round trip), its
    bounce-0 shadow rays the 64-B records (wave packets), so the ceiling is the time-weighted mix of
    mcrt_ctx_gather_chase_compact (packed 32 / 48-B records, leaf_frac = the oracle's share of leaf
    visits) and mcrt_ctx_gather_chase (64-B records as four 16-B loads).  A node visit also does the
    slab / triangle arithmetic and stack work the probes leave out.  hint_frac: the share of the
    launch's shadow rays answered by their occluder hint (two record fetches instead of a walk)."""
    rays = rl["rays_per_launch"]
    hinted = rays["shadow"] * hint_frac
    v_ext = rays["extension"] * vq["k_extend"]
    v_sh = (rays["shadow"] - hinted) * vq["k_shadow"] + 2 * hinted
    visits = v_ext + v_sh
    rate = visits / (avg_ms * 1e-3) / 1e9
    out = {"unit": "G dependent record fetches / s", "node_visits_per_launch": int(visits),
           "node_visits_per_s": round(rate, 1), "shadow_rays_hinted": round(hint_frac, 4), "ceilings": {},
           "visits": {"extension_compact": int(v_ext), "shadow_64b": int(v_sh)}}
    if leaf_frac is not None:
        out["extension_leaf_visit_share"] = round(leaf_frac, 4)
    try:
        for name, recs in (("l2_resident_2MiB", 32768), ("infinity_cache_resident_122MiB", 2_000_000),
                           ("hbm_tree_size", int(rl["nodes_total"]))):
            c64 = ctx.gather_chase_gsteps(recs, 256, 3)
            cq = ctx.gather_chase_compact_gsteps(recs, leaf_frac if leaf_frac is not None else 0.5, 256, 3)
            mix = visits / (v_ext / cq + v_sh / c64)   # G visits / s if every visit ran at the probes' rates
            out["ceilings"][name] = {"chase_64b": round(c64, 1), "chase_compact": round(cq, 1), "launch_mix": round(mix, 1)}
        for name in out["ceilings"]:
            out["frac_of_" + name] = round(rate / out["ceilings"][name]["launch_mix"], 4)
    except Exception as e:   # noqa: BLE001 -- reported, not fatal
        log(f"[bench] gather-chase probe failed: {e}")
    return out


def survey_8d_figure(value_mpaths, rays_per_path, vq, D):
    """SURVEY.md §8(d)'s literal algorithmic bytes per path, B_path = 112 + sum_closest (48 + 32 + 64 V)
    + sum_any (48 + 4 + 64 V) + sum_shade 388 + sum_bounce 132 + 72, with the line's rays per path and
    the oracle's visits per query V, and GB/s_alg = Mpaths/s x B_path / 1000.  Reported beside the
    roofline, not as it: 64 V prices EVERY node visit as an HBM fetch, while the walks revisit the
    upper tree from L1 / L2 (the counters put the dominant launch's memory-side traffic at ~8x its
    compulsory bytes but ~1/8 of 64 V), so the figure exceeds the HBM peak."""
    n_cl, n_any, n_sh = rays_per_path["closest"], rays_per_path["any"], rays_per_path["shaded"]
    n_prim = 1.0
    n_ext = max(n_cl - n_prim, 0.0)
    b = (112 + n_prim * (80 + 64 * vq["k_primary"]) + n_ext * (80 + 64 * vq["k_extend"])
         + n_any * (52 + 64 * vq["k_shadow"]) + n_sh * 388 + n_any * 132 + 72)
    gbs = value_mpaths * b / 1000.0
    return {"bytes_per_path": round(b, 1), "gb_s_alg": round(gbs, 1), "frac_of_peak": round(gbs / HBM_PEAK_GBS, 3),
            "note": "SURVEY 8(d) B_path with V = the oracle's node visits per query: every visit priced as a 64-B "
                    "HBM fetch; the walks re-read the upper tree from L1 / L2, so this visit bandwidth exceeds the "
                    "8 TB/s peak -- the roofline above uses the compulsory bytes and the measured traffic instead"}


# FETCH_SIZE x 1024 is exact for the traversal's 64-B node gathers but reports half of a coalesced
# 16-B/lane streamed read (profiles/r03/fetch_size_calibration.json, MI355X_MICROARCH.md "HBM"):
# memory-side bytes = raw fetch + the unreported half of the launch's streamed reads + writes.
def calibrated_traffic(fetch_raw, write, streamed_read_bytes):
    return fetch_raw + 0.5 * streamed_read_bytes + write


def pmc_traffic(kernel, summary="pmc_latest.json", last_launches=0):
    """Raw FETCH_SIZE / WRITE_SIZE bytes per launch of `kernel` (and the SQ limiter summary, if
    measured) from a committed rocprofv3 counter summary under profiles/ (tools/pmc_json.py).
    last_launches > 0: also the summed bytes of the kernel's last `last_launches` dispatches (one
    BDPT frame).  Callers apply calibrated_traffic with their launch's streamed-read bytes."""
    path = os.path.join(ROOT, "profiles", summary)
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        k = d.get("kernels", {}).get(kernel)
        if k is None:
            return None
        c = k.get("counters", {})
        r = {"fetch_raw": float(c["FETCH_SIZE"]) * 1024, "write": float(c["WRITE_SIZE"]) * 1024,
             "source": f"profiles/{summary} ({d.get('config', 'config not recorded')})"}
        raw = k.get("last_dispatches", {})
        if last_launches and len(raw.get("FETCH_SIZE", [])) >= last_launches and \
                len(raw.get("WRITE_SIZE", [])) >= last_launches:
            r["fetch_raw_last"] = sum(f * 1024 for f in raw["FETCH_SIZE"][-last_launches:])
            r["write_last"] = sum(w * 1024 for w in raw["WRITE_SIZE"][-last_launches:])
        if "limiter" in k:
            r["limiter"] = k["limiter"]
        return r
    except Exception:
        return None


def bdpt_section(ctx, ds, cam_of, W, H, D, sampler, world, rank, steps, warmup, kernel_timing, split="band",
                 batch=8, sparse=False):
    """Config 4's integrator on the same scene and GPU(s): BDPT (RTBDPTPass::update), 1 spp per
    step, split over the ranks by frames (rank r renders frames r, r + N, ...; light-tracing splats
    land anywhere in the image) or by 8-row bands (one splat reduce-scatter per frame,
    mcrt.dist.exchange_splats), and the same single reduce of the accumulators.  Returns the
    measured numbers plus an untimed one-slot per-kernel timing pass."""
    import torch
    import torch.distributed as dist
    from mcrt import dist as mdist
    from mcrt import lib
    from mcrt import types as T
    fb = lib.FrameBuffer(ctx, W, H)
    filt = T.make_filter(T.BOX)
    first = [True]
    band = split == "band" and world > 1
    xstats = [0, 0, 0]   # sparse exchange: calls, records sent, records received (this rank)
    if band and sparse:   # the few splats into other ranks' rows as records, one all-to-all per call
        fb.set_splat_exchange(True)
        sbufs = mdist.SparseSplatBuffers("cuda")
    elif band:   # rank-major splats (chunks of this rank count x 8-row blocks x batch frames) + own chunk
        cr = mdist.splat_chunk_rows(H, 8, world)   # uninitialised: mcrt_bdpt_splats_copy zeroes on its stream
        splat_full = torch.empty(mdist.SPLAT_CHANNELS * W * cr * batch * world, dtype=torch.float32, device="cuda")
        splat_own = torch.empty(mdist.SPLAT_CHANNELS * W * cr * batch, dtype=torch.float32, device="cuda")

    last = [1]   # frames of the last call (fb.stats() counts that call's queues)

    def run(i0, count):
        # calls of up to `batch` consecutive frames (mcrt_render_frames): band split: every rank the
        # same frames; frame split: rank r its own consecutive block of frame indices (its RNG streams)
        i = i0
        while i < i0 + count:
            k = min(batch, i0 + count - i)
            last[0] = k
            f = i if band else rank * (1 << 20) + i
            cams = [cam_of(f + j) for j in range(k)]
            bands = dict(band_rows=8, num_bands=world, band_index=rank) if band else {}
            fb.render_frames(ds, cams, frame=f, max_depth=D, sampler=sampler, integrator=T.INTEGRATOR_BDPT, **bands)
            if band and sparse:
                sent, got = mdist.exchange_splats_sparse(fb, sbufs)
                xstats[0] += 1
                xstats[1] += sent
                xstats[2] += got
            elif band:
                mdist.exchange_splats(fb, splat_full, splat_own)
            fb.accumulate_frames([filt] * k, 0 if first[0] else f)
            first[0] = False
            i += k

    f0 = max(warmup, 3 * batch)   # every frame slot holds a whole batch before timing
    run(0, f0)
    ctx.sync()
    if world > 1:
        acc_buf, acc_s, acc_w = mdist.packed_accumulators(W * H, "cuda")

    def end_of_job(warm):   # ONE reduce of the packed accumulators into rank 0
        fb.copy_device(1, acc_s.data_ptr())
        fb.copy_device(3, acc_w.data_ptr())
        ctx.sync()
        mdist.reduce_packed(acc_buf, dst=0)
        if rank == 0 and not warm:
            torch.cuda.synchronize()
            fb.set_accumulation(acc_s.data_ptr(), acc_w.data_ptr())

    def sync():
        ctx.sync()
        torch.cuda.synchronize()

    el = timed_region(lambda: run(f0, steps), end_of_job, world, sync)
    st = fb.stats()
    out = {"value": round(W * H * steps * (1 if band else world) / el / 1e6, 3), "unit": "Mpaths/s", "steps": steps,
           # the band split divides each frame (strong scaling, also its 1-rank case); --bdpt-split
           # frame gives each rank whole frames of its own (weak)
           "ms_per_step": round(el / steps * 1e3, 4), "scaling": "strong" if split == "band" else "weak",
           "workload": f"same scene {W}x{H}, BDPT, maxDepth {D}, 1 spp per step (SURVEY config 4's integrator), "
                       f"{batch} frames per mcrt_render_frames call, "
                       + (f"band split x {world} + 1 sparse splat all-to-all per call + 1 RCCL reduce" if band and sparse
                          else f"band split x {world} + 1 splat reduce-scatter per call + 1 RCCL reduce" if band else
                          f"frame split x {world} + 1 RCCL reduce" if world > 1 else "1 GPU"),
           "rays_per_path": {"subpath": round(st["closest_rays"] / (W * H * last[0]), 4),
                             "connection": round(st["any_rays"] / (W * H * last[0]), 4)}}
    if kernel_timing:   # one slot, one call of `batch` frames (the timed calls' shape)
        kb = min(batch, steps)
        fb.set_frames_in_flight(1)
        run(f0 + steps, kb)
        ctx.sync()
        ctx.set_profiling(True)
        ctx.reset_stats()
        run(f0 + steps + kb, kb)
        ctx.sync()
        ks = ctx.kernel_stats()
        ctx.set_profiling(False)
        out["kernels"] = {k: {"avg_ms": round(v["ms"] / max(v["launches"], 1), 4), "launches": v["launches"],
                              "ms_per_frame": round(v["ms"] / kb, 4)} for k, v in ks.items()}
        out["kernels_note"] = f"one frame slot, one call of {kb} frames (per-kernel HIP events)"
    out["frames_per_call"] = batch
    if band and sparse and xstats[0]:
        out["splat_exchange"] = {"kind": "sparse all-to-all of (target, rgb) records, 16 B each",
                                 "records_sent_per_frame_rank0": round(xstats[1] / (xstats[0] * batch), 1),
                                 "bytes_sent_per_frame_rank0": round(16 * xstats[1] / (xstats[0] * batch)),
                                 "dense_bytes_per_frame_per_rank": 12 * W * H}
    out["_fb"] = fb
    return out


def bdpt_roofline_and_cpu(scene, oracle, cam_of, W, H, D, res, target_s, quant=False):
    """BDPT's dominant kernel is k_extend (the closest-hit launches over both subpaths' rays, D + 1
    per frame).  Compulsory bytes per frame: 48 B per subpath ray (read o, d; write the hit) + 64 B
    per DISTINCT BVH node the frame's subpath rays visit (counted by the oracle's BDPT on frame 0),
    over k_extend's time per frame in the one-slot pass.  CPU baseline: the oracle's BDPT on whole
    frames (its splats land anywhere) of the same cameras, ~target_s of CPU work."""
    from oracle import pyoracle as po
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    o = oracle
    if o is None:
        o = po.OracleScene(scene)
        o.build()
    out = {}
    b = po.OracleBDPT(o, W, H, D)
    touched = o.track_touched(True)
    t0 = time.perf_counter()
    _, _, _, st0 = b.render(cam_of(0), frame=0, threads=threads)
    first_s = time.perf_counter() - t0
    o.track_touched(False)
    n_nodes = int((touched[1] != 0).sum())
    ks = res.get("kernels", {}).get("k_extend")
    if ks:
        ms_frame = ks["ms_per_frame"]
        rays = res["rays_per_path"]["subpath"] * W * H
        if quant:   # compact records: 32 B per internal node, 48 B per leaf
            leaf = o.nodes()["addr_left"] == 0xFFFFFFFF
            ext = touched[1] != 0
            node_bytes = 32 * int((ext & ~leaf).sum()) + 48 * int((ext & leaf).sum())
        else:
            node_bytes = 64 * n_nodes
        alg = rays * 48 + node_bytes
        ach = alg / (ms_frame * 1e-3) / 1e9
        out["roofline"] = {"bound": "hbm", "kernel": "k_extend (BDPT, D+1 launches per frame)", "achieved": round(ach, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                           "alg_bytes_per_frame": int(alg), "kernel_ms_per_frame": ms_frame,
                           "distinct_nodes_per_frame": n_nodes,
                           "model": "compulsory bytes per frame: 48 B per subpath ray + each DISTINCT BVH record the "
                                    "frame's subpath rays visit once (oracle BDPT, frame 0), " +
                                    ("32 B per internal / 48 B per leaf compact record" if quant else "64 B per record"),
                           "node_bytes_per_frame": int(node_bytes)}
        pm = pmc_traffic("k_extend", "pmc_bdpt.json", last_launches=2 * (D + 1))
        rs = pmc_traffic("k_walk_resume", "pmc_bdpt.json", last_launches=2 * (D + 1))
        if pm and rs and "fetch_raw_last" in pm and "fetch_raw_last" in rs:   # the stopped walks' launches
            pm["fetch_raw_last"] += rs["fetch_raw_last"]
            pm["write_last"] += rs["write_last"]
            out["roofline"]["kernel"] = "k_extend + k_walk_resume (BDPT, D+1 launches each per frame)"
        if pm and "fetch_raw_last" in pm:
            # the counter run's last two calls (2 x (D + 1) k_extend dispatches, interleaved by the
            # two frames in flight; res["frames_per_call"] frames each, the timed calls' shape)
            fpc = 2 * max(int(res.get("frames_per_call", 1)), 1)
            tr = calibrated_traffic(pm["fetch_raw_last"] / fpc, pm["write_last"] / fpc, rays * 32)   # streamed: ray (o, d)
            out["roofline"].update(traffic=int(tr), traffic_source=pm["source"], traffic_over_alg=round(tr / alg, 2),
                                   traffic_rule="FETCH_SIZE x 1024 + half the streamed ray reads + WRITE_SIZE x 1024")
        if pm and "limiter" in pm:
            out["roofline"]["limiter"] = pm["limiter"]
    # CPU baseline: whole frames 1, 2, ... until ~target_s (frame 0 above carried the node marks)
    el, frames = 0.0, 0
    while frames == 0 or el + el / frames <= target_s:
        t0 = time.perf_counter()
        b.render(cam_of(1 + frames), frame=1 + frames, threads=threads)
        el += time.perf_counter() - t0
        frames += 1
    out["cpu_baseline"] = {"value": round(W * H * frames / el / 1e6, 4), "unit": "Mpaths/s", "cores": threads,
                           "kind": "port",
                           "sample": f"{frames} whole {W}x{H} frames (1..{frames}), D={D}; oracle = C restatement of "
                                     f"BDPT.cl (RTBDPTPass order) + RR Bvh2/LDS traversal, {threads} threads, {el:.1f}s "
                                     f"(frame 0, {first_s:.1f}s with node marking, not timed)"}
    return out


def timed_region(render, end_of_job, world, sync, device="cuda", trace=None):
    """The bench contract's timed region: barrier + sync, render, the job's ONE end collective, sync +
    barrier, max over ranks.  With N > 1 ranks the end collective runs once more BEFORE the timed
    region, untimed and without applying its result (end_of_job(warm=True)): RCCL sets up a pair of
    ranks' point-to-point connections on their first send/recv, and the gather is the job's only
    send/recv (dist.barrier() is an all-reduce), so without this the first-use setup would fall inside
    the ~24 ms N = 8 timed region.  render(): the timed steps; end_of_job(warm): the collective;
    sync(): every device stream of this rank drained.  trace (a list): the events in order, for the
    tests.  Returns the elapsed seconds (max over ranks)."""
    import torch
    import torch.distributed as dist
    ev = trace.append if trace is not None else (lambda e: None)
    if world > 1:
        end_of_job(True)
        ev("end_collective:warm")
        sync()
        dist.barrier()
    sync()
    ev("t_start")
    t0 = time.perf_counter()
    render()
    ev("render")
    if world > 1:
        end_of_job(False)
        ev("end_collective:timed")
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    ev("t_end")
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def launch_ranks(n):
    """Runs this script under `python -m torch.distributed.run --nproc-per-node n` (one process
    per GPU, rendezvous on 127.0.0.1 at a free port) as a child process with the same arguments,
    and returns its exit status.  Called before torch is imported: this process never initialises
    a GPU, and it waits for the child instead of replacing itself."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--tris", type=int, default=10_000_000)
    ap.add_argument("--max-depth", type=int, default=2)
    ap.add_argument("--scene", default="san_miguel_proxy", choices=["san_miguel_proxy", "dragon_proxy", "sponza_proxy",
                                                                   "instanced_proxy"])
    ap.add_argument("--sampler", default="random", choices=["random", "sobol"])
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--end-collective", default="gather", choices=["gather", "reduce"],
                    help="tile split: gather each rank's band rows to rank 0, or sum-reduce the full frames")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-reference-parity", action="store_true",
                    help="skip the reference-kernel render of the first timed frame (parity_vs_reference)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-roofline-model", action="store_true",
                    help="skip the oracle pass that counts the distinct BVH nodes of one launch")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--stats-launches", type=int, default=2,
                    help="launch sequences of the untimed per-kernel timing pass (one frame slot)")
    ap.add_argument("--integrator", default="pt", choices=["pt", "bdpt"])
    ap.add_argument("--no-bdpt", action="store_true", help="skip the BDPT object (config 4) of the PT run")
    ap.add_argument("--bdpt-steps", type=int, default=32, help="timed BDPT frames of the BDPT object")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = N frames per step (1 per GPU), each tile-split over the ranks (PT) or whole "
                         "frames per rank (BDPT); strong = one frame per step split over the ranks")
    ap.add_argument("--bdpt-split", default=None, choices=["frame", "band"],
                    help="multi-GPU BDPT (default: frame for --scaling weak, band for strong): 8-row bands per rank "
                         "with one splat reduce-scatter per call (the 1-GPU image up to splat summation order; "
                         "mcrt.dist.exchange_splats) or whole frames per rank (no per-call exchange; each rank's "
                         "sampled-light history differs, BDPT.cl:585)")
    ap.add_argument("--splat-exchange", default="dense", choices=["sparse", "dense"],
                    help="band-split BDPT: the rank-major full-frame buffers with one stream-ordered reduce-scatter "
                         "(dense, default: the exchange overlaps the next call), or the splats landing in other "
                         "ranks' rows as records with one all-to-all (sparse: 100x fewer bytes, but its host-side "
                         "split sizes stop the calls overlapping -- 13 %% slower per rank, profiles/r05/ab/splat_exchange)")
    ap.add_argument("--save-image", default=None, help="rank 0 saves the final accumulated image (.npy)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the product path); gloo only rehearses N ranks on one GPU")
    ap.add_argument("--device-build", action="store_true", help="on-device linear BVH instead of the RR-identical tree")
    ap.add_argument("--host-build", action="store_true",
                    help="build the RR-identical tree on the host (mcrt_bvh.cpp) instead of the device (mcrt_sahbuild.hip)")
    ap.add_argument("--force-flat", action="store_true",
                    help="flat BVH even for instanced scenes (RR bvh.forceflat); default: RR's auto selection")
    ap.add_argument("--russian-roulette", action="store_true",
                    help="opt-in RR on extension rays (perf mode; the reference has none, so not a parity run)")
    ap.add_argument("--rr-start", type=int, default=1, help="first bounce whose extension rays RR may cut")
    ap.add_argument("--pow2-calls", action="store_true",
                    help="A/B only: round every call's frame count down to a power of two (16 + 4 for 20 steps)")
    ap.add_argument("--chunks", default="",
                    help="A/B only: comma-separated frames per call of the timed region, cycled (e.g. 4,16)")
    ap.add_argument("--bvh-bins", type=int, default=64,
                    help="SAH bins (64 = RTScene::commit's setting; others are host-built A/B trees)")
    ap.add_argument("--perf-tree", action="store_true",
                    help="A/B: the host 3-axis SAH tree (device_build 4) instead of the reference's Bvh2")
    ap.add_argument("--bdpt-batch", type=int, default=16,
                    help="BDPT frames per mcrt_render_frames call (the BDPT object and --integrator bdpt; 16: "
                         "4.62 ms per frame against 4.79 at 8 and 4.74 at 32, profiles/r05/ab/bdpt_batch)")
    ap.add_argument("--batch", type=int, default=0,
                    help="PT frames per mcrt_render_frames call (one launch sequence for all of them); "
                         "0 = auto (32 up to 1080p, 16 above)")
    args = ap.parse_args()

    # --gpus N is the job's world size.  A plain `python bench.py --gpus N` (no launcher) starts
    # torch.distributed.run with N ranks as a CHILD process -- before torch is imported or any GPU
    # is touched here -- and exits with its status; rank 0 of the child prints the JSON line on
    # the inherited stdout.  Under a launcher, WORLD_SIZE must equal --gpus.  (The reference is
    # single-device: PlatformManager.cpp:59-79 picks one OpenCL device.)
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} from the launcher but --gpus {args.gpus}; they must agree")

    if args.bdpt_split is None:
        args.bdpt_split = "frame" if args.scaling == "weak" else "band"

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and args.dist_backend == "nccl" and torch.cuda.device_count() < world:
        # RCCL needs one GPU per rank (it refuses two ranks on one device); --dist-backend gloo
        # rehearses N ranks on one GPU
        sys.exit(f"bench.py: {world} ranks over nccl need {world} GPUs, {torch.cuda.device_count()} visible "
                 f"(use --dist-backend gloo to rehearse on one GPU)")
    if world > 1:
        if args.dist_backend == "gloo":   # rehearsal: every rank on cuda:0 of a 1-GPU box
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from mcrt import dist as mdist
    from mcrt import lib, scenes
    from mcrt import types as T
    from mcrt.camera import scene_camera

    W, H, D = args.width, args.height, args.max_depth
    t0 = time.perf_counter()
    if args.scene == "san_miguel_proxy":
        scene = scenes.san_miguel_proxy(tris=args.tris)
    elif args.scene == "sponza_proxy":
        scene = scenes.sponza_proxy()
    elif args.scene == "instanced_proxy":
        scene = scenes.instanced_proxy()
    else:
        scene = scenes.dragon_proxy(tris=min(args.tris, 871_414))
    sampler = T.SAMPLER_SOBOL if args.sampler == "sobol" else T.SAMPLER_RANDOM
    if sampler == T.SAMPLER_SOBOL:   # g_SobolMatrices32 (sobol.h:34), package data
        from mcrt import sobol_matrices
        scene.sobol = sobol_matrices()
    gen_s = time.perf_counter() - t0
    # TAA on (the reference default, PathTracingApp.cpp:208-215): every frame f has its own sub-pixel
    # jittered camera; computed once for all frames before timing
    ncams = 64
    cams = [scene_camera(args.scene, W, H, frame=f, jitter=True) for f in range(ncams)]
    cam_of = lambda f: cams[f % ncams]   # noqa: E731
    cam = cams[0]
    log(f"[bench] scene {scene.name}: {scene.num_triangles} tris, gen {gen_s:.1f}s")

    ctx = lib.Context(local)
    t0 = time.perf_counter()
    ds = lib.DeviceScene(ctx, scene, device_build=4 if args.perf_tree else 1 if args.device_build else
                         3 if args.host_build else 2,
                         force_flat=args.force_flat, bins=args.bvh_bins)
    info = ds.info()
    two_level = ds.layout()["two_level"] == 1
    quant = info["bytes"] > 64 * info["nodes"]   # compact records built (mcrt_traverse.h traverseQOct)
    log(f"[bench] upload+BVH {time.perf_counter() - t0:.1f}s (build {info['build_ms'] / 1e3:.1f}s, "
        f"{info['nodes']} nodes, {info['bytes'] / 1e6:.0f} MB)")
    fb = lib.FrameBuffer(ctx, W, H)
    filt = T.make_filter(T.BOX)
    bdpt = args.integrator == "bdpt"
    band_bdpt = bdpt and args.bdpt_split == "band" and world > 1
    sparse_x = band_bdpt and args.splat_exchange == "sparse"
    if sparse_x:
        fb.set_splat_exchange(True)
        sbufs = mdist.SparseSplatBuffers("cuda")
    if band_bdpt:   # band split: every rank renders every frame's rows of its bands
        band = dict(band_rows=8, num_bands=world, band_index=rank, integrator=T.INTEGRATOR_BDPT)
        cr = mdist.splat_chunk_rows(H, 8, world)   # uninitialised: mcrt_bdpt_splats_copy zeroes on its stream
        splat_full = torch.empty(mdist.SPLAT_CHANNELS * W * cr * args.bdpt_batch * world, dtype=torch.float32, device="cuda")
        splat_own = torch.empty(mdist.SPLAT_CHANNELS * W * cr * args.bdpt_batch, dtype=torch.float32, device="cuda")
    elif bdpt:   # frame split: whole frames per rank
        band = dict(band_rows=8, num_bands=1, band_index=0, integrator=T.INTEGRATOR_BDPT)
    else:
        band = dict(band_rows=args.band_rows, num_bands=world, band_index=rank)
    first = [True]
    # auto: 32 frames per launch (MCRT_MAX_BATCH_FRAMES) up to 1080p, 16 above (slot memory).  The
    # camera and first-shading waves then hold 2 pixels x 32 jittered frames (packed waves); the
    # sweep tools/r2_gpu27.sh measured 1297 / 1315 Mpaths/s at 16 / 32 frames per launch, and a
    # 1/N band share x 32 frames keeps every multi-GPU launch at >= 4 whole images of paths
    batch = args.bdpt_batch if bdpt else (args.batch if args.batch > 0 else (32 if W * H <= 2_100_000 else 16))
    # PT, weak scaling: a step is `world` frames, each tile-split over the ranks; a rank's calls take
    # world x as many frames (its 1/world band share of each), so they hold as many paths as one
    # GPU's calls (MCRT_MAX_BATCH_FRAMES = 256)
    fps = world if (args.scaling == "weak" and not bdpt) else 1   # frames per step
    batch = min(256, batch * fps)
    # the untimed per-kernel pass and the roofline price the TIMED launch shape: calls of
    # min(batch, frames) frames (the driver's 20 steps are one 20-frame call, 160 band-frames at N = 8)
    stats_batch = min(batch, args.steps * fps)

    def step(i, n=1):
        """frames i .. i+n-1 (one mcrt_render_frames call when n > 1)"""
        # BDPT frame split: rank r renders its own consecutive block of frame indices (RNG streams)
        frame = rank * (1 << 20) + i if bdpt and not band_bdpt else i
        kw = dict(max_depth=D, sampler=sampler, rr=args.russian_roulette, rr_start=args.rr_start, **band)
        if n == 1:
            fb.render(ds, cam_of(frame), frame=frame, **kw)
        else:
            fb.render_frames(ds, [cam_of(frame + k) for k in range(n)], frame=frame, **kw)
        if sparse_x:   # one splat exchange per call (all its frames)
            mdist.exchange_splats_sparse(fb, sbufs)
        elif band_bdpt:
            mdist.exchange_splats(fb, splat_full, splat_own)
        fb.accumulate(filt, 0 if first[0] else frame)   # 0: the first accumulation overwrites
        first[0] = False

    def run(i0, count, per=None):
        # calls of min(batch, remaining) frames: the camera and first-shading waves pack 64 consecutive
        # (pixel, frame) paths for any frame count, so the driver's 20 steps are ONE 20-frame call
        # (1293 / 1282 Mpaths/s against 1264 / 1267 for 16 + 4, tools/r2_gpu41.sh); --pow2-calls
        # restores the earlier power-of-two split for A/B
        i = 0
        per = per or batch
        plan = [int(c) for c in args.chunks.split(",")] if args.chunks and per == batch else [per]
        calls = 0
        while i < count:
            n = min(plan[calls % len(plan)], count - i)
            if args.pow2_calls:
                n = 1 << (n.bit_length() - 1)
            calls += 1
            step(i0 + i, n)
            i += n

    # warmup: at least one call per frame slot (MCRT_MAX_FRAMES_IN_FLIGHT = 4), so no slot
    # allocation falls inside the timed region
    warm = max(args.warmup, 4 * batch)
    run(0, warm)
    ctx.sync()
    warm_frames = warm + 1   # + the untimed statistics frame below (the driver's W is a minimum)
    # per-frame path statistics (device queue sizes, occluder-hint counts) from one untimed frame
    ctx.set_profiling(2)
    step(warm)
    ctx.sync()
    ctx.set_profiling(False)
    fstats = fb.stats()
    qcounts = fb.queue_counts(max(D, 8)) if not bdpt else None
    hcounts = fb.hint_counts(max(D, 8)) if not bdpt else None   # shadow rays answered by their occluder hint
    rcounts = fb.retrace_counts(max(D, 8)) if not bdpt else None   # compact walks repeated on exact records
    frame0 = warm + 1

    ctx.reset_stats()
    if world > 1:
        if args.end_collective == "gather" and dist.get_backend() not in ("nccl", "gloo"):
            args.end_collective = "reduce"   # decided from the backend, identically on every rank
        if args.end_collective == "gather":   # packed own rows -> one gather (no full-frame copies)
            band_send, band_recv = mdist.band_buffers(H, W, args.band_rows, world, "cuda")
        else:
            acc_buf, acc_s, acc_w = mdist.packed_accumulators(W * H, "cuda")   # one buffer -> one reduce

    def end_of_job(warm):
        # one collective: each rank's own band rows gathered to rank 0 (north star).  No try/except:
        # a fallback taken by one rank while the others sit in the gather would hang the job; an
        # error exits this rank and torch.distributed.run stops the others.  warm: the untimed first
        # use before the timed region, result not applied (timed_region)
        if args.end_collective == "gather":
            # rows packed straight from the frame buffer, unpacked in place on rank 0 (+ image)
            mdist.gather_bands_fb(ctx, fb, H, W, args.band_rows, band_send, band_recv, dst=0, apply=not warm)
        else:
            fb.copy_device(1, acc_s.data_ptr())
            fb.copy_device(3, acc_w.data_ptr())
            ctx.sync()
            mdist.reduce_packed(acc_buf, dst=0)
            if rank == 0 and not warm:
                torch.cuda.synchronize()
                fb.set_accumulation(acc_s.data_ptr(), acc_w.data_ptr())

    def sync():
        ctx.sync()
        torch.cuda.synchronize()

    elapsed = timed_region(lambda: run(frame0, args.steps * fps), end_of_job, world, sync)
    if args.save_image and rank == 0:
        np.save(args.save_image, fb.read(2))
    kstats = {}
    if not args.no_kernel_timing:
        # per-kernel HIP-event durations in a separate, untimed pass: one frame slot (kernels do not
        # share the GPU with another frame's launches, so each duration is the kernel's own), calls
        # of the timed region's shape (stats_batch frames each)
        fb.set_frames_in_flight(1)
        run(frame0 + args.steps * fps, stats_batch, stats_batch)   # the slot re-binds outside the profiled launches
        ctx.sync()
        ctx.set_profiling(True)
        ctx.reset_stats()
        run(frame0 + args.steps * fps + stats_batch, args.stats_launches * stats_batch, stats_batch)
        ctx.sync()
        kstats = ctx.kernel_stats()
        ctx.set_profiling(False)
        fb.set_frames_in_flight(0)

    bd = None
    if not bdpt and not args.no_bdpt and not two_level:   # config 4's integrator beside the PT headline
        bd = bdpt_section(ctx, ds, cam_of, W, H, D, sampler, world, rank, args.bdpt_steps, args.warmup,
                          not args.no_kernel_timing, args.bdpt_split, args.bdpt_batch, args.splat_exchange == "sparse")

    gb = world if bdpt and not band_bdpt else fps   # frames per step (global batch)
    paths = W * H * args.steps * gb
    value = paths / elapsed / 1e6
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "warmup_frames_run": warm_frames,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": args.scaling, "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: deterministic {args.scene} ({scene.num_triangles} tris, seeded generator mcrt/scenes.py)",
        "config": {"workload": f"{args.scene} {W}x{H}, {'BDPT' if bdpt else 'unidirectional PT'}, maxDepth {D}, "
                               f"{args.sampler} sampler, "
                               + (f"{gb} spp per step (1 per GPU)" if gb > 1 else "1 spp per step")
                               + ", box-filter accumulate"
                               + (f", Russian roulette from bounce {args.rr_start} (perf mode)"
                                  if args.russian_roulette and not bdpt else ""), "width": W, "height": H,
                   "triangles": scene.num_triangles, "max_depth": D, "spp_per_step": gb, "global_batch": gb,
                   "bvh": ("two-level (instanced), RadeonRays-identical Bvh trees" if two_level else
                           "device LBVH" if args.device_build else
                           "RadeonRays-identical SAH, " + ("host build" if args.host_build else "device build")),
                   "bvh_build_ms": round(info["build_ms"], 1),
                   "parallelism": (f"band split x {world}, 1 sparse splat all-to-all per call + 1 RCCL reduce" if sparse_x
                                   else f"band split x {world}, 1 splat reduce-scatter per call + 1 RCCL reduce" if band_bdpt
                                   else f"frame split x {world} + 1 RCCL reduce" if bdpt else
                                   f"tile-split {args.band_rows}-row bands x {world}"
                                   + (f", {fps} frames per step" if fps > 1 else "") + " + 1 RCCL "
                                   + ("band gather" if args.end_collective == "gather" else "reduce")),
                   "frames_per_launch": stats_batch, "max_frames_per_call": batch},
    }
    if rank == 0:
        rays = {"closest": fstats["closest_rays"] / (W * H / world), "any": fstats["any_rays"] / (W * H / world),
                "shaded": fstats["shaded_paths"] / (W * H / world)}
        out["rays_per_path"] = {k: round(v, 4) for k, v in rays.items()}
        if hcounts is not None and qcounts is not None:   # occluder hints
            out["shadow_hints"] = {f"bounce{b}": round(hcounts[b] / max(qcounts[0][b], 1), 4) for b in range(D)}
            # the wavefront's queues per bounce (one untimed frame): compaction keeps only live paths,
            # so the launches shrink with depth (and with --russian-roulette)
            # closest-hit walks over the compact records that ended on a near tie and were repeated on
            # the exact 64-B records (mcrt_traverse.h traverseQOct), per extension bounce
            out["near_tie_retraces"] = {f"bounce{b + 1}": int(rcounts[b]) for b in range(D - 1)}
            out["queues_per_frame"] = {"shadow": [int(v) for v in qcounts[0][:D]],
                                       "extension": [int(v) for v in qcounts[1][:max(D - 1, 0)]],
                                       "pixels": int(W * H / world)}
        # (the CPU oracle and the roofline's node counts price the flat structure)
        oracle_ok = world == 1 and not bdpt and sampler == T.SAMPLER_RANDOM and not two_level
        cpu = None
        if oracle_ok and not args.no_cpu_baseline:
            cpu = cpu_baseline(scene, cam_of, W, H, D, args.cpu_seconds)
            st = cpu["_stats"]
            # the port's fidelity: the product renders the port's first sampled frame again.  The
            # port is an IEEE restatement (no fma contraction, exact 1/x where the reference uses
            # native_recip), so it is NOT bit-exact at this scene size; the product's
            # parity is measured against the reference itself (parity_vs_reference)
            f0 = cpu["_frame0"]
            fb.render(ds, cam_of(f0), frame=f0, max_depth=D, **band)
            g = fb.read(0)[cpu["_rows"]]
            r = cpu["_radiance"][cpu["_rows"]]
            dlt = np.abs(g[..., :3].astype(np.float64) - r[..., :3])
            ok = (dlt <= 1e-4 * np.maximum(1.0, np.abs(r[..., :3]))).all(-1).mean()
            out["visits_per_query"] = {"k_primary": round(st[1] / max(st[0], 1), 2),
                                       "k_extend": round(st[3] / max(st[2], 1), 2),
                                       "k_shadow": round(st[5] / max(st[4], 1), 2)}
            out["leaf_visit_share"] = {"k_extend": round(st[6] / max(st[3], 1), 4), "k_shadow": round(st[7] / max(st[5], 1), 4)}
            out["cpu_baseline"] = {k: v for k, v in cpu.items() if not k.startswith("_")}
            out["cpu_baseline"]["value"] = round(out["cpu_baseline"]["value"], 4)
            out["cpu_baseline"]["fidelity"] = {
                "pixels_within_1e-4_of_product": round(float(ok), 5), "rows": int(len(cpu["_rows"])), "frame": int(f0),
                "note": "the port (IEEE C restatement) against the product; the product against the reference "
                        "itself is parity_vs_reference"}
            if not args.russian_roulette and not args.no_reference_parity:   # the reference has no RR
                out["parity_vs_reference"] = reference_parity(args.scene, args.tris, fb, ds, cam_of, W, H, D, frame0,
                                                              band)
        if kstats:
            out["kernels"] = {k: {"avg_ms": round(v["ms"] / max(v["launches"], 1), 4), "launches": v["launches"],
                                  "items_per_launch": round(v["items"] / max(v["launches"], 1), 1),
                                  "ms_per_frame": round(v["ms"] / (args.stats_launches * stats_batch), 4)}
                              for k, v in kstats.items()}
            out["kernels_note"] = ("HIP-event durations from an untimed pass after the timed region: one frame slot "
                                   f"(no overlap with another frame's launches), {args.stats_launches} calls of "
                                   f"{stats_batch} frames, the timed region's launch shape")
            dom = max(kstats, key=lambda k: kstats[k]["ms"])
            if oracle_ok and dom == "k_shadow_extend" and not args.no_roofline_model:
                avg_ms = kstats[dom]["ms"] / max(kstats[dom]["launches"], 1)
                out["roofline"] = roofline_shadow_extend(scene, cam_of, W, H, D, stats_batch, avg_ms, qcounts, ctx,
                                                         cpu["_oracle"] if cpu else None, quant)
                if "visits_per_query" in out:
                    hf = hcounts[0] / max(qcounts[0][0], 1) if hcounts else 0.0
                    out["roofline"]["gather_ceiling"] = gather_ceiling(ctx, out["roofline"], out["visits_per_query"],
                                                                       avg_ms, hf, out["leaf_visit_share"]["k_extend"])
                    out["roofline"]["survey_8d"] = survey_8d_figure(value, out["rays_per_path"],
                                                                    out["visits_per_query"], D)
        if bd is not None:
            bdo = {k: v for k, v in bd.items() if not k.startswith("_")}
            if oracle_ok and sampler == T.SAMPLER_RANDOM and not args.no_cpu_baseline:
                bdo.update(bdpt_roofline_and_cpu(scene, cpu["_oracle"] if cpu else None, cam_of, W, H, D, bdo,
                                                 args.cpu_seconds, quant))
            out["bdpt"] = bdo
        print(json.dumps(out), flush=True)
    if bd is not None:
        bd["_fb"].close()
    fb.close()
    ds.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
