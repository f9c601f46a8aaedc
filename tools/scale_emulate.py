"""Per-rank work of the N-GPU tile split, emulated on ONE GPU, plus the modelled collectives.

For N in --ns, renders each rank's bands (band_index = r of num_bands = N) one rank at a time on
cuda:0 and reports the slowest rank's ms per band-frame next to the 1-GPU ms/frame; efficiency =
base / (N x that), the compute part of the scaling efficiency (the launch gaps of concurrent
processes are not in it).  --scaling strong: K frames per rank (a step = one frame split over the
ranks); weak (bench.py's default): K x N frames per rank, calls of N x the --chunks frames (capped
at 256), as a step = N frames.  --integrator bdpt: the band-split BDPT frame
of each rank (render, rank-major splat pack, gather of its own chunk) and the bytes of the one
splat reduce-scatter per frame, against the full-frame all-reduce it replaced.  Prints one JSON
line.

The collectives cannot run here (one GPU; RCCL refuses two ranks on one device), so their time is
MODELLED from the bytes each rank moves over xGMI: LINK_GBS per direction per link
(a conservative 50 GB/s, about two thirds of one direction of the ~153 GB/s bidirectional link
figure of the task brief) and STEP_US of latency per collective step.
  PT:   ONE gather of every rank's own rows to rank 0 at the end of the job (mcrt.dist.gather_bands_fb):
        rank 0 receives N - 1 shares over N - 1 links at once -> share / LINK + STEP.
  BDPT: ONE reduce-scatter of the rank-major splats per call (mcrt.dist.exchange_splats), RCCL rings
        striped over min(N - 1, 7) links: (N - 1) / N x buffer / (links x LINK) + 2 (N - 1) STEP.  The
        exchange of a call runs on its frame slot's stream while the next call renders on the other
        slot, so only the last call's exchange is exposed ("overlapped"); "serial" adds every one.
The model has no term for a collective's first-use setup (RCCL connects a pair of ranks on their
first send / recv): bench.py runs its end-of-job collective once before the timed region
(bench.timed_region, tests/test_dist_cpu.py::test_bench_warms_end_collective_before_timing), and the
BDPT band split's per-call reduce-scatters already run in its warm-up calls, so setup falls outside
the timed region there too.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)


LINK_GBS = 50.0   # per direction per xGMI link (model assumption, see the docstring)
STEP_US = 10.0    # latency per collective step


def pt_gather_ms(n, W, H, band_rows, steps):
    """Modelled end-of-job band gather, ms per (band-)frame of the job (steps = its frames)."""
    if n == 1:
        return 0.0
    from mcrt import dist as mdist
    share = mdist.splat_chunk_rows(H, band_rows, n) * W * 5 * 4   # packed rows: sum(w L) float4 + sum(w)
    return (share / (LINK_GBS * 1e9) * 1e3 + STEP_US * 1e-3) / steps


def bdpt_exchange_ms(n, W, H, band_rows, batch):
    """Modelled splat reduce-scatter of one call of `batch` frames (ms)."""
    if n == 1:
        return 0.0, 0
    from mcrt import dist as mdist
    full = mdist.SPLAT_CHANNELS * 4 * W * mdist.splat_chunk_rows(H, band_rows, n) * batch * n
    links = min(n - 1, 7)
    return ((n - 1) / n * full / (links * LINK_GBS * 1e9) * 1e3 + 2 * (n - 1) * STEP_US * 1e-3), full


def sparse_exchange_ms(n, rec, batch):
    """Modelled sparse splat exchange of one call (ms): an all-to-all of the counts, then one of the
    16-B records; each rank sends to N - 1 receivers over N - 1 links at once, so the largest
    per-receiver share bounds it.  The measured rank time already holds the host wait for the counts."""
    if n == 1 or rec["calls"] == 0:
        return 0.0, 0
    per_call = rec["records"] / rec["calls"] * 16
    biggest = rec["to_rank_max"] * 16
    return (biggest / (LINK_GBS * 1e9) * 1e3 + 2 * STEP_US * 1e-3), int(per_call / batch)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--scene", default="san_miguel_proxy")
    ap.add_argument("--fif", type=int, default=0, help="frames in flight (0 = the library's auto choice)")
    ap.add_argument("--batch", type=int, default=1, help="frames per mcrt_render_frames call (0 = N)")
    ap.add_argument("--chunks", default="", help="frames per call, cycled (overrides --batch)")
    ap.add_argument("--pow2", action="store_true", help="round each call of --chunks down to a power of two")
    ap.add_argument("--kernels", action="store_true",
                    help="also report rank 0's per-kernel HIP-event ms per frame (a separate profiled pass)")
    ap.add_argument("--integrator", default="pt", choices=["pt", "bdpt"])
    ap.add_argument("--splat-exchange", default="dense", choices=["sparse", "dense"],
                    help="band-split BDPT: record lists + all-to-all (sparse) or rank-major planes + reduce-scatter")
    ap.add_argument("--ranks", default="", help="only these ranks (comma list; profiling one rank's call)")
    ap.add_argument("--base-ms", type=float, default=None,
                    help="1-GPU ms/frame (the efficiency base) when --ns does not include 1")
    args = ap.parse_args()
    import torch
    torch.cuda.init()   # torch's HIP runtime before the library's context (as bench.py)
    from mcrt import lib, scenes
    from mcrt import types as T
    from mcrt.camera import scene_camera
    W, H = 1920, 1080
    scene = scenes.san_miguel_proxy() if args.scene == "san_miguel_proxy" else scenes.dragon_proxy()
    cams = [scene_camera(args.scene, W, H, frame=f, jitter=True) for f in range(64)]   # TAA as bench.py
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, scene)
    fb = lib.FrameBuffer(ctx, W, H)
    filt = T.make_filter(T.BOX)
    fb.set_frames_in_flight(args.fif)
    out = {"fif": args.fif, "batch": args.batch, "chunks": args.chunks, "scene": args.scene, "steps": args.steps,
           "scaling": args.scaling if args.integrator == "pt" else "strong",
           "band_rows": args.band_rows, "integrator": args.integrator, "per_n": {}}
    if args.integrator == "bdpt":
        bdpt_sweep(args, ctx, ds, fb, cams, filt, W, H, out)
        return
    for n in [int(x) for x in args.ns.split(",")]:
        per_rank = []
        for r in ranks_of(args, n):
            band = dict(band_rows=args.band_rows, num_bands=n, band_index=r)
            B = args.batch if args.batch > 0 else n
            mult = n if args.scaling == "weak" else 1   # frames per step
            plan = [min(256, int(c) * mult) for c in args.chunks.split(",")] if args.chunks else [min(256, B * mult)]
            frames = args.steps * mult

            def run(f0, count):
                i = calls = 0
                while i < count:
                    k = min(plan[calls % len(plan)], count - i)
                    if args.chunks and args.pow2:
                        k = 1 << (k.bit_length() - 1)
                    calls += 1
                    if k == 1:
                        fb.render(ds, cams[(f0 + i) % 64], frame=f0 + i, max_depth=2, **band)
                    else:
                        fb.render_frames(ds, [cams[(f0 + i + j) % 64] for j in range(k)], frame=f0 + i, max_depth=2,
                                         **band)
                    fb.accumulate(filt, f0 + i)
                    i += k
            run(0, max(3, 4 * max(plan)))   # every frame slot allocated before timing
            ctx.sync()
            t0 = time.perf_counter()
            run(16, frames)
            ctx.sync()
            per_rank.append((time.perf_counter() - t0) / frames * 1e3)
            if args.kernels and len(per_rank) == 1:
                ctx.set_profiling(True)
                ctx.reset_stats()
                run(16 + frames, frames)
                ctx.sync()
                ks = ctx.kernel_stats()
                ctx.set_profiling(False)
                kern = {k: round(v["ms"] / frames, 4) for k, v in ks.items()}
        out["per_n"][n] = {"max_ms": round(max(per_rank), 4), "mean_ms": round(sum(per_rank) / len(per_rank), 4),
                           "min_ms": round(min(per_rank), 4), "rank_ms": [round(x, 4) for x in per_rank],
                           "frames_per_rank": frames, "frames_per_call": plan}
        if args.kernels:
            out["per_n"][n]["rank0_kernel_ms_per_frame"] = kern
    # efficiency is relative to ONE GPU rendering the whole image: the N = 1 run of this sweep, or
    # --base-ms from a separate N = 1 run (never the smallest N of the sweep, which may be > 1)
    base = out["per_n"][1]["max_ms"] if 1 in out["per_n"] else args.base_ms
    out["base_ms_n1"] = base
    out["model"] = {"link_gbs_per_direction": LINK_GBS, "step_us": STEP_US}
    for n, v in out["per_n"].items():
        v["compute_eff"] = round(base / (n * v["max_ms"]), 4) if base else None
        g = pt_gather_ms(n, W, H, args.band_rows, v["frames_per_rank"])
        v["gather_ms_per_frame_modelled"] = round(g, 5)
        v["eff_with_collective"] = round(base / (n * (v["max_ms"] + g)), 4) if base else None
    print(json.dumps(out), flush=True)
    fb.close()
    ds.close()
    ctx.close()


def ranks_of(args, n):
    return [int(x) for x in args.ranks.split(",")] if args.ranks else list(range(n))


def bdpt_sweep(args, ctx, ds, fb, cams, filt, W, H, out):
    """Band-split BDPT per rank: render the rank's bands, pack its splats rank-major, complete its
    rows from its own chunk (the values do not matter for the timing), accumulate."""
    import torch
    from mcrt import dist as mdist
    from mcrt import types as T
    B = max(args.batch, 1)   # BDPT frames per mcrt_render_frames call
    sparse = args.splat_exchange == "sparse"
    fb.set_splat_exchange(sparse)
    for n in [int(x) for x in args.ns.split(",")]:
        per_rank = []
        cr = mdist.splat_chunk_rows(H, args.band_rows, n)
        C = mdist.SPLAT_CHANNELS
        full = None if sparse else torch.zeros(C * W * cr * n * B, dtype=torch.float32, device="cuda")
        sbufs = mdist.SparseSplatBuffers("cuda")
        rec = {"records": 0, "to_rank_max": 0, "calls": 0}   # sparse: records each rank sends per call
        for r in ranks_of(args, n):
            band = dict(band_rows=args.band_rows, num_bands=n, band_index=r, integrator=T.INTEGRATOR_BDPT)
            own = None if sparse else full[r * C * W * cr * B:(r + 1) * C * W * cr * B]

            def run(f0, count, timed=False):
                i = 0
                while i < count:
                    k = min(B, count - i)
                    fb.render_frames(ds, [cams[(f0 + i + j) % 64] for j in range(k)], frame=f0 + i, max_depth=2,
                                     **band)
                    if n > 1 and sparse:
                        # the rank's records grouped by receiver (their host counts: the all-to-all's
                        # split sizes); the receive side is the model's: its own splats are in place
                        send = sbufs.get("send", 0)
                        cnt = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
                        if cnt.sum() > send.numel() // 4:
                            send = sbufs.get("send", int(cnt.sum()))
                            cnt = fb.bdpt_splats_sparse(send.data_ptr(), send.numel() // 4)
                        fb.bdpt_gather_sparse(0, 0)
                        if timed:
                            rec["records"] += int(cnt.sum())
                            rec["to_rank_max"] = max(rec["to_rank_max"], int(cnt.max()))
                            rec["calls"] += 1
                    elif n > 1:
                        fb.bdpt_splats_copy(full.data_ptr())
                        fb.bdpt_gather(own.data_ptr())
                    fb.accumulate_frames([filt] * k, f0 + i)
                    i += k
            run(0, 3 * B)
            ctx.sync()
            t0 = time.perf_counter()
            run(16 * B, args.steps, timed=True)
            ctx.sync()
            per_rank.append((time.perf_counter() - t0) / args.steps * 1e3)
        if sparse:
            call_ms, call_bytes = sparse_exchange_ms(n, rec, B)
        else:
            call_ms, call_bytes = bdpt_exchange_ms(n, W, H, args.band_rows, B)
        calls = -(-args.steps // B)
        out["per_n"][n] = {"max_ms": round(max(per_rank), 4), "mean_ms": round(sum(per_rank) / n, 4),
                           "min_ms": round(min(per_rank), 4),
                           "splat_exchange": {"kind": "sparse all-to-all" if sparse else "dense reduce-scatter",
                                              "bytes_per_rank_per_frame": call_bytes if sparse else call_bytes // B,
                                              "ms_per_call_modelled": round(call_ms, 4),
                                              "calls": calls,
                                              "exposed_ms_per_frame_overlapped": round(call_ms / args.steps, 5),
                                              "exposed_ms_per_frame_serial": round(call_ms * calls / args.steps, 5)}}
    base = out["per_n"][1]["max_ms"] if 1 in out["per_n"] else args.base_ms
    out["base_ms_n1"] = base
    out["model"] = {"link_gbs_per_direction": LINK_GBS, "step_us": STEP_US, "frames_per_call": B}
    for n, v in out["per_n"].items():
        v["compute_eff"] = round(base / (n * v["max_ms"]), 4) if base else None
        x = v["splat_exchange"]
        # sparse: the host waits for each call's counts, so every call's exchange is exposed (its host
        # wait is already in max_ms, the RCCL part is modelled); dense: all but the last call's overlap
        # the next call's render on the other frame slot
        exposed = x["exposed_ms_per_frame_serial"] if sparse else x["exposed_ms_per_frame_overlapped"]
        v["eff_with_collective"] = round(base / (n * (v["max_ms"] + exposed)), 4) if base else None
        v["eff_with_collective_serial"] = round(base / (n * (v["max_ms"] + x["exposed_ms_per_frame_serial"])), 4) \
            if base else None
    print(json.dumps(out), flush=True)
    fb.close()
    ds.close()
    ctx.close()


if __name__ == "__main__":
    main()
