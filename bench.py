"""Benchmark: Mpaths/s of the MI355X path tracer on the San-Miguel proxy at 1920x1080
(BASELINE.json metric), PT with maxDepth 2 (the reference default), random sampler.
`--integrator bdpt` measures the BDPT integrator instead: one path =
one camera + one light subpath with all their connections; N GPUs split frames (each rank
renders whole frames f = rank + N*i, "scaling": "weak"), since light-tracing splats land anywhere.

One step = one 1-spp frame of the whole image (mcrt_render_frame + mcrt_accumulate).
N GPUs: one process per GPU (torch.distributed.run), the image is tile-split into 8-row bands
dealt round-robin to the ranks (north star), each rank accumulates its bands, and one RCCL
reduce of the accumulators (sum) to rank 0 ends the job (inside the timed region).
Total work per step is fixed -> "scaling": "strong".

Also reported (one JSON line on rank 0):
  roofline      dominant kernel: algorithmic bytes per launch (rays x (48 + 32 + 64 V)
                for closest, rays x (48 + 4 + 64 V) for any-hit, V = node visits per query of the
                reference Bvh2 + LDS traversal measured by the oracle on the same scene/camera) over its
                average HIP-event duration, vs the 8 TB/s HBM peak; traffic from rocprofv3 PMC if present
  cpu_baseline  the oracle (C restatement of the reference kernels) on a bounded sample of rows of
                the same frame, all host cores (rank 0, N = 1 only)
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


def per_query_bytes(kernel, V):
    """SURVEY.md §8d algorithmic bytes per query."""
    if kernel == "k_shadow":
        return 48 + 4 + 64.0 * V
    return 48 + 32 + 64.0 * V


def b_path(stats_per_path, D):
    """B_path = 112 + sum_closest(48+32+64V) + sum_any(48+4+64V) + sum_shade 388 + sum_bounce 132 + 72."""
    s = stats_per_path
    return (112 + s["closest"] * 80 + 64 * s["closest_visits"] + s["any"] * 52 + 64 * s["any_visits"]
            + s["shaded"] * 388 + D * 132 + 72)


def cpu_baseline(scene, cam, W, H, D, target_s=15.0):
    """Times the oracle on a bounded, evenly spread sample of rows of frame 0."""
    from oracle import pyoracle as po
    # the box exposes all host CPUs but one GPU job owns a share of them (OMP_NUM_THREADS there)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    o = po.OracleScene(scene)
    t0 = time.perf_counter()
    o.build()
    build_s = time.perf_counter() - t0
    # calibrate on 8 rows, then size the sample to ~target_s
    cal_rows = np.linspace(0, H - 1, 8).astype(np.int32)
    t0 = time.perf_counter()
    o.render_rows(cam, cal_rows, frame=0, max_depth=D, threads=threads)
    dt = max(time.perf_counter() - t0, 1e-3)
    nrows = int(np.clip(8 * target_s / dt, 8, H))
    rows = np.unique(np.linspace(0, H - 1, nrows).astype(np.int32))
    t0 = time.perf_counter()
    rad, st = o.render_rows(cam, rows, frame=0, max_depth=D, threads=threads)
    el = time.perf_counter() - t0
    paths0 = paths = len(rows) * W
    frames = 1
    # a whole frame can take well under target_s: render further frames (1, 2, ...) of the same
    # rows until the sample is ~target_s of CPU work
    while len(rows) == H and el + el / frames <= target_s:
        t0 = time.perf_counter()
        o.render_rows(cam, rows, frame=frames, max_depth=D, threads=threads)
        el += time.perf_counter() - t0
        paths += paths0
        frames += 1
    return {
        "value": paths / el / 1e6, "unit": "Mpaths/s", "cores": threads, "kind": "port",
        "sample": f"{len(rows)} of {H} rows (evenly spaced) of frames 0..{frames - 1}, {paths} paths, D={D}, "
                  f"random sampler; oracle = C restatement of PathTracing.cl + RR Bvh2/LDS traversal, {threads} "
                  f"threads, {el:.1f}s (BVH build {build_s:.1f}s not timed)",
        "_rows": rows, "_radiance": rad, "_stats": st, "_paths": paths0,
    }


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from a committed rocprofv3 PMC summary (tools/pmc.py)."""
    path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        k = d.get("kernels", {}).get(kernel)
        return None if k is None else float(k["hbm_bytes_per_launch"])
    except Exception:
        return None


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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--integrator", default="pt", choices=["pt", "bdpt"])
    ap.add_argument("--save-image", default=None, help="rank 0 saves the final accumulated image (.npy)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the product path); gloo only rehearses N ranks on one GPU")
    ap.add_argument("--device-build", action="store_true", help="on-device linear BVH instead of the RR-identical host build")
    ap.add_argument("--force-flat", action="store_true",
                    help="flat BVH even for instanced scenes (RR bvh.forceflat); default: RR's auto selection")
    ap.add_argument("--russian-roulette", action="store_true",
                    help="opt-in RR on extension rays (perf mode; the reference has none, so not a parity run)")
    ap.add_argument("--rr-start", type=int, default=1, help="first bounce whose extension rays RR may cut")
    ap.add_argument("--batch", type=int, default=0,
                    help="PT frames per mcrt_render_frames call (one launch sequence for all of them); "
                         "0 = auto (min(16, 4 x ranks))")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    if sampler == T.SAMPLER_SOBOL:   # g_SobolMatrices32 (sobol.h:34), committed as a data fixture
        scene.sobol = np.load(os.path.join(ROOT, "tests", "golden", "sobol_1024x52.npy"))
    gen_s = time.perf_counter() - t0
    cam = scene_camera(args.scene, W, H)
    log(f"[bench] scene {scene.name}: {scene.num_triangles} tris, gen {gen_s:.1f}s")

    ctx = lib.Context(local)
    t0 = time.perf_counter()
    ds = lib.DeviceScene(ctx, scene, device_build=args.device_build, force_flat=args.force_flat)
    info = ds.info()
    two_level = ds.layout()["two_level"] == 1
    log(f"[bench] upload+BVH {time.perf_counter() - t0:.1f}s (build {info['build_ms'] / 1e3:.1f}s, "
        f"{info['nodes']} nodes, {info['bytes'] / 1e6:.0f} MB)")
    fb = lib.FrameBuffer(ctx, W, H)
    filt = T.make_filter(T.BOX)
    bdpt = args.integrator == "bdpt"
    if bdpt:   # frame split: whole frames per rank
        band = dict(band_rows=8, num_bands=1, band_index=0, integrator=T.INTEGRATOR_BDPT)
    else:
        band = dict(band_rows=args.band_rows, num_bands=world, band_index=rank)
    first = [True]
    # auto: 4 frames per launch on one GPU, 16 from 4 GPUs on (a 1/N band share x 16 frames keeps
    # every launch at >= 4 whole images of paths; tools/scale_emulate.py sweeps)
    batch = 1 if bdpt else (args.batch if args.batch > 0 else min(16, 4 * world))

    def step(i, n=1):
        """frames i .. i+n-1 (one mcrt_render_frames call when n > 1)"""
        frame = rank + world * i if bdpt else i
        kw = dict(max_depth=D, sampler=sampler, rr=args.russian_roulette, rr_start=args.rr_start, **band)
        if n == 1:
            fb.render(ds, cam, frame=frame, **kw)
        else:
            fb.render_frames(ds, [cam] * n, frame=frame, **kw)
        fb.accumulate(filt, 0 if first[0] else frame)   # 0: the first accumulation overwrites
        first[0] = False

    def run(i0, count):
        i = 0
        while i < count:
            n = min(batch, count - i)
            step(i0 + i, n)
            i += n

    # warmup: at least one call per frame slot (MCRT_MAX_FRAMES_IN_FLIGHT = 4), so no slot
    # allocation falls inside the timed region
    warm = max(args.warmup, 4 * batch)
    run(0, warm)
    ctx.sync()
    # per-frame path statistics (device queue sizes) from one untimed frame
    step(warm)
    ctx.sync()
    fstats = fb.stats()
    qcounts = fb.queue_counts() if not bdpt else None
    frame0 = warm + 1

    if not args.no_kernel_timing:
        ctx.set_profiling(True)
    ctx.reset_stats()
    if world > 1:
        acc_buf, acc_s, acc_w = mdist.packed_accumulators(W * H, "cuda")   # one buffer -> one reduce
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    run(frame0, args.steps)
    if world > 1:   # single RCCL reduce of the tile accumulators (north star)
        fb.copy_device(1, acc_s.data_ptr())
        fb.copy_device(3, acc_w.data_ptr())
        ctx.sync()
        mdist.reduce_packed(acc_buf, dst=0)
        if rank == 0:
            torch.cuda.synchronize()
            fb.set_accumulation(acc_s.data_ptr(), acc_w.data_ptr())
    ctx.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if args.save_image and rank == 0:
        np.save(args.save_image, fb.read(2))
    kstats = ctx.kernel_stats() if not args.no_kernel_timing else {}
    ctx.set_profiling(False)

    paths = W * H * args.steps * (world if bdpt else 1)
    value = paths / elapsed / 1e6
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Mpaths/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak" if bdpt else "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: deterministic {args.scene} ({scene.num_triangles} tris, seeded generator mcrt/scenes.py)",
        "config": {"workload": f"{args.scene} {W}x{H}, {'BDPT' if bdpt else 'unidirectional PT'}, maxDepth {D}, "
                               f"{args.sampler} sampler, 1 spp per step, box-filter accumulate"
                               + (f", Russian roulette from bounce {args.rr_start} (perf mode)"
                                  if args.russian_roulette and not bdpt else ""), "width": W, "height": H,
                   "triangles": scene.num_triangles, "max_depth": D, "spp_per_step": 1,
                   "bvh": ("two-level (instanced), RadeonRays-identical Bvh trees" if two_level else
                           "device LBVH" if args.device_build else "host RadeonRays-identical SAH"),
                   "bvh_build_ms": round(info["build_ms"], 1),
                   "parallelism": (f"frame split x {world} + 1 RCCL reduce" if bdpt else
                                   f"tile-split {args.band_rows}-row bands x {world} + 1 RCCL reduce"),
                   "frames_per_launch": batch},
    }
    if rank == 0:
        rays = {"closest": fstats["closest_rays"] / (W * H / world), "any": fstats["any_rays"] / (W * H / world),
                "shaded": fstats["shaded_paths"] / (W * H / world)}
        out["rays_per_path"] = {k: round(v, 4) for k, v in rays.items()}
        cpu = None
        # (the CPU oracle and the roofline's visit counts price the flat structure)
        if world == 1 and not args.no_cpu_baseline and not bdpt and sampler == T.SAMPLER_RANDOM and not two_level:
            cpu = cpu_baseline(scene, cam, W, H, D, args.cpu_seconds)
            st = cpu["_stats"]
            V = {"k_primary": st[1] / max(st[0], 1), "k_extend": st[3] / max(st[2], 1),
                 "k_shadow": st[5] / max(st[4], 1)}
            # parity spot check of the timed product frames is not possible (different frame
            # indices); render frame 0 again and compare the sampled rows
            fb.render(ds, cam, frame=0, max_depth=D, **band)
            g = fb.read(0)[cpu["_rows"]]
            r = cpu["_radiance"][cpu["_rows"]]
            dlt = np.abs(g[..., :3].astype(np.float64) - r[..., :3])
            ok = (dlt <= 1e-4 * np.maximum(1.0, np.abs(r[..., :3]))).all(-1).mean()
            out["parity_vs_oracle"] = {"pixels_within_1e-4": round(float(ok), 5), "rows": int(len(cpu["_rows"]))}
            per_path = {"closest": (st[0] + st[2]) / cpu["_paths"], "any": st[4] / cpu["_paths"],
                        "closest_visits": (st[1] + st[3]) / cpu["_paths"], "any_visits": st[5] / cpu["_paths"],
                        "shaded": (st[0] + st[2]) / cpu["_paths"]}
            bp = b_path(per_path, D)
            out["b_path_bytes"] = round(bp, 1)
            out["achieved_hbm_gbs_alg"] = round(value * 1e6 * bp / 1e9, 1)
            out["visits_per_query"] = {k: round(v, 2) for k, v in V.items()}
            out["cpu_baseline"] = {k: v for k, v in cpu.items() if not k.startswith("_")}
            out["cpu_baseline"]["value"] = round(out["cpu_baseline"]["value"], 4)
        else:
            V = None
        if kstats:
            dom = max(kstats, key=lambda k: kstats[k]["ms"])
            ks = kstats[dom]
            avg_ms = ks["ms"] / max(ks["launches"], 1)
            items_per_launch = ks["items"] / max(ks["launches"], 1)
            out["kernels"] = {k: {"avg_ms": round(v["ms"] / max(v["launches"], 1), 4), "launches": v["launches"],
                                  "items_per_launch": round(v["items"] / max(v["launches"], 1), 1)}
                              for k, v in kstats.items()}
            alg = None
            fpl = args.steps / max(ks["launches"], 1)   # frames per launch (mcrt_render_frames batches)
            if V is not None and dom == "k_shadow_extend":
                # one launch = the extension rays for bounce 1 + the shadow rays of bounce 0, of fpl frames
                alg = fpl * (qcounts[1][0] * per_query_bytes("k_extend", V["k_extend"])
                             + qcounts[0][0] * per_query_bytes("k_shadow", V["k_shadow"]))
            elif V is not None and dom in V:
                alg = items_per_launch * per_query_bytes(dom, V[dom])
            if alg is not None:
                achieved = alg / (avg_ms * 1e-3) / 1e9
                tr = pmc_traffic(dom)
                out["roofline"] = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                                   "traffic": tr, "alg_bytes_per_launch": round(alg),
                                   "avg_launch_ms": round(avg_ms, 4)}
                try:   # attainable HBM bandwidth of an in-repo stream copy
                    att = ctx.stream_copy_gbps(2 << 30, 5)
                    out["roofline"]["attainable"] = round(att, 1)
                    out["roofline"]["frac_of_attainable"] = round(achieved / att, 4)
                except Exception as e:   # noqa: BLE001 -- reported, not fatal
                    log(f"[bench] stream copy failed: {e}")
        print(json.dumps(out), flush=True)
    fb.close()
    ds.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
