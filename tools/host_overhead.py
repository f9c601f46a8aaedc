"""Host-side cost of one bench step call (analysis tool, GPU): how long the Python + C-ABI calls of
bench.py's timed region take on the host (camera records, mcrt_render_frames, mcrt_accumulate), and
the wall time of a whole synchronised call against its GPU span (HIP events on the frame's stream).
Small scene so the GPU work is short and the fixed host costs stand out.
usage: python tools/host_overhead.py [frames_per_call] [repeats]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd")]


def main():
    import numpy as np
    import torch
    torch.cuda.init()
    from mcrt import lib, scenes
    from mcrt import types as T
    from mcrt.camera import scene_camera
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    W, H = 480, 272
    sc = scenes.dragon_proxy(tris=200_000)
    cams = [scene_camera("dragon_proxy", W, H, frame=f, jitter=True) for f in range(64)]
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, sc)
    fb = lib.FrameBuffer(ctx, W, H)
    filt = T.make_filter(T.BOX)
    out = {"frames_per_call": n, "W": W, "H": H}
    rec, call, acc, wall = [], [], [], []
    for r in range(reps + 3):
        f0 = r * n
        ctx.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cl = [cams[(f0 + k) % 64] for k in range(n)]
        t1 = time.perf_counter()
        fb.render_frames(ds, cl, frame=f0, max_depth=2)
        t2 = time.perf_counter()
        fb.accumulate(filt, f0)
        t3 = time.perf_counter()
        ctx.sync()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if r >= 3:
            rec.append(t1 - t0)
            call.append(t2 - t1)
            acc.append(t3 - t2)
            wall.append(t4 - t0)
    ctx.set_profiling(True)
    ctx.reset_stats()
    fb.set_frames_in_flight(1)
    for r in range(reps):
        fb.render_frames(ds, [cams[(k + r) % 64] for k in range(n)], frame=r * n, max_depth=2)
        fb.accumulate(filt, r * n)
    ctx.sync()
    ks = ctx.kernel_stats()
    ctx.set_profiling(False)
    gpu = sum(v["ms"] for v in ks.values()) / reps
    med = lambda a: round(float(np.median(a)) * 1e6, 1)   # noqa: E731  (us)
    out.update({"camera_list_us": med(rec), "render_frames_call_us": med(call), "accumulate_call_us": med(acc),
                "wall_per_call_us": med(wall), "kernel_time_per_call_us": round(gpu * 1e3, 1),
                "wall_minus_kernels_us": round(float(np.median(wall)) * 1e6 - gpu * 1e3, 1)})
    print(json.dumps(out))
    fb.close()
    ds.close()
    ctx.close()


if __name__ == "__main__":
    main()
