"""Launch tails of the PT call at N ranks, from per-workgroup clocks (MCRT_WAVE_CLOCK=1,
mcrt_framebuffer_wave_clock): renders one rank's bands (band split of N) with the bench's call shape
(one call of --steps TAA frames) and reports, per launch (camera, shadow+extension, last shadow):
the span, the wave-duration distribution, the mean number of waves in flight over the span and
over its last 10 %, and how long the launch runs after 90 % / 99 % of its waves have ended.
usage: MCRT_WAVE_CLOCK=1 python tools/wave_tail.py --ns 1,8 > out.json"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)

NAMES = ["k_primary", "k_shadow_extend (extension)", "k_shadow"]


def stats(clk):
    ok = clk[:, 1] != 0
    c = clk[ok].astype(np.int64)
    if len(c) == 0:
        return None
    t0 = c[:, 0].min()
    s, e = c[:, 0] - t0, c[:, 1] - t0
    e = np.where(e < s, e + (1 << 32), e)   # 32-bit wrap
    span = e.max()
    dur = e - s
    ends = np.sort(e)
    # waves in flight over time (10-ns ticks)
    ev = np.concatenate([np.stack([s, np.ones_like(s)], 1), np.stack([e, -np.ones_like(e)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    conc = np.cumsum(ev[:, 1])
    tt = ev[:, 0]
    area = np.sum(conc[:-1] * np.diff(tt))
    cut = int(span * 0.9)
    m = tt[:-1] >= cut
    tail_area = np.sum(conc[:-1][m] * np.diff(tt)[m])
    return {"waves": int(len(c)), "span_us": span / 100.0, "mean_in_flight": round(area / max(span, 1), 1),
            "mean_in_flight_last10pct": round(tail_area / max(span - cut, 1), 1),
            "dur_us": {"p50": float(np.percentile(dur, 50)) / 100, "p90": float(np.percentile(dur, 90)) / 100,
                       "p99": float(np.percentile(dur, 99)) / 100, "max": float(dur.max()) / 100},
            "after_90pct_done_us": (span - ends[int(0.9 * (len(ends) - 1))]) / 100.0,
            "after_99pct_done_us": (span - ends[int(0.99 * (len(ends) - 1))]) / 100.0}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,8")
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    if os.environ.get("MCRT_WAVE_CLOCK") != "1":
        sys.exit("set MCRT_WAVE_CLOCK=1")
    import torch
    torch.cuda.init()
    from mcrt import lib, scenes
    from mcrt.camera import scene_camera
    W, H = 1920, 1080
    scene = scenes.san_miguel_proxy()
    cams = [scene_camera("san_miguel_proxy", W, H, frame=f, jitter=True) for f in range(64)]
    ctx = lib.Context(0)
    ds = lib.DeviceScene(ctx, scene)
    fb = lib.FrameBuffer(ctx, W, H)
    fb.set_frames_in_flight(1)
    out = {"steps": args.steps, "per_n": {}}
    for n in [int(x) for x in args.ns.split(",")]:
        band = dict(band_rows=8, num_bands=n, band_index=min(args.rank, n - 1))
        for rep in range(3):   # the last call is read (earlier ones warm the slot and the hint tables)
            f0 = 64 * rep
            fb.render_frames(ds, [cams[(f0 + j) % 64] for j in range(args.steps)], frame=f0, max_depth=2, **band)
            ctx.sync()
        out["per_n"][n] = {NAMES[w]: stats(fb.wave_clock(w)) for w in range(3)}
    print(json.dumps(out), flush=True)
    fb.close()
    ds.close()
    ctx.close()


if __name__ == "__main__":
    main()
