"""Per-kernel durations of bench.py's timed render_frames call from a rocprofv3 --kernel-trace
database of `bench.py --no-kernel-timing ...` (the timed call is the last launch of each PT kernel:
20 frames packed per launch), beside the all-dispatch averages that mix in the overlapped warm-up.
usage: python tools/timed_call_trace.py results.db > profiles/r03/timed_call_trace.txt"""
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import dispatches  # noqa: E402

PT = ["k_primary", "k_shade0", "k_shadow_extend", "k_walk_resume", "k_shadeN", "k_shadow", "k_accumulate"]


def short(name):
    return next((k for k in sorted(PT, key=len, reverse=True) if k in name), None)


def main(db):
    ds = dispatches(db)
    per = defaultdict(list)
    for d in ds:
        k = short(d["kernel"])
        if k:
            per[k].append(d)
    frames = None
    print(f"# {os.path.basename(db)}: rocprofv3 --kernel-trace of bench.py --no-kernel-timing (timed call = last dispatch)")
    print(f"{'kernel':18s} {'grid':>10s} {'timed ms':>10s} {'ms/frame':>9s}   {'all-dispatch avg ms':>20s} {'n':>3s}")
    tot = 0.0
    for k in PT:
        if k not in per:
            continue
        last = per[k][-1]
        if k == "k_primary":
            frames = last["grid"] // 2073600 if last["grid"] >= 2073600 else 1
        f = frames or 1
        tot += last["ms"]
        avg = statistics.mean(x["ms"] for x in per[k])
        print(f"{k:18s} {last['grid']:10d} {last['ms']:10.4f} {last['ms'] / f:9.4f}   {avg:20.4f} {len(per[k]):3d}")
    print(f"{'sum':18s} {'':10s} {tot:10.4f} {tot / (frames or 1):9.4f}   (frames in the timed call: {frames})")
    if "k_shadow_extend" in per and "k_walk_resume" in per:   # the bench's K_SHADOW_EXTEND events span both
        both = per["k_shadow_extend"][-1]["ms"] + per["k_walk_resume"][-1]["ms"]
        print(f"k_shadow_extend + k_walk_resume (the bench's kernel): {both:.4f} ms, {both / (frames or 1):.4f} ms/frame")


if __name__ == "__main__":
    main(sys.argv[1])
