"""Compares bench.py's HIP-event kernel durations with a rocprofv3 --kernel-trace of the same command.

  python tools/timing_pass_compare.py TRACE_results.db PROFILED_RUN_STDOUT [UNPROFILED_BENCH_JSON]

bench.py's untimed one-slot kernel-timing pass is the `--stats-launches` (4) dispatches of each traversal
kernel right before the last one (the CPU-baseline parity re-render of one frame); the BDPT section launches
other kernels.  Prints the per-dispatch durations of that pass next to the avg_ms the JSON line reports."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import dispatches  # noqa: E402


def last_json(path):
    for line in reversed(open(path).read().strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def main():
    db, prof = sys.argv[1], sys.argv[2]
    plain = last_json(sys.argv[3]) if len(sys.argv) > 3 else None
    pj = last_json(prof)
    ds = dispatches(db)
    print("rocprofv3 --kernel-trace of the default `python3 bench.py` vs the HIP-event durations bench.py reports for the "
          "same run.  The one-slot kernel-timing pass (4 launches x 4 frames) is the 4 dispatches of each kernel before "
          "the last one (the single-frame parity re-render after the CPU baseline).")
    for k in ("k_shadow_extend", "k_primary", "k_shade0", "k_shadeN", "k_shadow"):
        ms = [d["ms"] for d in ds if d["kernel"].startswith(f"_Z{len(k)}{k}")]   # Itanium mangling: length + name
        tp = ms[-5:-1]
        avg = sum(tp) / len(tp)
        rep = pj["kernels"][k]["avg_ms"]
        line = (f"{k}: {len(ms)} dispatches; timing pass average {avg:.4f} ms ({', '.join(f'{x:.4f}' for x in tp)}); "
                f"bench.py avg_ms in the profiled run {rep:.4f} (ratio {avg / rep:.4f})")
        if plain:
            line += f"; unprofiled default run {plain['kernels'][k]['avg_ms']:.4f}"
        print(line)


if __name__ == "__main__":
    main()
