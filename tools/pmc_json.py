"""Builds profiles/pmc_latest.json (read by bench.py for roofline.traffic) from two rocprofv3
PMC passes of `bench.py` (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):

  rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f -- python3 bench.py ...
  rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w -- python3 bench.py ...
  python tools/pmc_json.py gpurun_out/pmc_fetch/f_results.db gpurun_out/pmc_write/w_results.db

Correction (MI355X_MICROARCH.md "HBM"): FETCH_SIZE counts 128-B memory-side read requests at
64 B, so it is doubled; WRITE_SIZE is taken as is.  Both are KB in rocprofv3.  Infinity-Cache
hits are counted as fetches by these L2 memory-side counters (same section), so the figure is
L2-miss traffic, an upper bound on HBM bytes.  Per kernel: median over its dispatches.
"""
import json
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import dispatches  # noqa: E402

# longest names first: "k_shadow" is a prefix of "k_shadow_extend"
KERNELS = ["k_shadow_extend", "k_primary", "k_extend", "k_shadow", "k_shade0", "k_shadeN", "k_accumulate",
           "k_bdpt_start", "k_bdpt_vertex", "k_bdpt_connect", "k_bdpt_vis", "k_bdpt_gather"]


def per_kernel(db, counter):
    out = {}
    for d in dispatches(db):
        name = next((k for k in KERNELS if k in d["kernel"]), None)
        if name is None or counter not in d["pmc"]:
            continue
        out.setdefault(name, []).append(d["pmc"][counter])
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (San-Miguel proxy 1080p, D=2)",
           "correction": "hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (MI355X_MICROARCH.md HBM section)",
           "kernels": {}}
    for k in KERNELS:
        if k in fetch and k in write:
            fb, wb = 2 * fetch[k] * 1024, write[k] * 1024
            res["kernels"][k] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                                 "fetch_size_kb_raw": fetch[k], "write_size_kb_raw": write[k]}
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                             "profiles", "pmc_latest.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
