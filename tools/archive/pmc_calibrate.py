"""FETCH_SIZE calibration for the traversal's access pattern.

MI355X_MICROARCH.md calibrates FETCH_SIZE only for coalesced 16-B/lane streaming reads (it reports
half their bytes) and calls other widths uncalibrated.  The traversal gathers one 64-B record per
lane per step as four dependent-free 16-B loads at a random address -- exactly the access pattern
of the dependent-gather probe (mcrt_ctx_gather_chase, mcrt_kernels.hip k_chase): 32 waves per CU,
every lane following its own chain of uniformly random records.  With the record array far larger
than every cache (the HBM case) nearly every step misses L2, so the memory-side demand is known:
one 64-B record per step.  This program runs the probe at L2 (2 MiB), Infinity-Cache (122 MiB)
and HBM (the 10 M-triangle tree's 1.28 GB) residency; run it under rocprofv3 --pmc passes and
summarise with `python tools/pmc_calibrate.py --summarise DIR`.

Result (profiles/r03/fetch_size_calibration.json, MI355X round 3): FETCH_SIZE x 1024 = 64 B x
TCC_MISS to 0.1 % at Infinity-Cache and HBM residency, i.e. a 64-B random gather is counted at
its full size (the streaming rule halves only 128-B requests), and L2 misses served by the
Infinity Cache are counted too.  The demand/fetch ratio is NOT 1 even at HBM residency because
random chains merge (a random functional graph): 19 % of the steps hit L2 there.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monte-carlo-raytracer_amd"), os.path.join(ROOT, "tools")]

CASES = [("l2_2MiB", 32768), ("infinity_cache_122MiB", 2_000_000), ("hbm_1.28GB", 19_969_571)]
STEPS, ITERS = 256, 2


def run():
    import torch
    torch.cuda.init()
    from mcrt import lib
    ctx = lib.Context(0)
    out = {}
    for name, recs in CASES:
        out[name] = ctx.gather_chase_gsteps(recs, STEPS, ITERS)
    print(json.dumps({"gsteps": out, "waves": None}), flush=True)
    ctx.close()


def summarise(d):
    from pmc_summary import dispatches
    res = {"pattern": "one random 64-B record per lane per step as four 16-B loads (k_chase, 32 waves/CU)",
           "cases": {}}
    dbs = sorted(glob.glob(os.path.join(d, "*", "*_results.db")))
    per = {}
    for db in dbs:
        ks = [x for x in dispatches(db) if "k_chase" in x["kernel"] and "init" not in x["kernel"]]
        for x in ks:
            per.setdefault(x["grid"], [])
        # launches per case: 1 warm-up (STEPS / 4 steps) + ITERS timed, in CASES order
        per_case = len(ks) // len(CASES)
        for i, (name, recs) in enumerate(CASES):
            timed = ks[i * per_case + 1:(i + 1) * per_case]
            c = res["cases"].setdefault(name, {"records": recs})
            for x in timed:
                for k, v in x["pmc"].items():
                    c.setdefault(k, []).append(v)
                c.setdefault("grid", x["grid"])
                c.setdefault("ms", []).append(x["ms"])
    for name, c in res["cases"].items():
        lanes = c["grid"]   # one lane per chain (grid_size_x = waves x 64)
        demand = lanes * STEPS * 64
        c["steps_per_dispatch"] = lanes * STEPS
        c["demand_bytes"] = demand
        for k in list(c):
            if isinstance(c[k], list) and k not in ("ms",):
                c[k] = sum(c[k]) / len(c[k])
        c["ms"] = min(c["ms"])
        if "FETCH_SIZE" in c:
            c["fetch_bytes_reported"] = c["FETCH_SIZE"] * 1024
            c["factor_demand_over_fetch"] = round(demand / max(c["fetch_bytes_reported"], 1), 4)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            c["l2_hit_rate"] = round(c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1), 4)
            c["l2_misses_per_step"] = round(c["TCC_MISS_sum"] / c["steps_per_dispatch"], 4)
    for c in res["cases"].values():
        if "FETCH_SIZE" in c and "TCC_MISS_sum" in c:
            c["fetch_bytes_per_l2_miss"] = round(c["FETCH_SIZE"] * 1024 / max(c["TCC_MISS_sum"], 1), 3)
    hbm = res["cases"].get("hbm_1.28GB", {})
    if "fetch_bytes_per_l2_miss" in hbm:
        res["factor"] = round(64.0 / hbm["fetch_bytes_per_l2_miss"], 4)
        res["rule"] = ("64-B random gathers: memory-side bytes = FETCH_SIZE x 1024 x factor (factor = 64 B per L2 miss / "
                       "reported bytes per L2 miss, HBM residency); coalesced 16-B/lane streams keep the guide's x2")
    out = os.path.join(ROOT, "profiles", "r03", "fetch_size_calibration.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--summarise":
        summarise(sys.argv[2])
    else:
        run()
