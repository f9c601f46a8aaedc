"""Builds profiles/pmc_latest.json (read by bench.py: roofline.traffic and roofline.limiter) from
rocprofv3 PMC passes of one bench.py command (tools/r2_gpu2.sh runs them, each pass in its own
process because FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):

  python tools/pmc_json.py DIR_WITH_RESULTS_DBS "bench command" [launches] [pass_dir_prefix (default pmc_)]
                           [output (default profiles/pmc_latest.json)] [description of those launches]

Per kernel the figures are the MEDIAN over the kernel's last `launches` dispatches.  Round 3: the
passes profile `bench.py --no-kernel-timing ...`, so the last dispatch of each PT kernel IS the
timed render_frames call (20 frames packed into one launch per kernel) and launches = 1.

Bytes (MI355X_MICROARCH.md "HBM" + profiles/r03/fetch_size_calibration.json): FETCH_SIZE counts a
128-B memory-side read request of a coalesced 16-B/lane stream at 64 B (the guide: double it), but
a 64-B random gather -- the traversal's node fetch -- exactly (calibrated here: FETCH_SIZE x 1024 =
64 B x TCC_MISS to 0.1 % on the dependent-gather probe at HBM and Infinity-Cache residency).  So
the JSON keeps the raw figure (fetch_bytes_raw = FETCH_SIZE x 1024, exact for the gathers) and
the streaming-rule upper bound (2x); bench.py adds back the unreported half of the launch's known
streamed reads (ray records).  WRITE_SIZE is exact for 16-B stores and float atomics.  These
L2-to-fabric counters also count Infinity-Cache hits: the figure is bytes beyond L2.
Limiter (SQ block, per dispatch; SQ_WAVE_CYCLES / WAIT_* / ACTIVE_INST_* in the same unit, so
their ratios are unit-free): share of wave time waiting on memory (SQ_WAIT_ANY), stalled at issue
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY); VALU pipe busy = SQ_INSTS_VALU x 2 cycles
(a wave64 VALU op occupies a SIMD32 for 2 cycles) / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).
"""
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import dispatches  # noqa: E402

# longest names first: "k_shadow" is a prefix of "k_shadow_extend"
KERNELS = ["k_shadow_extend", "k_walk_resume", "k_primary", "k_extend", "k_shadow", "k_shade0", "k_shadeN", "k_accumulate",
           "k_bdpt_start", "k_bdpt_vertex", "k_bdpt_connect", "k_bdpt_vis", "k_bdpt_gather"]


def collect(dbs, last, keep=12):
    """kernel -> counter -> median over the kernel's last `last` dispatches (per pass db); also the
    raw values of the last `keep` dispatches per counter (consumers that sum a frame's launches)."""
    out, ms, raw = {}, {}, {}
    for db in dbs:
        per = {}
        for d in dispatches(db):
            name = next((k for k in KERNELS if "_Z" in d["kernel"] and k in d["kernel"].split("ILb")[0] or
                         d["kernel"].endswith(k)), None)
            name = name or next((k for k in KERNELS if k in d["kernel"]), None)
            if name is None:
                continue
            per.setdefault(name, []).append(d)
        for name, ds in per.items():
            for c in ds[0]["pmc"]:
                raw.setdefault(name, {})[c] = [x["pmc"][c] for x in ds[-keep:]]
            ds = ds[-last:]
            for c in ds[0]["pmc"]:
                out.setdefault(name, {})[c] = statistics.median(x["pmc"][c] for x in ds)
            ms.setdefault(name, []).extend(x["ms"] for x in ds)
    return out, {k: statistics.median(v) for k, v in ms.items()}, raw


def main():
    d = sys.argv[1]
    cmd = sys.argv[2] if len(sys.argv) > 2 else "bench.py"
    last = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    prefix = sys.argv[4] if len(sys.argv) > 4 else "pmc_"
    dbs = sorted(glob.glob(os.path.join(d, prefix + "*", "*_results.db")))
    pmc, ms, raw = collect(dbs, last)
    res = {"source": f"rocprofv3 --kernel-trace --pmc passes ({', '.join(os.path.basename(os.path.dirname(x)) for x in dbs)})",
           "config": f"{cmd}; medians over the last {last} dispatch(es) of each kernel = " +
                     (sys.argv[6] if len(sys.argv) > 6 else "the timed render_frames call (one launch per kernel)"),
           "correction": ("fetch_bytes_raw = FETCH_SIZE x 1024 (exact for 64-B gathers, half of coalesced 16-B/lane "
                          "streams: profiles/r03/fetch_size_calibration.json); fetch_bytes_stream_rule = 2 x raw "
                          "(upper bound); write_bytes = WRITE_SIZE x 1024"),
           "kernels": {}}
    for k, c in pmc.items():
        r = {"dispatch_ms_median": round(ms[k], 4), "counters": {n: v for n, v in sorted(c.items())},
             "last_dispatches": {n: raw[k][n] for n in ("FETCH_SIZE", "WRITE_SIZE") if n in raw.get(k, {})}}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            fb, wb = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
            r.update(fetch_bytes_raw=fb, fetch_bytes_stream_rule=2 * fb, write_bytes=wb,
                     memory_side_bytes_bounds=[fb + wb, 2 * fb + wb])
        if all(x in c for x in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")):
            wc = c["SQ_WAVE_CYCLES"]
            cyc = c["GRBM_GUI_ACTIVE"] / 8.0
            lim = {"wave_time_waiting_on_memory": round(c["SQ_WAIT_ANY"] / wc, 3),
                   "wave_time_issue_stalled": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
                   "valu_busy": round(c["SQ_INSTS_VALU"] * 2 / (1024 * cyc), 3),
                   "clock_ghz": round(cyc / (ms[k] * 1e-3) / 1e9, 3)}
            if "SQ_INSTS_SALU" in c:   # one scalar unit per CU issues one SALU instruction per cycle
                lim["salu_busy"] = round(c["SQ_INSTS_SALU"] / (256 * cyc), 3)
            if "SQ_ACTIVE_INST_ANY" in c:
                lim["wave_time_issuing"] = round(c["SQ_ACTIVE_INST_ANY"] / wc, 3)
            if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
                lim["l2_hit_rate"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 3)
            if "memory_side_bytes_bounds" in r:
                lim["memory_side_tb_s_bounds"] = [round(x / (ms[k] * 1e-3) / 1e12, 3) for x in r["memory_side_bytes_bounds"]]
            if "TA_TA_BUSY_sum" in c:   # vector-memory address path, per CU (256 CUs)
                lim["ta_busy"] = round(c["TA_TA_BUSY_sum"] / (256 * cyc), 3)
                if "TA_ADDR_STALLED_BY_TC_CYCLES_sum" in c:
                    lim["ta_stalled_by_tcp"] = round(c["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / (256 * cyc), 3)
            if "TCP_TCC_READ_REQ_sum" in c and c["TCP_TCC_READ_REQ_sum"] > 0:
                lim["l1_miss_latency_cycles"] = round(c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"], 1)
                lim["l1_hit_rate"] = round(1 - c["TCP_TCC_READ_REQ_sum"] / max(c["TCP_TOTAL_CACHE_ACCESSES_sum"], 1), 3)
            mem, iss = lim["wave_time_waiting_on_memory"], lim["wave_time_issue_stalled"]
            bw = lim.get("memory_side_tb_s_bounds", [0.0, 0.0])[1]
            lim["binding"] = ("HBM bandwidth" if bw >= 5.0 else
                              "dependent-fetch latency, scalar unit busy (wave packets)" if lim.get("salu_busy", 0.0) >= 0.7 else
                              "vector-memory pipeline (TA busy) + memory latency"
                              if lim.get("ta_busy", 0.0) >= 0.85 and mem >= 0.4 else
                              "memory latency" if mem >= 0.4 and lim["valu_busy"] < 0.6 else
                              "VALU issue" if lim["valu_busy"] >= 0.6 else "mixed")
            r["limiter"] = lim
        res["kernels"][k] = r
    out = sys.argv[5] if len(sys.argv) > 5 else \
        os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_latest.json")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v.get("limiter") for k, v in res["kernels"].items()}, indent=1))


if __name__ == "__main__":
    main()
