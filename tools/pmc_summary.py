"""Per-dispatch PMC values from a rocprofv3 SQLite results file (kernel, grid, duration, counters).
usage: python tools/pmc_summary.py results.db [kernel-substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def dispatches(db):
    c = sqlite3.connect(db)
    q = """select d.id, d.event_id, s.kernel_name, d.grid_size_x, d.end - d.start
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""
    rows = {}
    for did, eid, name, grid, dur in c.execute(q):
        rows[eid] = {"kernel": name.split("(")[0], "grid": grid, "ms": dur / 1e6, "pmc": defaultdict(float)}
    q = """select e.event_id, p.name, e.value from rocpd_pmc_event e join rocpd_info_pmc p on e.pmc_id = p.id"""
    for eid, name, val in c.execute(q):
        if eid in rows:
            rows[eid]["pmc"][name] += val
    return list(rows.values())


if __name__ == "__main__":
    filt = sys.argv[2:]
    for r in dispatches(sys.argv[1]):
        if filt and not any(f in r["kernel"] for f in filt):
            continue
        p = r["pmc"]
        print(f"{r['kernel'][:40]:40s} grid {r['grid']:8d} {r['ms']:7.3f} ms  " +
              " ".join(f"{k.replace('SQ_', '')}={v:.3g}" for k, v in sorted(p.items())))
