"""Per-kernel summary (count, total/avg/min ms, grid) of a rocprofv3 SQLite results file.
usage: python tools/prof_summary.py results.db [out.csv]"""
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    q = """select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.grid_size_x),
                  s.arch_vgpr_count, s.sgpr_count, s.group_segment_size
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by sum(d.end - d.start) desc"""
    rows = []
    for name, n, tot, mn, grid, vgpr, sgpr, lds in c.execute(q):
        rows.append((name.split("(")[0][:60], n, tot / 1e6, tot / n / 1e6, mn / 1e6, grid, vgpr, sgpr, lds))
    return rows


if __name__ == "__main__":
    rows = summary(sys.argv[1])
    hdr = "kernel,calls,total_ms,avg_ms,min_ms,max_grid_x,arch_vgpr,sgpr,lds_bytes"
    lines = [hdr] + [f"{r[0]},{r[1]},{r[2]:.4f},{r[3]:.4f},{r[4]:.4f},{r[5]},{r[6]},{r[7]},{r[8]}" for r in rows]
    print("\n".join(lines))
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write("\n".join(lines) + "\n")
