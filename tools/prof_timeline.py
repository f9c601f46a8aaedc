"""Timeline of the last dispatches in a rocprofv3 SQLite results file: start offset, duration,
queue and the idle gap before each launch (where frames in flight overlap, and where the GPU
waits on the host).  Also prints the busy fraction of the window (union of kernel intervals).
usage: python tools/prof_timeline.py results.db [last_n]"""
import sqlite3
import sys


def dispatches(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
    qcol = "d.queue_id" if "queue_id" in cols else "0"
    q = f"""select s.kernel_name, d.start, d.end, {qcol}, d.grid_size_x
            from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
            order by d.start"""
    rows = [(n.split("(")[0].replace("_Z", "")[:32], st, en, qu, g) for n, st, en, qu, g in c.execute(q)]
    # memory copies (rocprofv3 --memory-copy-trace), merged into the timeline
    tables = {r[0] for r in c.execute("select name from sqlite_master where type = 'table'")}
    if "rocpd_memory_copy" in tables:
        mc = [r[1] for r in c.execute("pragma table_info(rocpd_memory_copy)")]
        size = "size" if "size" in mc else "0"
        for st, en, sz in c.execute(f"select start, end, {size} from rocpd_memory_copy"):
            rows.append(("memcpy", st, en, -1, sz))
        rows.sort(key=lambda r: r[1])
    return rows


def main():
    rows = dispatches(sys.argv[1])
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = rows[-last:]
    t0 = rows[0][1]
    busy_end = t0
    busy = 0
    for n, st, en, qu, g in rows:
        gap = max(0, st - busy_end)
        print(f"{(st - t0) / 1e3:9.1f} us  {(en - st) / 1e3:8.1f} us  gap {gap / 1e3:7.1f}  q{qu}  {n:32s} grid {g}")
        if en > busy_end:
            busy += en - max(st, busy_end)
            busy_end = en
    span = rows[-1][2] - t0
    print(f"window {span / 1e3:.1f} us, busy {busy / span * 100:.1f} %")


if __name__ == "__main__":
    main()
