"""Do kernels of different streams overlap?  From a rocprofv3 --kernel-trace database: the last
--last dispatches with their queue / stream, start and end (µs, relative), and over them the sum of
kernel durations against the union of their intervals (sum > union <=> concurrent kernels).
usage: python tools/kernel_overlap.py results.db [--last 60]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=60)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
    qcol = "d.queue_id" if "queue_id" in cols else "0"
    scol = "d.stream_id" if "stream_id" in cols else "0"
    q = f"""select s.kernel_name, {qcol}, {scol}, d.start, d.end, d.grid_size_x
            from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""
    rows = [(n.split("(")[0].split("<")[0].replace("void ", ""), qi, si, st, en, g) for n, qi, si, st, en, g in c.execute(q)]
    rows = rows[-a.last:]
    t0 = rows[0][3]
    for n, qi, si, st, en, g in rows:
        print(f"{n[:22]:22s} q{qi} s{si} {(st - t0) / 1e3:10.1f} {(en - t0) / 1e3:10.1f}  {(en - st) / 1e3:8.1f} us  grid {g}")
    tot = sum(en - st for _, _, _, st, en, _ in rows)
    union, cur_s, cur_e = 0, None, None
    for _, _, _, st, en, _ in sorted(rows, key=lambda r: r[3]):
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
    union += cur_e - cur_s
    span = max(r[4] for r in rows) - t0
    print(f"sum of kernel time {tot / 1e3:.1f} us, union {union / 1e3:.1f} us, span {span / 1e3:.1f} us, "
          f"overlap {(tot - union) / 1e3:.1f} us, idle {(span - union) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
