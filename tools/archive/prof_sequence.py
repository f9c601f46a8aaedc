"""Dispatch-ordered kernel durations of a rocprofv3 SQLite results file (one frame's launch
sequence, e.g. the per-depth k_extend launches of a BDPT frame).
usage: python tools/prof_sequence.py results.db [last_n]"""
import sqlite3
import sys


def sequence(db):
    c = sqlite3.connect(db)
    q = """select s.kernel_name, d.end - d.start, d.grid_size_x
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           order by d.start"""
    return [(n.split("(")[0][:40], dt / 1e6, g) for n, dt, g in c.execute(q)]


if __name__ == "__main__":
    rows = sequence(sys.argv[1])
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    for n, ms, g in rows[-last:]:
        print(f"{n:40s} {ms:8.4f} ms  grid {g}")
