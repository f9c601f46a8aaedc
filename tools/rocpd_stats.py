"""Kernel statistics (rocprofv3 --stats equivalent) from a rocprofv3 --kernel-trace database:
one CSV row per kernel -- name, calls, total / average / min / max duration (us), share of the
total.  usage: python tools/rocpd_stats.py results.db > profiles/.../kernel_stats.csv"""
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    print("kernel,calls,total_us,avg_us,min_us,max_us,percent")
    for name, n, tot, avg, mn, mx in rows:
        short = name.split("(")[0].replace("void ", "")
        print(f"\"{short}\",{n},{tot / 1e3:.3f},{avg / 1e3:.3f},{mn / 1e3:.3f},{mx / 1e3:.3f},{100.0 * tot / total:.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
