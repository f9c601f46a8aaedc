"""Per-phase kernel durations from a rocprofv3 --kernel-trace CSV (<name>_kernel_trace.csv) of
bench.py: the LAST `k` dispatches of a kernel are the untimed one-slot kernel-timing pass whose
HIP-event average bench.py divides roofline.achieved by; prints all-dispatch and last-k averages so
the two can be compared.  skip = dispatches after the pass (bench.py's parity spot-check frame
renders one more k_shadow_extend / k_primary launch after it).
usage: python tools/prof_phase.py kernel_trace.csv KERNEL_SUBSTRING k [skip]"""
import csv
import sys


def durations(path, sub):
    out = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if sub in row["Kernel_Name"]:
                out.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
    return [d for _, d in sorted(out)]


if __name__ == "__main__":
    path, sub, k = sys.argv[1], sys.argv[2], int(sys.argv[3])
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    d = durations(path, sub)
    last = d[len(d) - skip - k:len(d) - skip]
    print(f"{sub}: {len(d)} dispatches, average {sum(d) / len(d):.4f} ms; last {k} (one-slot timing pass) "
          f"average {sum(last) / len(last):.4f} ms: " + ", ".join(f"{x:.4f}" for x in last))
