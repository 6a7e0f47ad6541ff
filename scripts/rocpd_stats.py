"""Per-kernel statistics CSV from a rocprofv3 rocpd database (the default
output of `rocprofv3 --kernel-trace` on this image): Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs -- the columns of
rocprofv3's kernel_stats.csv.

    python scripts/rocpd_stats.py gpurun_out/x/k_results.db > profiles/x.csv
"""
import csv
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), min(end - start), max(end - start) "
                     f"from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, k, s, lo, hi in rows:
        w.writerow([n, k, s, round(s / k, 3), round(100.0 * s / tot, 4), lo, hi])


if __name__ == "__main__":
    main(sys.argv[1])
