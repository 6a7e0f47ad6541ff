#!/usr/bin/env python
"""Summarise rocprofv3 *_kernel_stats.csv files into a markdown table.

    python scripts/summarize_prof.py gpurun_out/prof/train_kernel_stats.csv [--top 30] [--div N]
--div divides totals by N (e.g. number of profiled steps) to give per-step ms.
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    ours = sum(float(r["TotalDurationNs"]) for r in rows if "rs::" in r["Name"])
    print(f"### {a.title or a.csv}\n")
    print(f"total kernel time {tot / 1e6 / a.div:.2f} ms per unit (div={a.div:g}); "
          f"hand-written rs:: kernels {100 * ours / tot:.1f}%\n")
    print("| ms/unit | % | calls/unit | avg us | kernel |\n|---:|---:|---:|---:|---|")
    for r in rows[:a.top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 120:
            name = name[:117] + "..."
        print(f"| {float(r['TotalDurationNs']) / 1e6 / a.div:.3f} | {float(r['Percentage']):.1f} | "
              f"{int(r['Calls']) / a.div:.0f} | {float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
