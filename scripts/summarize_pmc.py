#!/usr/bin/env python
"""Sum rocprofv3 counter_collection.csv files per kernel: python scripts/summarize_pmc.py DIR [TAG]"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
tag = sys.argv[2] if len(sys.argv) > 2 else ""
tot = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, f"{tag}*.csv"))):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "?")[:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add((f, r.get("Dispatch_Id")))
for k, c in tot.items():
    n = len({x[1] for x in disp[k]}) or 1
    print(k, f"dispatches~{n}")
    for name, v in sorted(c.items()):
        print(f"   {name:28s} {v:14.4g}")
