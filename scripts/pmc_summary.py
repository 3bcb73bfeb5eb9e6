#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc output dirs: median counter value per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if filt and filt not in k:
            continue
        short = k.split("(")[0].replace("void ", "")
        agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
        dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (k, c), v in sorted(agg.items()):
    v.sort()
    print(f"{k[:40]:40s} {c:40s} {v[len(v) // 2]:.6g}")
for k, v in dur.items():
    v.sort()
    print(f"{k[:40]:40s} {'duration_us(median)':40s} {v[len(v) // 2]:.2f}")
