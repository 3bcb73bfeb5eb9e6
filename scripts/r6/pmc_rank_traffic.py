#!/usr/bin/env python3
"""Fold scripts/r6/gpu_rank_pmc.sh's runs into profiles/pmc_traffic.json as
'<config>@p<p>r<r>': the median per-launch HBM bytes of rank r's tiled
kernel (2 x FETCH_SIZE + WRITE_SIZE, KiB -> B: the guide's gfx950 FETCH_SIZE
half-count correction, as scripts/pmc_traffic.py), the traffic bench.py
reports beside an N-GPU line for its slowest rank.  Copies the counter CSVs
to <keep>.

usage: pmc_rank_traffic.py <run dir (gpurun_out/r6_rankpmc)> <config> <keep dir>"""
import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys

run, config, keep = sys.argv[1:4]
os.makedirs(keep, exist_ok=True)
path = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "profiles",
                    "pmc_traffic.json")
db = json.load(open(path)) if os.path.exists(path) else {}
found = {}
for d in sorted(glob.glob(os.path.join(run, f"{config}_p*r*_*"))):
    m = re.search(r"_p(\d+)r(\d+)_(FETCH_SIZE|WRITE_SIZE)$", d)
    if not m or not os.path.isdir(d):
        continue
    p, r, ctr = int(m.group(1)), int(m.group(2)), m.group(3)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        vals, kname = [], None
        for row in csv.DictReader(open(f)):
            if "k_rows_ws" in row["Kernel_Name"] and row["Counter_Name"] == ctr:
                vals.append(float(row["Counter_Value"]))
                kname = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if vals:
            found.setdefault((p, r), {})[ctr] = (statistics.median(vals), len(vals), kname)
        shutil.copy(f, os.path.join(keep, f"{config}_p{p}r{r}_{ctr}_counter_collection.csv"))
for (p, r), v in sorted(found.items()):
    if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
        continue
    fs, n, kname = v["FETCH_SIZE"]
    ws, _, _ = v["WRITE_SIZE"]
    key = f"{config}@p{p}r{r}"
    db[key] = {"kernel": kname, "fetch_size_kib_median": fs, "write_size_kib_median": ws, "launches": n,
               "traffic_bytes_per_launch": round((2.0 * fs + ws) * 1024.0),
               "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)",
               "source": os.path.relpath(keep, os.path.dirname(os.path.dirname(path))) +
                         f" (bench.py --rank-plans {p} --rank-only {r})"}
    print(key, db[key]["traffic_bytes_per_launch"], kname)
json.dump(db, open(path, "w"), indent=1, sort_keys=True)
