#!/usr/bin/env python3
"""Fold a rocprofv3 FETCH_SIZE / WRITE_SIZE run (scripts/gpu_pmc.sh) into
profiles/pmc_traffic.json, the per-launch HBM traffic bench.py reports as
roofline.traffic.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE counts half the bytes of a 16-B/lane coalesced read -> doubled;
WRITE_SIZE is exact for 16-B/lane stores; both are in KiB.

usage: pmc_traffic.py <pmc_dir> <config> <kernel-substring> <profile-copy-dir>
"""
import csv
import glob
import json
import os
import shutil
import sys

pmc_dir, config, ksub, keep = sys.argv[1:5]
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
kname = None
for f in glob.glob(f"{pmc_dir}/*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if ksub in r["Kernel_Name"] and r["Counter_Name"] in vals:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            kname = r["Kernel_Name"].split("(")[0].replace("void ", "")
med = {k: sorted(v)[len(v) // 2] for k, v in vals.items()}
traffic = (2.0 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024.0
os.makedirs(keep, exist_ok=True)
for f in glob.glob(f"{pmc_dir}/*/pmc_counter_collection.csv"):
    shutil.copy(f, os.path.join(keep, os.path.basename(os.path.dirname(f)) + "_counter_collection.csv"))
path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
db = json.load(open(path)) if os.path.exists(path) else {}
db[config] = {"kernel": kname, "fetch_size_kib_median": med["FETCH_SIZE"],
              "write_size_kib_median": med["WRITE_SIZE"], "launches": len(vals["FETCH_SIZE"]),
              "traffic_bytes_per_launch": round(traffic),
              "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)",
              "source": os.path.relpath(keep, os.path.dirname(path) + "/..")}
json.dump(db, open(path, "w"), indent=1, sort_keys=True)
print(config, db[config])
