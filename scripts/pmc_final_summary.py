#!/usr/bin/env python3
"""Per-launch PMC summary of scripts/gpu_evidence_r04.sh output:
   python scripts/pmc_final_summary.py <evidence dir> <config>
Counter values are summed over a dispatch's rows, then the median over the
dispatches of each kernel; HBM bytes = FETCH_SIZE x 2 (gfx950 correction for
16-B-per-lane streams, MI355X_MICROARCH.md) + WRITE_SIZE, in KiB."""
import collections
import csv
import glob
import sys

root, cfg = sys.argv[1], sys.argv[2]
per = collections.defaultdict(float)
for f in sorted(glob.glob(f"{root}/pmc_{cfg}/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(k, r["Counter_Name"], f, r["Dispatch_Id"])] += float(r["Counter_Value"])
agg = collections.defaultdict(list)
for (k, c, _, _), v in per.items():
    agg[(k, c)].append(v)
med = {}
print(f"# rocprofv3 PMC (separate passes), bench.py --config {cfg} --no-warm --no-rebind --steps 20; median per launch")
for (k, c), v in sorted(agg.items()):
    v.sort()
    med[(k, c)] = v[len(v) // 2]
    print(f"{k[:60]:60s} {c:22s} {med[(k, c)]:14.1f}  (n={len(v)})")
for k in sorted({k for k, _ in med}):
    if "k_rows_ws" not in k:
        continue
    fs, ws = med.get((k, "FETCH_SIZE")), med.get((k, "WRITE_SIZE"))
    if fs is not None and ws is not None:
        rd, wr = 2 * fs * 1024 / 1e6, ws * 1024 / 1e6
        print(f"\n{k}: HBM bytes per launch = FETCH_SIZE x2 + WRITE_SIZE = {rd:.1f} + {wr:.1f} = {rd + wr:.1f} MB")
    wc = med.get((k, "SQ_WAVE_CYCLES"))
    if wc:
        print(f"{k}: wave time: SQ_WAIT_ANY {med[(k, 'SQ_WAIT_ANY')] / wc:.3f}, SQ_WAIT_INST_ANY "
              f"{med[(k, 'SQ_WAIT_INST_ANY')] / wc:.3f}, SQ_ACTIVE_INST_ANY {med[(k, 'SQ_ACTIVE_INST_ANY')] / wc:.3f}; "
              f"VALU instr {med[(k, 'SQ_ACTIVE_INST_VALU')]:.3g}, LDS instr {med[(k, 'SQ_ACTIVE_INST_LDS')]:.3g}")
