#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 --kernel-trace CSV (r6):
launch count, mean AND median duration, min, max.  The median is the figure
to set beside a bench line's ms_per_step: the mean of a profile of the bench
also averages the untimed replays (clock ramp, first launches), so it can sit
above the timed region's per-launch time.

usage: kernel_trace_summary.py <kernel_trace.csv> [<name substring> ...]"""
import csv
import statistics
import sys


def summarise(path, subs=()):
    by = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        by.setdefault(name, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        rows.append({"kernel": name.split("(")[0].replace("void ", ""), "launches": len(d),
                     "total_ms": round(sum(d) / 1e6, 3), "mean_ns": round(statistics.fmean(d), 1),
                     "median_ns": statistics.median(d), "min_ns": min(d), "max_ns": max(d)})
    return rows


if __name__ == "__main__":
    rows = summarise(sys.argv[1], sys.argv[2:])
    print(f"{'kernel':70s} {'launches':>8s} {'total_ms':>10s} {'mean_ns':>12s} {'median_ns':>12s} {'min_ns':>10s} {'max_ns':>10s}")
    for r in rows:
        print(f"{r['kernel'][:70]:70s} {r['launches']:8d} {r['total_ms']:10.3f} {r['mean_ns']:12.1f} "
              f"{r['median_ns']:12.1f} {r['min_ns']:10d} {r['max_ns']:10d}")
