#!/usr/bin/env python3
"""Effective clock of each kernel from a rocprofv3 run with --pmc GRBM_GUI_ACTIVE
and --kernel-trace (MI355X_MICROARCH.md 'DVFS give-back': clock ~ GRBM_GUI_ACTIVE
/ 8 XCDs / kernel wall time; within 3 % of the in-kernel clock on dispatches of
10 ms or more, reads high below ~0.3 ms).  The bulk update launches (the
largest grid of k_update_multi) are reported on their own line.

usage: python tools/clock_pmc.py ROCPROF_DIR [min_ms]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
    grbm, name, grid = {}, {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            k = (os.path.dirname(f), int(row["Dispatch_Id"]))
            grbm[k] = grbm.get(k, 0.0) + float(row["Counter_Value"])
            name[k] = row["Kernel_Name"]
            grid[k] = int(row.get("Grid_Size", 0) or 0)
    dur = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = (os.path.dirname(f), int(row["Dispatch_Id"]))
            dur[k] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
    gmax = defaultdict(int)
    for k, n in name.items():
        gmax[n.split("(")[0]] = max(gmax[n.split("(")[0]], grid[k])
    agg = defaultdict(list)
    for k, g in grbm.items():
        if k not in dur or dur[k] * 1e3 < min_ms:
            continue
        short = name[k].split("(")[0]
        if short.endswith("k_update_multi<false>") and grid[k] == gmax[short]:
            short += "[bulk]"
        agg[short].append((dur[k], g / 8.0 / dur[k] / 1e9))
    print(f"{'kernel':60s} {'n':>4s} {'avg ms':>8s} {'GHz (GRBM_GUI_ACTIVE/8/wall)':>30s}")
    for short, v in sorted(agg.items(), key=lambda kv: -sum(x for x, _ in kv[1])):
        t = sum(x for x, _ in v)
        ghz = sum(x * c for x, c in v) / t
        print(f"{short[:60]:60s} {len(v):4d} {t / len(v) * 1e3:8.3f} {ghz:30.3f}")


if __name__ == "__main__":
    main()
