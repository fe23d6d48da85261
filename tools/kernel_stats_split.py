"""rocprofv3 kernel stats with the two-step update kernel split by role.

k_update_multi (round 3; k_update_pair before) runs as the bulk sweep update
(every lower tile: the largest grid) and as the side stream's lookahead cross
(a few hundred tiles), so its --stats line averages two different launch
sizes.  This recomputes the per-kernel summary from the --kernel-trace CSV
with the bulk launches on their own line (`k_update_multi[bulk]`), which is
the launch the bench's roofline times with HIP events.

usage: python tools/kernel_stats_split.py DIR > profiles/rNN_kernel_stats_split.csv
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
    split = {"k_update_multi<false>(": "ace::k_update_multi", "k_update_pair(": "ace::k_update_pair"}
    gmax = {key: max((int(r["Grid_Size_X"]) for r in rows if key in r["Kernel_Name"]), default=0)
            for key in split}
    dur = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        for key, short in split.items():
            if key in name:
                name = short + ("[bulk]" if int(r["Grid_Size_X"]) == gmax[key] else "[cross]")
        dur[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    total = sum(sum(v) for v in dur.values())
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total, min(v), max(v)])


if __name__ == "__main__":
    main()
