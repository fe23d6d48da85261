"""Launch sequence of the last evaluation in a rocprofv3 --kernel-trace CSV:
start / end (us from the evaluation's first launch), duration, kernel, grid.
usage: python tools/chain_timeline.py DIR [max_lines]"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ace::", "")
rows.sort(key=lambda r: r["s"])
aug = [i for i, r in enumerate(rows) if "k_aug_init" in r["n"]]
grad = [i for i, r in enumerate(rows) if "k_grad_mm" in r["n"]]
a = aug[-1]
b = max(i for i in grad if i > a)
t0 = rows[a]["s"]
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 400
print(f"evaluation span {(rows[b]['e'] - t0) / 1e3:.1f} us, {b - a + 1} launches")
for r in rows[a:b + 1][:lim]:
    print(f"{(r['s'] - t0) / 1e3:9.1f} {(r['e'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f}  "
          f"{r['n'][:40]:40s} {r.get('Grid_Size', r.get('Grid_Size_X', ''))}")
