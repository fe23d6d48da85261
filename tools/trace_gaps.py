"""Idle gaps between kernels inside one evaluation, from a rocprofv3
--kernel-trace CSV (usage: python tools/trace_gaps.py DIR)."""
import csv
import glob
import os
import sys
from collections import Counter

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r["Kind"] == "KERNEL_DISPATCH"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
rows.sort(key=lambda r: r["s"])
asm = [i for i, r in enumerate(rows) if "k_asm_mm" in r["n"]]
per = 2 if len(asm) >= 4 and rows[asm[-1]]["s"] - rows[asm[-2]]["e"] < 1e6 else 1  # split assembly
a, b = asm[-1 - 2 * per + 1] if per == 2 else asm[-2], asm[-1 - per + 1] if per == 2 else asm[-1]
ev = rows[a:b + 1]
iv = sorted((r["s"], r["e"], r["n"]) for r in ev)
gaps, tot = Counter(), Counter()
ce, prev = iv[0][1], iv[0][2]
idle = 0
for s, e, nm in iv[1:]:
    if s > ce:
        gaps[(prev, nm)] += 1
        tot[(prev, nm)] += s - ce
        idle += s - ce
    if e > ce:
        ce, prev = e, nm
print("eval span ms %.3f, idle ms %.3f" % ((rows[b]["s"] - rows[a]["s"]) / 1e6, idle / 1e6))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:8]:
    print(k, gaps[k], "%.1f us" % (v / 1e3))
ups = [r for r in ev if r["n"] == "ace::k_update"]
d = [ups[i + 1]["s"] - ups[i]["e"] for i in range(len(ups) - 1)]
print("update->update gaps: n %d mean %.1f us" % (len(d), sum(d) / len(d) / 1e3))
asm_e = max(r["e"] for r in ev if "k_asm_mm" in r["n"] and r["s"] < ups[0]["s"])
print("last assembly launch end -> first update start: %.1f us" % ((ups[0]["s"] - asm_e) / 1e3))
ch = [r for r in ev if r["n"] in ("ace::k_gather", "ace::k_pivot", "ace::k_panel", "ace::k_panel_gemm")
      and r["s"] < ups[0]["s"]]
if ch:
    print("first chain: %.1f us .. %.1f us after the first assembly start" %
          ((min(r["s"] for r in ch) - ev[0]["s"]) / 1e3, (max(r["e"] for r in ch) - ev[0]["s"]) / 1e3))
