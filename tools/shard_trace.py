"""Where one evaluation's time goes, from a rocprofv3 --kernel-trace CSV:
per-kernel time per evaluation and the idle gaps (no kernel running) in the
last evaluation's span (first assembly launch to the last k_final_sums).
usage: python tools/shard_trace.py DIR [NGAPS]  (NGAPS: list the largest idle gaps)"""
import csv
import glob
import os
import sys
from collections import defaultdict

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
rows.sort(key=lambda r: r["s"])
fin = [i for i, r in enumerate(rows) if "k_final_sums" in r["n"]]
# the last evaluation: after the previous k_final_sums
a = fin[-2] + 1 if len(fin) >= 2 else 0
b = fin[-1]
ev = rows[a:b + 1]
t = defaultdict(float)
cnt = defaultdict(int)
for r in ev:
    t[r["n"]] += (r["e"] - r["s"]) / 1e6
    cnt[r["n"]] += 1
span = (ev[-1]["e"] - ev[0]["s"]) / 1e6
busy_end, idle, gaps, last = ev[0]["e"], 0.0, [], ev[0]
for r in ev[1:]:
    if r["s"] > busy_end:
        idle += (r["s"] - busy_end) / 1e6
        gaps.append(((r["s"] - busy_end) / 1e6, last["n"], r["n"], (busy_end - ev[0]["s"]) / 1e6))
    if r["e"] > busy_end:
        busy_end, last = r["e"], r

print(f"last evaluation span {span:.3f} ms, idle {idle:.3f} ms, {len(ev)} launches")
for n, v in sorted(t.items(), key=lambda kv: -kv[1]):
    print(f"  {n:28s} {cnt[n]:5d} launches {v:9.3f} ms")
ng = int(sys.argv[2]) if len(sys.argv) > 2 else 0
for g, x, y, at in sorted(gaps, reverse=True)[:ng]:
    print(f"  gap {g * 1e3:7.1f} us at {at:7.3f} ms: {x} -> {y}")
