"""Per-group timeline of the group-schedule sweep (any Z) of the last
evaluation in a rocprofv3 --kernel-trace CSV (usage: python tools/group_timeline.py DIR [NGROUPS]).

Bulk launches are the update launches (k_update_pair / k_update_multi /
k_update) with the largest grids.  For each group: bulk duration, the gap
to the next bulk launch, and every other kernel that started during it as
name:start-end (us from the bulk's start).
"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
nshow = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("ace::", "")
    r["g"] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
rows.sort(key=lambda r: r["s"])
asm = [i for i, r in enumerate(rows) if "k_asm_mm" in r["n"]]
last = asm[-1]
while last - 1 >= 0 and (last - 1 in asm or rows[last]["s"] - rows[last - 1]["e"] < 2e5):
    last -= 1
    if "k_grad" in rows[last]["n"]:
        last += 1
        break
ev = [r for r in rows[last:]]
upd = [r for r in ev if r["n"] in ("k_update_pair", "k_update_multi", "k_update")]
gmax = max(r["g"] for r in upd)
bulk = [r for r in upd if r["g"] > gmax // 4]
t0 = ev[0]["s"]
print("eval span %.3f ms, %d bulk launches, sum bulk %.3f ms, first bulk at %.3f ms" % (
    (ev[-1]["e"] - t0) / 1e6, len(bulk), sum(r["e"] - r["s"] for r in bulk) / 1e6,
    (bulk[0]["s"] - t0) / 1e6))
pre = [r for r in ev if r["e"] <= bulk[0]["s"] and "k_asm" not in r["n"]]
asm_end = max(r["e"] for r in ev if "k_asm_mm" in r["n"])
print("assembly end %.3f ms; before the first bulk: %s" % (
    (asm_end - t0) / 1e6,
    " ".join("%s:%.0f-%.0f" % (r["n"].replace("k_", ""), (r["s"] - t0) / 1e3, (r["e"] - t0) / 1e3)
             for r in pre)))
tot = 0.0
for i, b in enumerate(bulk):
    nxt = bulk[i + 1]["s"] if i + 1 < len(bulk) else None
    side = [r for r in ev if r is not b and r["s"] >= b["s"] - 1000 and r["s"] < (nxt or b["e"])
            and "k_grad" not in r["n"]]
    last_side = max((r["e"] for r in side), default=b["s"])
    gap = (nxt - b["e"]) / 1e3 if nxt else 0.0
    tot += gap
    if i < nshow or i >= len(bulk) - 2:
        print("g%02d bulk %7.1f us  gap %6.1f us  side end %+7.1f us vs bulk end" % (
            i, (b["e"] - b["s"]) / 1e3, gap, (last_side - b["e"]) / 1e3))
        print("     " + " ".join("%s:%.0f-%.0f" % (r["n"].replace("k_", "").replace("update_", "u"),
                                                  (r["s"] - b["s"]) / 1e3, (r["e"] - b["s"]) / 1e3)
                                 for r in side))
print("sum of gaps between bulk launches %.3f ms" % (tot / 1e3))
