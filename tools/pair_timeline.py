"""Per-group timeline of the pair-step sweep of one evaluation, from a
rocprofv3 --kernel-trace CSV (usage: python tools/pair_timeline.py DIR).

Bulk launches are the k_update_pair dispatches with the largest grids; for
each group: bulk duration, the gap to the next bulk launch (~17 us when the
bulk is the critical path, more when the next group's panels were late), and
the side kernels that ran during it.
"""
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if r.get("Kind", "KERNEL_DISPATCH") == "KERNEL_DISPATCH"]
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("ace::", "")
    r["g"] = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
rows.sort(key=lambda r: r["s"])
asm = [i for i, r in enumerate(rows) if "k_asm_mm" in r["n"]]
grd = [i for i, r in enumerate(rows) if "k_grad" in r["n"] or "grad" in r["n"]]
# the last evaluation: from the last assembly launch group to the end
last_asm = asm[-1]
first_asm = last_asm
while first_asm - 1 in asm or (first_asm - 2 in asm and rows[first_asm]["s"] - rows[first_asm - 2]["e"] < 1e6):
    first_asm -= 1 if first_asm - 1 in asm else 2
ev = [r for r in rows if r["s"] >= rows[first_asm]["s"]]
pairs = [r for r in ev if r["n"] == "k_update_pair"]
gmax = max(r["g"] for r in pairs)
bulk = [r for r in pairs if r["g"] > gmax // 8]
print("eval span %.3f ms, %d bulk launches, sum bulk %.3f ms" % (
    (ev[-1]["e"] - ev[0]["s"]) / 1e6, len(bulk), sum(r["e"] - r["s"] for r in bulk) / 1e6))
asm_end = max(r["e"] for r in ev if "k_asm_mm" in r["n"])
print("assembly end -> first bulk start %.1f us" % ((bulk[0]["s"] - asm_end) / 1e3))
gaps = []
for i, b in enumerate(bulk):
    nxt = bulk[i + 1]["s"] if i + 1 < len(bulk) else None
    side = [r for r in ev if r is not b and r["s"] >= b["s"] - 1000 and r["s"] < (nxt or b["e"])]
    last_side = max((r["e"] for r in side), default=b["s"])
    gap = (nxt - b["e"]) / 1e3 if nxt else float("nan")
    gaps.append(gap)
    print("g%02d bulk %7.1f us  gap %6.1f us  side end %+7.1f us vs bulk end  [%s]" % (
        i, (b["e"] - b["s"]) / 1e3, gap, (last_side - b["e"]) / 1e3,
        " ".join("%s:%.0f" % (r["n"].replace("k_", ""), (r["e"] - r["s"]) / 1e3) for r in side)))
g = [x for x in gaps[:-1]]
print("mean gap %.1f us, sum gaps %.3f ms" % (sum(g) / len(g), sum(g) / 1e3))
after = [r for r in ev if r["s"] > bulk[-1]["e"]]
print("after last bulk: %.1f us in %d kernels: %s" % (
    (ev[-1]["e"] - bulk[-1]["e"]) / 1e3, len(after),
    " ".join("%s:%.0f" % (r["n"].replace("k_", ""), (r["e"] - r["s"]) / 1e3) for r in after)))
