"""Gaps between consecutive bulk launches (k_update_multi longer than 2 ms)
of the last evaluation in a rocprofv3 kernel trace: the main stream's
per-boundary cost (packets between the launches).
  python tools/bulk_gaps.py <trace dir>"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").replace("ace::", "")
rows.sort(key=lambda r: r["s"])
fin = [i for i, r in enumerate(rows) if "k_final_sums" in r["n"]]
ev = rows[fin[-2] + 1:fin[-1] + 1]
bulk = [r for r in ev if r["n"] == "k_update_multi" and r["e"] - r["s"] > 2e6]
gaps = [(y["s"] - x["e"]) / 1e3 for x, y in zip(bulk, bulk[1:])]
print("bulk launches %d, gaps (us): %s" % (len(bulk), " ".join("%.1f" % g for g in gaps)))
print("sum %.1f us, mean %.1f us" % (sum(gaps), sum(gaps) / max(1, len(gaps))))
