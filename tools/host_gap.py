"""The host side of the gap between two evaluations, from one rocprofv3 run
with --kernel-trace and --hip-trace: every HIP API call (and its duration)
between the end of the next-to-last evaluation's k_final_sums and the first
k_asm_mm launch of the last evaluation, and the host time not spent in any
HIP call.  usage: python tools/host_gap.py DIR"""
import csv
import glob
import os
import sys


def load(pat):
    f = glob.glob(os.path.join(sys.argv[1], "**", pat), recursive=True)[0]
    return list(csv.DictReader(open(f)))


ker = load("*kernel_trace.csv")
api = load("*hip_api_trace.csv")
for r in ker + api:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
fin = sorted(r["e"] for r in ker if "k_final_sums" in r["Kernel_Name"])
asm = sorted(r["s"] for r in ker if "k_asm_mm" in r["Kernel_Name"])
t0 = fin[-2]
t1 = min(s for s in asm if s > t0)
print(f"gap: k_final_sums end -> next k_asm_mm start = {(t1 - t0) / 1e3:.1f} us")
calls = sorted((r for r in api if r["e"] > t0 and r["s"] < t1), key=lambda r: r["s"])
inside, prev = 0.0, t0
for r in calls:
    s, e = max(r["s"], t0), min(r["e"], t1)
    print(f"  +{(s - t0) / 1e3:8.1f} us  {r['Function']:32s} {(e - s) / 1e3:8.1f} us  (host idle before: {max(0, s - prev) / 1e3:.1f})")
    inside += (e - s) / 1e3
    prev = max(prev, e)
print(f"in HIP calls {inside:.1f} us, outside {(t1 - t0) / 1e3 - inside:.1f} us")
