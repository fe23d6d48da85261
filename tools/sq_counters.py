"""Per-kernel averages of rocprofv3 SQ counter passes (diagnostics for the
pair kernels).  Usage: python tools/sq_counters.py DIR [DIR ...] where each DIR
holds one `rocprofv3 --pmc ... --output-format csv` pass."""
import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = ("k_grad_mm", "k_asm_mm", "k_grad2", "k_assembly", "k_update(", "k_update_x", "k_update_multi")


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    for k in KERNELS:
                        if "ace::" + k in row["Kernel_Name"]:
                            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in vals.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"  {c:32s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
