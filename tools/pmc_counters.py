"""Per-launch PMC counters of the bench's kernels from rocprofv3 --pmc passes
(any counters; one directory per pass), with the bulk update launches
(k_update_multi, the largest grid) on their own line.

usage: python tools/pmc_counters.py DIR [DIR ...] > profiles/rNN_pmc_counters.json

For every kernel and counter: launches, the mean per launch of the summed
counter, and the mean per launch of each counter instance (rocprofv3 writes
one row per hardware instance, e.g. per TCC channel / XCD, in a fixed order),
so L2 hit / miss can be attributed per instance."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {
    "k_update_multi": "ace::k_update_multi<false>(",
    "k_update_q": "ace::k_update_q(",
    "k_panel_gemm_t": "ace::k_panel_gemm_t(",
    "k_asm_mm": "ace::k_asm_mm<",
    "k_grad_mm": "ace::k_grad_mm<",
    "k_gather": "ace::k_gather<",
}


def collect(dirs):
    rows = defaultdict(lambda: defaultdict(list))  # (kernel, dispatch) -> counter -> [instances]
    grid = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    for short, key in KERNELS.items():
                        if key in row["Kernel_Name"]:
                            k = (short, f, int(row["Dispatch_Id"]))
                            rows[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                            grid[k] = int(row.get("Grid_Size", 0) or 0)
    return rows, grid


def summarize(rows, grid):
    out = defaultdict(lambda: defaultdict(list))
    gmax = defaultdict(int)
    for (short, f, d), g in grid.items():
        gmax[short] = max(gmax[short], g)
    for k, cnts in rows.items():
        short = k[0]
        names = [short]
        if short == "k_update_multi":
            names = ["k_update_multi_bulk" if grid[k] == gmax[short] else "k_update_multi_side"]
        for nm in names:
            for c, inst in cnts.items():
                out[nm][c].append(inst)
    res = {}
    for nm, cnts in out.items():
        res[nm] = {}
        for c, launches in cnts.items():
            n = len(launches)
            width = max(len(x) for x in launches)
            per_inst = [sum(x[i] for x in launches if i < len(x)) / n for i in range(width)]
            res[nm][c] = {"launches": n, "mean_per_launch": sum(sum(x) for x in launches) / n,
                          "instances": width, "mean_per_instance": per_inst}
    return res


if __name__ == "__main__":
    r, g = collect(sys.argv[1:])
    json.dump({"source": "rocprofv3 --pmc (one pass per directory)", "kernels": summarize(r, g)},
              sys.stdout, indent=1)
