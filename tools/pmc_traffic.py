"""Per-launch HBM traffic of the bench's dominant kernel from rocprofv3 PMC passes.

Usage (on the GPU box, two separate passes -- FETCH_SIZE and WRITE_SIZE do not
fit one pass on gfx950, MI355X_MICROARCH.md "TCC" row):
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f -o run -- python3 bench.py ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w -o run -- python3 bench.py ...
  python tools/pmc_traffic.py gpurun_out/pmc_f gpurun_out/pmc_w > profiles/rNN_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are reported in KiB per dispatch.  On gfx950 FETCH_SIZE
counts half the bytes of wide (16 B/lane) coalesced reads, so it is doubled
(the guide's HBM section); WRITE_SIZE is exact for 16-B stores.  The
calibration kernel k_gather (reads one naug x 256 panel, writes two) is
reported beside it so the correction can be checked on a known byte count.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {
    "k_update": "ace::k_update(",
    "k_update_pair": "ace::k_update_pair(",
    "k_update_multi": "ace::k_update_multi<false>(",
    "k_update_multi_r": "ace::k_update_multi_r<false>(",
    "k_update_x": "ace::k_update_x(",
    "k_gather": "ace::k_gather(",
    "k_panel_gemm": "ace::k_panel_gemm(",
    "k_grad2": "ace::k_grad2<",
    "k_asm_mm": "ace::k_asm_mm<",
    "k_asm_mm_q": "ace::k_asm_mm_q<",
    "k_grad_mm": "ace::k_grad_mm<",
}


def read(d, counter):
    """Per kernel, the counter summed per dispatch (a counter comes as one row
    per dimension instance), in dispatch order."""
    per = defaultdict(dict)
    grid = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                for short, key in KERNELS.items():
                    if key in row["Kernel_Name"]:
                        k = (f, int(row["Dispatch_Id"]))
                        per[short][k] = per[short].get(k, 0.0) + float(row["Counter_Value"])
                        grid[short][k] = int(row.get("Grid_Size", 0) or 0)
    vals = {s: [v for _, v in sorted(m.items())] for s, m in per.items()}
    # the two-step update kernel runs both as the bulk update (every lower
    # tile: the largest grid) and as the side stream's lookahead cross (a few
    # hundred tiles): report the bulk launches, selected by grid size, on
    # their own
    for kn in ("k_update_pair", "k_update_multi"):
        if kn in per:
            g = grid[kn]
            gmax = max(g.values())
            vals[kn + "_bulk"] = [v for k, v in sorted(per[kn].items()) if g[k] == gmax]
    # small n: the bulk launches are the persistent k_update_multi_r (the plain
    # kernel's launches there are the side streams' crosses)
    if "k_update_multi_r" in vals:
        vals["k_update_multi_bulk"] = vals["k_update_multi_r"]
    return vals


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    # the bench configuration both passes ran (bench.py takes roofline.traffic
    # only from a record of its own configuration)
    config = sys.argv[3] if len(sys.argv) > 3 else "C2"
    fetch = read(fdir, "FETCH_SIZE")
    write = read(wdir, "WRITE_SIZE")
    out = {"unit": "bytes per launch", "fetch_correction": 2.0, "config": config, "kernels": {}}
    for k in list(KERNELS) + ["k_update_pair_bulk", "k_update_multi_bulk"]:
        if not fetch.get(k) or not write.get(k):
            continue
        f = sum(fetch[k]) / len(fetch[k]) * 1024.0
        w = sum(write[k]) / len(write[k]) * 1024.0
        out["kernels"][k] = {"launches": len(fetch[k]), "fetch_raw": f, "fetch": 2.0 * f,
                             "write": w, "traffic": 2.0 * f + w}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
