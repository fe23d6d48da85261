"""CU sharing of the chain's critical workgroups in one evaluation, from the raw
per-workgroup records tools/wg_timeline.py dumps (WGT_DUMP=path.npy):

  python tools/wgt_cu.py gpurun_out/r5t/wgt_c1.npy

For every k_panel_split workgroup that runs the fused sub-sweep (marks 0..3)
and every k_update_q workgroup with the fused D_0 sweep (marks 0..2): its
phases (us) and the workgroups of other launches resident on the same CU
(same XCC and HW_ID cu / sh / se) at any time during its life, by kernel.
Splits whose phases stretch with co-resident bulk / cross workgroups share
issue with them; stretched phases without co-residents point at memory."""
import sys
from collections import Counter

import numpy as np

KIND = {1: "pivot", 2: "split", 3: "gemm_t", 4: "update_q", 5: "update_multi", 6: "update",
        7: "grad", 8: "grad(diag)"}
TICK_US = 0.01


def parse(recs):
    out = []
    for r in recs:
        r = [int(x) for x in r]
        kid, bx, gx = r[0] & 0xFF, (r[0] >> 8) & 0xFFFFFFF, r[0] >> 36
        hw, xcc, nw = r[1] & 0xFFFFFFFF, (r[1] >> 32) & 0xFF, (r[1] >> 40) & 0xFF
        ends = [x for x in r[4:4 + nw] if x > 0]
        out.append({"kid": kid, "bx": bx, "grid": gx, "cu": (xcc, (hw >> 8) & 0xFF), "t0": r[2],
                    "t1": max(ends) if ends else r[2], "marks": [x for x in r[12:16]]})
    return out


def main():
    w = parse(np.load(sys.argv[1]))
    t0 = min(x["t0"] for x in w)
    crit = [x for x in w if (x["kid"] == 2 and all(x["marks"][:4])) or
            (x["kid"] == 4 and all(x["marks"][:3]))]
    crit.sort(key=lambda x: x["t0"])
    rows = []
    for c in crit:
        co = Counter()
        for x in w:
            if x is c or x["cu"] != c["cu"] or x["t1"] <= c["t0"] or x["t0"] >= c["t1"]:
                continue
            name = KIND.get(x["kid"], str(x["kid"]))
            if x["kid"] == 5:
                name = "bulk" if x["grid"] == 512 else "cross/T"
            co[name] += 1
        nm = 4 if c["kid"] == 2 else 3
        ts = [c["t0"]] + c["marks"][:nm] + [c["t1"]]
        ph = np.diff(ts) * TICK_US
        rows.append((c, ph, co))
        print("%8.1f us %-8s total %6.1f | %s | beside: %s" % (
            (c["t0"] - t0) * TICK_US, KIND[c["kid"]], ph.sum(),
            " ".join("%5.1f" % v for v in ph), dict(co) or "-"))
    for kid, label in ((2, "split"), (4, "update_q")):
        alone = [ph for c, ph, co in rows if c["kid"] == kid and not co]
        shared = [ph for c, ph, co in rows if c["kid"] == kid and co]
        for tag, lst in (("alone", alone), ("shared", shared)):
            if lst:
                a = np.asarray(lst)
                print("%-8s %-6s %3d wgs: median phases %s, total %.1f" % (
                    label, tag, len(a), " ".join("%.1f" % v for v in np.median(a, axis=0)),
                    np.median(a.sum(axis=1))))


if __name__ == "__main__":
    main()
