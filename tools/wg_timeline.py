"""Per-workgroup timeline of the sweep's kernels in one C2 evaluation, from a
-DACE_DIAG_WGTIME build (tools/build_variant.sh wgt -DACE_DIAG_WGTIME):
  ACE_LIB_PATH=ab/libace_wgt.so python tools/wg_timeline.py [n [p B kernel]]

For every launch of the chain kernels (k_pivot, k_panel_split) and the head
launches (k_panel_gemm_t, k_update_q): the launch span (first workgroup
entry to last wave exit), each workgroup's own duration (entry to its last
wave's exit) and the spread of the workgroups' entry times.  A span much
longer than the workgroups' own durations means the workgroups waited for a
CU slot (dispatch); a workgroup duration much longer than the kernel's
uncontended time means it ran slowly beside the bulk tiles (issue sharing).
The bulk update launches are sampled (every 32nd workgroup)."""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import additivecausalexpansion_amd as ace  # noqa: E402
from additivecausalexpansion_amd._lib import lib  # noqa: E402
from additivecausalexpansion_amd.synthetic import make_problem  # noqa: E402

KIND = {1: "pivot", 2: "panel_split", 3: "panel_gemm_t", 4: "update_q", 5: "update_multi",
        6: "update", 7: "grad_mm", 8: "grad_mm(diag)"}
REC = 16
TICK_US = 0.01  # wall_clock64: 100 MHz


def read(L, reset):
    """Both translation units' records (sweep kernels, pair kernels)."""
    out = []
    for name in ("ace_diag_wgtime", "ace_diag_wgtime_pairs"):
        f = getattr(L, name)
        f.restype = ctypes.c_longlong
        f.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int]
        cnt = f(None, 0, 0)
        buf = np.zeros((max(cnt, 1), REC), dtype=np.uint64)
        got = f(buf.ctypes.data, cnt, 1 if reset else 0)
        assert got >= 0, name + " failed"
        out.append(buf[:min(cnt, buf.shape[0])])
    return np.concatenate(out)


def launches(recs):
    """Records -> list of launches (kid, grid, [records]) in start order: per
    (kid, grid), a new launch starts when a block index repeats."""
    by = defaultdict(list)
    for r in recs:
        kid, bx, gx = int(r[0]) & 0xFF, (int(r[0]) >> 8) & 0xFFFFFFF, int(r[0]) >> 36
        by_, gy = int(r[3]) & 0xFFFFFFFF, int(r[3]) >> 32
        by[(kid, gx * max(gy, 1))].append((int(r[2]), (bx, by_), r))
    out = []
    for (kid, grid), lst in by.items():
        lst.sort(key=lambda t: t[0])
        cur, seen = [], set()
        for t0, blk, r in lst:
            if blk in seen:
                out.append((kid, grid, cur))
                cur, seen = [], set()
            seen.add(blk)
            cur.append(r)
        if cur:
            out.append((kid, grid, cur))
    out.sort(key=lambda L: min(int(r[2]) for r in L[2]))
    return out


def wg_end(r):
    nw = (int(r[1]) >> 40) & 0xFF
    ends = [int(x) for x in r[4:4 + nw] if int(x) > 0]
    return max(ends) if ends else int(r[2])


def phases(ls, kid, label):
    """Median per-phase durations of kid's workgroups (wave 0's marks), per
    set of marks present: entry -> mark i -> ... -> exit."""
    groups = defaultdict(list)
    for k, grid, rs in ls:
        if k != kid:
            continue
        for r in rs:
            marks = [(i, int(r[12 + i])) for i in range(4) if int(r[12 + i])]
            key = tuple(i for i, _ in marks)
            ts = [int(r[2])] + [t for _, t in marks] + [wg_end(r)]
            groups[key].append(np.diff(ts) * TICK_US)
    for key, rows in sorted(groups.items()):
        a = np.asarray(rows)
        names = ["entry"] + ["m%d" % i for i in key] + ["exit"]
        segs = "  ".join("%s->%s %.2f" % (names[i], names[i + 1], np.median(a[:, i]))
                         for i in range(a.shape[1]))
        print("  %-14s marks %-10s %5d wgs  total %.2f us | %s" % (
            label, ",".join(map(str, key)) or "-", len(a), np.median(a.sum(axis=1)), segs))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    kern = sys.argv[4] if len(sys.argv) > 4 else "Matern32"
    L = lib()
    y, X, Z, th, sy = make_problem(n, p, B, seed=5)
    m = ace.DeviceModel(kern, n, p, B)
    m.set_data(y, X, Z, sy)
    theta = th.copy()
    for it in (1, 2):
        m.para_update(it, theta)
    read(L, True)
    m.para_update(3, theta)
    recs = read(L, True)
    if os.environ.get("WGT_DUMP"):  # raw records for offline analysis (tools/wgt_cu.py)
        np.save(os.environ["WGT_DUMP"], recs)
    print(f"n={n}: {len(recs)} workgroup records")
    ls = launches(recs)
    t0 = min(int(r[2]) for r in recs)
    bulk_grid = max(g for k, g, _ in ls if k == 5)
    stats = defaultdict(lambda: {"span": [], "wg": [], "spread": [], "t": []})
    for kid, grid, rs in ls:
        st = min(int(r[2]) for r in rs)
        en = max(wg_end(r) for r in rs)
        durs = [wg_end(r) - int(r[2]) for r in rs]
        name = KIND.get(kid, str(kid))
        if kid == 5:
            name = "bulk(sampled)" if grid == bulk_grid else "update_multi(cross/T)"
        s = stats[name]
        s["span"].append((en - st) * TICK_US)
        s["wg"].append(np.median(durs) * TICK_US)
        s["spread"].append((max(int(r[2]) for r in rs) - st) * TICK_US)
        s["t"].append((st - t0) * TICK_US)
    print("%-24s %6s %10s %12s %12s   (us; medians over launches, then [p10, p90])" % (
        "kernel", "launch", "span", "wg duration", "entry spread"))
    for name, s in sorted(stats.items()):
        def q(v):
            v = np.asarray(v)
            return "%7.1f [%5.1f,%6.1f]" % (np.median(v), np.percentile(v, 10), np.percentile(v, 90))
        print("%-24s %6d %s %s %s" % (name, len(s["span"]), q(s["span"]), q(s["wg"]), q(s["spread"])))
    # k_panel_gemm_t phases (wave 0): entry -> staged first chunk -> K loop done -> exit
    ph = []
    for kid, grid, rs in ls:
        if kid != 3:
            continue
        for r in rs:
            m0, m1 = int(r[12]), int(r[13])
            if m0 and m1:
                ph.append(((m0 - int(r[2])) * TICK_US, (m1 - m0) * TICK_US, (wg_end(r) - m1) * TICK_US))
    if ph:
        a = np.asarray(ph)
        print("panel_gemm_t phases (median us): prologue %.1f  K loop %.1f  epilogue %.1f  (%d wgs)" % (
            np.median(a[:, 0]), np.median(a[:, 1]), np.median(a[:, 2]), len(a)))
    # gradient tiles (wave 0): entry -> staged (prologue) -> slice loop done -> exit
    gp = []
    for kid, grid, rs in ls:
        if kid != 7:
            continue
        for r in rs:
            m0, m1 = int(r[12]), int(r[13])
            if m0 and m1:
                gp.append(((m0 - int(r[2])) * TICK_US, (m1 - m0) * TICK_US, (wg_end(r) - m1) * TICK_US))
    if gp:
        a = np.asarray(gp)
        tot = a.sum(axis=1)
        print("grad_mm tiles (us): prologue median %.1f mean %.1f | slice loop median %.1f | finish median %.1f"
              " | prologue share of workgroup time %.1f %% (%d tiles)" % (
                  np.median(a[:, 0]), a[:, 0].mean(), np.median(a[:, 1]), np.median(a[:, 2]),
                  100.0 * a[:, 0].sum() / tot.sum(), len(a)))
    print("per-workgroup phases (wave 0 marks; us, medians):")
    phases(ls, 1, "pivot")
    phases(ls, 2, "panel_split")
    phases(ls, 4, "update_q")
    bulks = sorted((min(int(r[2]) for r in rs) - t0) * TICK_US for k, g, rs in ls
                   if k == 5 and g == bulk_grid)
    if len(bulks) > 9:
        print("launch sequence during bulk 8 (%.1f - %.1f us):" % (bulks[8], bulks[9]))
        sequence(ls, t0, bulks[8] - 50.0, bulks[9])
    # the first group (under the assembly) against the rest
    for name in ("panel_split", "pivot"):
        s = stats.get(name)
        if not s:
            continue
        t = np.asarray(s["t"])
        first = t < 3000.0
        for lab, sel in (("first 3 ms", first), ("after", ~first)):
            if sel.any():
                print("  %-12s %-10s span %6.1f  wg %6.1f  spread %6.1f  (%d launches)" % (
                    name, lab, np.median(np.asarray(s["span"])[sel]), np.median(np.asarray(s["wg"])[sel]),
                    np.median(np.asarray(s["spread"])[sel]), int(sel.sum())))


def sequence(ls, t0, lo_us, hi_us):
    """Every launch starting in [lo, hi) us: name, grid, first entry, last
    exit, median workgroup duration (us from the evaluation's first record)."""
    for kid, grid, rs in ls:
        st = (min(int(r[2]) for r in rs) - t0) * TICK_US
        if not lo_us <= st < hi_us:
            continue
        en = (max(wg_end(r) for r in rs) - t0) * TICK_US
        d = np.median([wg_end(r) - int(r[2]) for r in rs]) * TICK_US
        print("    %-14s grid %6d  %9.1f - %9.1f  (wg %6.1f, %d recs)" % (
            KIND.get(kid, str(kid)), grid, st, en, d, len(rs)))


if __name__ == "__main__":
    main()
