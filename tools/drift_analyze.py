#!/usr/bin/env python3
"""Numeric-drift analysis (CPU side) of tools/drift_probe.py's outputs: the
error of every library's gradient / stats / mu against the extended-precision
referee (tests/referee_ld.py), per case, with the worst gradient component.
usage: python tools/drift_analyze.py DIR [tag ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from drift_probe import CASES  # noqa: E402
from referee_ld import para_update_ld, rel_err  # noqa: E402

from additivecausalexpansion_amd.synthetic import make_problem  # noqa: E402


def main():
    d = sys.argv[1]
    tags = sys.argv[2:] or sorted(f[:-4] for f in os.listdir(d) if f.endswith(".npz"))
    runs = {t: dict(np.load(os.path.join(d, t + ".npz"))) for t in tags}
    print(f"{'case':<16}" + "".join(f"{t:>26}" for t in tags))
    for name, n, p, B, seed in CASES:
        for kernel in ("SE", "Matern32"):
            y, X, Z, th, sy = make_problem(n, p, B, seed=seed)
            g, st, mu = para_update_ld(kernel, y, X, Z, th, sy)
            row = f"{name + '_' + kernel:<16}"
            for t in tags:
                r = runs[t]
                k = f"{name}_{kernel}"
                gg = r[k + "_g"]
                eg = rel_err(gg, g)
                i = int(np.argmax(np.abs(gg - g) / (np.abs(g) + 1e-9 * np.abs(g).max())))
                es = rel_err(r[k + "_st"], st, 0)
                em = abs(float(r[k + "_mu"][0]) - float(mu)) / abs(float(mu))
                row += f"  g{eg:8.1e}@{i:<3d} s{es:7.1e} m{em:7.1e}"
            print(row, flush=True)


if __name__ == "__main__":
    main()
