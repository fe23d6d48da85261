"""Generates tests/golden/referee_*.npz: one iteration-1 para_update in
extended precision (tests/referee_ld.py, numpy longdouble) at every feature
bucket the pair kernels are compiled for (p = 3, 8, 12, 16, 20, 24, 32, 48,
64) and on the smoke problem, for both kernels.  Inputs come from the
seeded generator (additivecausalexpansion_amd/synthetic.py) and are stored
with the outputs, so the GPU test needs neither the generator's numpy
version nor the referee.

The outputs are the referee's longdouble values split into an fp64 head and
an fp64 tail (head + tail carries ~19 significant digits), so a test can
measure an fp64 result's error well below 1 ulp of the value.

Run:  python tests/golden/make_referee.py [--big | --only-big]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from referee_ld import para_update_ld  # noqa: E402

from additivecausalexpansion_amd.synthetic import make_problem  # noqa: E402

CASES = [("smoke", 300, 3, 5, 42)] + [(f"p{p}", 200, p, 4, 100 + p)
                                      for p in (3, 8, 12, 16, 20, 24, 32, 48, 64)]
# a multi-group sweep (round 6): n = 2600 is 11 steps of 256, four groups at
# Z = 3 (n <= 8192), so the persistent bulk queue, the fused D_0 pivot at the
# group boundaries and the blocked pivot across groups are held to the
# referee, not only to their own variants.  Its inputs (0.5 MB) are not
# stored: the test regenerates them from the seed and checks their SHA-256.
BIG = [("p20_n2600", 2600, 20, 4, 2600)]


def input_digest(y, X, Z, th, sy):
    import hashlib
    h = hashlib.sha256()
    for a in (y, X, Z, th, np.array([sy])):
        h.update(np.ascontiguousarray(a, dtype=np.float64).tobytes())
    return h.hexdigest()


def split(x):
    hi = np.asarray(x, dtype=np.float64)
    lo = np.asarray(np.asarray(x, dtype=np.longdouble) - hi.astype(np.longdouble), dtype=np.float64)
    return hi, lo


def main():
    cases = CASES + BIG if "--big" in sys.argv else CASES
    if "--only-big" in sys.argv:
        cases = BIG
    for name, n, p, B, seed in cases:
        y, X, Z, th, sy = make_problem(n, p, B, seed=seed)
        if (name, n, p, B, seed) in BIG:
            out = {"gen": np.array([n, p, B, seed]), "input_sha256": np.array([input_digest(y, X, Z, th, sy)])}
        else:
            out = {"y": y, "X": X, "Z": Z, "theta": th, "std_y": np.array([sy])}
        for kernel in ("SE", "Matern32"):
            g, st, mu = para_update_ld(kernel, y, X, Z, th, sy)
            for key, val in (("g", g), ("st", st), ("mu", np.array([mu]))):
                hi, lo = split(val)
                out[f"{kernel}_{key}_hi"] = hi
                out[f"{kernel}_{key}_lo"] = lo
        path = os.path.join(HERE, f"referee_{name}.npz")
        np.savez_compressed(path, **out)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
