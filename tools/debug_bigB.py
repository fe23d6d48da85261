"""Diagnostic: fused-model para_update vs the oracle at large B (per-component
errors of the gradient, stats and inverse).  Run on the GPU box:
    python tools/debug_bigB.py [ACE_PAIRS=valu|mm via env]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import additivecausalexpansion_amd as A  # noqa: E402
from additivecausalexpansion_amd.synthetic import make_problem  # noqa: E402
from oracle import ace_oracle as O  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


def main():
    A.default_context()
    cases = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]] or [
        (200, 4, 32), (200, 50, 8), (200, 50, 16), (200, 50, 24), (200, 50, 32), (200, 4, 20),
        (200, 20, 28)]
    for kernel in ("SE", "Matern32"):
        for n, p, B in cases:
            y, X, Z, th, sy = make_problem(n, p, B, seed=7)
            m = A.DeviceModel(kernel, n, p, B)
            m.set_data(y, X, Z, sy)
            t_dev = th.copy()
            g, st, _ = m.para_update(2, t_dev)
            sym, _, grad = O.KERNELS[kernel]
            Kl = sym(X, Z, th)
            inv = O.invkernel_cpp(Kl["full"], th[0])
            st_ref = np.zeros(2)
            g_ref = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], th.copy(),
                         st_ref, B, sy)
            print(f"{kernel:8s} n={n} p={p:2d} B={B:2d}  inv {rel(m.inverse(), inv['inv']):.1e}  "
                  f"stats {rel(st, st_ref):.1e}  g0 {rel(g[:1], g_ref[:1]):.1e}  "
                  f"lam {rel(g[2:2 + B], g_ref[2:2 + B]):.1e}  L {rel(g[2 + B:], g_ref[2 + B:]):.1e}",
                  flush=True)


if __name__ == "__main__":
    main()
