#!/usr/bin/env python3
"""Inverse-accuracy analysis (CPU side) of tools/inverse_probe.py's outputs:
per library and problem, the GPU inverse's error against the extended-
precision referee inverse, the gradient error that inverse alone causes
(the referee's gradient arithmetic fed the GPU inverse), and the rest (the
gradient kernel's own rounding).  usage: python tools/inverse_analyze.py DIR [tag ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import referee_ld as R  # noqa: E402

LD = np.longdouble


def main():
    d = sys.argv[1]
    tags = sys.argv[2:] or sorted(f[:-4] for f in os.listdir(d) if f.endswith(".npz"))
    runs = {t: dict(np.load(os.path.join(d, t + ".npz"))) for t in tags}
    for name in ("referee_smoke", "referee_p8", "referee_p3"):
        f = np.load(os.path.join(ROOT, "tests", "golden", name + ".npz"))
        y, X, Z, th, sy = f["y"], f["X"], f["Z"], f["theta"], float(f["std_y"][0])
        n = X.shape[0]
        for kernel in ("SE", "Matern32"):
            if f"{name}_{kernel}_inv" not in runs[tags[0]]:
                continue
            Kb = R._kernel_slices(kernel, X, np.asarray(Z).reshape(n, -1), th)
            A = Kb.sum(0) + np.exp(LD(th[0])) * np.eye(n, dtype=LD)
            inv_ref, logdet = R._chol_inverse(A)
            g_ref = f[kernel + "_g_hi"].astype(LD) + f[kernel + "_g_lo"]
            gmax = float(np.max(np.abs(g_ref)))
            for t in tags:
                r = runs[t]
                inv = r[f"{name}_{kernel}_inv"].astype(LD)
                e_inv = float(np.max(np.abs(inv - inv_ref)) / np.max(np.abs(inv_ref)))
                asym = float(np.max(np.abs(inv - inv.T)))
                g_inv, _, _ = R.grad_from_inverse(kernel, y, X, Z, th, sy, inv, logdet, 1, Kb)
                g = r[f"{name}_{kernel}_g"].astype(LD)
                e_from_inv = float(np.max(np.abs(g_inv - g_ref))) / gmax
                e_kernel = float(np.max(np.abs(g - g_inv))) / gmax
                e_tot = float(np.max(np.abs(g - g_ref))) / gmax
                print(f"{name:14s} {kernel:8s} {t:6s} inv {e_inv:.2e} (asym {asym:.1e})  grad/max: "
                      f"total {e_tot:.2e} = inverse {e_from_inv:.2e} + kernel {e_kernel:.2e}", flush=True)


if __name__ == "__main__":
    main()
