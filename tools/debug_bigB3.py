"""Diagnostic: the ABI gradient (oracle Kfull / inverse in, with and without
the K cube) vs the oracle at p = 50, to split a fused-model fault from a
gradient-kernel fault."""
import os, sys
import numpy as np
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
from oracle import ace_oracle as O
A.default_context()
np.set_printoptions(precision=6, linewidth=200)
for kernel, B in (("Matern32", 8), ("SE", 16), ("Matern32", 16)):
    n, p = 200, 50
    y, X, Z, th, sy = make_problem(n, p, B, seed=7)
    sym, _, grad = O.KERNELS[kernel]
    Kl = sym(X, Z, th); inv = O.invkernel_cpp(Kl["full"], th[0])
    st = np.zeros(2)
    g_ref = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], th.copy(), st, B, sy)
    f = A.grad_SE_cpp if kernel == "SE" else A.grad_Matern_cpp
    for cube in (Kl["elements"], None):
        s2 = np.zeros(2)
        g = f(y, X, Z, Kl["full"], cube, inv["inv"], inv["eigenval"], th.copy(), s2, B, sy)
        print(kernel, B, "cube" if cube is not None else "fused", "lam dev", g[2:2 + B])
    print(kernel, B, "ref      lam", g_ref[2:2 + B])
    m = A.DeviceModel(kernel, n, p, B); m.set_data(y, X, Z, sy)
    t = th.copy(); gm, stm, _ = m.para_update(2, t)
    print(kernel, B, "model    lam", gm[2:2 + B])
    Kd = A.kernmat_Matern32_symmetric_cpp(X, Z, th) if kernel != "SE" else A.kernmat_SE_symmetric_cpp(X, Z, th)
    print("kernmat full rel err", np.abs(Kd["full"] - Kl["full"]).max() / np.abs(Kl["full"]).max(),
          "diag dev/ref", np.diag(Kd["full"])[:4], np.diag(Kl["full"])[:4])
