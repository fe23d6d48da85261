import os, sys
import numpy as np
ROOT='/root/repo'
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT+'/tests')
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
from oracle import ace_oracle as O
A.default_context()
for kernel in ("SE", "Matern32"):
    n,p,B=200,50,8
    y, X, Z, th, sy = make_problem(n, p, B, seed=7)
    m = A.DeviceModel(kernel, n, p, B); m.set_data(y, X, Z, sy)
    t_dev = th.copy(); g, st, _ = m.para_update(2, t_dev)
    sym, _, grad = O.KERNELS[kernel]
    Kl = sym(X, Z, th); inv = O.invkernel_cpp(Kl["full"], th[0])
    st_ref = np.zeros(2)
    g_ref = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], th.copy(), st_ref, B, sy)
    np.set_printoptions(precision=6, linewidth=200)
    print(kernel, "lam dev", g[2:2+B]); print(kernel, "lam ref", g_ref[2:2+B])
    K=Kl["elements"]; off=K.copy()
    for b in range(B): np.fill_diagonal(off[:,:,b],0)
    print("max offdiag K_b", [float(np.abs(off[:,:,b]).max()) for b in range(B)])
    print("theta lam", th[2:2+B])
