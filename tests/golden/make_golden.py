"""Generates the golden fixtures in tests/golden/ from the CPU oracle
(oracle/ace_oracle.py, a restatement of the reference arithmetic).

PARITY UNPINNED: the reference (R/Rcpp/Armadillo) cannot run in this image
and ships no fixtures, so these vectors come from the oracle, which is
itself cross-checked against the literal C restatement (oracle/ace_ref.c)
and against finite differences (tests/test_oracle.py).

Run:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

from oracle import ace_oracle as O  # noqa: E402


def rand_case(rng, n, p, B, zero_frac=0.3, n2=None):
    X = rng.uniform(-1, 1, (n, p))
    Z = rng.normal(size=(n, B - 1))
    Z[rng.random((n, B - 1)) < zero_frac] = 0.0
    theta = np.concatenate([[math.log(rng.uniform(0.05, 0.5)), rng.normal(0, 0.2)],
                            rng.normal(0, 0.4, B), rng.normal(0.5, 0.8, B * p)])
    out = {"X": X, "Z": Z, "theta": theta}
    if n2:
        X2 = rng.uniform(-1, 1, (n2, p))
        Z2 = rng.normal(size=(n2, B - 1))
        Z2[rng.random((n2, B - 1)) < zero_frac] = 0.0
        out.update(X2=X2, Z2=Z2)
    return out


def main():
    rng = np.random.default_rng(20261015)
    files = {}
    # (1) assembly, symmetric + cross, both kernels, zeros and negative z (Q7)
    for kernel in ("SE", "Matern32"):
        sym, cross, grad = O.KERNELS[kernel]
        for (n, p, B) in ((7, 1, 2), (33, 2, 3), (40, 5, 6), (128, 3, 5), (70, 2, 1)):
            c = rand_case(rng, n, p, B, n2=max(5, n // 3))
            ks = sym(c["X"], c["Z"], c["theta"])
            kc = cross(c["X2"], c["X"], c["Z2"], c["Z"], c["theta"])
            d = dict(c, sym_full=ks["full"], cross_full=kc["full"])
            if n <= 40:
                d.update(sym_elements=ks["elements"], cross_elements=kc["elements"])
            files[f"asm_{kernel}_n{n}_p{p}_B{B}"] = d
    # (2)+(3) inverse, gradient and stats (Q1-Q3), (4) stats_cpp, mu_solution (Q4)
    for kernel in ("SE", "Matern32"):
        sym, cross, grad = O.KERNELS[kernel]
        for (n, p, B) in ((60, 3, 4), (97, 2, 5), (33, 1, 1)):
            c = rand_case(rng, n, p, B)
            y = rng.normal(size=n)
            ks = sym(c["X"], c["Z"], c["theta"])
            inv = O.invkernel_cpp(ks["full"], c["theta"][0])
            st = np.zeros(2)
            g = grad(y, c["X"], c["Z"], ks["full"], ks["elements"], inv["inv"], inv["eigenval"],
                     c["theta"], st, B, 1.7)
            files[f"grad_{kernel}_n{n}_p{p}_B{B}"] = dict(
                c, y=y, std_y=1.7, Kfull=ks["full"], inv=inv["inv"],
                logdet=float(np.sum(np.log(inv["eigenval"]))), grad=g, stats=st,
                stats_cpp=O.stats_cpp(y, ks["full"], inv["inv"], inv["eigenval"], c["theta"][1], 1.7),
                mu=O.mu_solution_cpp(y, inv["inv"]))
    # (5) prediction incl. ATE/ATT/ATU on binary Z_x
    for kernel in ("SE", "Matern32"):
        sym, cross, grad = O.KERNELS[kernel]
        n, nx, p = 50, 23, 2
        X = rng.uniform(-1, 1, (n, p))
        Zb = (rng.random((n, 1)) < 0.5).astype(float)
        theta = np.concatenate([[math.log(0.2), 0.1], [0.1, -0.2], rng.normal(0.8, 0.3, 2 * p)])
        y = rng.normal(size=n)
        ks = sym(X, Zb, theta)
        inv = O.invkernel_cpp(ks["full"], theta[0])["inv"]
        X2 = rng.uniform(-1, 1, (nx, p))
        Z2 = (rng.random((nx, 1)) < 0.4).astype(float)
        Z2[0] = 1.0
        Z2[1] = 0.0
        dZ2 = np.ones((nx, 1))
        K_xX = cross(X2, X, Z2, Zb, theta)["full"]
        K_xx = sym(X2, Z2, theta)["full"]
        pr = O.pred_cpp(y, theta[0], theta[1], inv, K_xX, K_xx, 0.3, 1.9)
        cX = cross(X2, X, dZ2, Zb, theta)["elements"]
        cx = sym(X2, dZ2, theta)["elements"]
        pm = O.pred_marginal_cpp(y, Z2, theta[0], theta[1], inv, cX, cx, 0.3, 1.9, 0.8, True)
        files[f"pred_{kernel}"] = dict(
            X=X, Z=Zb, theta=theta, y=y, inv=inv, X2=X2, Z2=Z2, dZ2=dZ2, K_xX=K_xX, K_xx=K_xx,
            cube_xX=cX, cube_xx=cx, map=pr["map"], ci=pr["ci"], var=pr["var"],
            m_map=pm["map"], m_ci=pm["ci"], m_var=pm["var"],
            avg=np.concatenate([[pm[k]["map"], pm[k]["ci"][0], pm[k]["ci"][1], pm[k]["var"]]
                                for k in ("ate", "att", "atu")]))
    # (6) optimizer steps, clip on/off (Q5, Q8)
    P = 17
    g = rng.normal(0, 3, P)
    para = rng.normal(size=P)
    m = rng.normal(0, 0.1, P)
    v = np.abs(rng.normal(0, 0.1, P))
    nu = rng.normal(0, 0.1, P)
    opt = {"g": g, "para": para, "m": m, "v": v, "nu": nu}
    for clip in (0, 1):
        gg = g.copy()
        O.norm_clip_cpp(bool(clip), gg, 1.0)
        for name, fn in (("nadam", O.Nadam_cpp), ("adam", O.Adam_cpp)):
            mm, vv, pp = m.copy(), v.copy(), para.copy()
            fn(3.0, 0.01, 0.9, 0.999, 1e-8, mm, vv, gg, pp)
            opt[f"{name}_clip{clip}"] = np.concatenate([mm, vv, pp])
        nn, pp = nu.copy(), para.copy()
        O.Nesterov_cpp(0.01, 0.5, nn, gg, pp)
        opt[f"nesterov_clip{clip}"] = np.concatenate([nn, pp])
    files["optim"] = opt
    # (7) README-config trajectory: n=300, d=2, cubic (ns) n.knots=2, Nadam lr 0.01
    from additivecausalexpansion_amd.synthetic import readme_data
    yraw, Xraw, Zraw = readme_data()
    y = yraw.copy()
    X = np.asfortranarray(Xraw.copy())
    Z = np.asfortranarray(Zraw.copy())
    mom = O.normalize_train(y, X, Z)
    z = Z[:, 0]
    ik = np.quantile(z, np.arange(1, 3) / 3, method="linear")
    knots = np.concatenate([ik, [-1.0, 1.0]])
    Bm = O.ncs_basis(z, knots)
    dBm = O.ncs_basis_deriv(z, knots)
    B = Bm.shape[1] + 1
    theta0 = O.set_initial_parameters(2, B, 300, y, X, Z)
    for kernel in ("SE", "Matern32"):
        optim = O.OracleOptimizer("Nadam", theta0.shape[0], 0.01, norm_clip=True, clip_at=1.0)
        th, st, gr, inv = O.train_trajectory(kernel, y, X, Bm, theta0, mom[0, 1], 20, optim)
        sym, cross, grad = O.KERNELS[kernel]
        pr = O.pred_cpp(y, th[-1][0], th[-1][1], inv, cross(X, X, Bm, Bm, th[-1])["full"],
                        sym(X, Bm, th[-1])["full"], mom[0, 0], mom[0, 1])
        files[f"traj_{kernel}"] = dict(
            yraw=yraw, Xraw=Xraw, Zraw=Zraw, y=y, X=X, Z=Z, moments=mom, knots=knots, basis=Bm,
            dbasis=dBm, theta0=theta0, thetas=th, stats=st, grads=gr, pred_map=pr["map"],
            pred_var=pr["var"])
    for name, d in files.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    total = sum(os.path.getsize(os.path.join(HERE, f + ".npz")) for f in files)
    print(f"wrote {len(files)} fixtures, {total / 1e6:.2f} MB")


if __name__ == "__main__":
    main()
