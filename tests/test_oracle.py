"""CPU tests of the oracle itself (PARITY UNPINNED: no reference outputs
exist, so the oracle is pinned by (a) an independent literal C restatement,
(b) finite differences on the components the reference's quirks leave
exact, (c) the documented quirks Q1-Q8, (d) its own golden fixtures)."""
import ctypes
import math

import numpy as np
import pytest
from conftest import golden, golden_names

from oracle import ace_oracle as O

D = ctypes.POINTER(ctypes.c_double)


def P(a):
    return a.ctypes.data_as(D)


def case(rng, n, p, B, zero_frac=0.3):
    X = np.asfortranarray(rng.uniform(-1, 1, (n, p)))
    Z = np.asfortranarray(rng.normal(size=(n, B - 1)))
    Z[rng.random((n, B - 1)) < zero_frac] = 0.0
    th = np.concatenate([[math.log(0.2), 0.1], rng.normal(0, 0.3, B), rng.normal(0.3, 0.5, B * p)])
    return X, Z, th


@pytest.mark.parametrize("kind,name", [(0, "SE"), (1, "Matern32")])
@pytest.mark.parametrize("n,p,B", [(1, 1, 2), (9, 2, 1), (41, 3, 4), (64, 5, 6)])
def test_numpy_oracle_matches_literal_c(ref_c, kind, name, n, p, B):
    rng = np.random.default_rng(n * 10 + B + kind)
    X, Z, th = case(rng, n, p, B)
    Kf = np.zeros((n, n), order="F")
    Ke = np.zeros((n, n, B), order="F")
    ref_c.ref_kernmat_sym(kind, n, p, B, P(X), P(Z), P(th), P(Kf), P(Ke))
    o = O.KERNELS[name][0](X, Z, th)
    assert np.allclose(Kf, o["full"], rtol=1e-14, atol=1e-15)
    assert np.allclose(Ke, o["elements"], rtol=1e-14, atol=1e-15)
    # cross
    n2 = max(1, n // 2 + 3)
    X2 = np.asfortranarray(rng.uniform(-1, 1, (n2, p)))
    Z2 = np.asfortranarray(rng.normal(size=(n2, B - 1)))
    Cf = np.zeros((n2, n), order="F")
    Ce = np.zeros((n2, n, B), order="F")
    ref_c.ref_kernmat_cross(kind, n2, n, p, B, P(X2), P(X), P(Z2), P(Z), P(th), P(Cf), P(Ce))
    oc = O.KERNELS[name][1](X2, X, Z2, Z, th)
    assert np.allclose(Cf, oc["full"], rtol=1e-14, atol=1e-15)
    assert np.allclose(Ce, oc["elements"], rtol=1e-14, atol=1e-15)
    if n < 3:
        return
    inv = O.invkernel_cpp(o["full"], th[0])
    y = rng.normal(size=n)
    st = np.zeros(2)
    g = O.KERNELS[name][2](y, X, Z, o["full"], o["elements"], inv["inv"], inv["eigenval"], th, st,
                           B, 1.3)
    st2 = np.zeros(2)
    g2 = np.zeros(th.shape[0])
    invF = np.asfortranarray(inv["inv"])
    ref_c.ref_grad(kind, n, p, B, P(y), P(X), P(Kf), P(Ke), P(invF),
                   float(np.sum(np.log(inv["eigenval"]))), P(th), P(st2), 1.3, P(g2))
    assert np.allclose(g, g2, rtol=1e-10, atol=1e-12 * np.abs(g).max())
    assert np.allclose(st, st2, rtol=1e-12)
    mu_c = ref_c.ref_mu_solution(n, P(y), P(invF))
    assert mu_c == pytest.approx(O.mu_solution_cpp(y, inv["inv"]), rel=1e-10)


def _true_evidence(kernel, X, Z, th, y):
    """log evidence with ybar.alpha (the textbook form; Q3 uses y.alpha)."""
    K = O.KERNELS[kernel][0](X, Z, th)["full"]
    A = K + math.exp(th[0]) * np.eye(K.shape[0])
    ybar = y - th[1]
    s, ld = np.linalg.slogdet(A)
    return -0.5 * (len(y) * math.log(2 * math.pi) + ld + ybar @ np.linalg.solve(A, ybar))


def test_gradients_against_finite_differences():
    """sigma and lambda gradients are exact (except lambda_{B-1}, see below); SE length-scale gradient j is the
    derivative w.r.t. the KERNEL's parameter j-1 rescaled by e^-(th_j - th_{j-1})
    (Q1: kernel index 1+b+B(i+1), gradient index 2+B+b+B i)."""
    rng = np.random.default_rng(5)
    n, p, B = 30, 2, 3
    X, Z, th = case(rng, n, p, B, zero_frac=0.2)
    y = rng.normal(size=n)
    Kl = O.kernmat_SE_symmetric_cpp(X, Z, th)
    inv = O.invkernel_cpp(Kl["full"], th[0])
    st = np.zeros(2)
    g = O.grad_SE_cpp(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], th, st, B, 1)
    h = 1e-6
    # theta[1+B] is lambda_{B-1} AND the kernel's (i=0, b=0) length scale (Q1): skip it
    for j in [0] + list(range(2, 1 + B)):
        e = np.zeros_like(th)
        e[j] = h
        fd = (_true_evidence("SE", X, Z, th + e, y) - _true_evidence("SE", X, Z, th - e, y)) / (2 * h)
        assert g[j] == pytest.approx(fd, rel=1e-6, abs=1e-7)
    for i in range(p):
        for b in range(B):
            j = 2 + B + b + B * i
            if j - 1 < 2 + B:
                continue  # maps onto a lambda slot: not a length scale of the kernel
            e = np.zeros_like(th)
            e[j - 1] = h
            fd = (_true_evidence("SE", X, Z, th + e, y) - _true_evidence("SE", X, Z, th - e, y)) / (2 * h)
            assert g[j] * math.exp(th[j]) * math.exp(-th[j - 1]) == pytest.approx(fd, rel=1e-5, abs=1e-7)
    # the last theta entry is never read by the kernel but has a non-zero gradient (Q1)
    assert g[-1] != 0.0


def test_quirks_evidence_mu_clip():
    rng = np.random.default_rng(7)
    n, p, B = 25, 2, 2
    X, Z, th = case(rng, n, p, B)
    th[1] = 0.4
    y = rng.normal(size=n)
    K = O.kernmat_SE_symmetric_cpp(X, Z, th)["full"]
    inv = O.invkernel_cpp(K, th[0])
    st = O.stats_cpp(y, K, inv["inv"], inv["eigenval"], th[1], 1.0)
    alpha = inv["inv"] @ (y - th[1])
    q3 = -0.5 * (n * math.log(2 * math.pi) + np.sum(np.log(inv["eigenval"])) + y @ alpha)
    assert st[1] == pytest.approx(q3, rel=1e-13)                    # Q3: y . alpha
    gls = np.sum(inv["inv"] @ y) / np.sum(inv["inv"])
    assert O.mu_solution_cpp(y, inv["inv"]) == pytest.approx(0.5 * gls, rel=1e-13)  # Q4
    g = np.array([3.0, 4.0])
    O.norm_clip_cpp(True, g, 2.0)
    assert np.allclose(g, [0.6, 0.8])                               # Q5: unit norm, not clip.at
    g = np.array([0.3, 0.4])
    O.norm_clip_cpp(True, g, 2.0)
    assert np.allclose(g, [0.3, 0.4])
    para, m, v = np.zeros(2), np.zeros(2), np.zeros(2)
    O.Nadam_cpp(1.0, 0.1, 0.9, 0.999, 1e-8, m, v, np.array([1.0, -1.0]), para)
    assert para[0] > 0 and para[1] < 0                               # Q8: ascent


def test_invkernel_matches_direct_inverse():
    rng = np.random.default_rng(3)
    X, Z, th = case(rng, 50, 3, 4)
    K = O.kernmat_Matern32_symmetric_cpp(X, Z, th)["full"]
    inv = O.invkernel_cpp(K, th[0])
    A = K + math.exp(th[0]) * np.eye(50)
    assert np.allclose(inv["inv"], np.linalg.inv(A), rtol=1e-9, atol=1e-11)
    assert np.all(np.diff(inv["eigenval"]) >= 0)  # ascending (dsyevd)


@pytest.mark.parametrize("name", golden_names("asm_") + golden_names("grad_"))
def test_golden_fixtures_reproduce(name):
    d = golden(name)
    kernel = "SE" if "_SE_" in name else "Matern32"
    sym, cross, grad = O.KERNELS[kernel]
    if name.startswith("asm_"):
        assert np.array_equal(sym(d["X"], d["Z"], d["theta"])["full"], d["sym_full"])
        assert np.array_equal(cross(d["X2"], d["X"], d["Z2"], d["Z"], d["theta"])["full"],
                              d["cross_full"])
    else:
        Kl = sym(d["X"], d["Z"], d["theta"])
        inv = O.invkernel_cpp(Kl["full"], d["theta"][0])
        st = np.zeros(2)
        g = grad(d["y"], d["X"], d["Z"], Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"],
                 d["theta"], st, Kl["elements"].shape[2], float(d["std_y"]))
        assert np.allclose(g, d["grad"], rtol=1e-9, atol=1e-12)
        assert np.allclose(st, d["stats"], rtol=1e-10)


def test_golden_trajectory_is_an_ascent():
    for k in ("SE", "Matern32"):
        d = golden(f"traj_{k}")
        ev = d["stats"][:, 1]
        assert np.all(np.isfinite(ev)) and ev[-1] > ev[0]
        assert d["thetas"].shape == (20, d["theta0"].shape[0])


def test_sweep_model_inverts_and_logdets():
    """The device algorithm (blocked Gauss-Jordan sweep with AUG rows) in numpy,
    same blocking as the HIP kernels."""
    import sweep_model as S
    rng = np.random.default_rng(11)
    for n in (37, 300):
        X, Z, th = case(rng, n, 3, 4)
        K = O.kernmat_SE_symmetric_cpp(X, Z, th)["full"]
        y = rng.normal(size=n)
        r = S.invert_with_aug(K, th[0], y)
        ref = O.invkernel_cpp(K, th[0])
        scale = np.abs(ref["inv"]).max()
        assert np.abs(r["inv"] - ref["inv"]).max() < 1e-10 * scale
        assert r["logdet"] == pytest.approx(np.sum(np.log(ref["eigenval"])), rel=1e-12, abs=1e-9)
        assert np.allclose(r["u"], ref["inv"] @ y, rtol=1e-9, atol=1e-10 * scale)
        assert r["oK1"] == pytest.approx(ref["inv"].sum(), rel=1e-10)
        assert r["yK1"] == pytest.approx(np.sum(ref["inv"] @ y), rel=1e-9, abs=1e-9 * scale)


@pytest.mark.parametrize("zx_val", [0.0, 1.0])
def test_pred_marginal_empty_group_is_c_semantics(zx_val):
    """src/pred_cpp.cpp:95-110 divides doubles by `unsigned int` counts: with
    no treated (ntx = 0) or no untreated (nux = 0) test point the reference
    returns NaN / inf, it does not fail.  The oracle must do the same."""
    rng = np.random.default_rng(4)
    n, nx, B = 12, 7, 3
    X = rng.uniform(-1, 1, (n, 2))
    Z = rng.normal(size=(n, B - 1))
    X2 = rng.uniform(-1, 1, (nx, 2))
    Z2 = rng.normal(size=(nx, B - 1))
    th = np.concatenate([[math.log(0.1), 0.2], np.zeros(B), np.full(2 * B, math.log(2.0))])
    inv = O.invkernel_cpp(O.kernmat_SE_symmetric_cpp(X, Z, th)["full"], th[0])["inv"]
    out = O.pred_marginal_cpp(rng.normal(size=n), np.full(nx, zx_val), th[0], th[1], inv,
                              O.kernmat_SE_cpp(X2, X, Z2, Z, th)["elements"],
                              O.kernmat_SE_symmetric_cpp(X2, Z2, th)["elements"], 0.0, 1.3, 0.7,
                              True)
    assert np.isfinite(out["ate"]["map"])
    if zx_val == 0.0:  # ntx = 0: 0/0
        assert np.isnan(out["att"]["map"]) and np.isnan(out["att"]["var"])
        assert np.isnan(out["atu"]["map"])  # (ate nx - NaN * 0) / nx
    else:  # nux = 0
        assert np.isfinite(out["att"]["map"])
        assert not np.isfinite(out["atu"]["map"]) and np.isnan(out["atu"]["var"])
