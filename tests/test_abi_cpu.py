"""CPU-side checks of the C ABI library: it loads, exports every symbol
include/ace_hip.h declares, fails loudly without a GPU, and its host-only
entry points (optimizers, norm clip, ncs basis, normalisation) match the
oracle.  No GPU compute here."""
import ctypes
import os
import re

import numpy as np
import pytest
from conftest import ROOT, golden

from oracle import ace_oracle as O


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.lib()
    return pkg


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "ace_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ace_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol(A):
    from additivecausalexpansion_amd._lib import SIGNATURES, lib
    syms = header_symbols()
    assert len(syms) >= 28
    L = lib()
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(SIGNATURES), set(syms) ^ set(SIGNATURES)
    assert L.ace_abi_version() == 1


def test_no_gpu_fails_loudly(A):
    from additivecausalexpansion_amd._lib import AceError, lib
    h = ctypes.c_void_p()
    st = lib().ace_create(0, ctypes.byref(h))
    if st == 0:
        lib().ace_destroy(h)
        pytest.skip("a GPU is visible")
    assert st == 2
    assert b"device" in lib().ace_last_error(None)
    with pytest.raises(AceError):
        A.Context(0)


def test_optimizers_match_oracle(A):
    d = golden("optim")
    for clip in (0, 1):
        g = d["g"].copy()
        A.norm_clip_cpp(bool(clip), g, 1.0)
        for name, fn in (("nadam", A.Nadam_cpp), ("adam", A.Adam_cpp)):
            m, v, p = d["m"].copy(), d["v"].copy(), d["para"].copy()
            assert fn(3.0, 0.01, 0.9, 0.999, 1e-8, m, v, g, p)
            exp = d[f"{name}_clip{clip}"]
            P = g.size
            assert np.array_equal(m, exp[:P]) and np.array_equal(v, exp[P:2 * P])
            assert np.allclose(p, exp[2 * P:], rtol=0, atol=1e-15)
        nu, p = d["nu"].copy(), d["para"].copy()
        assert A.Nesterov_cpp(0.01, 0.5, nu, g, p)
        exp = d[f"nesterov_clip{clip}"]
        assert np.array_equal(nu, exp[:g.size]) and np.array_equal(p, exp[g.size:])
    # non-finite gradient -> False, parameters still updated (as the reference)
    g = np.array([np.nan, 1.0])
    m, v, p = np.zeros(2), np.zeros(2), np.zeros(2)
    assert A.Nadam_cpp(1.0, 0.1, 0.9, 0.999, 1e-8, m, v, g, p) is False


def test_norm_clip_edge_cases(A):
    for g0, cl in (([0.0, 0.0], 0.5), ([np.inf, 1.0], 1.0), ([3.0, 4.0], 5.0), ([3.0, 4.0], 4.9)):
        a = np.array(g0)
        b = np.array(g0)
        A.norm_clip_cpp(True, a, cl)
        O.norm_clip_cpp(True, b, cl)
        assert np.array_equal(a, b, equal_nan=True)
    a = np.array([3.0, 4.0])
    A.norm_clip_cpp(False, a, 1.0)
    assert np.array_equal(a, [3.0, 4.0])


@pytest.mark.parametrize("knots", [[-1, 1], [-0.3, 0.2, -1, 1], [0.1, 0.1, -1, 1, 0.5]])
def test_ncs_basis_matches_oracle(A, knots):
    x = np.linspace(-1.2, 1.2, 57)
    for f, g in ((A.ncs_basis, O.ncs_basis), (A.ncs_basis_deriv, O.ncs_basis_deriv)):
        a = f(x, np.array(knots, dtype=float))
        b = g(x, np.array(knots, dtype=float))
        assert a.shape == b.shape
        assert np.allclose(a, b, rtol=1e-14, atol=1e-15)
    # exact zeros below the lowest knot survive (Q7 branch)
    assert np.sum(A.ncs_basis(x, np.array(knots, float))[:, 1:] == 0) > 0


def test_normalize_train_test_match_oracle(A):
    rng = np.random.default_rng(4)
    n = 41
    X = np.asfortranarray(np.column_stack([rng.normal(size=n), (rng.random(n) < .5) * 3.0 + 2.0,
                                           rng.uniform(0, 5, n)]))
    Z = np.asfortranarray(rng.normal(3, 2, (n, 1)))
    y = rng.normal(10, 3, n)
    Xa, Za, ya = X.copy(order="F"), Z.copy(order="F"), y.copy()
    Xb, Zb, yb = X.copy(order="F"), Z.copy(order="F"), y.copy()
    ma = A.normalize_train(ya, Xa, Za)
    mb = O.normalize_train(yb, Xb, Zb)
    assert np.allclose(ma, mb, rtol=1e-13)
    assert np.allclose(Xa, Xb, rtol=1e-13) and np.allclose(Za, Zb, rtol=1e-13)
    assert np.allclose(ya, yb, rtol=1e-12)
    # binary X column 1: flag in row 2, but its location went to row 1
    # (moments(i, 0), quirk kept), where column 0's median then overwrote it
    assert mb[2, 2] == 1 and mb[2, 0] == 0.0 and mb[1, 0] != 2.0
    assert set(np.unique(Xb[:, 1])) == {0.0, 1.0}
    Xt, Zt = X[:5].copy(order="F"), Z[:5].copy(order="F")
    Xu, Zu = Xt.copy(order="F"), Zt.copy(order="F")
    A.normalize_test(Xt, Zt, ma)
    O.normalize_test(Xu, Zu, mb)
    assert np.allclose(Xt, Xu) and np.allclose(Zt, Zu)


def test_trajectory_host_preprocessing_matches_golden(A):
    """normalize_train + ns basis of the README config through the C ABI."""
    d = golden("traj_SE")
    y, X, Z = d["yraw"].copy(), np.asfortranarray(d["Xraw"].copy()), np.asfortranarray(d["Zraw"].copy())
    mom = A.normalize_train(y, X, Z)
    assert np.allclose(mom, d["moments"], rtol=1e-12)
    assert np.allclose(X, d["X"], rtol=1e-12) and np.allclose(y, d["y"], rtol=1e-12)
    assert np.allclose(A.ncs_basis(Z[:, 0], d["knots"]), d["basis"], rtol=1e-12, atol=1e-14)
