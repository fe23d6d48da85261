"""The device-fused training loop (ace_model_train on an unsharded model):
theta, the optimizer moments and the stats matrix stay in HBM, and each
iteration is the evaluation pipeline with tables built from the device theta
plus one k_train_step (compose_grad + stats + norm clip + optimizer + mu
overwrite + convergence test; csrc/ace_train.hip).  The reference loop is
R/main_ace.R:213-235 with R/optimizer_classes.R:54-63 and
src/optimizer_cpp.cpp:23-42.

Checked against the golden 20-iteration README trajectory (not against
another caller of the same library), plus the properties of the loop's host
syncs: the sync cadence (ACE_TRAIN_SYNC) never changes a result.
"""
import os
import subprocess
import sys

import numpy as np

from conftest import run_child
import pytest
from conftest import golden
from test_gpu import close

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.default_context()
    return pkg


@pytest.fixture(scope="module")
def O():
    from oracle import ace_oracle
    return ace_oracle


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_device_loop_matches_golden_trajectory(A, O, kernel):
    """README config (n=300, d=2, ns n.knots=2, Nadam lr 0.01, norm clip 1),
    20 iterations entirely on the device.  Tolerances as the host-driven
    free run of tests/test_gpu.py::test_training_trajectory_matches_golden
    (Nadam amplifies last-bit gradient differences along the loop)."""
    d = golden(f"traj_{kernel}")
    y, X, Bm = d["y"], np.asfortranarray(d["X"]), np.asfortranarray(d["basis"])
    B = Bm.shape[1] + 1
    sy = float(d["moments"][0, 1])
    m = A.DeviceModel(kernel, 300, 2, B)
    m.set_data(y, X, Bm, sy)
    th = d["theta0"].copy()
    stats, it, conv = m.train(th, "Nadam", 0.01, 0.0, 0.9, 0.999, True, 1.0, maxiter=20, tol=-1.0)
    assert it == 20 and not conv
    close(stats[:, 1:21].T, d["stats"], 1e-6, 1e-9)
    close(th, d["thetas"][19], 1e-5, 1e-9)
    assert np.all(stats[:, 0] == 0.0)
    # final column: get_train_stats at theta_T (R/kernel_SE_R6.R:63-74)
    sym = O.kernmat_SE_symmetric_cpp if kernel == "SE" else O.kernmat_Matern32_symmetric_cpp
    K = sym(X, Bm, th)
    inv = O.invkernel_cpp(K["full"], th[0])
    ref = O.stats_cpp(y, K["full"], inv["inv"], inv["eigenval"], th[1], sy)
    close(stats[:, 21], ref, 1e-6, 1e-9)


_LOOP = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import readme_data
y, X, Z = readme_data(seed=11, n=240)
f = A.ace_train(y, X, Z, kernel={kernel!r}, basis="cubic", n_knots=2, optimizer="Adam",
                maxiter=25, tol={tol!r}, learning_rate=0.03, norm_clip=True, verbose=False,
                native_loop=True)
np.savez({out!r}, stats=f["train_stats"]["stats"], theta=f["Kernel"].parameters,
         conv=f["train_stats"]["convergence"])
"""


def _loop(tmp_path, kernel, tol, sync):
    out = str(tmp_path / f"t{sync}_{tol}.npz")
    env = dict(os.environ, ACE_TRAIN_SYNC=str(sync))
    run_child(_LOOP.format(root=ROOT, kernel=kernel, tol=tol, out=out), env=env, timeout=100)
    return np.load(out)


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_sync_cadence_is_neutral(A, tmp_path, kernel):
    """Iterations enqueued after the converged one run but change nothing:
    syncing every iteration, every 4th (default) and every 7th give the same
    stopping iteration, stats and theta bit for bit.  The tolerance is picked
    from a full run so that the loop stops at an iteration that is a multiple
    of neither cadence."""
    # ace.train returns the stats of iterations 2..it and the final column
    # (train.py, as R/main_ace.R); the test at iteration j > 3 is
    # |evidence_j - evidence_{j-1}| < tol
    ev = _loop(tmp_path, kernel, -1.0, 1)["stats"][1, :-1]  # iterations 2..25
    d = {j: abs(ev[j - 2] - ev[j - 3]) for j in range(3, 26)}
    tol = None
    for j in range(5, 25):
        lo = min(d[i] for i in range(4, j))
        if j % 4 and j % 7 and d[j] < lo:
            tol = float(0.5 * (d[j] + lo))
            break
    assert tol is not None, d
    outs = {k: _loop(tmp_path, kernel, tol, k) for k in (1, 4, 7)}
    s1 = outs[1]["stats"]
    assert outs[1]["conv"] and s1.shape[1] == j  # stopped at iteration j
    for k in (4, 7):
        assert np.array_equal(outs[k]["stats"], s1)
        assert np.array_equal(outs[k]["theta"], outs[1]["theta"])


_FIT = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd import native
from additivecausalexpansion_amd.synthetic import make_problem
n, p, B, nx = 260, 2, 4, 90
y, X, Z, th, sy = make_problem(n, p, B, seed=11)
m = A.DeviceModel({kernel!r}, n, p, B)
m.set_data(y, X, Z, sy)
t = th.copy()
if {mode!r} == "device":
    stats, it, conv = m.train(t, "Adam", 0.03, 0.0, 0.9, 0.999, True, 1.0, maxiter={maxiter},
                              tol={tol!r})
    ev = stats[1, 1:it + 1]
else:  # the host-driven loop: R/main_ace.R:215-227 over para_update + Optim$update
    m1, m2, ev = np.zeros_like(t), np.zeros_like(t), [0.0]
    for it in range(1, {maxiter} + 1):
        g, st, mu = m.para_update(it, t)
        native.norm_clip_cpp(True, g, 1.0)
        assert native.Adam_cpp(it, 0.03, 0.9, 0.999, 1e-8, m1, m2, g, t)
        t[1] = mu
        ev.append(st[1])
        if abs(ev[-1] - ev[-2]) < {tol!r} and it > 3:
            break
    ev = np.array(ev[1:])
_, X2, Z2, _, _ = make_problem(nx, p, B, seed=12)
zx = (np.arange(nx) % 3 == 0).astype(float)
pr = m.predict(t, X2, Z2, 0.3, 1.7)
pm = m.predict_marginal(t, X2, np.asfortranarray(0.7 * Z2 + 0.1), zx, 1.7, 0.8, True)
V = np.random.default_rng(3).normal(size=(n, 3))
avg = np.array([[pm[k]["map"], pm[k]["var"], *pm[k]["ci"]] for k in ("ate", "att", "atu")])
np.savez({out!r}, theta=t, it=it, ev=ev, inv=m.inverse(), ainv=m.apply_inverse(V),
         map=pr["map"], var=pr["var"], ci=pr["ci"], mmap=pm["map"], mvar=pm["var"], avg=avg)
"""


def _fit(tmp_path, kernel, mode, tol, maxiter, sync=1):
    out = str(tmp_path / f"{mode}_{sync}_{maxiter}_{tol}.npz")
    env = dict(os.environ, ACE_TRAIN_SYNC=str(sync))
    src = _FIT.format(root=ROOT, kernel=kernel, mode=mode, tol=tol, maxiter=maxiter, out=out)
    run_child(src, env=env, timeout=100)
    return np.load(out)


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_device_loop_keeps_last_update_inverse(A, O, tmp_path, kernel):
    """Q6 after a converged device loop: predict / predict_marginal (ATE,
    ATT, ATU) / apply_inverse / the inverse itself use the inverse of the
    LAST para_update, A(theta_{T-1})^-1, with kernels at the final theta_T
    (R/main_ace.R:215-227, R/kernel_SE_R6.R:37,75-97), whatever the host
    sync cadence.  The loop is made to stop at an iteration that is a
    multiple of neither 4 nor 7, so the cadences 4 and 7 enqueue iterations
    past the stopping one (their evaluations overwrite the resident inverse
    and the library re-runs the stopping one).  Checked:
    * cadences 1, 4, 7: every output bit-identical;
    * the oracle fed A(theta_{T-1})^-1 (theta_{T-1} from a run stopped by
      maxiter = T - 1, the same trajectory bit for bit) and kernels at
      theta_T, to 1e-6 -- and the inverse at theta_T would fail that;
    * the host-driven loop (para_update + host Adam): same stopping
      iteration and the same predictions to the loops' rounding difference."""
    full = _fit(tmp_path, kernel, "device", -1.0, 25)
    ev = full["ev"]  # evidence of iterations 1..25
    d = {j: abs(ev[j - 1] - ev[j - 2]) for j in range(2, 26)}
    tol, T = None, None
    for j in range(5, 25):
        lo = min(d[i] for i in range(4, j))
        if j % 4 and j % 7 and d[j] < lo:
            tol, T = float(0.5 * (d[j] + lo)), j
            break
    assert tol is not None, d
    outs = {k: _fit(tmp_path, kernel, "device", tol, 25, sync=k) for k in (1, 4, 7)}
    assert int(outs[1]["it"]) == T
    keys = ("theta", "inv", "ainv", "map", "var", "ci", "mmap", "mvar", "avg")
    for k in (4, 7):
        assert int(outs[k]["it"]) == T
        for key in keys:
            assert np.array_equal(outs[k][key], outs[1][key], equal_nan=True), (k, key)
    got = outs[1]
    th_T = got["theta"]
    th_prev = _fit(tmp_path, kernel, "device", -1.0, T - 1)["theta"]  # theta_{T-1}
    from additivecausalexpansion_amd.synthetic import make_problem
    n, p, B, nx = 260, 2, 4, 90
    y, X, Z, _, _ = make_problem(n, p, B, seed=11)
    _, X2, Z2, _, _ = make_problem(nx, p, B, seed=12)
    sym, cross = O.KERNELS[kernel][0], O.KERNELS[kernel][1]
    inv = O.invkernel_cpp(sym(X, Z, th_prev)["full"], th_prev[0])["inv"]
    inv_T = O.invkernel_cpp(sym(X, Z, th_T)["full"], th_T[0])["inv"]
    close(got["inv"], inv, 1e-6, 1e-9)
    assert np.max(np.abs(inv_T - inv)) > 1e-4 * np.max(np.abs(inv))  # the test can tell them apart
    V = np.random.default_rng(3).normal(size=(n, 3))
    close(got["ainv"], inv @ V, 1e-6, 1e-9)
    K_xX = cross(X2, X, Z2, Z, th_T)["full"]
    ref = O.pred_cpp(y, th_T[0], th_T[1], inv, K_xX, sym(X2, Z2, th_T)["full"], 0.3, 1.7)
    close(got["map"], ref["map"])
    close(got["ci"], ref["ci"], 1e-6, 1e-8)
    kxx = np.diag(sym(X2, Z2, th_T)["full"])
    terms = 1.7 ** 2 * (np.abs(kxx) + np.abs(np.sum((K_xX @ inv) * K_xX, axis=1)) + np.exp(th_T[0]))
    assert np.all(np.abs(got["var"] - ref["var"]) <= 1e-6 * terms)
    dZ2 = np.asfortranarray(0.7 * Z2 + 0.1)
    zx = (np.arange(nx) % 3 == 0).astype(float)
    Km_xX = cross(X2, X, dZ2, Z, th_T)["elements"]
    rm = O.pred_marginal_cpp(y, zx, th_T[0], th_T[1], inv, Km_xX, sym(X2, dZ2, th_T)["elements"],
                             0.3, 1.7, 0.8, True)
    close(got["mmap"], rm["map"])
    KmX = Km_xX[:, :, 1:].sum(axis=2)
    Kmx = sym(X2, dZ2, th_T)["elements"][:, :, 1:].sum(axis=2)
    tmp = KmX @ inv
    for j, (k, w) in enumerate((("ate", np.ones(nx)), ("att", zx), ("atu", 1.0 - zx))):
        a = got["avg"][j]
        close(a[0], rm[k]["map"])
        # the posterior quadratic form w^T (Kmx - tmp KmX^T) w cancels under
        # the Q6 theta mix: held to 1e-6 of the cancelled terms; a negative
        # form makes the reference's sqrt NaN, which must match
        terms = (1.7 / w.sum()) ** 2 * (abs(w @ Kmx @ w) + abs(w @ tmp @ KmX.T @ w))
        assert np.isnan(a[1]) == np.isnan(rm[k]["var"])
        if not np.isnan(a[1]):
            assert abs(a[1] - rm[k]["var"]) <= 1e-6 * terms, (k, a[1], rm[k]["var"])
    host = _fit(tmp_path, kernel, "host", tol, 25)
    assert int(host["it"]) == T
    # device vs host exp / clip-norm rounding, amplified over T Adam steps
    close(got["map"], host["map"], 1e-4, 1e-6)
    close(got["inv"], host["inv"], 1e-4, 1e-6)


def test_device_loop_nonfinite_keeps_theta(A):
    """A non-finite gradient ends the loop with ACE_ERR_NONFINITE (the
    optimizer classes' stop(), R/optimizer_classes.R:26-29); as in R, the
    parameters keep their value from before the failing update (theta[1] is
    the iteration-1 mean_solution, which para_update assigns before the
    optimizer runs: R/kernel_SE_R6.R:45)."""
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th, sy = make_problem(200, 2, 3, seed=2)
    m = A.DeviceModel("SE", 200, 2, 3)
    m.set_data(y, X, Z, sy)
    th = th.copy()
    th[0] = 800.0  # e^800 overflows on the diagonal: not positive definite
    before = th.copy()
    with pytest.raises(A.AceError, match="NONFINITE"):
        m.train(th, "Nadam", maxiter=5)
    assert np.array_equal(np.delete(th, 1), np.delete(before, 1))
