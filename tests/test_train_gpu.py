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
    subprocess.run([sys.executable, "-c", _LOOP.format(root=ROOT, kernel=kernel, tol=tol, out=out)],
                   env=env, check=True, timeout=100)
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
