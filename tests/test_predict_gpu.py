"""GPU parity tests of the device-resident prediction path
(ace_model_predict / ace_model_predict_marginal / ace_model_apply_inverse):
the resident inverse of the last para_update (Q6: theta_{T-1}) with kernels
at the caller's theta_T, against the oracle's pred_cpp / pred_marginal_cpp
(src/pred_cpp.cpp:8-126) fed the oracle's own kernels and inverse.

Tolerances (north star 1e-6 relative fp64): map relative 1e-6; the
variance is |K_xx - tmp K_xX^T (+ e^sigma)|, a difference of terms up to
cond x larger than the result under Q6's theta mix, so it is held to a
fraction of the cancelled terms std_y^2 (|K_xx,rr| + q_r) -- VAR_TOL, and the
ATE/ATT/ATU intervals map -+ 1.96 sd to CI_TOL of |map| + 1.96 sd, both set
at <= 5x the largest error measured (profiles/r06_error_table.txt).
"""
import numpy as np

from conftest import record_error, run_child
import pytest
from test_gpu import close

pytestmark = pytest.mark.gpu

# Round 6: the variance and interval bounds at <= 5x the largest error
# measured (profiles/r06_error_table.txt): variances 3.5e-10 of the terms
# their quadratic forms cancel, ATE/ATT/ATU intervals 5.2e-8 of |map| + 1.96 sd
# (round 5: 1e-6 of each, the north star's tolerance)
VAR_TOL = 1.5e-9
CI_TOL = 2.5e-7


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.default_context()
    return pkg


@pytest.fixture(scope="module")
def O():
    from oracle import ace_oracle
    return ace_oracle


def _fit_state(O, kernel, n, p, B, seed, sharded=False, world=1, A=None, mix=True):
    """A model whose resident inverse is at theta_{T-1} = th, and theta_T:
    th + 0.02 (mix, Q6), or th itself (then the marginal posterior
    covariance is positive semidefinite and ATE/ATT/ATU's square roots exist,
    which the Q6 mix does not guarantee -- the reference then returns NaN)."""
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th, sy = make_problem(n, p, B, seed=seed)
    m = A.DeviceModel(kernel, n, p, B, world=world, sharded=sharded)
    m.set_data(y, X, Z, sy)
    th_prev = th.copy()
    m.para_update(2, th_prev)             # resident inverse at theta_{T-1}
    th_now = th + 0.02 if mix else th.copy()  # kernels at theta_T (Q6)
    th_now[1] = 0.13
    inv = O.invkernel_cpp(O.KERNELS[kernel][0](X, Z, th)["full"], th[0])["inv"]
    return m, y, X, Z, th_now, sy, inv


def _test_points(p, B, nx, seed):
    from additivecausalexpansion_amd.synthetic import make_problem
    _, X2, Z2, _, _ = make_problem(nx, p, B, seed=seed)
    return X2, Z2


def _var_terms(O, kernel, X2, Z2, th, sy, inv, K_xX, extra):
    kxx = np.diag(O.KERNELS[kernel][0](X2, Z2, th)["full"])
    q = np.abs(np.sum((K_xX @ inv) * K_xX, axis=1))
    return sy ** 2 * (np.abs(kxx) + q + extra)


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
@pytest.mark.parametrize("n,p,B,nx", [(300, 3, 5, 70), (700, 20, 10, 257), (130, 1, 1, 9)])
def test_device_predict_matches_oracle(A, O, kernel, n, p, B, nx):
    m, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=n, A=A)
    X2, Z2 = _test_points(p, B, nx, seed=n + 1)
    sym, cross = O.KERNELS[kernel][0], O.KERNELS[kernel][1]
    K_xX = cross(X2, X, Z2, Z, th)["full"]
    ref = O.pred_cpp(y, th[0], th[1], inv, K_xX, sym(X2, Z2, th)["full"], 0.3, 1.7)
    got = m.predict(th, X2, Z2, 0.3, 1.7)
    close(got["map"], ref["map"])
    close(got["ci"], ref["ci"], 1e-6, 1e-8)
    terms = _var_terms(O, kernel, X2, Z2, th, 1.7, inv, K_xX, np.exp(th[0]))
    record_error("predict var: max |err| / terms", np.max(np.abs(got["var"] - ref["var"]) / terms), VAR_TOL)
    assert np.all(np.abs(got["var"] - ref["var"]) <= VAR_TOL * terms)


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
@pytest.mark.parametrize("B", [1, 2, 6])
def test_device_predict_marginal_ate_matches_oracle(A, O, kernel, B):
    n, p, nx = 400, 3, 150
    m, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=5 + B, A=A, mix=False)
    X2, Z2 = _test_points(p, B, nx, seed=77)
    dZ2 = np.asfortranarray(Z2 * 0.7 + 0.1)  # a stand-in derivative basis
    zx = (np.arange(nx) % 3 == 0).astype(float)
    sym, cross = O.KERNELS[kernel][0], O.KERNELS[kernel][1]
    Km_xX = cross(X2, X, dZ2, Z, th)["elements"]
    Km_xx = sym(X2, dZ2, th)["elements"]
    ref = O.pred_marginal_cpp(y, zx, th[0], th[1], inv, Km_xX, Km_xx, 0.3, 1.7, 0.8, True)
    got = m.predict_marginal(th, X2, dZ2, zx, 1.7, 0.8, True)
    close(got["map"], ref["map"])
    sl = slice(1, B) if B > 1 else slice(0, 1)
    KmX = Km_xX[:, :, sl].sum(axis=2)
    kxx = np.diag(Km_xx[:, :, sl].sum(axis=2))
    q = np.abs(np.sum((KmX @ inv) * KmX, axis=1))
    terms = (1.7 / 0.8) ** 2 * (np.abs(kxx) + q)
    record_error("marginal var: max |err| / terms", np.max(np.abs(got["var"] - ref["var"]) / terms), VAR_TOL)
    assert np.all(np.abs(got["var"] - ref["var"]) <= VAR_TOL * terms)
    for k in ("ate", "att", "atu"):
        close(got[k]["map"], ref[k]["map"])
        close(got[k]["var"], ref[k]["var"], 1e-6, 1e-10)
        # ci = map -+ 1.96 sd: where the two nearly cancel (|ci| << |map|), a
        # bound relative to ci itself is below the inverse's rounding; bound
        # it by the terms it is formed from (as the variance check above)
        sd = np.sqrt(abs(ref[k]["var"]))
        tol = CI_TOL * (abs(ref[k]["map"]) + 1.96 * sd)
        record_error(f"{k} ci: max |err| / (|map| + 1.96 sd)",
                     np.max(np.abs(got[k]["ci"] - ref[k]["ci"])) / (abs(ref[k]["map"]) + 1.96 * sd), CI_TOL)
        assert np.all(np.abs(got[k]["ci"] - ref[k]["ci"]) <= tol), (k, got[k]["ci"], ref[k]["ci"], tol)
    plain = m.predict_marginal(th, X2, dZ2, zx, 1.7, 0.8, False)
    assert "ate" not in plain and np.array_equal(plain["map"], got["map"])


def _check_avg_edge(got, ref, case):
    """ATE/ATT/ATU with a zero treated (ntx = 0) or untreated (nux = 0) count:
    the reference divides doubles by the unsigned count, so its outputs are
    the C results (src/pred_cpp.cpp:95-110): 0/0 = NaN for the empty group's
    sd, NaN for ATT's map when ntx = 0 (and so for ATU's, via NaN * 0), and a
    non-finite ATU map when nux = 0 (0/0 or +-tiny/0, by summation rounding)."""
    close(got["ate"]["map"], ref["ate"]["map"])
    close(got["ate"]["var"], ref["ate"]["var"], 1e-6, 1e-10)
    if case == "none_treated":
        for k in ("map", "var"):
            assert np.isnan(got["att"][k]) and np.isnan(ref["att"][k])
        assert np.all(np.isnan(got["att"]["ci"])) and np.all(np.isnan(ref["att"]["ci"]))
        assert np.isnan(got["atu"]["map"]) and np.isnan(ref["atu"]["map"])
        close(got["atu"]["var"], ref["atu"]["var"], 1e-6, 1e-10)
    else:
        close(got["att"]["map"], ref["att"]["map"])
        close(got["att"]["var"], ref["att"]["var"], 1e-6, 1e-10)
        assert not np.isfinite(got["atu"]["map"]) and not np.isfinite(ref["atu"]["map"])
        assert np.isnan(got["atu"]["var"]) and np.isnan(ref["atu"]["var"])
        assert np.all(~np.isfinite(got["atu"]["ci"])) and np.all(~np.isfinite(ref["atu"]["ci"]))


@pytest.mark.parametrize("case", ["none_treated", "all_treated"])
@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_predict_marginal_empty_group_semantics(A, O, kernel, case):
    """Z_x all 0 (ntx = 0) or all 1 (nux = 0): the device-resident
    predict_marginal and the pred_marginal_cpp ABI reproduce the reference's
    inf / NaN outputs instead of raising."""
    n, p, B, nx = 300, 3, 4, 64
    m, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=31, A=A, mix=False)
    X2, Z2 = _test_points(p, B, nx, seed=32)
    dZ2 = np.asfortranarray(Z2 * 0.5 + 0.2)
    zx = np.zeros(nx) if case == "none_treated" else np.ones(nx)
    sym, cross = O.KERNELS[kernel][0], O.KERNELS[kernel][1]
    Km_xX = cross(X2, X, dZ2, Z, th)["elements"]
    Km_xx = sym(X2, dZ2, th)["elements"]
    ref = O.pred_marginal_cpp(y, zx, th[0], th[1], inv, Km_xX, Km_xx, 0.3, 1.7, 0.8, True)
    got = m.predict_marginal(th, X2, dZ2, zx, 1.7, 0.8, True)
    close(got["map"], ref["map"])
    _check_avg_edge(got, ref, case)
    abi = A.pred_marginal_cpp(y, zx, th[0], th[1], inv, Km_xX, Km_xx, 0.3, 1.7, 0.8, True)
    close(abi["map"], ref["map"])
    _check_avg_edge(abi, ref, case)


def test_device_predict_chunks_and_padding(A, O):
    """nx above one 8192-point chunk plus a ragged tail, n not a multiple of
    the 128-row product tile."""
    kernel, n, p, B, nx = "SE", 333, 2, 3, 8192 + 77
    m, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=3, A=A)
    X2, Z2 = _test_points(p, B, nx, seed=4)
    K_xX = O.KERNELS[kernel][1](X2, X, Z2, Z, th)["full"]
    tmp = K_xX @ inv  # src/pred_cpp.cpp:19-28 without the nx x nx K_xx
    mp = 0.5 + 1.5 * (tmp @ (y - th[1]) + th[1])
    # diag(K_xx): r2 = 0, slice 0 exp(lam_0) plus z^2 exp(lam_b) (SE, z != 0)
    kxx = np.exp(th[2]) + sum(Z2[:, b - 1] ** 2 * np.exp(th[2 + b]) for b in range(1, B))
    q = np.sum(tmp * K_xX, axis=1)
    var = (1.5 * np.sqrt(np.abs(kxx - q + np.exp(th[0])))) ** 2
    got = m.predict(th, X2, Z2, 0.5, 1.5)
    close(got["map"], mp)
    assert np.all(np.abs(got["var"] - var) <= 1e-6 * 1.5 ** 2 * (np.abs(kxx) + np.abs(q) + 1))


@pytest.mark.parametrize("world", [1, 3])
def test_sharded_predict_matches_single(A, O, world):
    """Sharded models multiply by the inverse entries each rank stores and
    all-reduce the per-point sums: same result as one GPU."""
    kernel, n, p, B, nx = "Matern32", 1100, 4, 5, 300
    single, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=21, A=A, mix=False)
    sh, *_ = _fit_state(O, kernel, n, p, B, seed=21, sharded=True, world=world, A=A, mix=False)
    X2, Z2 = _test_points(p, B, nx, seed=22)
    a, b = single.predict(th, X2, Z2, 0.1, 1.3), sh.predict(th, X2, Z2, 0.1, 1.3)
    # the sharded sweep's operand order differs: inverses agree to ~1e-10 of
    # their scale (test_shard_gpu), the predictions to 1e-9 of theirs
    close(b["map"], a["map"], 1e-8, 1e-9)
    close(b["var"], a["var"], 1e-7, 1e-9)
    zx = (np.arange(nx) % 2).astype(float)
    a = single.predict_marginal(th, X2, Z2, zx, 1.3, 0.9, True)
    b = sh.predict_marginal(th, X2, Z2, zx, 1.3, 0.9, True)
    close(b["map"], a["map"], 1e-8, 1e-9)
    for k in ("ate", "att", "atu"):
        close(b[k]["var"], a[k]["var"], 1e-7, 1e-12)
    V = np.random.default_rng(0).normal(size=(n, 5))
    close(sh.apply_inverse(V), single.apply_inverse(V), 1e-8, 1e-9)


def test_sharded_rccl_world1_predict(A, O):
    kernel, n, p, B, nx = "SE", 700, 3, 4, 120
    single, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=8, A=A)
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th0, sy = make_problem(n, p, B, seed=8)
    sh = A.DeviceModel(kernel, n, p, B, world=1, rank=0, unique_id=A.comm_unique_id(),
                       sharded=True)
    sh.set_data(y, X, Z, sy)
    sh.para_update(2, th0.copy())
    X2, Z2 = _test_points(p, B, nx, seed=9)
    c0 = sh.comm_calls()["allreduce"]
    close(sh.predict(th, X2, Z2, 0.0, 1.0)["map"], single.predict(th, X2, Z2, 0.0, 1.0)["map"],
          1e-8, 1e-9)
    c1 = sh.comm_calls()["allreduce"]
    V = np.random.default_rng(1).normal(size=(n, 3))
    close(sh.apply_inverse(V), single.apply_inverse(V), 1e-8, 1e-9)
    # the rank-partial products are summed by RCCL all-reduces (world 1 included)
    assert c1 > c0 and sh.comm_calls()["allreduce"] > c1


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_apply_inverse_matches_oracle(A, O, kernel):
    n, p, B = 513, 3, 4
    m, y, X, Z, th, sy, inv = _fit_state(O, kernel, n, p, B, seed=2, A=A)
    V = np.random.default_rng(5).normal(size=(n, 70))
    close(m.apply_inverse(V), inv @ V, 1e-9, 1e-9)
    v = np.random.default_rng(6).normal(size=n)
    close(m.apply_inverse(v), inv @ v, 1e-9, 1e-9)


def test_predict_before_para_update_raises(A):
    m = A.DeviceModel("SE", 100, 2, 3)
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th, sy = make_problem(100, 2, 3, seed=1)
    m.set_data(y, X, Z, sy)
    with pytest.raises(A.AceError, match="ARG"):
        m.predict(th, X[:5], Z[:5], 0.0, 1.0)


_TRI_SNIPPET = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
y, X, Z, th, sy = make_problem({n}, 8, 6, seed=41)
m = A.DeviceModel({kernel!r}, {n}, 8, 6)
m.set_data(y, X, Z, sy)
m.para_update(2, th.copy())
th2 = th + 0.01
_, X2, Z2, _, _ = make_problem({nx}, 8, 6, seed=42)
p = m.predict(th2, X2, Z2, 0.2, 1.4)
zx = (np.arange({nx}) % 2 == 0).astype(float)
q = m.predict_marginal(th2, X2, np.asfortranarray(0.5 * Z2), zx, 1.4, 0.9, True)
out = [p["map"], p["var"], q["map"], q["var"]]
for k in ("ate", "att", "atu"):
    out += [np.atleast_1d(q[k]["map"]), np.atleast_1d(q[k]["var"])]
np.save({out!r}, np.concatenate([np.ravel(v) for v in out]))
"""


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_triangular_variance_matches_full_product(tmp_path, kernel):
    """The single-GPU prediction's triangular form (ACE_PRED_TRI=1, default:
    Y = L K_xX^T with L the strictly lower part of A^-1, d = K (2Y + D K),
    the map from A^-1 w, u_j = A^-1 s_j) against the full symmetric product
    (ACE_PRED_TRI=0): predict and predict_marginal with ATE/ATT/ATU at
    n = 2300 (a diagonal block cut by n), nx = 700, to 1e-9 of the scale of
    each output (the two forms only round differently)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for v in ("0", "1"):
        out = str(tmp_path / f"p{v}.npy")
        env = dict(os.environ, ACE_PRED_TRI=v)
        run_child(_TRI_SNIPPET.format(root=root, n=2300, nx=700, kernel=kernel, out=out), env=env, timeout=100)
        outs[v] = np.load(out)
    a, b = outs["0"], outs["1"]
    assert a.shape == b.shape and np.all(np.isfinite(a) == np.isfinite(b))
    f = np.isfinite(a)
    scale = np.max(np.abs(a[f]))
    assert np.max(np.abs(a[f] - b[f])) <= 1e-9 * scale
