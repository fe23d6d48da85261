"""The extended-precision referee (tests/referee_ld.py) and its fixtures
(tests/golden/referee_*.npz, tests/golden/make_referee.py) against the fp64
oracle: the oracle restates the reference's fp64 arithmetic (eigen-inverse
and all), the referee the same mathematics in 80-bit; they must agree to the
fp64 oracle's own rounding (~cond(A) eps, measured <= 2e-12 here), which
pins the referee to the oracle before the GPU test holds the kernels to it."""
import numpy as np
import pytest
from conftest import golden, golden_names

from referee_ld import para_update_ld

ALL = golden_names("referee_")
# fixtures with stored inputs (the multi-group n = 2600 fixture stores a seed
# and an input digest instead; its check is the GPU test and the digest below)
NAMES = [n for n in ALL if "gen" not in golden(n)]


def _ld(d, key):
    return d[key + "_hi"].astype(np.longdouble) + d[key + "_lo"]


def _rel(a, ref, floor):
    a = np.asarray(a, dtype=np.longdouble)
    return float(np.max(np.abs(a - ref) / (np.abs(ref) + floor * np.max(np.abs(ref)))))


def test_referee_fixtures_cover_every_feature_bucket():
    assert {"referee_p%d" % p for p in (3, 8, 12, 16, 20, 24, 32, 48, 64)} <= set(NAMES)
    assert "referee_smoke" in NAMES


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_fp64_oracle_matches_referee(name, kernel):
    from oracle import ace_oracle as O
    d = golden(name)
    y, X, Z, th, sy = d["y"], d["X"], d["Z"], d["theta"], float(d["std_y"][0])
    B = Z.shape[1] + 1
    sym, _, grad = O.KERNELS[kernel]
    t = th.copy()
    K = sym(X, Z, t)
    inv = O.invkernel_cpp(K["full"], t[0])
    t[1] = O.mu_solution_cpp(y, inv["inv"])
    st = np.zeros(2)
    g = grad(y, X, Z, K["full"], K["elements"], inv["inv"], inv["eigenval"], t, st, B, sy)
    assert _rel(g, _ld(d, kernel + "_g"), 1e-9) < 1e-11
    assert _rel(st, _ld(d, kernel + "_st"), 0.0) < 1e-12
    assert _rel([t[1]], _ld(d, kernel + "_mu"), 0.0) < 1e-10


def test_multigroup_referee_inputs_regenerate():
    """The n = 2600 fixture's inputs come from the seeded generator: their
    digest is the one stored beside the referee's outputs."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    from make_referee import input_digest
    from additivecausalexpansion_amd.synthetic import make_problem
    big = [n for n in ALL if n not in NAMES]
    assert big == ["referee_p20_n2600"]
    d = golden(big[0])
    n, p, B, seed = (int(v) for v in d["gen"])
    assert n >= 2600 and -(-n // 256) >= 3 * 3  # at least three groups of Z = 3 steps
    assert input_digest(*make_problem(n, p, B, seed=seed)) == str(d["input_sha256"][0])
    for kernel in ("SE", "Matern32"):
        assert d[kernel + "_g_hi"].size == 2 + B * (p + 1)


def test_referee_fixture_regenerates():
    """The smallest fixture recomputed by the referee: the committed values
    are what tests/golden/make_referee.py's arithmetic gives."""
    d = golden("referee_p3")
    for kernel in ("SE", "Matern32"):
        g, st, mu = para_update_ld(kernel, d["y"], d["X"], d["Z"], d["theta"], float(d["std_y"][0]))
        assert np.array_equal(np.asarray(g, dtype=np.float64), d[kernel + "_g_hi"])
        assert np.array_equal(np.asarray(st, dtype=np.float64), d[kernel + "_st_hi"])
