"""The fused model's gradient, statistics and mu at every compiled feature
bucket, against the extended-precision referee (tests/referee_ld.py via
tests/golden/referee_*.npz) rather than the fp64 oracle, whose own rounding
(<= 2e-12 here, tests/test_referee_cpu.py) would otherwise hide a kernel's.

The bound is 1e-10 relative with the smoke's 1e-9 * max floor: fifty times
the fp64 oracle's error, and ten times below the 8.6e-10 the round-4 kernels
reached on the smoke problem ("numeric drift"), so a change
that is claimed bit-identical or ulp-level is checked at every PM bucket,
not only at p = 20."""
import numpy as np
import pytest
from conftest import golden, golden_names

pytestmark = pytest.mark.gpu

GRAD_TOL = 1e-10
STATS_TOL = 1e-12
MU_TOL = 1e-10


def _ld(d, key):
    return d[key + "_hi"].astype(np.longdouble) + d[key + "_lo"]


def _rel(a, ref, floor):
    a = np.asarray(a, dtype=np.longdouble)
    den = np.abs(ref) + floor * np.max(np.abs(ref))
    e = np.abs(a - ref) / den
    return float(np.max(e)), int(np.argmax(e))


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.default_context()
    return pkg


@pytest.mark.parametrize("name", golden_names("referee_"))
@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_fused_model_matches_extended_precision_referee(A, name, kernel):
    d = golden(name)
    y, X, Z, th, sy = d["y"], d["X"], d["Z"], d["theta"], float(d["std_y"][0])
    n, p = X.shape
    B = Z.shape[1] + 1
    m = A.DeviceModel(kernel, n, p, B)
    m.set_data(y, X, Z, sy)
    g, st, mu = m.para_update(1, th.copy())
    m.close()
    eg, ig = _rel(g, _ld(d, kernel + "_g"), 1e-9)
    es, _ = _rel(st, _ld(d, kernel + "_st"), 0.0)
    em, _ = _rel([mu], _ld(d, kernel + "_mu"), 0.0)
    assert eg <= GRAD_TOL, f"gradient rel err {eg:.2e} at index {ig} (P = {g.size})"
    assert es <= STATS_TOL, f"stats rel err {es:.2e}"
    assert em <= MU_TOL, f"mu rel err {em:.2e}"
