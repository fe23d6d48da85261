"""Pins the full-size checker (tests/torch_ref.py, the PyTorch fp64
restatement the C2 full-size GPU test compares against) to the oracle at
small n on the CPU: gradient, stats and mu to 1e-10 relative."""
import numpy as np
import pytest


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
@pytest.mark.parametrize("it", [1, 2])
@pytest.mark.parametrize("n,p,B", [(300, 3, 5), (257, 20, 10), (70, 1, 1)])
def test_torch_ref_matches_oracle(kernel, it, n, p, B):
    torch = pytest.importorskip("torch")
    import torch_ref
    from additivecausalexpansion_amd.synthetic import make_problem
    from oracle import ace_oracle as O
    torch.set_num_threads(4)
    y, X, Z, th, sy = make_problem(n, p, B, seed=n + it)
    th = th + 0.03 * np.arange(th.shape[0]) / th.shape[0]
    r = torch_ref.para_update(kernel, y, X, Z, th, sy, it, dev="cpu", chunk=100)
    sym, _, grad = O.KERNELS[kernel]
    t = th.copy()
    Kl = sym(X, Z, t)
    inv = O.invkernel_cpp(Kl["full"], t[0])
    if it == 1:
        t[1] = O.mu_solution_cpp(y, inv["inv"])
        assert r["mu"] == pytest.approx(t[1], rel=1e-10, abs=1e-13)
    st = np.zeros(2)
    g = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], t, st, B, sy)
    scale = np.abs(g).max()
    assert np.all(np.abs(r["grad"] - g) <= 1e-10 * np.abs(g) + 1e-12 * scale)
    assert np.allclose(r["stats"], st, rtol=1e-10, atol=0)
    assert r["logdet"] == pytest.approx(float(np.sum(np.log(inv["eigenval"]))), rel=1e-12)
