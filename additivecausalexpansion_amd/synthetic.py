"""Seeded synthetic inputs for the benchmark configurations
and the README example shape (README.md:41-51).  numpy's PCG64 generator is
used; R RNG parity is not required (no reference outputs exist to match)."""
from __future__ import annotations

import math

import numpy as np

CONFIGS = {
    # name: (n, p, B, kernel)    BASELINE.json configs[1..4]
    "C1": (4096, 10, 6, "SE"),
    "C2": (16384, 20, 10, "Matern32"),
    "C3": (32768, 32, 12, "SE"),
    "C4": (65536, 50, 16, "Matern32"),
}


def _ncs(x, knots):
    """Natural cubic spline design (same algebra as src/ncs_basis_cpp.cpp)."""
    kn = np.unique(knots)
    K = kn.shape[0]
    f = lambda k: (x > k) * (x - k) ** 3  # noqa: E731
    d = np.zeros((x.shape[0], K))
    d[:, K - 1] = f(kn[K - 1])
    for i in range(K - 1):
        d[:, i] = (f(kn[i]) - d[:, K - 1]) / (kn[K - 1] - kn[i])
    d[:, K - 1] = 0
    N = np.zeros((x.shape[0], K - 1))
    for i in range(K - 2):
        N[:, i] = d[:, i] - d[:, K - 2]
    N[:, K - 2] = -d[:, K - 2]
    return np.column_stack([x, N])


def make_problem(n, p, B, seed=0):
    """Returns (y, X, Zbasis, theta, std_y) in the post-normalisation domain:
    X ~ U(-1,1), z ~ N(0,1) median-centred / max-abs scaled, ns basis with
    B-3 internal type-7 quantile knots (B-1 columns), y = sin(3 x1) + x2 z +
    N(0, 0.1^2) standardised, theta = [log 0.1, 0, 0 x B, log 20 x B p]."""
    rng = np.random.default_rng(seed)
    X = np.asfortranarray(rng.uniform(-1.0, 1.0, size=(n, p)))
    z = rng.normal(size=n)
    z = z - np.median(z)
    z = z / np.max(np.abs(z))
    nk = B - 3
    if nk >= 1:
        ik = np.quantile(z, np.arange(1, nk + 1) / (nk + 1), method="linear")
        Zb = _ncs(z, np.concatenate([ik, [-1.0, 1.0]]))
    elif B == 3:
        Zb = np.column_stack([z, z ** 2])
    elif B == 2:
        Zb = z.reshape(n, 1)
    else:
        Zb = np.zeros((n, 0))
    Zb = np.asfortranarray(Zb[:, :B - 1])
    x2 = X[:, 1] if p > 1 else X[:, 0]
    y = np.sin(3 * X[:, 0]) + x2 * z + rng.normal(scale=0.1, size=n)
    y = (y - y.mean())
    std_y = float(np.std(y, ddof=1))
    y = y / std_y
    theta = np.concatenate([[math.log(0.1), 0.0], np.zeros(B), np.full(B * p, math.log(20.0))])
    return y, X, Zb, theta, std_y


def readme_data(seed=1234, n=300):
    """README.md:41-51 shape: x ~ U(1,2), x2 ~ U(-1,1), z ~ N(exp(x)-14, 1),
    y = sqrt(x) + 3 x2 ((z+8)^2 - 2z) + N(0,1).  Returns raw (y, X, Z)."""
    rng = np.random.default_rng(seed)
    x = rng.uniform(1, 2, n)
    x2 = rng.uniform(-1, 1, n)
    z = rng.normal(np.exp(x) - 14, 1)
    y = np.sqrt(x) + x2 * 3 * ((z + 8) ** 2 - 2 * z) + rng.normal(0, 1, n)
    return y, np.column_stack([x, x2]), z.reshape(n, 1)
