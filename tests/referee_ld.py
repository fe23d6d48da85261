"""Extended-precision (x87 80-bit, numpy longdouble: 64-bit significand)
restatement of one `para_update` evaluation -- TEST INFRASTRUCTURE ONLY.
Nothing in the product path imports it.

Why it exists: the fp64 oracle (oracle/ace_oracle.py) inverts by an fp64
eigendecomposition, so its own gradient carries ~cond(A)*eps of rounding,
and a GPU-vs-oracle difference cannot say which side moved.  This referee
evaluates the same mathematics with 2^11 = 2048x less rounding per
operation, so the errors of the fp64 oracle and of the GPU kernels can each
be measured against it ("numeric drift").

Mathematics (the reference's, quirks included):
  * kernel length scale of (feature i, slice b) at theta[1+b+B(i+1)] (Q1,
    src/kernel_SE_cpp.cpp:89, src/kernel_Matern_cpp.cpp:210);
  * SE K_b = z_r z_c exp(lambda_b - r2_b), z_0 = 1 -- the exact value of
    the reference's sign / log|z| form (Q7, src/kernel_SE_cpp.cpp:96,119);
  * Matern32 K_b = z_r z_c (1 + sqrt3 t) exp(lambda_b - sqrt3 t), t = sqrt(r2_b)
    (src/kernel_Matern_cpp.cpp:215-227);
  * A = K + e^theta0 I; A^-1 and log det A (src/kernel_SE_cpp.cpp:137-157),
    here by Cholesky in extended precision;
  * iteration 1: theta1 = 0.5 sum(A^-1 y) / sum(A^-1) (Q4, src/utilities_cpp.cpp:6-10);
  * alpha = A^-1 (y - mu), T = A^-1 - alpha alpha^T; g0 = -0.5 e^theta0 tr T,
    g_{2+b} = -0.5 sum T K_b, SE g_{2+B+b+Bi} = -0.5 e^-L sum T K_b d_i^2,
    Matern -2.25 e^-L sum T K_b d_i^2 / (1 + sqrt(3 r~2_b)) with the
    gradient-indexed scales (Q1, Q2); g1 = sum alpha (SE), 0 (Matern)
    (src/kernel_SE_cpp.cpp:161-243, src/kernel_Matern_cpp.cpp:340-467);
  * stats = [std_y ||ybar - K alpha|| / sqrt(n), -0.5 (n log 2pi + log det + y.alpha)]
    (Q3, src/include/ace_kernel_utils.hpp:33-36).
Inputs are fp64 and converted exactly; outputs are returned in longdouble.
"""
from __future__ import annotations

import numpy as np

LD = np.longdouble
PI_LD = np.longdouble("3.14159265358979323846264338327950288")


def _kernel_slices(kernel, X, Z, theta):
    n, p = X.shape
    B = Z.shape[1] + 1
    X = X.astype(LD)
    th = theta.astype(LD)
    K = np.empty((B, n, n), dtype=LD)
    for b in range(B):
        r2 = np.zeros((n, n), dtype=LD)
        for i in range(p):
            d = X[:, i][:, None] - X[:, i][None, :]
            r2 += d * d * np.exp(-th[1 + b + B * (i + 1)])
        if kernel == "SE":
            k = np.exp(th[2 + b] - r2)
        else:
            t = np.sqrt(r2)
            s3 = np.sqrt(LD(3))
            k = (1 + s3 * t) * np.exp(th[2 + b] - s3 * t)
        if b >= 1:
            z = Z[:, b - 1].astype(LD)
            k = k * z[:, None] * z[None, :]
        K[b] = k
    return K


def _chol_inverse(A):
    """(A^-1, log det A) by a right-looking Cholesky in longdouble."""
    n = A.shape[0]
    L = A.copy()
    for k in range(n):
        L[k, k] = np.sqrt(L[k, k])
        L[k + 1:, k] /= L[k, k]
        L[k + 1:, k + 1:] -= np.outer(L[k + 1:, k], L[k + 1:, k])
    L = np.tril(L)
    logdet = 2 * np.sum(np.log(np.diag(L)))
    # L^-1 by forward substitution (columns of the identity, vectorised over them)
    Li = np.zeros_like(L)
    eye = np.eye(n, dtype=LD)
    for i in range(n):
        Li[i] = (eye[i] - L[i, :i] @ Li[:i]) / L[i, i]
    return Li.T @ Li, logdet


def para_update_ld(kernel, y, X, Z, theta, std_y, it=1):
    """Returns (grad, stats, mu) in longdouble for one para_update at theta
    (theta[1] replaced by the mu solution when it == 1, as the R6 class does)."""
    X = np.asarray(X, dtype=np.float64)
    n, p = X.shape
    Z = np.asarray(Z, dtype=np.float64).reshape(n, -1)
    B = Z.shape[1] + 1
    th = np.array(theta, dtype=np.float64).astype(LD)
    Kb = _kernel_slices(kernel, X, Z, np.asarray(theta, dtype=np.float64))
    K = Kb.sum(axis=0)
    A = K + np.exp(th[0]) * np.eye(n, dtype=LD)
    inv, logdet = _chol_inverse(A)
    return grad_from_inverse(kernel, y, X, Z, theta, std_y, inv, logdet, it, Kb)


def grad_from_inverse(kernel, y, X, Z, theta, std_y, inv, logdet, it=1, Kb=None):
    """The gradient / stats / mu of para_update_ld from a GIVEN inverse (e.g.
    the GPU's A^-1 converted exactly): separates an inverse's error from the
    gradient kernel's (tools/inverse_analyze.py)."""
    X = np.asarray(X, dtype=np.float64)
    n, p = X.shape
    Z = np.asarray(Z, dtype=np.float64).reshape(n, -1)
    B = Z.shape[1] + 1
    th = np.array(theta, dtype=np.float64).astype(LD)
    if Kb is None:
        Kb = _kernel_slices(kernel, X, Z, np.asarray(theta, dtype=np.float64))
    K = Kb.sum(axis=0)
    inv = np.asarray(inv).astype(LD)
    yl = np.asarray(y, dtype=np.float64).astype(LD)
    if it == 1:
        th[1] = LD(0.5) * np.sum(inv @ yl) / np.sum(inv)
    mu = th[1]
    ybar = yl - mu
    alpha = inv @ ybar
    T = inv - np.outer(alpha, alpha)
    P = 2 + B * (p + 1)
    g = np.zeros(P, dtype=LD)
    g[0] = LD(-0.5) * np.trace(T) * np.exp(th[0])
    g[1] = np.sum(alpha) if kernel == "SE" else LD(0)
    Xl = X.astype(LD)
    D2 = [(Xl[:, i][:, None] - Xl[:, i][None, :]) ** 2 for i in range(p)]
    for b in range(B):
        g[2 + b] = LD(-0.5) * np.sum(T * Kb[b])
        if kernel == "SE":
            TK = T * Kb[b]
            for i in range(p):
                j = 2 + B + b + B * i
                g[j] = LD(-0.5) * np.exp(-th[j]) * np.sum(TK * D2[i])
        else:
            rt2 = np.zeros((n, n), dtype=LD)
            for i in range(p):
                rt2 += D2[i] * np.exp(-th[2 + B + b + B * i])
            F = T * Kb[b] / (1 + np.sqrt(3 * rt2))
            for i in range(p):
                j = 2 + B + b + B * i
                g[j] = LD(-2.25) * np.exp(-th[j]) * np.sum(F * D2[i])
    res = ybar - K @ alpha
    stats = np.array([LD(std_y) * np.sqrt(np.sum(res * res)) / np.sqrt(LD(n)),
                      LD(-0.5) * (n * np.log(2 * PI_LD) + logdet + yl @ alpha)], dtype=LD)
    return g, stats, mu


def rel_err(a, ref, floor=1e-9):
    """max |a - ref| / (|ref| + floor * max|ref|) -- the smoke's measure."""
    a = np.asarray(a, dtype=LD)
    ref = np.asarray(ref, dtype=LD)
    den = np.abs(ref) + LD(floor) * np.max(np.abs(ref))
    return float(np.max(np.abs(a - ref) / den))
