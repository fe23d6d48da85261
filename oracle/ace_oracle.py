"""CPU oracle: a numpy restatement of the reference `ace` 0.4.1 numerics.

TEST INFRASTRUCTURE ONLY.  Nothing in the product package imports this file;
only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg
may use it, and only as the checker.

PARITY UNPINNED: the reference (R + Rcpp + RcppArmadillo) cannot be built or
run in this image (no R, no Rcpp, no Armadillo) and its own
tree holds no tests, fixtures or golden vectors.  This file is
therefore a line-by-line restatement of the reference arithmetic, quirks
included, cross-checked against an independent literal
C restatement (`oracle/ace_ref.c`) and against finite differences on the
components the quirks do not touch (tests/test_oracle.py).

Array conventions follow Armadillo: matrices are 2-D numpy arrays indexed
[row, col]; cubes are (n1, n2, B) arrays with cube[:, :, b] == slice(b);
column-major memory order is irrelevant here (the C-ABI handles layout).

Every function cites the reference file:line it follows.
"""
from __future__ import annotations

import math

import numpy as np

SQRT3 = math.sqrt(3.0)  # `sqrt(3)` in src/kernel_Matern_cpp.cpp:79 (int promoted to double)


# --------------------------------------------------------------------------
# src/include/ace_kernel_utils.hpp
# --------------------------------------------------------------------------
def _sign(x):
    """`sign` (src/include/ace_kernel_utils.hpp:38-40): (0 < x) - (x < 0)."""
    return (x > 0).astype(np.float64) - (x < 0).astype(np.float64)


def evid_grad(Kaa, dK):
    """-0.5 * trace(Kaa * dK)  (src/include/ace_kernel_utils.hpp:23-26)."""
    return -0.5 * float(np.einsum("ij,ji->", Kaa, dK))


def sigma_gradient(Kaa, sigma):
    """-0.5 * trace(Kaa) * exp(sigma)  (src/include/ace_kernel_utils.hpp:29-31)."""
    return -0.5 * float(np.trace(Kaa)) * math.exp(sigma)


def logevidence(y, alpha, eigenval, n):
    """Q3: uses y . alpha, not ybar . alpha (src/include/ace_kernel_utils.hpp:33-36)."""
    return -0.5 * (n * math.log(2.0 * math.pi) + float(np.sum(np.log(eigenval)))
                   + float(np.dot(np.ravel(y), np.ravel(alpha))))


# --------------------------------------------------------------------------
# Distance accumulation shared by every assembly routine.
# The kernel reads length scale (i, b) at theta[1 + b + B*(i+1)]   (Q1)
# src/kernel_SE_cpp.cpp:27-36, 82-94; src/kernel_Matern_cpp.cpp:66-75, 203-214
# --------------------------------------------------------------------------
def _scaled_sqdist(X1, X2, theta, B):
    X1 = np.asarray(X1, dtype=np.float64)
    X2 = np.asarray(X2, dtype=np.float64)
    theta = np.ravel(theta).astype(np.float64)
    p = X2.shape[1]
    n1, n2 = X1.shape[0], X2.shape[0]
    acc = np.zeros((n1, n2, B))
    for i in range(p):
        tmp = (X1[:, i][:, None] - X2[:, i][None, :]) ** 2
        for b in range(B):
            acc[:, :, b] += tmp * math.exp(-theta[1 + b + B * (i + 1)])
    return acc


def _as2d(Z, n):
    Z = np.asarray(Z, dtype=np.float64)
    if Z.ndim == 1:
        Z = Z.reshape(n, 1)
    return Z


# --------------------------------------------------------------------------
# src/kernel_SE_cpp.cpp
# --------------------------------------------------------------------------
def _se_slices(acc, Z1, Z2, theta, B):
    """slice 0: exp(theta[2] - r2); slice b>=1: the sign/log|z| form (Q7)."""
    theta = np.ravel(theta)
    out = np.empty_like(acc)
    out[:, :, 0] = np.exp(theta[2] - acc[:, :, 0])
    for b in range(1, B):
        z1 = Z1[:, b - 1]
        z2 = Z2[:, b - 1]
        with np.errstate(divide="ignore"):
            l1 = np.log(np.abs(z1))
            l2 = np.log(np.abs(z2))
        val = (_sign(z1)[:, None] * _sign(z2)[None, :]) * np.exp(
            ((theta[2 + b] - acc[:, :, b]) + l1[:, None]) + l2[None, :])
        mask = (z1 == 0)[:, None] | (z2 == 0)[None, :]
        val[mask] = 0.0
        out[:, :, b] = val
    return out


def _sum_slices(S):
    """Kfull = slice0 + slice1 + ... in order (src/kernel_SE_cpp.cpp:126-130)."""
    full = S[:, :, 0].copy()
    for b in range(1, S.shape[2]):
        full = full + S[:, :, b]
    return full


def kernmat_SE_cpp(X1, X2, Z1, Z2, parameters):
    """Cross kernel (src/kernel_SE_cpp.cpp:9-64).  B = Z1.n_cols + 1."""
    X1 = np.asarray(X1, dtype=np.float64)
    X2 = np.asarray(X2, dtype=np.float64)
    Z1 = _as2d(Z1, X1.shape[0])
    Z2 = _as2d(Z2, X2.shape[0])
    B = Z1.shape[1] + 1
    S = _se_slices(_scaled_sqdist(X1, X2, parameters, B), Z1, Z2, parameters, B)
    return {"full": _sum_slices(S), "elements": S}


def kernmat_SE_symmetric_cpp(X, Z, parameters):
    """Train kernel (src/kernel_SE_cpp.cpp:67-134); computed on the upper
    triangle and mirrored, so the result is exactly symmetric."""
    X = np.asarray(X, dtype=np.float64)
    Z = _as2d(Z, X.shape[0])
    B = Z.shape[1] + 1
    S = _se_slices(_scaled_sqdist(X, X, parameters, B), Z, Z, parameters, B)
    S = _mirror_upper(S)
    return {"full": _sum_slices(S), "elements": S}


def _mirror_upper(S):
    """uppertri2symmat (src/include/ace_kernel_utils.hpp:7-20) applied per slice."""
    n = S.shape[0]
    iu = np.triu_indices(n, 1)
    S = S.copy()
    for b in range(S.shape[2]):
        sl = S[:, :, b]
        sl[(iu[1], iu[0])] = sl[iu]
    return S


# --------------------------------------------------------------------------
# src/kernel_Matern_cpp.cpp (Matern 3/2 only; 5/2 and 1/2 are dead code)
# --------------------------------------------------------------------------
def _matern_slices(acc, Z1, Z2, theta, B, symmetric):
    theta = np.ravel(theta)
    t = np.sqrt(acc)
    out = np.empty_like(acc)
    out[:, :, 0] = (1 + SQRT3 * t[:, :, 0]) * np.exp(theta[2] - SQRT3 * t[:, :, 0])
    for b in range(1, B):
        z1 = Z1[:, b - 1]
        z2 = Z2[:, b - 1]
        tb = t[:, :, b]
        val = (((1 + SQRT3 * tb) * np.exp(theta[2 + b] - SQRT3 * tb)) * z1[:, None]) * z2[None, :]
        val[z1 == 0, :] = 0.0
        if not symmetric:  # src/kernel_Matern_cpp.cpp:85 (the symmetric form has no column test)
            val[:, z2 == 0] = 0.0
        out[:, :, b] = val
    return out


def kernmat_Matern32_cpp(X1, X2, Z1, Z2, parameters):
    """Cross kernel (src/kernel_Matern_cpp.cpp:52-93)."""
    X1 = np.asarray(X1, dtype=np.float64)
    X2 = np.asarray(X2, dtype=np.float64)
    Z1 = _as2d(Z1, X1.shape[0])
    Z2 = _as2d(Z2, X2.shape[0])
    B = Z1.shape[1] + 1
    S = _matern_slices(_scaled_sqdist(X1, X2, parameters, B), Z1, Z2, parameters, B, False)
    return {"full": _sum_slices(S), "elements": S}


def kernmat_Matern32_symmetric_cpp(X, Z, parameters):
    """Train kernel (src/kernel_Matern_cpp.cpp:190-240)."""
    X = np.asarray(X, dtype=np.float64)
    Z = _as2d(Z, X.shape[0])
    B = Z.shape[1] + 1
    S = _matern_slices(_scaled_sqdist(X, X, parameters, B), Z, Z, parameters, B, True)
    S = _mirror_upper(S)
    return {"full": _sum_slices(S), "elements": S}


# --------------------------------------------------------------------------
# src/kernel_SE_cpp.cpp:137-157
# --------------------------------------------------------------------------
def invkernel_cpp(pdmat, sigma):
    """A = pdmat + e^sigma I; (w, V) = eig_sym(A) (LAPACK syevd, ascending);
    inv = (V diag(w^-1/2)) (V diag(w^-1/2))^T."""
    A = np.array(pdmat, dtype=np.float64, copy=True)
    A[np.diag_indices_from(A)] += math.exp(float(np.ravel([sigma])[0]))
    w, V = np.linalg.eigh(A)
    with np.errstate(invalid="ignore", divide="ignore"):
        Vs = V / np.sqrt(w)[None, :]
    return {"eigenval": w, "inv": Vs @ Vs.T}


# --------------------------------------------------------------------------
# Gradients: src/kernel_SE_cpp.cpp:161-243, src/kernel_Matern_cpp.cpp:340-467
# --------------------------------------------------------------------------
def _alpha_T(y, invK, mu):
    ybar = np.ravel(y) - mu
    alpha = invK @ ybar
    T = invK - np.outer(alpha, alpha)
    return ybar, alpha, T


def _sqd(X, i):
    x = X[:, i]
    return (x[:, None] - x[None, :]) ** 2  # tmpX.col(r) = pow(X(r,i) - X.col(i), 2): symmetric


def _grad_stats(y, Kfull, ybar, alpha, eigenval, stats, std_y):
    n = ybar.shape[0]
    stats[0] = std_y * float(np.linalg.norm(ybar - Kfull @ alpha)) / math.sqrt(n)
    stats[1] = logevidence(y, alpha, eigenval, n)


def grad_SE_cpp(y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y):
    """Returns the P-gradient; writes stats[0:2] in place (src/kernel_SE_cpp.cpp:192-243)."""
    X = np.asarray(X, dtype=np.float64)
    theta = np.ravel(parameters).astype(np.float64)
    n, px = X.shape
    g = np.zeros(theta.shape[0])
    ybar, alpha, T = _alpha_T(y, invKmatn, theta[1])
    g[0] = sigma_gradient(T, theta[0])
    for b in range(B):
        g[2 + b] = evid_grad(T, K[:, :, b])
    # evid_scale_gradients (src/kernel_SE_cpp.cpp:161-188): gradient index 2+B+b+B*i (Q1)
    for i in range(px):
        D2 = _sqd(X, i)
        for b in range(B):
            L = theta[2 + B + b + B * i]
            g[2 + B + b + B * i] = evid_grad(T, (K[:, :, b] * D2) * math.exp(-L))
    g[1] = float(np.sum(invKmatn @ ybar))
    _grad_stats(y, Kfull, ybar, alpha, eigenval, stats, std_y)
    return g


def grad_Matern_cpp(y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y):
    """src/kernel_Matern_cpp.cpp:420-467 with evid_scale_Matern32_gradients (340-377):
    r~2 uses the GRADIENT-indexed scales and the prefactor is -0.25*9 (Q2)."""
    X = np.asarray(X, dtype=np.float64)
    theta = np.ravel(parameters).astype(np.float64)
    n, px = X.shape
    g = np.zeros(theta.shape[0])
    ybar, alpha, T = _alpha_T(y, invKmatn, theta[1])
    g[0] = sigma_gradient(T, theta[0])
    for b in range(B):
        g[2 + b] = evid_grad(T, K[:, :, b])
    acc = np.zeros((n, n, B))
    for i in range(px):
        D2 = _sqd(X, i)
        for b in range(B):
            acc[:, :, b] += D2 * math.exp(-theta[2 + B + b + B * i])
    F = np.empty_like(acc)
    for b in range(B):
        F[:, :, b] = K[:, :, b] / (1 + np.sqrt(3 * acc[:, :, b]))
    for i in range(px):
        D2 = _sqd(X, i)
        for b in range(B):
            L = theta[2 + B + b + B * i]
            g[2 + B + b + B * i] = (-0.25 * 9 * float(np.einsum("ij,ji->", T, F[:, :, b] * D2))
                                    * math.exp(-L))
    g[1] = 0.0
    _grad_stats(y, Kfull, ybar, alpha, eigenval, stats, std_y)
    return g


# --------------------------------------------------------------------------
# src/stats_cpp.cpp:9-32 ; src/utilities_cpp.cpp:6-10
# --------------------------------------------------------------------------
def stats_cpp(y, Kmat, invKmatn, eigenval, mu, std_y=1.0):
    ybar = np.ravel(y) - mu
    alpha = invKmatn @ ybar
    n = ybar.shape[0]
    return np.array([std_y * float(np.linalg.norm(ybar - Kmat @ alpha)) / math.sqrt(n),
                     logevidence(y, alpha, eigenval, n)])


def mu_solution_cpp(y, invKmat):
    """Q4: 0.5 * sum(inv y) / accu(inv)."""
    return 0.5 * float(np.sum(invKmat @ np.ravel(y))) / float(np.sum(invKmat))


# --------------------------------------------------------------------------
# src/pred_cpp.cpp
# --------------------------------------------------------------------------
def pred_cpp(y_X, sigma, mu, invK_XX, K_xX, K_xx, mean_y, std_y):
    """src/pred_cpp.cpp:8-34."""
    tmp = K_xX @ invK_XX
    y_x = mean_y + std_y * (tmp @ (np.ravel(y_X) - mu) + mu)
    Kp = K_xx - tmp @ K_xX.T
    d = np.diag(Kp) + math.exp(sigma)
    var = std_y * np.sqrt(np.abs(d))
    ci = np.stack([y_x - 1.96 * var, y_x + 1.96 * var], axis=1)
    return {"map": y_x, "ci": ci, "var": var ** 2}


def pred_marginal_cpp(y_X, Z_x, sigma, mu, invK_XX, K_xX, K_xx, mean_y, std_y, std_Z,
                      calculate_ate):
    """src/pred_cpp.cpp:37-126 (slices 1..B-1, or slice 0 when B == 1)."""
    B = K_xx.shape[2]
    if B > 1:
        Km_xX = K_xX[:, :, 1].copy()
        Km_xx = K_xx[:, :, 1].copy()
        for b in range(2, B):
            Km_xX = Km_xX + K_xX[:, :, b]
            Km_xx = Km_xx + K_xx[:, :, b]
    else:
        Km_xX = K_xX[:, :, 0].copy()
        Km_xx = K_xx[:, :, 0].copy()
    nx = Km_xx.shape[0]
    tmp = Km_xX @ invK_XX
    y_x = std_y * (tmp @ (np.ravel(y_X) - mu)) / std_Z
    Km_xx = Km_xx - tmp @ Km_xX.T
    var = std_y * np.sqrt(np.abs(np.diag(Km_xx))) / std_Z
    ci = np.stack([y_x - 1.96 * var, y_x + 1.96 * var], axis=1)
    out = {"map": y_x, "ci": ci, "var": var ** 2}
    if not calculate_ate:
        return out
    zx = np.ravel(Z_x).astype(np.float64)
    # C double semantics: sqrt of a negative quadratic form is NaN and a
    # division by a zero count is +-inf / NaN (no exception), as in the
    # reference's doubles; the counts are `unsigned int` (src/pred_cpp.cpp:43,95,104)
    f64 = np.float64
    with np.errstate(divide="ignore", invalid="ignore"):
        ate = float(np.mean(y_x))
        ate_sd = float(std_y * np.sqrt(f64(np.sum(Km_xx))) / f64(nx))
        ntx = int(np.sum(zx)) % 2 ** 32  # truncation toward zero, like the C conversion
        att = float(f64(np.dot(y_x, zx)) / f64(ntx))
        att_sd = float(std_y * np.sqrt(f64(np.dot(Km_xx @ zx, zx))) / f64(ntx))
        nux = (nx - ntx) % 2 ** 32  # unsigned subtraction (src/pred_cpp.cpp:104)
        atu = float((f64(ate) * f64(nx) - f64(att) * f64(ntx)) / f64(nux))
        u = (zx == 0).astype(np.float64)
        atu_sd = float(std_y * np.sqrt(f64(np.dot(Km_xx @ u, u))) / f64(nux))
    for key, m, sd in (("ate", ate, ate_sd), ("att", att, att_sd), ("atu", atu, atu_sd)):
        out[key] = {"map": m, "ci": np.array([m - 1.96 * sd, m + 1.96 * sd]), "var": sd ** 2}
    return out


# --------------------------------------------------------------------------
# src/optimizer_cpp.cpp ; src/utilities_cpp.cpp:121-129  (in place, Q5/Q8)
# --------------------------------------------------------------------------
def Nesterov_cpp(learn_rate, momentum, nu, grad, para):
    flag = bool(np.all(np.isfinite(grad)))
    nu[:] = momentum * nu + learn_rate * grad
    para[:] = para + nu
    return flag


def Nadam_cpp(it, learn_rate, beta1, beta2, eps, m, v, grad, para):
    flag = bool(np.all(np.isfinite(grad)))
    m[:] = beta1 * m + (1 - beta1) * grad
    v[:] = beta2 * v + (1 - beta2) * grad ** 2
    para[:] = para + learn_rate * ((beta1 * m + (1 - beta1) * grad) / (1 - beta1 ** it)) / (
        np.sqrt(v / (1 - beta2 ** it)) + eps)
    return flag


def Adam_cpp(it, learn_rate, beta1, beta2, eps, m, v, grad, para):
    flag = bool(np.all(np.isfinite(grad)))
    m[:] = beta1 * m + (1 - beta1) * grad
    v[:] = beta2 * v + (1 - beta2) * grad ** 2
    para[:] = para + learn_rate * (m / (1 - beta1 ** it)) / (np.sqrt(v / (1 - beta2 ** it)) + eps)
    return flag


def norm_clip_cpp(flag, grads, max_length):
    """Q5: rescales to UNIT norm when ||g|| > max_length."""
    if flag:
        L2 = float(np.linalg.norm(grads))
        if L2 > max_length and math.isfinite(L2) and L2 != 0:
            grads[:] = grads / L2


# --------------------------------------------------------------------------
# Host preprocessing: src/utilities_cpp.cpp:13-118, src/ncs_basis_cpp.cpp
# --------------------------------------------------------------------------
def normalize_train(y, X, Z):
    """In place on y, X, Z; returns moments ((1+px+pz) x 3).  Quirks kept:
    binary columns write their location/scale one row up (moments(i, .)),
    and the Z rescale tests isbinary(i - px - 1), i.e. X's flags
    (src/utilities_cpp.cpp:32-36, 60-63, 106-110)."""
    px = X.shape[1]
    pz = Z.shape[1]
    mom = np.zeros((1 + px + pz, 3))
    mom[:, 1] = 1.0
    isb = np.zeros(px + pz, dtype=np.int64)
    for i in range(px):
        u = np.unique(X[:, i])
        if u.size == 2:
            isb[i] = 1
            mom[i + 1, 2] = 1
            if u.min() != 0:
                mom[i, 0] = u.min()
            if u.max() != 1:
                mom[i, 1] = u.max() - u.min()
            X[:, i] -= mom[i, 0]
            X[:, i] /= mom[i, 1]
        elif u.size == 1:
            X[:, i] = 0.0
    for i in range(px, px + pz):
        u = np.unique(Z[:, i - px])
        if u.size == 2:
            isb[i] = 1
            mom[i + 1, 2] = 1
            if u.min() != 0:
                mom[i, 0] = u.min()
            if u.max() != 1:
                mom[i, 1] = u.max() - u.min()
            Z[:, i - px] -= mom[i, 0]
            Z[:, i - px] /= mom[i, 1]
        elif u.size == 1:
            if i >= Z.shape[1]:
                raise IndexError("Mat::col(): index out of bounds")  # Z.col(i) with i >= pz
            Z[:, i] = 0.0
    mom[0, 0] = float(np.mean(y))
    y -= mom[0, 0]
    for i in range(1, px + 1):
        if isb[i - 1] == 0:
            mom[i, 0] = float(np.median(X[:, i - 1]))
            X[:, i - 1] -= mom[i, 0]
    for i in range(px + 1, px + pz + 1):
        if isb[i - 1] == 0:
            mom[i, 0] = float(np.median(Z[:, i - px - 1]))
            Z[:, i - px - 1] -= mom[i, 0]
    mom[0, 1] = float(np.std(y, ddof=1))
    y /= mom[0, 1]
    for i in range(1, px + 1):
        if isb[i - 1] == 0:
            mom[i, 1] = float(np.max(np.abs(X[:, i - 1])))
            X[:, i - 1] /= mom[i, 1]
    for i in range(px + 1, px + pz + 1):
        if isb[i - px - 1] == 0:
            mom[i, 1] = float(np.max(np.abs(Z[:, i - px - 1])))
            Z[:, i - px - 1] = Z[:, i - px - 1] / mom[i, 1]
    return mom


def normalize_test(X, Z, moments):
    """src/utilities_cpp.cpp:108-118 (in place)."""
    px = X.shape[1]
    for i in range(px):
        X[:, i] = (X[:, i] - moments[i + 1, 0]) / moments[i + 1, 1]
    for i in range(Z.shape[1]):
        Z[:, i] = (Z[:, i] - moments[i + 1 + px, 0]) / moments[i + 1 + px, 1]


def _ncs_cols(x, knots, deriv):
    K = knots.shape[0]
    n = x.shape[0]
    d = np.zeros((n, K))
    if deriv:
        f = lambda kk: 3 * (x > kk) * (x - kk) ** 2
    else:
        f = lambda kk: (x > kk) * (x - kk) ** 3
    d[:, K - 1] = f(knots[K - 1])
    for i in range(K - 1):
        d[:, i] = (f(knots[i]) - d[:, K - 1]) / (knots[K - 1] - knots[i])
    d[:, K - 1] = 0.0
    N = np.zeros((n, K - 1))
    for i in range(K - 2):
        N[:, i] = d[:, i] - d[:, K - 2]
    N[:, K - 2] = -d[:, K - 2]
    return N


def ncs_basis(x, knots):
    """src/ncs_basis_cpp.cpp:61-79 (+ generate_ncs_matrix 5-28)."""
    x = np.ravel(x).astype(np.float64)
    knots = np.unique(np.ravel(knots).astype(np.float64))
    design = np.empty((x.shape[0], knots.shape[0]))
    design[:, 0] = x
    design[:, 1:] = _ncs_cols(x, knots, False)
    return design


def ncs_basis_deriv(x, knots):
    """src/ncs_basis_cpp.cpp:82-99 (+ generate_ncs_derivative_matrix 30-58)."""
    x = np.ravel(x).astype(np.float64)
    knots = np.unique(np.ravel(knots).astype(np.float64))
    design = np.empty((x.shape[0], knots.shape[0]))
    design[:, 0] = 1.0
    design[:, 1:] = _ncs_cols(x, knots, True)
    return design


# --------------------------------------------------------------------------
# One para_update (R/kernel_SE_R6.R:40-62, R/kernel_Matern32_R6.R:39-60)
# and the training loop (R/main_ace.R:213-235), Nadam/Adam/Nesterov classes
# (R/optimizer_classes.R).
# --------------------------------------------------------------------------
KERNELS = {
    "SE": (kernmat_SE_symmetric_cpp, kernmat_SE_cpp, grad_SE_cpp),
    "Matern32": (kernmat_Matern32_symmetric_cpp, kernmat_Matern32_cpp, grad_Matern_cpp),
}


class OracleOptimizer:
    """R/optimizer_classes.R: update() = norm_clip_cpp then the step, stop() on non-finite."""

    def __init__(self, kind, P, lr, beta1=0.9, beta2=0.999, momentum=0.0, norm_clip=True,
                 clip_at=1.0):
        self.kind, self.lr, self.beta1, self.beta2 = kind, lr, beta1, beta2
        self.momentum, self.norm_clip, self.clip_at = momentum, norm_clip, clip_at
        self.m = np.zeros(P)
        self.v = np.zeros(P)
        self.nu = np.zeros(P)

    def update(self, it, para, grads):
        norm_clip_cpp(self.norm_clip, grads, self.clip_at)
        if self.kind == "Adam":
            ok = Adam_cpp(float(it), self.lr, self.beta1, self.beta2, 1e-8, self.m, self.v, grads, para)
        elif self.kind == "Nadam":
            ok = Nadam_cpp(float(it), self.lr, self.beta1, self.beta2, 1e-8, self.m, self.v, grads, para)
        else:
            ok = Nesterov_cpp(self.lr, self.momentum, self.nu, grads, para)
        if not ok:
            raise FloatingPointError("Some gradients are not finite, NaN, or NA. "
                                     "Often this is due to too large learning rates.")
        return para


def para_update(kernel, it, theta, y, X, Z, B, optim, std_y):
    """Returns (stats, gradients_before_clip, mutated theta).  Sequence of
    R/kernel_SE_R6.R:40-62: kernel_mat_sym -> invkernel -> [iter==1: mu] ->
    grad -> Optim$update -> mu overwrite (with the pre-update inverse)."""
    sym, _, grad = KERNELS[kernel]
    Kl = sym(X, Z, theta)
    inv = invkernel_cpp(Kl["full"], theta[0])
    if it == 1:
        theta[1] = mu_solution_cpp(y, inv["inv"])
    stats = np.zeros(2)
    g = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], theta, stats, B, std_y)
    graw = g.copy()
    optim.update(it, theta, g)
    theta[1] = mu_solution_cpp(y, inv["inv"])
    return stats, graw, inv["inv"]


def train_trajectory(kernel, y, X, Z, theta0, std_y, iters, optim):
    """First `iters` iterations of R/main_ace.R:215-227 (no convergence stop)."""
    theta = np.array(theta0, dtype=np.float64)
    B = Z.shape[1] + 1
    thetas, stats_l, grads_l = [], [], []
    inv = None
    for it in range(1, iters + 1):
        st, g, inv = para_update(kernel, it, theta, y, X, Z, B, optim, std_y)
        thetas.append(theta.copy())
        stats_l.append(st)
        grads_l.append(g)
    return np.array(thetas), np.array(stats_l), np.array(grads_l), inv


def set_initial_parameters(p, B, n, y, X, Z, init_length_scale=20.0):
    """R/parameters.R:1-23.  `init.sigma` is always passed by ace.train
    (R/main_ace.R:199-202), so `!missing(init.sigma)` is TRUE and the OLS
    residual variance is always used."""
    Xm = np.column_stack([X, Z, np.ones(n)])
    Q, R = np.linalg.qr(Xm)
    rank = int(np.sum(np.abs(np.diag(R)) > 1e-7 * np.abs(R).max()))
    Q = Q[:, :rank]
    yv = np.ravel(y)
    resid = yv - Q @ (Q.T @ yv)
    init_sigma = math.log(float(yv @ resid) / (n - 1))
    return np.concatenate([[init_sigma, 0.0], -np.log(np.ones(B)),
                           np.log(np.full(B * p, init_length_scale))])
