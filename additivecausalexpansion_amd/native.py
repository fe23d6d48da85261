"""The reference's `.Call` surface (R/RcppExports.R:4-78), same names and
argument order, implemented over the C ABI (include/ace_hip.h).

Return values mirror the Rcpp lists (`dict` with the same keys); arguments
the reference takes by non-const reference (`stats` in grad_*_cpp, m/v/nu/
para in the optimizers, grads in norm_clip_cpp, y/X/Z in normalize_*) are
mutated in place, so they must be writable float64 numpy arrays.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KIND, AceError, check, default_context, fmat, lib, ptr


def _ctx(ctx):
    return (ctx or default_context()).handle


# ---------------------------------------------------------------- device handles
class DMat:
    """An ace_dmat handle: a device-resident matrix / cube, or a virtual
    `elements` cube (X, Z, theta recorded; values assembled only if read).
    What the R shim wraps in an ALTREP vector: reading it (np.asarray, or
    any numpy use) materialises it, passing it back to a *_cpp routine does
    not (include/ace_hip.h "device-matrix handles")."""

    def __init__(self, handle, ctx):
        self.handle, self.ctx = handle, ctx
        r, c, sl = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        check(lib().ace_dmat_dims(handle, ctypes.byref(r), ctypes.byref(c), ctypes.byref(sl)))
        self.shape = (r.value, c.value) if sl.value == 1 else (r.value, c.value, sl.value)

    @classmethod
    def upload(cls, a, ctx=None):
        a = np.asarray(a, dtype=np.float64)
        dims = a.shape + (1,) * (3 - a.ndim)
        af = np.asfortranarray(a)
        h = ctypes.c_void_p()
        check(lib().ace_dmat_upload(_ctx(ctx), dims[0], dims[1], dims[2], ptr(af),
                                    ctypes.byref(h)), _ctx(ctx))
        return cls(h, _ctx(ctx))

    def read(self):
        out = np.empty(self.shape, order="F")
        check(lib().ace_dmat_read(self.handle, 0, out.size, ptr(out)), self.ctx)
        return out

    def __array__(self, dtype=None, copy=None):
        a = self.read()
        return a if dtype is None else a.astype(dtype)

    @property
    def on_device(self):
        return bool(lib().ace_dmat_materialized(self.handle) & 1)

    @property
    def read_to_host(self):
        return bool(lib().ace_dmat_materialized(self.handle) & 2)

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                lib().ace_dmat_free(self.handle)
                self.handle = None
        except Exception:
            pass


def _dmat(a, ctx, keep):
    """A handle for a matrix argument: DMat as is, a host array uploaded (the
    R shim does the same for a plain R matrix); `keep` holds temporaries."""
    if isinstance(a, DMat):
        return a.handle
    d = DMat.upload(a, ctx)
    keep.append(d)
    return d.handle


def _any_dev(*xs):
    return any(isinstance(x, DMat) for x in xs)


def _zmat(Z, n):
    Z = np.asarray(Z, dtype=np.float64)
    if Z.ndim == 1:
        Z = Z.reshape(n, 1)
    return np.asfortranarray(Z)


def _theta(parameters):
    return np.ascontiguousarray(np.ravel(parameters), dtype=np.float64)


def _check_theta(theta, B, p, grad=False):
    """The kernel reads theta up to P - 2 (P = 2 + B (p + 1)), so the kernmat_*
    routines accept P - 1 entries like the reference's; the gradient also
    reads the last, gradient-indexed length scale (Q1) and needs all P."""
    need = 2 + B * (p + 1) - (0 if grad else 1)
    if theta.shape[0] < need:
        raise AceError(f"parameters too short for B={B} and p={p}: {theta.shape[0]} < {need}")


# ---------------------------------------------------------------- kernels
def _kernmat_cross(kind, X1, X2, Z1, Z2, parameters, ctx=None, elements=True, device=False):
    X1 = fmat(X1)
    X2 = fmat(X2)
    n1, n2, p = X1.shape[0], X2.shape[0], X2.shape[1]
    Z1 = _zmat(Z1, n1)
    Z2 = _zmat(Z2, n2)
    B = Z1.shape[1] + 1
    th = _theta(parameters)
    _check_theta(th, B, p)
    if device:
        hf, he = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().ace_kernmat_cross_dev(_ctx(ctx), kind, n1, n2, p, B, ptr(X1), ptr(X2), ptr(Z1),
                                          ptr(Z2), ptr(th), ctypes.byref(hf), ctypes.byref(he)),
              _ctx(ctx))
        return {"full": DMat(hf, _ctx(ctx)), "elements": DMat(he, _ctx(ctx))}
    full = np.empty((n1, n2), order="F")
    el = np.empty((n1, n2, B), order="F") if elements else None
    check(lib().ace_kernmat_cross(_ctx(ctx), kind, n1, n2, p, B, ptr(X1), ptr(X2), ptr(Z1),
                                  ptr(Z2), ptr(th), ptr(full), ptr(el)), _ctx(ctx))
    return {"full": full, "elements": el}


def _kernmat_sym(kind, X, Z, parameters, ctx=None, elements=True, device=False):
    X = fmat(X)
    n, p = X.shape
    Z = _zmat(Z, n)
    B = Z.shape[1] + 1
    th = _theta(parameters)
    _check_theta(th, B, p)
    if device:
        hf, he = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().ace_kernmat_sym_dev(_ctx(ctx), kind, n, p, B, ptr(X), ptr(Z), ptr(th),
                                        ctypes.byref(hf), ctypes.byref(he)), _ctx(ctx))
        return {"full": DMat(hf, _ctx(ctx)), "elements": DMat(he, _ctx(ctx))}
    full = np.empty((n, n), order="F")
    el = np.empty((n, n, B), order="F") if elements else None
    check(lib().ace_kernmat_sym(_ctx(ctx), kind, n, p, B, ptr(X), ptr(Z), ptr(th), ptr(full),
                                ptr(el)), _ctx(ctx))
    return {"full": full, "elements": el}


def kernmat_SE_cpp(X1, X2, Z1, Z2, parameters, ctx=None, device=False):
    """src/kernel_SE_cpp.cpp:9-64"""
    return _kernmat_cross(KIND["SE"], X1, X2, Z1, Z2, parameters, ctx, device=device)


def kernmat_SE_symmetric_cpp(X, Z, parameters, ctx=None, device=False):
    """src/kernel_SE_cpp.cpp:67-134"""
    return _kernmat_sym(KIND["SE"], X, Z, parameters, ctx, device=device)


def kernmat_Matern32_cpp(X1, X2, Z1, Z2, parameters, ctx=None, device=False):
    """src/kernel_Matern_cpp.cpp:52-93"""
    return _kernmat_cross(KIND["Matern32"], X1, X2, Z1, Z2, parameters, ctx, device=device)


def kernmat_Matern32_symmetric_cpp(X, Z, parameters, ctx=None, device=False):
    """src/kernel_Matern_cpp.cpp:190-240"""
    return _kernmat_sym(KIND["Matern32"], X, Z, parameters, ctx, device=device)


def invkernel_cpp(pdmat, sigma, ctx=None):
    """src/kernel_SE_cpp.cpp:137-157.  `eigenval` holds the elimination
    pivots (sum(log(.)) == log det, the only use the reference makes of it)."""
    sig = float(np.ravel([sigma])[0])
    if _any_dev(pdmat):  # handle in, handle out: the inverse stays in HBM
        n = pdmat.shape[0]
        ev = np.empty(n)
        h = ctypes.c_void_p()
        check(lib().ace_invkernel_dev(_ctx(ctx), pdmat.handle, sig, ptr(ev), ctypes.byref(h)),
              _ctx(ctx))
        return {"eigenval": ev, "inv": DMat(h, _ctx(ctx))}
    K = fmat(pdmat)
    n = K.shape[0]
    if K.shape != (n, n):
        raise AceError("pdmat must be square")
    ev = np.empty(n)
    inv = np.empty((n, n), order="F")
    check(lib().ace_invkernel(_ctx(ctx), n, ptr(K), float(np.ravel([sigma])[0]), ptr(ev),
                              ptr(inv)), _ctx(ctx))
    return {"eigenval": ev, "inv": inv}


def _grad(kind, y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y, ctx):
    X = fmat(X)
    n, p = X.shape
    Z = _zmat(Z, n)
    if Z.shape[1] + 1 != B:
        raise AceError("B != ncol(Z) + 1")
    yv = np.ascontiguousarray(np.ravel(y), dtype=np.float64)
    th = _theta(parameters)
    _check_theta(th, B, p, grad=True)
    dev = _any_dev(Kfull, K, invKmatn)
    Kf = fmat(Kfull) if not dev else None
    Kc = fmat(K) if (K is not None and not dev) else None
    inv = fmat(invKmatn) if not dev else None
    ev = np.ascontiguousarray(np.ravel(eigenval), dtype=np.float64)
    if not (isinstance(stats, np.ndarray) and stats.dtype == np.float64 and stats.size >= 2):
        raise AceError("stats must be a float64 numpy array of length 2 (mutated in place)")
    st = np.ascontiguousarray(stats)
    g = np.empty(th.shape[0])
    if dev:
        keep = []
        hK = _dmat(Kfull, ctx, keep)
        hC = _dmat(K, ctx, keep) if K is not None else None
        hI = _dmat(invKmatn, ctx, keep)
        check(lib().ace_grad_dev(_ctx(ctx), kind, n, p, B, ptr(yv), ptr(X), ptr(Z), hK, hC, hI,
                                 ptr(ev), ptr(th), ptr(st), float(std_y), ptr(g)), _ctx(ctx))
    else:
        check(lib().ace_grad(_ctx(ctx), kind, n, p, B, ptr(yv), ptr(X), ptr(Z), ptr(Kf), ptr(Kc),
                             ptr(inv), ptr(ev), ptr(th), ptr(st), float(std_y), ptr(g)), _ctx(ctx))
    stats.flat[0:2] = st.flat[0:2]
    return g


def grad_SE_cpp(y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y, ctx=None):
    """src/kernel_SE_cpp.cpp:192-243 (stats written in place)."""
    return _grad(KIND["SE"], y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B,
                 std_y, ctx)


def grad_Matern_cpp(y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y,
                    ctx=None):
    """src/kernel_Matern_cpp.cpp:420-467 (stats written in place)."""
    return _grad(KIND["Matern32"], y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B,
                 std_y, ctx)


def stats_cpp(y, Kmat, invKmatn, eigenval, mu, std_y=1.0, ctx=None):
    """src/stats_cpp.cpp:9-32"""
    yv = np.ascontiguousarray(np.ravel(y), dtype=np.float64)
    n = yv.shape[0]
    out = np.empty(2)
    if _any_dev(Kmat, invKmatn):
        keep = []
        check(lib().ace_stats_dev(_ctx(ctx), n, ptr(yv), _dmat(Kmat, ctx, keep),
                                  _dmat(invKmatn, ctx, keep),
                                  ptr(np.ascontiguousarray(np.ravel(eigenval), dtype=np.float64)),
                                  float(np.ravel([mu])[0]), float(std_y), ptr(out)), _ctx(ctx))
        return out
    check(lib().ace_stats(_ctx(ctx), n, ptr(yv), ptr(fmat(Kmat)), ptr(fmat(invKmatn)),
                          ptr(np.ascontiguousarray(np.ravel(eigenval), dtype=np.float64)),
                          float(np.ravel([mu])[0]), float(std_y), ptr(out)), _ctx(ctx))
    return out


def mu_solution_cpp(y, invKmat, ctx=None):
    """src/utilities_cpp.cpp:6-10"""
    yv = np.ascontiguousarray(np.ravel(y), dtype=np.float64)
    out = ctypes.c_double()
    if _any_dev(invKmat):
        check(lib().ace_mu_solution_dev(_ctx(ctx), yv.shape[0], ptr(yv), invKmat.handle,
                                        ctypes.cast(ctypes.pointer(out),
                                                    ctypes.POINTER(ctypes.c_double))), _ctx(ctx))
        return out.value
    check(lib().ace_mu_solution(_ctx(ctx), yv.shape[0], ptr(yv), ptr(fmat(invKmat)),
                                ctypes.cast(ctypes.pointer(out), ctypes.POINTER(ctypes.c_double))),
          _ctx(ctx))
    return out.value


def pred_cpp(y_X, sigma, mu, invK_XX, K_xX, K_xx, mean_y, std_y, ctx=None):
    """src/pred_cpp.cpp:8-34"""
    yv = np.ascontiguousarray(np.ravel(y_X), dtype=np.float64)
    if _any_dev(invK_XX, K_xX, K_xx):
        keep = []
        nx, nX = K_xX.shape if isinstance(K_xX, DMat) else np.shape(K_xX)
        mp, var = np.empty(nx), np.empty(nx)
        ci = np.empty((nx, 2), order="F")
        check(lib().ace_pred_dev(_ctx(ctx), nX, nx, ptr(yv), float(sigma), float(mu),
                                 _dmat(invK_XX, ctx, keep), _dmat(K_xX, ctx, keep),
                                 _dmat(K_xx, ctx, keep), float(mean_y), float(std_y), ptr(mp),
                                 ptr(ci), ptr(var)), _ctx(ctx))
        return {"map": mp, "ci": ci, "var": var}
    KxX = fmat(K_xX)
    nx, nX = KxX.shape
    mp = np.empty(nx)
    ci = np.empty((nx, 2), order="F")
    var = np.empty(nx)
    check(lib().ace_pred(_ctx(ctx), nX, nx, ptr(yv), float(sigma), float(mu),
                         ptr(fmat(invK_XX)), ptr(KxX), ptr(fmat(K_xx)), float(mean_y),
                         float(std_y), ptr(mp), ptr(ci), ptr(var)), _ctx(ctx))
    return {"map": mp, "ci": ci, "var": var}


def pred_marginal_cpp(y_X, Z_x, sigma, mu, invK_XX, K_xX, K_xx, mean_y, std_y, std_Z,
                      calculate_ate, ctx=None):
    """src/pred_cpp.cpp:37-126"""
    yv = np.ascontiguousarray(np.ravel(y_X), dtype=np.float64)
    zx = np.ascontiguousarray(np.ravel(Z_x), dtype=np.float64) if Z_x is not None else None
    avg = np.empty(12)
    if _any_dev(invK_XX, K_xX, K_xx):
        keep = []
        nx, nX = (K_xX.shape if isinstance(K_xX, DMat) else np.shape(K_xX))[:2]
        mp, var = np.empty(nx), np.empty(nx)
        ci = np.empty((nx, 2), order="F")
        check(lib().ace_pred_marginal_dev(_ctx(ctx), nX, nx, ptr(yv), ptr(zx), float(sigma),
                                          float(mu), _dmat(invK_XX, ctx, keep),
                                          _dmat(K_xX, ctx, keep), _dmat(K_xx, ctx, keep),
                                          float(mean_y), float(std_y),
                                          float(np.ravel([std_Z])[0]), 1 if calculate_ate else 0,
                                          ptr(mp), ptr(ci), ptr(var), ptr(avg)), _ctx(ctx))
    else:
        cX = fmat(K_xX)
        cx = fmat(K_xx)
        nx, nX, B = cX.shape
        mp = np.empty(nx)
        ci = np.empty((nx, 2), order="F")
        var = np.empty(nx)
        check(lib().ace_pred_marginal(_ctx(ctx), nX, nx, B, ptr(yv), ptr(zx), float(sigma),
                                      float(mu), ptr(fmat(invK_XX)), ptr(cX), ptr(cx),
                                      float(mean_y), float(std_y), float(np.ravel([std_Z])[0]),
                                      1 if calculate_ate else 0, ptr(mp), ptr(ci), ptr(var),
                                      ptr(avg)), _ctx(ctx))
    out = {"map": mp, "ci": ci, "var": var}
    if calculate_ate:
        for j, key in enumerate(("ate", "att", "atu")):
            a = avg[4 * j:4 * j + 4]
            out[key] = {"map": a[0], "ci": np.array([a[1], a[2]]), "var": a[3]}
    return out


# ---------------------------------------------------------------- host-only
def _inplace(a, name):
    if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and
            (a.flags.c_contiguous or a.flags.f_contiguous) and a.flags.writeable):
        raise AceError(f"{name} must be a writable contiguous float64 numpy array")
    return a


def Nesterov_cpp(learn_rate, momentum, nu, grad, para):
    """src/optimizer_cpp.cpp:8-20 (nu, para in place)."""
    g = np.ascontiguousarray(np.ravel(grad), dtype=np.float64)
    return bool(lib().ace_nesterov(g.shape[0], float(learn_rate), float(momentum),
                                   ptr(_inplace(nu, "nu")), ptr(g), ptr(_inplace(para, "para"))))


def Nadam_cpp(iter, learn_rate, beta1, beta2, eps, m, v, grad, para):  # noqa: A002
    """src/optimizer_cpp.cpp:23-42 (m, v, para in place)."""
    g = np.ascontiguousarray(np.ravel(grad), dtype=np.float64)
    return bool(lib().ace_nadam(g.shape[0], float(iter), float(learn_rate), float(beta1),
                                float(beta2), float(eps), ptr(_inplace(m, "m")),
                                ptr(_inplace(v, "v")), ptr(g), ptr(_inplace(para, "para"))))


def Adam_cpp(iter, learn_rate, beta1, beta2, eps, m, v, grad, para):  # noqa: A002
    """src/optimizer_cpp.cpp:45-63 (m, v, para in place)."""
    g = np.ascontiguousarray(np.ravel(grad), dtype=np.float64)
    return bool(lib().ace_adam(g.shape[0], float(iter), float(learn_rate), float(beta1),
                               float(beta2), float(eps), ptr(_inplace(m, "m")),
                               ptr(_inplace(v, "v")), ptr(g), ptr(_inplace(para, "para"))))


def norm_clip_cpp(flag, grads, max_length):
    """src/utilities_cpp.cpp:121-129 (grads in place)."""
    g = _inplace(grads, "grads")
    lib().ace_norm_clip(1 if flag else 0, g.size, ptr(g), float(max_length))


def _ncs(fn, x, knots):
    xv = np.ascontiguousarray(np.ravel(x), dtype=np.float64)
    kv = np.ascontiguousarray(np.ravel(knots), dtype=np.float64)
    nk = np.unique(kv).shape[0]
    out = np.empty((xv.shape[0], nk), order="F")
    ncols = ctypes.c_int64()
    check(fn(xv.shape[0], ptr(xv), kv.shape[0], ptr(kv), ptr(out), ctypes.byref(ncols)))
    return out[:, :ncols.value]


def ncs_basis(x, knots):
    """src/ncs_basis_cpp.cpp:61-79"""
    return _ncs(lib().ace_ncs_basis, x, knots)


def ncs_basis_deriv(x, knots):
    """src/ncs_basis_cpp.cpp:82-99"""
    return _ncs(lib().ace_ncs_basis_deriv, x, knots)


def normalize_train(y, X, Z):
    """src/utilities_cpp.cpp:13-104: y (n), X (n x px), Z (n x pz) in place
    (Fortran-ordered float64); returns the (1+px+pz) x 3 moments."""
    y = _inplace(y, "y")
    X = _inplace(X, "X")
    Z = _inplace(Z, "Z")
    if X.ndim != 2 or Z.ndim != 2 or not X.flags.f_contiguous or not Z.flags.f_contiguous:
        raise AceError("X and Z must be 2-D Fortran-ordered arrays")
    n, px = X.shape
    pz = Z.shape[1]
    mom = np.empty((1 + px + pz, 3), order="F")
    check(lib().ace_normalize_train(n, px, pz, ptr(y), ptr(X), ptr(Z), ptr(mom)))
    return mom


def normalize_test(X, Z, moments):
    """src/utilities_cpp.cpp:108-118 (X, Z in place)."""
    X = _inplace(X, "X")
    Z = _inplace(Z, "Z")
    mom = fmat(moments)
    check(lib().ace_normalize_test(X.shape[0], X.shape[1], Z.shape[1], ptr(X), ptr(Z), ptr(mom),
                                   mom.shape[0]))
