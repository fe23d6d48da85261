"""Host-side mirror of the reference's R6 classes on the hot path:
KernelClass_SE_R6 / KernelClass_Matern32_R6 (R/kernel_SE_R6.R,
R/kernel_Matern32_R6.R) and the optimizer classes (R/optimizer_classes.R).

The numerics all run through the C ABI.  `para_update` uses the
device-resident model (ace_model_para_update): X, Z and y stay in HBM, the
n x n x B cube is never built, and `Kmat`, `Karray` and `invKmatn` become
on-demand handles that are materialised (at the theta they refer to) only
when a caller reads them (SURVEY.md §7 hard part ii).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native
from ._lib import KIND, UNIQUE_ID_BYTES, AceError, check, default_context, fmat, lib, ptr


class DeviceModel:
    """ace_model handle: one fit's resident data and the last inverse."""

    def __init__(self, kind, n, p, B, ctx=None, world=1, rank=0, unique_id=None,
                 sharded=False, host_comm=None):
        """sharded=False: one GPU (ace_model_create).  sharded=True: rank
        `rank` of a `world`-rank block-column-sharded model
        (ace_model_create_sharded): unique_id = the 128 bytes rank 0 got from
        comm_unique_id() (RCCL, one process per GPU), or None to simulate all
        ranks in this process (validation mode).  host_comm (a HostComm):
        the collectives go through torch.distributed on host buffers
        (ace_model_create_sharded_host; validation over gloo)."""
        self.ctx = ctx or default_context()
        self.kind, self.n, self.p, self.B = kind, n, p, B
        self.P = 2 + B * (p + 1)
        self.world, self.rank = (world, rank) if sharded else (1, 0)
        h = ctypes.c_void_p()
        if sharded and host_comm is not None:
            self._host_comm = host_comm  # keeps the callbacks alive
            check(lib().ace_model_create_sharded_host(self.ctx.handle, KIND[kind], n, p, B,
                                                      int(world), int(rank),
                                                      ctypes.byref(host_comm.ops),
                                                      ctypes.byref(h)),
                  self.ctx.handle)
        elif sharded:
            if unique_id is not None and len(unique_id) != UNIQUE_ID_BYTES:
                raise ValueError("unique_id must be 128 bytes")
            check(lib().ace_model_create_sharded(self.ctx.handle, KIND[kind], n, p, B, int(world),
                                                 int(rank), unique_id, ctypes.byref(h)),
                  self.ctx.handle)
        else:
            check(lib().ace_model_create(self.ctx.handle, KIND[kind], n, p, B, ctypes.byref(h)),
                  self.ctx.handle)
        self.handle = h

    def set_data(self, y, X, Z, std_y):
        yv = np.ascontiguousarray(np.ravel(y), dtype=np.float64)
        Xf = fmat(X)
        Zf = np.asfortranarray(np.asarray(Z, dtype=np.float64).reshape(self.n, -1))
        check(lib().ace_model_set_data(self.handle, ptr(yv), ptr(Xf), ptr(Zf), float(std_y)),
              self.ctx.handle)

    def para_update(self, it, theta):
        """theta (float64, P) is mutated at it == 1 (mu overwrite)."""
        g = np.empty(self.P)
        st = np.empty(2)
        mu = ctypes.c_double()
        check(lib().ace_model_para_update(self.handle, int(it), ptr(theta), ptr(g), ptr(st),
                                          ctypes.cast(ctypes.pointer(mu),
                                                      ctypes.POINTER(ctypes.c_double))),
              self.ctx.handle)
        return g, st, mu.value

    def train(self, theta, optimizer="Nadam", learning_rate=0.01, momentum=0.0, beta1=0.9,
              beta2=0.999, norm_clip=True, clip_at=1.0, maxiter=1000, tol=1e-4):
        """ace_model_train: the whole ace.train loop natively (R/main_ace.R:213-235).
        theta (float64, P) is updated in place; returns (stats 2 x (maxiter+2),
        iterations, converged)."""
        from ._lib import OPTIMIZER
        if optimizer == "GD":
            momentum = 0.0
        stats = np.zeros((2, maxiter + 2), order="F")
        it = ctypes.c_int()
        conv = ctypes.c_int()
        check(lib().ace_model_train(self.handle, OPTIMIZER[optimizer], float(learning_rate),
                                    float(momentum), float(beta1), float(beta2),
                                    1 if norm_clip else 0, float(clip_at), int(maxiter),
                                    float(tol), ptr(theta), ptr(stats), ctypes.byref(it),
                                    ctypes.byref(conv)), self.ctx.handle)
        return stats, it.value, bool(conv.value)

    def train_stats(self, theta):
        th = np.ascontiguousarray(theta, dtype=np.float64)
        st = np.empty(2)
        check(lib().ace_model_train_stats(self.handle, ptr(th), ptr(st)), self.ctx.handle)
        return st

    def inverse(self):
        out = np.empty((self.n, self.n), order="F")
        check(lib().ace_model_get_inverse(self.handle, ptr(out)), self.ctx.handle)
        return out

    def apply_inverse(self, V):
        """ace_model_apply_inverse: A^-1 V with the resident inverse (V n x k)."""
        Vf = np.asfortranarray(np.asarray(V, dtype=np.float64).reshape(self.n, -1))
        out = np.empty_like(Vf, order="F")
        check(lib().ace_model_apply_inverse(self.handle, Vf.shape[1], ptr(Vf), ptr(out)),
              self.ctx.handle)
        return out if np.ndim(V) == 2 else out.ravel()

    def predict(self, theta, X2, Z2, mean_y, std_y):
        """ace_model_predict: pred_cpp with the resident inverse (Q6), kernels at theta."""
        th = np.ascontiguousarray(np.ravel(theta), dtype=np.float64)
        X2f = fmat(X2)
        nx = X2f.shape[0]
        Z2f = np.asfortranarray(np.asarray(Z2, dtype=np.float64).reshape(nx, -1))
        mp, var = np.empty(nx), np.empty(nx)
        ci = np.empty((nx, 2), order="F")
        check(lib().ace_model_predict(self.handle, ptr(th), nx, ptr(X2f), ptr(Z2f), float(mean_y),
                                      float(std_y), ptr(mp), ptr(ci), ptr(var)), self.ctx.handle)
        return {"map": mp, "ci": ci, "var": var}

    def predict_marginal(self, theta, X2, dZ2, Z_x, std_y, std_Z, calculate_ate):
        """ace_model_predict_marginal: pred_marginal_cpp with the resident inverse."""
        th = np.ascontiguousarray(np.ravel(theta), dtype=np.float64)
        X2f = fmat(X2)
        nx = X2f.shape[0]
        dZf = np.asfortranarray(np.asarray(dZ2, dtype=np.float64).reshape(nx, -1))
        zx = (np.ascontiguousarray(np.ravel(Z_x), dtype=np.float64)
              if calculate_ate else None)
        mp, var, avg = np.empty(nx), np.empty(nx), np.empty(12)
        ci = np.empty((nx, 2), order="F")
        check(lib().ace_model_predict_marginal(self.handle, ptr(th), nx, ptr(X2f), ptr(dZf),
                                               ptr(zx), float(std_y),
                                               float(np.ravel([std_Z])[0]),
                                               1 if calculate_ate else 0, ptr(mp), ptr(ci),
                                               ptr(var), ptr(avg)), self.ctx.handle)
        out = {"map": mp, "ci": ci, "var": var}
        if calculate_ate:
            for j, key in enumerate(("ate", "att", "atu")):
                a = avg[4 * j:4 * j + 4]
                out[key] = {"map": a[0], "ci": np.array([a[1], a[2]]), "var": a[3]}
        return out

    def comm_calls(self):
        """ace_model_comm_calls: collectives this rank issued since creation,
        {"broadcast", "allgather", "allreduce", "groups"} (zeros when simulated)."""
        c = (ctypes.c_int64 * 4)()
        check(lib().ace_model_comm_calls(self.handle, c), self.ctx.handle)
        return dict(zip(("broadcast", "allgather", "allreduce", "groups"), c))

    def profile(self, enable):
        check(lib().ace_model_profile(self.handle, 1 if enable else 0), self.ctx.handle)

    def kernel_time(self, which):
        ms = ctypes.c_double()
        nl = ctypes.c_int64()
        work = ctypes.c_double()
        check(lib().ace_model_kernel_time(self.handle, which, ctypes.byref(ms), ctypes.byref(nl),
                                          ctypes.byref(work)), self.ctx.handle)
        return ms.value, nl.value, work.value

    def close(self):
        if getattr(self, "handle", None):
            lib().ace_model_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def comm_unique_id():
    """ace_comm_unique_id: the RCCL bootstrap id (rank 0 calls it and sends
    the bytes to every rank out of band)."""
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    check(lib().ace_comm_unique_id(buf), None)
    return buf.raw


class _KernelClass:
    """Common body of KernelClass_SE_R6 / KernelClass_Matern32_R6."""

    kernel = None  # "SE" | "Matern32"

    def __init__(self, p_arg, B_arg, ext_init_parameters, std_y_arg=1.0, verbose=False,
                 ctx=None):
        if verbose:
            print("Using SE kernel" if self.kernel == "SE" else "Using Matern 3/2 kernel")
        self.B = int(B_arg)
        self.p = int(p_arg)
        self.parameters = np.array(np.ravel(ext_init_parameters), dtype=np.float64)
        self.stdy = float(std_y_arg)
        self.ctx = ctx
        self._model = None
        self._data_id = None
        self._kern_theta = None   # theta of the current Kmat / Karray handle
        self._kern_data = None    # (X, Z) they are evaluated on
        self._kcache = None
        self._inv = None          # explicit inverse (getinv_kernel path)
        self._inv_from_model = False

    # ----------------------------------------------------------- R6 fields
    @property
    def Kmat(self):
        return self._materialise()["full"] if self._kern_theta is not None else None

    @property
    def Karray(self):
        return self._materialise()["elements"] if self._kern_theta is not None else None

    @property
    def invKmatn(self):
        if self._inv_from_model:
            if self._inv is None:
                self._inv = self._model.inverse()
            return self._inv
        return self._inv

    def _materialise(self):
        if self._kcache is None:
            X, Z = self._kern_data
            f = (native.kernmat_SE_symmetric_cpp if self.kernel == "SE"
                 else native.kernmat_Matern32_symmetric_cpp)
            self._kcache = f(X, Z, self._kern_theta, ctx=self.ctx)
        return self._kcache

    def _mark_kernel(self, X, Z):
        self._kern_theta = self.parameters.copy()
        self._kern_data = (X, Z)
        self._kcache = None

    # ----------------------------------------------------------- R6 methods
    def kernel_mat(self, X1, X2, Z1, Z2):
        f = native.kernmat_SE_cpp if self.kernel == "SE" else native.kernmat_Matern32_cpp
        return f(X1, X2, Z1, Z2, self.parameters, ctx=self.ctx)

    def kernel_mat_sym(self, X, Z):
        f = (native.kernmat_SE_symmetric_cpp if self.kernel == "SE"
             else native.kernmat_Matern32_symmetric_cpp)
        Klist = f(X, Z, self.parameters, ctx=self.ctx)
        self._kern_theta = self.parameters.copy()
        self._kern_data = (X, Z)
        self._kcache = Klist
        return Klist

    def getinv_kernel(self, X, Z):
        self.kernel_mat_sym(X, Z)
        lst = native.invkernel_cpp(self.Kmat, self.parameters[0], ctx=self.ctx)
        self._inv = lst["inv"]
        self._inv_from_model = False
        return lst

    def _ensure_model(self, y, X, Z):
        key = (id(y), id(X), id(Z))
        n = np.asarray(X).shape[0]
        if self._model is None or self._data_id != key:
            self._model = DeviceModel(self.kernel, n, self.p, self.B, self.ctx)
            self._model.set_data(y, X, Z, self.stdy)
            self._data_id = key
        return self._model

    def use_model(self, model, y, X, Z):
        """Attach an already-created DeviceModel (e.g. a sharded one) holding
        y, X, Z; para_update then runs on it."""
        model.set_data(y, X, Z, self.stdy)
        self._model = model
        self._data_id = (id(y), id(X), id(Z))
        return model

    def para_update(self, iter, y, X, Z, Optim, printevery=100, verbose=True):  # noqa: A002
        """R/kernel_SE_R6.R:40-62 (R/kernel_Matern32_R6.R:39-60)."""
        model = self._ensure_model(y, X, Z)
        self._mark_kernel(X, Z)
        gradients, stats, mu_post = model.para_update(iter, self.parameters)
        self._inv = None
        self._inv_from_model = True
        self.parameters = Optim.update(iter, self.parameters, gradients)
        self.parameters[1] = mu_post  # mean_solution with this iteration's inverse
        if verbose and iter % printevery == 0:
            print("%5d | log Evidence %9.4f | RMSE %9.4f | Norm. noise var: %3.4f | "
                  "Gradient L2: %3.4f" % (iter, stats[1], stats[0], np.exp(self.parameters[0]),
                                          np.linalg.norm(gradients)))
        return stats

    def get_train_stats(self, y, X, Z, invKmatList=None):
        """R/kernel_SE_R6.R:63-74: fresh kernel + inverse at the current theta,
        stats_cpp with mu = theta[1]; the stored inverse is NOT replaced (Q6)."""
        if invKmatList is not None:
            self.kernel_mat_sym(X, Z)
            return native.stats_cpp(y, self.Kmat, invKmatList["inv"], invKmatList["eigenval"],
                                    self.parameters[1], self.stdy, ctx=self.ctx)
        model = self._ensure_model(y, X, Z)
        self._mark_kernel(X, Z)
        return model.train_stats(self.parameters)

    def _resident(self, y, X, Z):
        """The device model holds this fit's inverse (invKmatn never replaced
        from outside) and was built on the same training data."""
        return (self._inv_from_model and self._model is not None and
                self._data_id == (id(y), id(X), id(Z)))

    def predict(self, y, X, Z, X2, Z2, mean_y, std_y):
        """R/kernel_SE_R6.R:75-83.  With the fit's device model the inverse
        stays in HBM (ace_model_predict); otherwise the pred_cpp ABI."""
        if self._resident(y, X, Z):
            return self._model.predict(self.parameters, X2, Z2, mean_y, std_y)
        K_xX = self.kernel_mat(X2, X, Z2, Z)["full"]
        f = (native.kernmat_SE_symmetric_cpp if self.kernel == "SE"
             else native.kernmat_Matern32_symmetric_cpp)
        K_xx = f(X2, Z2, self.parameters, ctx=self.ctx)["full"]
        return native.pred_cpp(y, self.parameters[0], self.parameters[1], self.invKmatn, K_xX,
                               K_xx, mean_y, std_y, ctx=self.ctx)

    def predict_marginal(self, y, X, Z, X2, Z2, dZ2, mean_y, std_y, std_Z, calculate_ate):
        """R/kernel_SE_R6.R:84-97 (device-resident like predict)."""
        if self._resident(y, X, Z):
            return self._model.predict_marginal(self.parameters, X2, dZ2, Z2, std_y, std_Z,
                                                calculate_ate)
        Km_xX = self.kernel_mat(X2, X, dZ2, Z)["elements"]
        f = (native.kernmat_SE_symmetric_cpp if self.kernel == "SE"
             else native.kernmat_Matern32_symmetric_cpp)
        Km_xx = f(X2, dZ2, self.parameters, ctx=self.ctx)["elements"]
        return native.pred_marginal_cpp(y, Z2, self.parameters[0], self.parameters[1],
                                        self.invKmatn, Km_xX, Km_xx, mean_y, std_y, std_Z,
                                        calculate_ate, ctx=self.ctx)

    def mean_solution(self, y):
        """R/kernel_SE_R6.R:99-102 (private in the SE class)."""
        self.parameters[1] = native.mu_solution_cpp(y, self.invKmatn, ctx=self.ctx)


class KernelClass_SE_R6(_KernelClass):
    kernel = "SE"


class KernelClass_Matern32_R6(_KernelClass):
    kernel = "Matern32"


# --------------------------------------------------------------------------
# R/optimizer_classes.R
# --------------------------------------------------------------------------
_NONFINITE = ("Some gradients are not finite, NaN, or NA. Often this is due to too large "
              "learning rates.")


class optAdam:
    def __init__(self, KernelObj, lr, beta1, beta2, norm_clip, clip_at):
        self.m = KernelObj.parameters * 0
        self.v = KernelObj.parameters * 0
        self.lr, self.beta1, self.beta2 = lr, beta1, beta2
        self.norm_clip, self.clip_at = norm_clip, clip_at

    def update(self, iter, parameters, gradients):  # noqa: A002
        native.norm_clip_cpp(self.norm_clip, gradients, self.clip_at)
        if not native.Adam_cpp(iter, self.lr, self.beta1, self.beta2, 1e-8, self.m, self.v,
                               gradients, parameters):
            raise AceError(_NONFINITE)
        return parameters


class optNadam(optAdam):
    def update(self, iter, parameters, gradients):  # noqa: A002
        native.norm_clip_cpp(self.norm_clip, gradients, self.clip_at)
        if not native.Nadam_cpp(iter, self.lr, self.beta1, self.beta2, 1e-8, self.m, self.v,
                                gradients, parameters):
            raise AceError(_NONFINITE)
        return parameters


class optNesterov:
    def __init__(self, KernelObj, lr, momentum, norm_clip, clip_at):
        self.nu = KernelObj.parameters * 0
        self.lr, self.momentum = lr, momentum
        self.norm_clip, self.clip_at = norm_clip, clip_at

    def update(self, iter, parameters, gradients):  # noqa: A002
        native.norm_clip_cpp(self.norm_clip, gradients, self.clip_at)
        if not native.Nesterov_cpp(self.lr, self.momentum, self.nu, gradients, parameters):
            raise AceError(_NONFINITE)
        return parameters


def set_optimizer(optimizer, myKernel, learning_rate, momentum, beta1, beta2, norm_clip,
                  clip_at):
    """R/utilities.R:8-21"""
    if optimizer == "Adam":
        return optAdam(myKernel, learning_rate, beta1, beta2, norm_clip, clip_at)
    if optimizer == "Nadam":
        return optNadam(myKernel, learning_rate, beta1, beta2, norm_clip, clip_at)
    if optimizer in ("GD", "NAG"):
        if optimizer == "GD":
            momentum = 0.0
        return optNesterov(myKernel, learning_rate, momentum, norm_clip, clip_at)
    raise AceError(f"unknown optimizer {optimizer!r}")
