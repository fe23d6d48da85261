"""User API mirror: ace.train / predict.ace (R/main_ace.R:132-254,
R/predict.ace.R:30-99), the basis classes (R/spline_*_R6.R) and the
parameter initialisation (R/parameters.R).  Host preprocessing; the hot
path underneath is the device-resident para_update (model.py).
"""
from __future__ import annotations

import math

import numpy as np

from . import native
from ._lib import AceError
from .model import KernelClass_Matern32_R6, KernelClass_SE_R6, set_optimizer


# --------------------------------------------------------------------------
# Basis classes
# --------------------------------------------------------------------------
class linear_spline:
    """R/spline_linear_R6.R"""

    def __init__(self):
        self.B = self.dB = None

    def dim(self):
        return self.B.shape[1] + 1

    def trainbasis(self, Z, n_knots, verbose=False):
        if verbose:
            print("Using binary/linear-basis")
        n = np.asarray(Z).size
        self.B = np.asfortranarray(np.asarray(Z, dtype=np.float64).reshape(n, 1))
        self.dB = np.ones((n, 1), order="F")
        return self.B

    def testbasis(self, Znew=None):
        if Znew is not None:
            z = np.ravel(np.asarray(Znew, dtype=np.float64))
            return {"B": z.reshape(-1, 1).copy(order="F"), "dB": np.ones((z.size, 1), order="F")}
        return {"B": self.B.copy(order="F"), "dB": self.dB.copy(order="F")}


class square_spline:
    """R/spline_square_R6.R"""

    def __init__(self):
        self.B = self.dB = None

    def dim(self):
        return self.B.shape[1] + 1

    def trainbasis(self, Z, n_knots, verbose=False):
        if verbose:
            print("Using square-basis")
        z = np.ravel(np.asarray(Z, dtype=np.float64))
        self.B = np.asfortranarray(np.column_stack([z, z ** 2]))
        self.dB = np.asfortranarray(np.column_stack([np.ones_like(z), 2 * z]))
        return self.B

    def testbasis(self, Znew=None):
        if Znew is not None:
            z = np.ravel(np.asarray(Znew, dtype=np.float64))
            return {"B": np.asfortranarray(np.column_stack([z, z ** 2])),
                    "dB": np.asfortranarray(np.column_stack([np.ones_like(z), 2 * z]))}
        return {"B": self.B, "dB": self.dB}


class ns_spline:
    """R/spline_ns_R6.R: internal knots at type-7 quantiles, boundary (-1, 1)."""

    def __init__(self):
        self.B = self.dB = self.myknots = None

    def dim(self):
        return self.B.shape[1] + 1

    def trainbasis(self, Z, n_knots, verbose=False):
        if verbose:
            print("Using natural cubic-spline")
        z = np.ravel(np.asarray(Z, dtype=np.float64))
        if n_knots > 0:
            ik = np.quantile(z, np.arange(1, n_knots + 1) / (n_knots + 1), method="linear")
        else:
            ik = np.array([])
        self.myknots = np.concatenate([ik, [-1.0, 1.0]])
        self.B = native.ncs_basis(z, self.myknots)
        self.dB = native.ncs_basis_deriv(z, self.myknots)
        return self.B

    def testbasis(self, Znew=None):
        if Znew is not None:
            return {"B": native.ncs_basis(Znew, self.myknots),
                    "dB": native.ncs_basis_deriv(Znew, self.myknots)}
        return {"B": self.B, "dB": self.dB}


def set_basis(basis, isuniv):
    """R/utilities.R:23-30.  "B" (splines2::bSpline) is not available here."""
    if basis in ("binary", "linear"):
        return linear_spline()
    if isuniv and basis == "B":
        raise AceError("basis 'B' needs splines2::bSpline (not available); use 'ns'")
    if isuniv and basis == "square":
        return square_spline()
    if isuniv:
        return ns_spline()  # "cubic", "ns" and anything else
    raise AceError("multivariate Z is not supported by the reference either")


def set_initial_parameters(p, B, n, y, X, Z, init_sigma=None, init_length_scale=20.0,
                           verbose=False):
    """R/parameters.R:1-23.  ace.train always passes init.sigma, so the OLS
    residual variance of y on [X, Z, 1] is always used (see oracle notes)."""
    Xm = np.column_stack([X, Z, np.ones(n)])
    Q, R = np.linalg.qr(Xm)
    rank = int(np.sum(np.abs(np.diag(R)) > 1e-7 * np.abs(R).max()))
    Q = Q[:, :rank]
    yv = np.ravel(y)
    init_sigma = math.log(float(yv @ (yv - Q @ (Q.T @ yv))) / (n - 1))
    if verbose:
        print("Initial noise variance: ", math.exp(init_sigma))
    return np.concatenate([[init_sigma, 0.0], -np.log(np.ones(B)),
                           np.log(np.full(B * p, init_length_scale))])


class AceFit(dict):
    """The S3 "ace" list (R/main_ace.R:242-253)."""


def ace_train(y, X, Z, pi=None, kernel="SE", basis="linear", n_knots=1, optimizer="Nadam",
              maxiter=1000, tol=1e-4, learning_rate=0.01, beta1=0.9, beta2=0.999, momentum=0.0,
              norm_clip=None, clip_at=1.0, init_sigma=None, init_length_scale=20.0,
              plot_stats=False, verbose=True, ctx=None, native_loop=False):
    """R/main_ace.R:132-254 (ace.train).  native_loop=True runs the optimisation
    loop inside the library (ace_model_train: no per-iteration round trip
    through Python; same arithmetic, so the same trajectory)."""
    if norm_clip is None:
        norm_clip = optimizer in ("Adam", "Nadam")  # R/main_ace.R:143 (Q5)
    yv = np.array(np.ravel(y), dtype=np.float64)
    n = yv.shape[0]
    Xi = np.array(X, dtype=np.float64, order="F", copy=True)
    if Xi.ndim == 1:
        Xi = Xi.reshape(n, 1, order="F")
    px = Xi.shape[1]
    Zi = np.array(Z, dtype=np.float64, order="F", copy=True)
    if Zi.ndim == 1:
        Zi = Zi.reshape(n, 1, order="F")
    pz = Zi.shape[1]
    if Xi.shape != (n, px):
        raise AceError("Dimension of X not correct.")
    if Zi.shape != (n, pz):
        raise AceError("Dimension of Z not correct.")
    moments = native.normalize_train(yv, Xi, Zi)
    isuniv = pz == 1
    isbinary = moments[1 + px:1 + px + pz, 2] == 1
    if np.all(isbinary):
        if verbose:
            print("Assuming binary Z")
        if pi is None:
            basis = "binary"
    elif verbose:
        print("Non-Binary Z detected")
    if pi is not None and isuniv:
        pint = np.ravel(np.asarray(pi, dtype=np.float64)).reshape(n, 1)
        if not isbinary[0]:
            pint = (pint - moments[1 + px, 0]) / moments[1 + px, 1]
        Zi = np.asfortranarray(Zi - pint)
    myBasis = set_basis(basis, isuniv)
    myBasis.trainbasis(Zi, n_knots, verbose)
    theta0 = set_initial_parameters(px, myBasis.dim(), n, yv, Xi, Zi, init_sigma,
                                    init_length_scale, verbose)
    Kc = KernelClass_Matern32_R6 if kernel == "Matern32" else KernelClass_SE_R6
    myKernel = Kc(px, myBasis.dim(), theta0, moments[0, 1], verbose, ctx=ctx)
    myOptimizer = set_optimizer(optimizer, myKernel, learning_rate, momentum, beta1, beta2,
                                norm_clip, clip_at)
    if native_loop:
        model = myKernel._ensure_model(yv, Xi, myBasis.B)
        theta = np.ascontiguousarray(myKernel.parameters, dtype=np.float64)
        stats, it, convergence = model.train(theta, optimizer, learning_rate, momentum, beta1,
                                             beta2, norm_clip, clip_at, maxiter, tol)
        myKernel.parameters = theta
        myKernel._mark_kernel(Xi, myBasis.B)
        myKernel._inv = None
        myKernel._inv_from_model = True
        if verbose:
            print("Final training log Evidence: ", stats[1, it + 1])
        stats = stats[:, 2:it + 2]
        return AceFit(Kernel=myKernel, Basis=myBasis,
                      OptimSettings={"optim": optimizer, "lr": learning_rate, "momentum": momentum,
                                     "beta1": beta1, "beta2": beta2},
                      moments=moments,
                      train_data={"y": yv, "X": Xi, "Z": Zi, "Zbinary": isbinary},
                      train_stats={"RIC_bias_corrected": pi is not None,
                                   "init.length_scale": init_length_scale,
                                   "convergence": convergence, "final_evidence": stats[1, -1],
                                   "stats": stats})
    stats = np.zeros((2, maxiter + 2))
    it = 0
    for it in range(1, maxiter + 1):
        stats[:, it] = myKernel.para_update(it, yv, Xi, myBasis.B, myOptimizer, verbose=verbose)
        change = abs(stats[1, it] - stats[1, it - 1])
        if change < tol and it > 3:
            if verbose:
                print(f"Stopped: change smaller than tolerance after {it} iterations")
            break
    convergence = it < maxiter
    stats[:, it + 1] = myKernel.get_train_stats(yv, Xi, myBasis.B)
    if verbose and not convergence:
        print("WARNING NO CONVERGENCE - Optimization stopped: maximum iterations reached")
    if verbose:
        print("Final training log Evidence: ", stats[1, it + 1])
    stats = stats[:, 2:it + 2]
    return AceFit(Kernel=myKernel, Basis=myBasis,
                  OptimSettings={"optim": optimizer, "lr": learning_rate, "momentum": momentum,
                                 "beta1": beta1, "beta2": beta2},
                  moments=moments,
                  train_data={"y": yv, "X": Xi, "Z": Zi, "Zbinary": isbinary},
                  train_stats={"RIC_bias_corrected": pi is not None,
                               "init.length_scale": init_length_scale,
                               "convergence": convergence, "final_evidence": stats[1, -1],
                               "stats": stats})


def predict_ace(obj, newX=None, newZ=None, marginal=False, return_average_treatments=False,
                normalize=True):
    """R/predict.ace.R:30-99 (predict.ace)."""
    isbinary = obj["train_data"]["Zbinary"]
    X = obj["train_data"]["X"]
    px = X.shape[1]
    pz = obj["train_data"]["Z"].shape[1]
    mom = obj["moments"]
    if newX is None and newZ is None:
        Xn = X
        Zn = obj["train_data"]["Z"]
    elif newX is None:
        Xn = np.array(X, order="F", copy=True)
        if np.size(newZ) == 1:
            Zn = np.full((Xn.shape[0], 1), float(np.ravel(newZ)[0]), order="F")
        else:
            Zn = np.asfortranarray(np.ravel(newZ).astype(np.float64).reshape(-1, 1))
            if normalize:
                native.normalize_test(Xn, Zn, mom)
            Xn = X
    elif newZ is None:
        Xn = np.array(newX, dtype=np.float64, order="F", copy=True)
        Zn = np.zeros((Xn.shape[0], 1), order="F")
        if normalize:
            native.normalize_test(Xn, Zn, mom)
        Zn = np.zeros((Xn.shape[0], 1), order="F")
    else:
        Xn = np.array(newX, dtype=np.float64, order="F", copy=True)
        if Xn.shape[1] != px:
            raise AceError("Dimension mismatch of X with newX")
        if np.size(newZ) == 1:
            Zn = np.full((Xn.shape[0], 1), float(np.ravel(newZ)[0]), order="F")
        else:
            Zn = np.array(newZ, dtype=np.float64, order="F", copy=True).reshape(-1, pz, order="F")
        if normalize:
            native.normalize_test(Xn, Zn, mom)
    K = obj["Kernel"]
    y = obj["train_data"]["y"]
    Btr = obj["Basis"].B
    if not marginal:
        return K.predict(y, X, Btr, Xn, obj["Basis"].testbasis(Zn)["B"], mom[0, 0], mom[0, 1])
    tb = obj["Basis"].testbasis(Zn)
    return K.predict_marginal(y, X, Btr, Xn, tb["B"], tb["dB"], mom[0, 0], mom[0, 1],
                              mom[1 + px:1 + px + pz, 1],
                              bool(np.all(isbinary)) and return_average_treatments)
