"""Line-by-line mirror of the reference's unchanged R6 kernel classes
(R/kernel_SE_R6.R:2-103, R/kernel_Matern32_R6.R:2-99), driving the Rcpp
surface exactly as the R code does -- kernmat_*_symmetric_cpp ->
invkernel_cpp -> mu_solution_cpp -> grad_*_cpp -> Optim$update ->
mu_solution_cpp, and kernmat + pred_cpp / pred_marginal_cpp for predict --
with the matrices held as device handles (native.DMat, the Python face of
the ace_dmat handles the R shim wraps in ALTREP vectors).

This is the drop-in path for an unmodified R package: no n x n matrix and
no n x n x B `elements` cube crosses PCIe unless R code reads one.  The
fused device model (model.py, ace_model_*) remains the fast path the
package's own classes use.
"""
from __future__ import annotations

import numpy as np

from . import native


class _R6Kernel:
    kernel = None  # "SE" | "Matern32"

    def __init__(self, p_arg, B_arg, ext_init_parameters, std_y_arg=1.0, verbose=False,
                 ctx=None, handles=True):
        if verbose:
            print("Using SE kernel" if self.kernel == "SE" else "Using Matern 3/2 kernel")
        self.B = int(B_arg)
        self.p = int(p_arg)
        self.parameters = np.array(np.ravel(ext_init_parameters), dtype=np.float64)
        self.stdy = float(std_y_arg)
        self.invKmatn = None
        self.Kmat = None
        self.Karray = None
        self.ctx = ctx
        self.handles = handles

    # the R class's .Call targets
    def _sym(self, X, Z):
        f = (native.kernmat_SE_symmetric_cpp if self.kernel == "SE"
             else native.kernmat_Matern32_symmetric_cpp)
        return f(X, Z, self.parameters, ctx=self.ctx, device=self.handles)

    def _cross(self, X1, X2, Z1, Z2):
        f = native.kernmat_SE_cpp if self.kernel == "SE" else native.kernmat_Matern32_cpp
        return f(X1, X2, Z1, Z2, self.parameters, ctx=self.ctx, device=self.handles)

    def _grad(self, *a):
        f = native.grad_SE_cpp if self.kernel == "SE" else native.grad_Matern_cpp
        return f(*a, ctx=self.ctx)

    # ------------------------------------------------------------ R6 methods
    def kernel_mat(self, X1, X2, Z1, Z2):
        """R/kernel_SE_R6.R:21-24"""
        return self._cross(X1, X2, Z1, Z2)

    def kernel_mat_sym(self, X, Z):
        """R/kernel_SE_R6.R:25-31"""
        Klist = self._sym(X, Z)
        self.Kmat = Klist["full"]
        self.Karray = Klist["elements"]
        return Klist

    def getinv_kernel(self, X, Z):
        """R/kernel_SE_R6.R:32-38"""
        self.kernel_mat_sym(X, Z)
        invKmatList = native.invkernel_cpp(self.Kmat, self.parameters[0], ctx=self.ctx)
        self.invKmatn = invKmatList["inv"]
        return invKmatList

    def para_update(self, iter, y, X, Z, Optim, printevery=100, verbose=True):  # noqa: A002
        """R/kernel_SE_R6.R:39-62 (R/kernel_Matern32_R6.R:39-60)"""
        stats = np.zeros(2)
        eigenval = self.getinv_kernel(X, Z)["eigenval"]
        if iter == 1:
            self.mean_solution(y)
        gradients = self._grad(y, X, Z, self.Kmat, self.Karray, self.invKmatn, eigenval,
                               self.parameters, stats, self.B, self.stdy)
        self.parameters = Optim.update(iter, self.parameters, gradients)
        self.mean_solution(y)
        if iter % printevery == 0 and verbose:
            print("%5d | log Evidence %9.4f | RMSE %9.4f | Norm. noise var: %3.4f | "
                  "Gradient L2: %3.4f" % (iter, stats[1], stats[0], np.exp(self.parameters[0]),
                                          np.linalg.norm(gradients)))
        return stats

    def get_train_stats(self, y, X, Z, invKmatList=None):
        """R/kernel_SE_R6.R:63-74"""
        if invKmatList is None:
            Klist = self.kernel_mat_sym(X, Z)
            invKmatList = native.invkernel_cpp(Klist["full"], self.parameters[0], ctx=self.ctx)
        return native.stats_cpp(y, self.Kmat, invKmatList["inv"], invKmatList["eigenval"],
                                self.parameters[1], self.stdy, ctx=self.ctx)

    def predict(self, y, X, Z, X2, Z2, mean_y, std_y):
        """R/kernel_SE_R6.R:75-83"""
        K_xX = self._cross(X2, X, Z2, Z)["full"]
        K_xx = self._sym(X2, Z2)["full"]
        return native.pred_cpp(y, self.parameters[0], self.parameters[1], self.invKmatn, K_xX,
                               K_xx, mean_y, std_y, ctx=self.ctx)

    def predict_marginal(self, y, X, Z, X2, Z2, dZ2, mean_y, std_y, std_Z, calculate_ate):
        """R/kernel_SE_R6.R:84-97"""
        Kmarginal_xX = self._cross(X2, X, dZ2, Z)["elements"]
        Kmarginal_xx = self._sym(X2, dZ2)["elements"]
        return native.pred_marginal_cpp(y, Z2, self.parameters[0], self.parameters[1],
                                        self.invKmatn, Kmarginal_xX, Kmarginal_xx, mean_y,
                                        std_y, std_Z, calculate_ate, ctx=self.ctx)

    def mean_solution(self, y):
        """R/kernel_SE_R6.R:99-102 (private in the SE class, public in Matern32)"""
        self.parameters[1] = native.mu_solution_cpp(y, self.invKmatn, ctx=self.ctx)


class R6KernelSE(_R6Kernel):
    kernel = "SE"


class R6KernelMatern32(_R6Kernel):
    kernel = "Matern32"
