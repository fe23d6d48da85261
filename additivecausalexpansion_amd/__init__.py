"""MI355X-native engine for the hot path of the R package `ace` 0.4.1
(ayotoasset/AdditiveCausalExpansion): reduced-kernel assembly, SPD inverse +
log-determinant and hyperparameter gradients as hand-written gfx950 HIP
kernels behind the C ABI in include/ace_hip.h.  See DESIGN.md."""
from ._lib import AceError, Context, default_context, lib  # noqa: F401
from .native import (  # noqa: F401
    DMat, Adam_cpp, Nadam_cpp, Nesterov_cpp, grad_Matern_cpp, grad_SE_cpp, invkernel_cpp,
    kernmat_Matern32_cpp, kernmat_Matern32_symmetric_cpp, kernmat_SE_cpp,
    kernmat_SE_symmetric_cpp, mu_solution_cpp, ncs_basis, ncs_basis_deriv, norm_clip_cpp,
    normalize_test, normalize_train, pred_cpp, pred_marginal_cpp, stats_cpp)
from .model import (  # noqa: F401
    DeviceModel, KernelClass_Matern32_R6, KernelClass_SE_R6, comm_unique_id, optAdam, optNadam,
    optNesterov, set_optimizer)
from .r6 import R6KernelMatern32, R6KernelSE  # noqa: F401
from .train import (  # noqa: F401
    AceFit, ace_train, linear_spline, ns_spline, predict_ace, set_basis,
    set_initial_parameters, square_spline)
