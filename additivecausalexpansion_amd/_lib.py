"""ctypes binding of the C ABI declared in include/ace_hip.h.

The shared library `libace_hip.so` is built in-tree (see build.py).  There is
no CPU fallback: if the library (or a GPU, for device entry points) is
missing, calls raise AceError.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ACE_LIB_PATH") or os.path.join(_HERE, "libace_hip.so")

ACE_KERNEL_SE = 0
ACE_KERNEL_MATERN32 = 1
KIND = {"SE": ACE_KERNEL_SE, "Matern32": ACE_KERNEL_MATERN32}

_D = ctypes.POINTER(ctypes.c_double)
_I64 = ctypes.c_int64
_vp = ctypes.c_void_p

# name -> (restype, argtypes); must match include/ace_hip.h exactly
SIGNATURES = {
    "ace_abi_version": (ctypes.c_int, []),
    "ace_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "ace_destroy": (None, [_vp]),
    "ace_last_error": (ctypes.c_char_p, [_vp]),
    "ace_set_interrupt_poll": (ctypes.c_int, [_vp, ctypes.c_void_p, ctypes.c_void_p]),
    "ace_kernmat_cross": (ctypes.c_int, [_vp, ctypes.c_int, _I64, _I64, ctypes.c_int, ctypes.c_int,
                                         _D, _D, _D, _D, _D, _D, _D]),
    "ace_kernmat_sym": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int,
                                       _D, _D, _D, _D, _D]),
    "ace_invkernel": (ctypes.c_int, [_vp, _I64, _D, ctypes.c_double, _D, _D]),
    "ace_grad": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int, _D, _D, _D,
                                _D, _D, _D, _D, _D, _D, ctypes.c_double, _D]),
    "ace_stats": (ctypes.c_int, [_vp, _I64, _D, _D, _D, _D, ctypes.c_double, ctypes.c_double,
                                 _D]),
    "ace_mu_solution": (ctypes.c_int, [_vp, _I64, _D, _D, _D]),
    "ace_pred": (ctypes.c_int, [_vp, _I64, _I64, _D, ctypes.c_double, ctypes.c_double, _D, _D,
                                _D, ctypes.c_double, ctypes.c_double, _D, _D, _D]),
    "ace_pred_marginal": (ctypes.c_int, [_vp, _I64, _I64, ctypes.c_int, _D, _D, ctypes.c_double,
                                         ctypes.c_double, _D, _D, _D, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_int, _D, _D,
                                         _D, _D]),
    "ace_dmat_upload": (ctypes.c_int, [_vp, _I64, _I64, _I64, _D, ctypes.POINTER(_vp)]),
    "ace_dmat_dims": (ctypes.c_int, [_vp, ctypes.POINTER(_I64), ctypes.POINTER(_I64),
                                     ctypes.POINTER(_I64)]),
    "ace_dmat_read": (ctypes.c_int, [_vp, _I64, _I64, _D]),
    "ace_dmat_materialized": (ctypes.c_int, [_vp]),
    "ace_dmat_free": (None, [_vp]),
    "ace_kernmat_sym_dev": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int,
                                           _D, _D, _D, ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "ace_kernmat_cross_dev": (ctypes.c_int, [_vp, ctypes.c_int, _I64, _I64, ctypes.c_int,
                                             ctypes.c_int, _D, _D, _D, _D, _D,
                                             ctypes.POINTER(_vp), ctypes.POINTER(_vp)]),
    "ace_invkernel_dev": (ctypes.c_int, [_vp, _vp, ctypes.c_double, _D, ctypes.POINTER(_vp)]),
    "ace_mu_solution_dev": (ctypes.c_int, [_vp, _I64, _D, _vp, _D]),
    "ace_stats_dev": (ctypes.c_int, [_vp, _I64, _D, _vp, _vp, _D, ctypes.c_double,
                                     ctypes.c_double, _D]),
    "ace_grad_dev": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int, _D, _D,
                                    _D, _vp, _vp, _vp, _D, _D, _D, ctypes.c_double, _D]),
    "ace_pred_dev": (ctypes.c_int, [_vp, _I64, _I64, _D, ctypes.c_double, ctypes.c_double, _vp,
                                    _vp, _vp, ctypes.c_double, ctypes.c_double, _D, _D, _D]),
    "ace_pred_marginal_dev": (ctypes.c_int, [_vp, _I64, _I64, _D, _D, ctypes.c_double,
                                             ctypes.c_double, _vp, _vp, _vp, ctypes.c_double,
                                             ctypes.c_double, ctypes.c_double, ctypes.c_int, _D,
                                             _D, _D, _D]),
    "ace_nesterov": (ctypes.c_int, [_I64, ctypes.c_double, ctypes.c_double, _D, _D, _D]),
    "ace_nadam": (ctypes.c_int, [_I64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, _D, _D, _D, _D]),
    "ace_adam": (ctypes.c_int, [_I64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_double, _D, _D, _D, _D]),
    "ace_norm_clip": (None, [ctypes.c_int, _I64, _D, ctypes.c_double]),
    "ace_ncs_basis": (ctypes.c_int, [_I64, _D, _I64, _D, _D, ctypes.POINTER(_I64)]),
    "ace_ncs_basis_deriv": (ctypes.c_int, [_I64, _D, _I64, _D, _D, ctypes.POINTER(_I64)]),
    "ace_normalize_train": (ctypes.c_int, [_I64, ctypes.c_int, ctypes.c_int, _D, _D, _D, _D]),
    "ace_normalize_test": (ctypes.c_int, [_I64, ctypes.c_int, ctypes.c_int, _D, _D, _D, _I64]),
    "ace_model_create": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int, ctypes.c_int,
                                        ctypes.POINTER(_vp)]),
    "ace_model_destroy": (None, [_vp]),
    "ace_model_set_data": (ctypes.c_int, [_vp, _D, _D, _D, ctypes.c_double]),
    "ace_model_para_update": (ctypes.c_int, [_vp, ctypes.c_int, _D, _D, _D, _D]),
    "ace_model_train_stats": (ctypes.c_int, [_vp, _D, _D]),
    "ace_model_get_inverse": (ctypes.c_int, [_vp, _D]),
    "ace_model_apply_inverse": (ctypes.c_int, [_vp, _I64, _D, _D]),
    "ace_model_predict": (ctypes.c_int, [_vp, _D, _I64, _D, _D, ctypes.c_double, ctypes.c_double,
                                         _D, _D, _D]),
    "ace_model_predict_marginal": (ctypes.c_int, [_vp, _D, _I64, _D, _D, _D, ctypes.c_double,
                                                  ctypes.c_double, ctypes.c_int, _D, _D, _D,
                                                  _D]),
    "ace_model_profile": (ctypes.c_int, [_vp, ctypes.c_int]),
    "ace_model_kernel_time": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(_I64),
                                             ctypes.POINTER(ctypes.c_double)]),
    "ace_model_train": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_int, ctypes.c_double, _D, _D,
                                       ctypes.POINTER(ctypes.c_int),
                                       ctypes.POINTER(ctypes.c_int)]),
    "ace_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "ace_model_create_sharded": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_char_p, ctypes.POINTER(_vp)]),
    "ace_model_shard_info": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_int)]),
    "ace_model_comm_calls": (ctypes.c_int, [_vp, ctypes.POINTER(_I64)]),
    "ace_model_create_sharded_host": (ctypes.c_int, [_vp, ctypes.c_int, _I64, ctypes.c_int,
                                                     ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                     ctypes.c_void_p, ctypes.POINTER(_vp)]),
}

# ace_comm_ops (include/ace_hip.h): host-callback collectives
BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _D, _I64, ctypes.c_int)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _D, _D, _I64)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _D, _I64, ctypes.c_int)


class CommOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("broadcast", BCAST_FN),
                ("allgather", ALLGATHER_FN), ("allreduce", ALLREDUCE_FN)]
UNIQUE_ID_BYTES = 128

STATUS = {0: "ACE_OK", 1: "ACE_ERR_ARG", 2: "ACE_ERR_HIP", 3: "ACE_ERR_OOM",
          4: "ACE_ERR_UNSUPPORTED", 5: "ACE_ERR_NONFINITE", 6: "ACE_ERR_INTERRUPTED", 7: "ACE_ERR_TIMEOUT"}
POLL_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
OPTIMIZER = {"GD": 0, "NAG": 0, "Adam": 1, "Nadam": 2}


class AceError(RuntimeError):
    """A non-zero ace_status (the Rcpp shim maps these to Rcpp::stop)."""


_lib = None
_lock = threading.Lock()


def lib():
    """Load libace_hip.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise AceError(f"{LIB_PATH} is missing: run __graft_entry__.build() "
                               "(there is no CPU fallback)")
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                # an older library built for an A/B run may lack newer entry
                # points: they stay unbound (calling one raises AttributeError);
                # tests/test_abi_cpu.py checks the in-tree library exports all
                f = getattr(L, name, None)
                if f is None:
                    continue
                f.restype = res
                f.argtypes = args
            _lib = L
    return _lib


def ptr(a):
    """double* of a contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    assert a.dtype == np.float64 and (a.flags.f_contiguous or a.flags.c_contiguous)
    return a.ctypes.data_as(_D)


def check(status, ctx=None):
    if status != 0:
        msg = lib().ace_last_error(ctx)
        raise AceError(f"{STATUS.get(status, status)}: {msg.decode() if msg else ''}")


class Context:
    """One ace_ctx (one HIP device, one stream) -- one process per GPU."""

    def __init__(self, device=None):
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = device
        h = _vp()
        check(lib().ace_create(device, ctypes.byref(h)), None)
        self.handle = h

    def set_interrupt_poll(self, fn):
        """fn() -> bool, polled between training iterations (ace_set_interrupt_poll);
        None removes it."""
        self._poll = None if fn is None else POLL_FN(lambda _u: 1 if fn() else 0)
        ptr_ = ctypes.cast(self._poll, ctypes.c_void_p) if self._poll is not None else None
        check(lib().ace_set_interrupt_poll(self.handle, ptr_, None), self.handle)

    def close(self):
        if getattr(self, "handle", None):
            lib().ace_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx = None


def default_context():
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context()
    return _default_ctx


def fmat(a, shape=None):
    """Column-major float64 copy/view (R/Armadillo layout)."""
    a = np.asarray(a, dtype=np.float64)
    if shape is not None:
        a = a.reshape(shape, order="F") if a.ndim != len(shape) else a
    return np.asfortranarray(a)
