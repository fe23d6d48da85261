import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as f:
        return {k: f[k] for k in f.files}


def golden_names(prefix):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


@pytest.fixture(scope="session")
def ref_c():
    """The literal C restatement (oracle/libace_ref.so), built on demand."""
    import ctypes
    import subprocess
    so = os.path.join(ROOT, "oracle", "libace_ref.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    L = ctypes.CDLL(so)
    D = ctypes.POINTER(ctypes.c_double)
    I64 = ctypes.c_int64
    L.ref_kernmat_sym.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D]
    L.ref_kernmat_cross.argtypes = [ctypes.c_int, I64, I64, ctypes.c_int, ctypes.c_int, D, D, D, D,
                                    D, D, D]
    L.ref_grad.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D,
                           ctypes.c_double, D, D, ctypes.c_double, D]
    L.ref_mu_solution.argtypes = [I64, D, D]
    L.ref_mu_solution.restype = ctypes.c_double
    return L
