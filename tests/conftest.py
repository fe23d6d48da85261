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


def record_error(check, measured, bound):
    """Appends one measured error beside the bound it is held to, as a JSON
    line to $ACE_ERROR_LOG (unset: nothing is written).  tools/error_table.py
    turns the log of a GPU run into the committed error table
    (profiles/r06_error_table.txt), so drift toward a bound is visible."""
    path = os.environ.get("ACE_ERROR_LOG")
    if not path:
        return
    import json
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, "check": check, "measured": float(measured),
                            "bound": float(bound)}) + "\n")


def run_child(code, env=None, timeout=100):
    """Runs a Python snippet in a fresh interpreter (a clean HIP runtime per
    A/B variant).  A child that stalls dumps every thread's Python stack
    (faulthandler) 10 s before its limit and exits, so a hang names the call
    it was blocked in; on any failure the child's stdout / stderr tail is in
    the assertion message.  The library's own bounded sync (ACE_SYNC_TIMEOUT)
    is set below the limit so a stalled stream reports which streams held
    work before faulthandler fires."""
    import subprocess
    env = dict(os.environ if env is None else env)
    env.setdefault("ACE_SYNC_TIMEOUT", str(max(5, timeout - 25)))
    pre = f"import faulthandler; faulthandler.dump_traceback_later({max(5, timeout - 10)}, exit=True)\n"
    try:
        r = subprocess.run([sys.executable, "-c", pre + code], env=env, timeout=timeout,
                           capture_output=True, text=True)
    except subprocess.TimeoutExpired as e:
        out = (e.stdout or b"")[-3000:] if isinstance(e.stdout, bytes) else (e.stdout or "")[-3000:]
        err = (e.stderr or b"")[-6000:] if isinstance(e.stderr, bytes) else (e.stderr or "")[-6000:]
        raise AssertionError(f"child timed out after {timeout} s\n--- stdout\n{out}\n--- stderr\n{err}")
    if r.returncode != 0:
        raise AssertionError(f"child exited {r.returncode}\n--- stdout\n{r.stdout[-3000:]}\n"
                             f"--- stderr\n{r.stderr[-6000:]}")
    return r
