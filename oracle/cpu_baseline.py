"""CPU baseline leg for bench.py (TEST/BENCH INFRASTRUCTURE ONLY).

Times the reference's algorithms on the host for one log-marg-lik + gradient
evaluation (one para_update's native work) on a BOUNDED sample of the bench
workload, and extrapolates to the full size:
  * pair loops (kernmat_*_symmetric_cpp + grad_*_cpp, single-threaded as in
    the reference): the literal C restatement oracle/ace_ref.c, scaled by n^2;
  * invkernel_cpp (eig_sym = LAPACK dsyevd, then V D^-1/2 (V D^-1/2)^T):
    numpy.linalg.eigh + matmul on all host BLAS threads, scaled by n^3.
The extrapolation exponents come from the measured scaling fit committed in
profiles/r*_cpu_baseline.json (oracle/cpu_scaling.py: full evaluations at
n = 2048, 4096, 8192 on the GPU box's host) when one is present -- the pair
loops grow faster than n^2 there (cube traffic) -- else n^2 / n^3.
Prints one JSON line.  PARITY UNPINNED note: see oracle/ace_oracle.py.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384, help="full-size n to extrapolate to")
    ap.add_argument("--sample-n", type=int, default=2048)
    ap.add_argument("--p", type=int, default=20)
    ap.add_argument("--B", type=int, default=10)
    ap.add_argument("--kernel", default="Matern32")
    ap.add_argument("--fit", default=None, help="measured scaling fit (JSON of cpu_scaling.py)")
    a = ap.parse_args()
    e_pairs, e_inv, fit = 2.0, 3.0, None
    if a.fit and os.path.exists(a.fit):
        fit = json.load(open(a.fit))
        e_pairs = fit["fit"]["pairs"]["exponent"]
        e_inv = fit["fit"]["inverse_eigh"]["exponent"]

    import numpy as np

    from additivecausalexpansion_amd.synthetic import make_problem

    so = os.path.join(HERE, "libace_ref.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    L = ctypes.CDLL(so)
    D = ctypes.POINTER(ctypes.c_double)
    I64 = ctypes.c_int64
    L.ref_kernmat_sym.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D]
    L.ref_grad.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D,
                           ctypes.c_double, D, D, ctypes.c_double, D]
    P = lambda x: x.ctypes.data_as(D)  # noqa: E731
    kind = 0 if a.kernel == "SE" else 1
    n, p, B = a.sample_n, a.p, a.B
    y, X, Z, th, sy = make_problem(n, p, B, seed=0)
    X = np.asfortranarray(X)
    Z = np.asfortranarray(Z)
    Kf = np.zeros((n, n), order="F")
    Ke = np.zeros((n, n, B), order="F")
    t0 = time.perf_counter()
    L.ref_kernmat_sym(kind, n, p, B, P(X), P(Z), P(th), P(Kf), P(Ke))
    t_asm = time.perf_counter() - t0
    t0 = time.perf_counter()
    A = Kf.copy()
    A[np.diag_indices(n)] += math.exp(th[0])
    w, V = np.linalg.eigh(A)
    Vs = V / np.sqrt(w)[None, :]
    inv = np.asfortranarray(Vs @ Vs.T)
    t_inv = time.perf_counter() - t0
    st = np.zeros(2)
    g = np.zeros(th.shape[0])
    t0 = time.perf_counter()
    L.ref_grad(kind, n, p, B, P(y), P(X), P(Kf), P(Ke), P(inv), float(np.sum(np.log(w))), P(th),
               P(st), sy, P(g))
    t_grad = time.perf_counter() - t0
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    try:
        cpu = [l for l in open("/proc/cpuinfo") if l.startswith("model name")][0].split(":")[1].strip()
    except Exception:
        cpu = "unknown"
    t_pairs = t_asm + t_grad
    if fit:
        # one C2 figure: the measured fit (full evaluations at n <= 8192 on
        # this host type, oracle/cpu_scaling.py) per component, calibrated by
        # today's sample against the fit's own prediction at the sample size
        f = fit["fit"]
        tgt = fit["c2_extrapolated"]["n"]
        pred_pairs = f["pairs"]["seconds_at_target"] * (n / tgt) ** e_pairs
        pred_inv = f["inverse_eigh"]["seconds_at_target"] * (n / tgt) ** e_inv
        pt = [q for q in fit["points_c2_shape"] if q["n"] == n and q["p"] == p and q["B"] == B]
        if pt:  # a measured point of the fit: compare like with like
            pred_pairs, pred_inv = pt[0]["pairs"], pt[0]["inverse_eigh"]
        r_pairs, r_inv = t_pairs / pred_pairs, t_inv / pred_inv
        sc = (a.n / tgt)
        c2_fit = (f["pairs"]["seconds_at_target"] * sc ** e_pairs +
                  f["inverse_eigh"]["seconds_at_target"] * sc ** e_inv)
        t_full = (f["pairs"]["seconds_at_target"] * sc ** e_pairs * r_pairs +
                  f["inverse_eigh"]["seconds_at_target"] * sc ** e_inv * r_inv)
        how = (f"measured fit {os.path.basename(a.fit)} ({c2_fit:.0f} s at n={a.n}) x today's "
               f"sample / the fit's {'measured point' if pt else 'prediction'} at n={n} (pairs "
               f"{r_pairs:.3f}, inverse {r_inv:.3f})")
    else:
        t_full = t_pairs * (a.n / n) ** e_pairs + t_inv * (a.n / n) ** e_inv
        how = "sample x (n/n_s)^2 pairs, ^3 inverse"
    out = {
        "value": 1.0 / t_full, "unit": "evals/s", "cores": threads, "host_nproc": os.cpu_count(),
        "kind": "port",
        "seconds_per_eval": t_full,
        "sample": (f"one {a.kernel} eval at n={n}, p={p}, B={B}: pair loops {t_pairs:.2f} s "
                   f"single-threaded (as the reference), eigh+inverse {t_inv:.2f} s on {threads} "
                   f"BLAS threads (host nproc {os.cpu_count()}); n={a.n}: {t_full:.0f} s per "
                   f"eval = {how}; host CPU: {cpu}"),
        "sample_seconds": {"assembly": t_asm, "inverse": t_inv, "gradient": t_grad},
        "extrapolated_seconds_per_eval": t_full}
    if fit:
        out["measured_fit"] = {
            "source": os.path.relpath(a.fit, os.path.dirname(HERE)),
            "exponents": {k: v["exponent"] for k, v in fit["fit"].items()},
            "points_seconds_per_eval": {str(q["n"]): q["eval_reference"]
                                        for q in fit["points_c2_shape"]},
            "c2_seconds_per_eval_fit": fit["c2_extrapolated"]["seconds_per_eval_reference"],
            "c2_seconds_per_eval_best_cpu_fit": fit["c2_extrapolated"]["seconds_per_eval_best_cpu"],
            "calibration": {"pairs": r_pairs, "inverse": r_inv},
            "c2_seconds_per_eval": t_full,
            "c1_median_seconds": fit["c1_measured"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
