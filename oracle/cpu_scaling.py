"""Measured CPU baseline points and their scaling fit (TEST/BENCH
INFRASTRUCTURE ONLY; run on the GPU box's host).

One log-marg-lik + gradient evaluation of the reference's algorithms, timed
in full (no sampling) at:
  * the C2 shape (p = 20, B = 10, Matern32) at n = 2048, 4096, 8192;
  * C1 (n = 4096, p = 10, B = 6, SE) three times (median reported).
Per evaluation:
  * pair loops: kernmat_*_symmetric_cpp + grad_*_cpp as the literal C
    restatement oracle/ace_ref.c (single-threaded, as the reference's
    Armadillo loops: src/kernel_SE_cpp.cpp:9-243, src/kernel_Matern_cpp.cpp);
  * inverse, two variants:
      "reference": eig_sym (LAPACK dsyevd via numpy.linalg.eigh) and
                   V D^-1/2 (V D^-1/2)^T (src/kernel_SE_cpp.cpp:137-157);
      "best_cpu":  dpotrf + dpotri (scipy LAPACK) + the log-det from the
                   Cholesky diagonal -- the fastest exact CPU route;
    both on every host BLAS thread (generous to the CPU: R's default
    reference BLAS is single-threaded).
The C2 (n = 16384) time is then extrapolated from a least-squares fit of
log t against log n over the three C2-shaped points, per component (pair
loops and each inverse variant separately), and the fitted exponents are
reported.  Prints one JSON document.

PARITY UNPINNED note: see oracle/ace_oracle.py.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import statistics
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def _lib():
    so = os.path.join(HERE, "libace_ref.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    L = ctypes.CDLL(so)
    D = ctypes.POINTER(ctypes.c_double)
    I64 = ctypes.c_int64
    L.ref_kernmat_sym.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D]
    L.ref_grad.argtypes = [ctypes.c_int, I64, ctypes.c_int, ctypes.c_int, D, D, D, D, D,
                           ctypes.c_double, D, D, ctypes.c_double, D]
    return L


def one_eval(L, n, p, B, kernel, seed=0):
    """Wall seconds of each component of one evaluation at (n, p, B)."""
    import numpy as np
    from scipy.linalg import lapack

    from additivecausalexpansion_amd.synthetic import make_problem
    D = ctypes.POINTER(ctypes.c_double)
    P = lambda x: x.ctypes.data_as(D)  # noqa: E731
    kind = 0 if kernel == "SE" else 1
    y, X, Z, th, sy = make_problem(n, p, B, seed=seed)
    X = np.asfortranarray(X)
    Z = np.asfortranarray(Z)
    Kf = np.zeros((n, n), order="F")
    Ke = np.zeros((n, n, B), order="F")
    t0 = time.perf_counter()
    L.ref_kernmat_sym(kind, n, p, B, P(X), P(Z), P(th), P(Kf), P(Ke))
    t_asm = time.perf_counter() - t0
    A = Kf.copy()
    A[np.diag_indices(n)] += math.exp(th[0])
    # reference inverse: symmetric eigendecomposition
    t0 = time.perf_counter()
    w, V = np.linalg.eigh(A)
    Vs = V / np.sqrt(w)[None, :]
    inv = np.asfortranarray(Vs @ Vs.T)
    logdet = float(np.sum(np.log(w)))
    t_eig = time.perf_counter() - t0
    del V, Vs
    # best-CPU inverse: Cholesky + triangular inverse product
    t0 = time.perf_counter()
    c, info = lapack.dpotrf(A, lower=1, overwrite_a=0)
    ld_chol = 2.0 * float(np.sum(np.log(np.diag(c))))
    ci, info2 = lapack.dpotri(c, lower=1, overwrite_c=1)
    t_chol = time.perf_counter() - t0
    ok_chol = info == 0 and info2 == 0 and abs(ld_chol - logdet) <= 1e-8 * abs(logdet)
    del c, ci, A
    st = np.zeros(2)
    g = np.zeros(th.shape[0])
    t0 = time.perf_counter()
    L.ref_grad(kind, n, p, B, P(y), P(X), P(Kf), P(Ke), P(inv), logdet, P(th), P(st), sy, P(g))
    t_grad = time.perf_counter() - t0
    return {"n": n, "p": p, "B": B, "kernel": kernel, "assembly": t_asm, "gradient": t_grad,
            "pairs": t_asm + t_grad, "inverse_eigh": t_eig, "inverse_chol": t_chol,
            "chol_logdet_agrees": bool(ok_chol),
            "eval_reference": t_asm + t_grad + t_eig, "eval_best_cpu": t_asm + t_grad + t_chol}


def fit(ns, ts):
    """Least-squares t = c n^a on log-log axes: (a, c)."""
    lx = [math.log(n) for n in ns]
    ly = [math.log(t) for t in ts]
    mx, my = sum(lx) / len(lx), sum(ly) / len(ly)
    a = sum((x - mx) * (y - my) for x, y in zip(lx, ly)) / sum((x - mx) ** 2 for x in lx)
    return a, math.exp(my - a * mx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="2048,4096,8192")
    ap.add_argument("--c1-reps", type=int, default=3)
    ap.add_argument("--target-n", type=int, default=16384)
    a = ap.parse_args()
    L = _lib()
    import threading
    t_start = time.perf_counter()

    def beat():  # progress line for long single-threaded points
        while True:
            time.sleep(60)
            print(f"# ... {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    try:
        cpu = [ln for ln in open("/proc/cpuinfo") if ln.startswith("model name")][0]
        cpu = cpu.split(":")[1].strip()
    except Exception:
        cpu = "unknown"
    pts = []
    for n in [int(x) for x in a.ns.split(",")]:
        pts.append(one_eval(L, n, 20, 10, "Matern32"))
        print(f"# C2-shape n={n}: {pts[-1]}", file=sys.stderr, flush=True)
    c1 = []
    for r in range(a.c1_reps):
        c1.append(one_eval(L, 4096, 10, 6, "SE", seed=r))
        print(f"# C1 rep {r}: {c1[-1]}", file=sys.stderr, flush=True)
    ns = [q["n"] for q in pts]
    out = {"host_cpu": cpu, "blas_threads": threads, "pair_loop_threads": 1,
           "points_c2_shape": pts, "c1_reps": c1}
    N = a.target_n
    ext = {}
    for comp in ("pairs", "inverse_eigh", "inverse_chol"):
        ex, c = fit(ns, [q[comp] for q in pts])
        ext[comp] = {"exponent": ex, "seconds_at_target": c * N ** ex}
    out["fit"] = ext
    t_ref = ext["pairs"]["seconds_at_target"] + ext["inverse_eigh"]["seconds_at_target"]
    t_best = ext["pairs"]["seconds_at_target"] + ext["inverse_chol"]["seconds_at_target"]
    out["c2_extrapolated"] = {
        "n": N, "seconds_per_eval_reference": t_ref, "evals_per_s_reference": 1.0 / t_ref,
        "seconds_per_eval_best_cpu": t_best, "evals_per_s_best_cpu": 1.0 / t_best}
    out["c1_measured"] = {
        "n": 4096, "median_seconds_reference": statistics.median(q["eval_reference"] for q in c1),
        "median_seconds_best_cpu": statistics.median(q["eval_best_cpu"] for q in c1)} if c1 else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
