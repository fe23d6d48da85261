"""PCIe-inclusive rate of one C2 evaluation through the host-buffer ABI (the
literal Rcpp surface: kernmat_Matern32_symmetric_cpp -> invkernel_cpp ->
mu_solution_cpp -> grad_Matern_cpp, every matrix a host numpy buffer, the
`elements` cube virtual).  DESIGN.md §8 quotes it beside the device-resident
`value`.  Usage: python tools/bench_abi.py [--reps 3]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import additivecausalexpansion_amd as ace
    from additivecausalexpansion_amd import native
    from additivecausalexpansion_amd.synthetic import CONFIGS, make_problem
    n, p, B, kernel = CONFIGS["C2"]
    y, X, Z, th, sy = make_problem(n, p, B, seed=1000)
    ctx = ace.default_context()
    times = []
    for _ in range(a.reps + 1):
        t0 = time.perf_counter()
        K = native._kernmat_sym(native.KIND[kernel], X, Z, th, ctx=ctx, elements=False)["full"]
        t1 = time.perf_counter()
        r = native.invkernel_cpp(K, th[0], ctx=ctx)
        t2 = time.perf_counter()
        th[1] = native.mu_solution_cpp(y, r["inv"], ctx=ctx)
        st = np.zeros(2)
        g = native.grad_Matern_cpp(y, X, Z, K, None, r["inv"], r["eigenval"], th, st, B, sy,
                                   ctx=ctx)
        t3 = time.perf_counter()
        times.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2))
    t = np.median(np.array(times[1:]), axis=0) * 1e3
    print(json.dumps({"config": "C2", "n": n, "evals_per_s": 1e3 / t[0], "ms_per_eval": t[0],
                      "ms": {"kernmat_sym": t[1], "invkernel": t[2], "mu+grad": t[3]},
                      "host_bytes_moved_per_eval": 5 * 8 * n * n,
                      "stats": [float(st[0]), float(st[1])], "grad_norm": float(np.linalg.norm(g))}))


if __name__ == "__main__":
    main()
