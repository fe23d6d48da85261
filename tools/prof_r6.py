"""Per-call wall times of the unchanged R6 para_update on device handles at
C2 (r6.py's sequence, R/kernel_Matern32_R6.R:39-60): where the drop-in path
spends the time beyond the fused model.  Usage: python tools/prof_r6.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import additivecausalexpansion_amd as ace
    from additivecausalexpansion_amd import native
    from additivecausalexpansion_amd.synthetic import CONFIGS, make_problem
    n, p, B, kernel = CONFIGS["C2"]
    y, X, Z, th, sy = make_problem(n, p, B, seed=1000)
    ctx = ace.default_context()
    k = ace.R6KernelMatern32(p, B, th, sy, ctx=ctx)
    opt = ace.set_optimizer("Nadam", k, 0.01, 0.0, 0.9, 0.999, True, 1.0)
    rows = []
    for it in range(1, 7):
        t = [time.perf_counter()]
        Kl = native.kernmat_Matern32_symmetric_cpp(X, Z, k.parameters, ctx=ctx, device=True)
        k.Kmat, k.Karray = Kl["full"], Kl["elements"]
        t.append(time.perf_counter())
        lst = native.invkernel_cpp(k.Kmat, k.parameters[0], ctx=ctx)
        k.invKmatn = lst["inv"]
        t.append(time.perf_counter())
        if it == 1:
            k.mean_solution(y)
        t.append(time.perf_counter())
        st = np.zeros(2)
        g = native.grad_Matern_cpp(y, X, Z, k.Kmat, k.Karray, k.invKmatn, lst["eigenval"],
                                   k.parameters, st, B, sy, ctx=ctx)
        t.append(time.perf_counter())
        k.parameters = opt.update(it, k.parameters, g)
        k.mean_solution(y)
        t.append(time.perf_counter())
        rows.append(np.diff(t) * 1e3)
    r = np.median(np.array(rows[1:]), axis=0)
    print(json.dumps({"config": "C2", "ms": dict(zip(["kernmat_sym", "invkernel", "mu_iter1", "grad",
                                                      "update+mu"], r.tolist())),
                      "total_ms": float(r.sum())}))


if __name__ == "__main__":
    main()
