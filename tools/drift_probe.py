#!/usr/bin/env python3
"""Numeric-drift probe (GPU side): one iteration-1 para_update of the fused
model on the smoke problem (n=300, p=3, B=5, seed 42) and at every compiled
feature bucket (p = 3, 8, 12, 16, 20, 24, 32, 48, 64; n = 200, B = 4), both
kernels, for each library given (each in its own process via ACE_LIB_PATH).
Saves gradient, stats and mu per case to OUT/<tag>.npz; tools/drift_analyze.py
compares them with the extended-precision referee (tests/referee_ld.py) on
the CPU.  usage: python tools/drift_probe.py OUT tag=lib.so [tag=lib.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [("smoke", 300, 3, 5, 42)] + [(f"p{p}", 200, p, 4, 100 + p)
                                      for p in (3, 8, 12, 16, 20, 24, 32, 48, 64)]

SNIP = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
out = {{}}
for name, n, p, B, seed in {cases!r}:
    for kernel in ("SE", "Matern32"):
        y, X, Z, th, sy = make_problem(n, p, B, seed=seed)
        m = A.DeviceModel(kernel, n, p, B)
        m.set_data(y, X, Z, sy)
        g, st, mu = m.para_update(1, th.copy())
        out[f"{{name}}_{{kernel}}_g"] = g
        out[f"{{name}}_{{kernel}}_st"] = st
        out[f"{{name}}_{{kernel}}_mu"] = np.array([mu])
        m.close()
np.savez({out!r}, **out)
"""


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    for spec in sys.argv[2:]:
        tag, lib = spec.split("=", 1)
        env = dict(os.environ, ACE_LIB_PATH=os.path.abspath(lib))
        code = SNIP.format(root=ROOT, cases=CASES, out=os.path.join(out, tag + ".npz"))
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
        print("probe", tag, "done", flush=True)


if __name__ == "__main__":
    main()
