#!/usr/bin/env python3
"""Inverse-accuracy probe (GPU side): one iteration-1 para_update of the
fused model on the referee problems (tests/golden/referee_{smoke,p8}.npz),
saving the resident inverse A^-1 (ace_model_get_inverse), the gradient and
the stats per library, so tools/inverse_analyze.py can split the gradient's
error into the inverse's share and the gradient kernel's share on the CPU.
usage: python tools/inverse_probe.py OUT tag=lib.so [tag=lib.so ...]"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ("referee_smoke", "referee_p8", "referee_p3")

SNIP = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
out = {{}}
for name in {names!r}:
    d = np.load({root!r} + "/tests/golden/" + name + ".npz")
    y, X, Z, th, sy = d["y"], d["X"], d["Z"], d["theta"], float(d["std_y"][0])
    n, p = X.shape
    B = Z.shape[1] + 1
    for kernel in ("SE", "Matern32"):
        m = A.DeviceModel(kernel, n, p, B)
        m.set_data(y, X, Z, sy)
        t = th.copy()
        g, st, mu = m.para_update(1, t)
        out[f"{{name}}_{{kernel}}_g"] = g
        out[f"{{name}}_{{kernel}}_st"] = st
        out[f"{{name}}_{{kernel}}_mu"] = np.array([mu])
        out[f"{{name}}_{{kernel}}_inv"] = m.inverse()
        m.close()
np.savez({out!r}, **out)
"""


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    for spec in sys.argv[2:]:
        tag, lib = spec.split("=", 1)
        env = dict(os.environ, ACE_LIB_PATH=os.path.abspath(lib))
        code = SNIP.format(root=ROOT, names=NAMES, out=os.path.join(out, tag + ".npz"))
        subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)
        print("inverse probe", tag, "done", flush=True)


if __name__ == "__main__":
    main()
