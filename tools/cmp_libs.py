#!/usr/bin/env python3
"""Bitwise comparison of two builds of libace_hip.so on the fused model:
two para_update evaluations (gradient, stats, mu) at a C2-shaped problem,
each build in its own process (ACE_LIB_PATH).  Used for bit-identical A/B
switches.  usage: python tools/cmp_libs.py libA.so libB.so [n] [kernel]; CMP_ENV_B="K=V ..."
sets environment switches for the second run only."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SNIP = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
y, X, Z, th, sy = make_problem({n}, 20, 10, seed=5)
m = A.DeviceModel({kernel!r}, {n}, 20, 10)
m.set_data(y, X, Z, sy)
outs = []
for it in (1, 2):
    g, st, mu = m.para_update(it, th)
    outs += [g, st, np.array([mu])]
    th = th + 0.01 * g / max(1.0, float(np.abs(g).max()))
np.save({out!r}, np.concatenate(outs))
"""


def main():
    a, b = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    kernel = sys.argv[4] if len(sys.argv) > 4 else "Matern32"
    res = []
    with tempfile.TemporaryDirectory() as d:
        for i, lib in enumerate((a, b)):
            out = os.path.join(d, f"o{i}.npy")
            env = dict(os.environ, ACE_LIB_PATH=os.path.abspath(lib))
            if i == 1 and os.environ.get("CMP_ENV_B"):  # "K=V ..." for the second run only
                env.update(kv.split("=", 1) for kv in os.environ["CMP_ENV_B"].split())
            subprocess.run([sys.executable, "-c", SNIP.format(root=ROOT, n=n, kernel=kernel, out=out)],
                           env=env, check=True, timeout=120)
            res.append(np.load(out))
    same = np.array_equal(res[0], res[1])
    rel = float(np.max(np.abs(res[0] - res[1]) / np.maximum(np.abs(res[0]), 1e-300)))
    print(f"n={n} {kernel}: bit-identical={same} max rel diff={rel:.3e} finite={bool(np.all(np.isfinite(res[1])))}")
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
