"""Timing probe of the prediction snippet whose subprocess timed out once
(tests/test_predict_gpu.py::test_triangular_variance_matches_full_product):
wall time of every phase, including interpreter exit, in fresh processes."""
import os
import subprocess
import sys
import time

SNIP = r"""
import sys, time, numpy as np
t0 = time.time()
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
def lap(s):
    print(f"  {{s}} {{time.time() - t0:.2f}} s", flush=True)
lap("import")
y, X, Z, th, sy = make_problem(2300, 8, 6, seed=41)
m = A.DeviceModel({kernel!r}, 2300, 8, 6)
m.set_data(y, X, Z, sy)
lap("model")
m.para_update(2, th.copy())
lap("para_update")
th2 = th + 0.01
_, X2, Z2, _, _ = make_problem(700, 8, 6, seed=42)
p = m.predict(th2, X2, Z2, 0.2, 1.4)
lap("predict")
zx = (np.arange(700) % 2 == 0).astype(float)
q = m.predict_marginal(th2, X2, np.asfortranarray(0.5 * Z2), zx, 1.4, 0.9, True)
lap("predict_marginal")
"""
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for kernel in ("SE", "Matern32"):
    for v in ("0", "1"):
        t = time.time()
        r = subprocess.run([sys.executable, "-c", SNIP.format(root=root, kernel=kernel)],
                           env=dict(os.environ, ACE_PRED_TRI=v), timeout=60, capture_output=True, text=True)
        print(kernel, "TRI", v, "rc", r.returncode, f"total {time.time() - t:.2f} s")
        print(r.stdout, r.stderr[-500:], flush=True)
