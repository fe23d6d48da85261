import sys, time, numpy as np
sys.path.insert(0, '/root/repo')
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
n = int(sys.argv[1]); kern = sys.argv[2]
y, X, Z, th, sy = make_problem(n, 20, 10, seed=5)
m = A.DeviceModel(kern, n, 20, 10)
m.set_data(y, X, Z, sy)
for it in (1, 2, 3):
    t = time.time()
    try:
        g, st, mu = m.para_update(it, th)
        print(it, f"{time.time()-t:.3f}s", np.all(np.isfinite(g)), mu, flush=True)
    except Exception as e:
        print(it, f"{time.time()-t:.3f}s", "EXC", e, flush=True)
        break
