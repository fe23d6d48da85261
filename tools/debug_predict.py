"""Debug helper: device predict vs the same quantities from apply_inverse and
the ABI kernels (GPU box)."""
import sys

import numpy as np

sys.path.insert(0, ".")
import additivecausalexpansion_amd as A  # noqa: E402
from additivecausalexpansion_amd.synthetic import make_problem  # noqa: E402

for kernel in ("SE", "Matern32"):
    n, p, B, nx = 300, 3, 5, 70
    y, X, Z, th, sy = make_problem(n, p, B, seed=n)
    m = A.DeviceModel(kernel, n, p, B)
    m.set_data(y, X, Z, sy)
    m.para_update(2, th.copy())
    _, X2, Z2, _, _ = make_problem(nx, p, B, seed=n + 1)
    cross = A.kernmat_SE_cpp if kernel == "SE" else A.kernmat_Matern32_cpp
    K = cross(X2, X, Z2, Z, th)["full"]
    inv = m.inverse()
    w = m.apply_inverse(y - th[1])
    print("w vs inv@(y-mu)", np.abs(w - inv @ (y - th[1])).max())
    ref = K @ w + th[1]
    got = m.predict(th, X2, Z2, 0.0, 1.0)["map"]
    print(kernel, "map err", np.abs(got - ref).max(), got[:4], ref[:4])
    T = m.apply_inverse(K.T)
    print("apply_inverse(K^T) vs inv K^T", np.abs(T - inv @ K.T).max())
    # predict at a single point repeated
    got1 = m.predict(th, X2[:1], Z2[:1], 0.0, 1.0)["map"]
    print("single point", got1, ref[0])
    got2 = m.predict(th, X[:5], Z[:5], 0.0, 1.0)["map"]
    K5 = cross(X[:5], X, Z[:5], Z, th)["full"]
    print("train points", got2, K5 @ w + th[1])
