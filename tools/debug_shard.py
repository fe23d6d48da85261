"""Debug: sharded (simulated) vs single-GPU model, block error map of the inverse."""
import sys
import numpy as np
sys.path.insert(0, ".")
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem

n, p, B = int(sys.argv[1]) if len(sys.argv) > 1 else 300, 2, 5
y, X, Z, th, sy = make_problem(n, p, B, seed=11)
single = A.DeviceModel("SE", n, p, B)
single.set_data(y, X, Z, sy)
g1, s1, m1 = single.para_update(2, th.copy())
inv1 = single.inverse()
for G in tuple(int(g) for g in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3").split(",")):
    sh = A.DeviceModel("SE", n, p, B, world=G, sharded=True)
    sh.set_data(y, X, Z, sy)
    g2, s2, m2 = sh.para_update(2, th.copy())
    inv2 = sh.inverse()
    nb = (n + 255) // 256
    emap = np.zeros((nb, nb))
    for i in range(nb):
        for j in range(nb):
            a = inv1[i*256:(i+1)*256, j*256:(j+1)*256]
            b = inv2[i*256:(i+1)*256, j*256:(j+1)*256]
            emap[i, j] = np.abs(a - b).max() / np.abs(inv1).max()
    print(f"G={G}: mu {m1:.6e} vs {m2:.6e}; stats {s1} vs {s2}; grad err "
          f"{np.abs(g1-g2).max()/np.abs(g1).max():.2e}\n  inv block err map\n{np.array2string(emap, precision=1)}",
          flush=True)
