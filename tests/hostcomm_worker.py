"""One rank of the host-callback sharded model (tests/test_hostcomm_gpu.py).

Launched as `python tests/hostcomm_worker.py OUT KIND N P B` with RANK,
WORLD_SIZE, MASTER_ADDR, MASTER_PORT in the environment: every rank joins a
gloo group, opens its own ace_ctx on GPU 0 and builds its shard of one
block-column-sharded model whose panel exchanges and all-reduces go through
torch.distributed on host buffers (ace_model_create_sharded_host).  Rank 0
writes what every check needs to OUT (npz).
"""
import datetime
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out, kind, n, p, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    import torch.distributed as dist
    # short timeout: a rank whose collective failed must not hang its peers long
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=60))
    rank, world = dist.get_rank(), dist.get_world_size()
    import additivecausalexpansion_amd as A
    from additivecausalexpansion_amd.hostcomm import HostComm
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th, sy = make_problem(n, p, B, seed=61)  # identical on every rank
    ctx = A.Context(0)
    m = A.DeviceModel(kind, n, p, B, ctx=ctx, world=world, rank=rank, sharded=True,
                      host_comm=HostComm())
    m.set_data(y, X, Z, sy)
    res = {}
    keys = ("broadcast", "allgather", "allreduce", "groups")
    c0 = m.comm_calls()
    th1 = th.copy()
    g1, st1, mu1 = m.para_update(1, th1)
    # host callbacks of one evaluation (the head / tail exchange split)
    res["calls_eval1"] = np.array([m.comm_calls()[k] - c0[k] for k in keys])
    th2 = th1 + 0.01 * np.sin(np.arange(th1.size))
    g2, st2, _ = m.para_update(2, th2)
    res.update(theta1=th1, g1=g1, st1=st1, mu1=np.array([mu1]), theta2=th2, g2=g2, st2=st2)
    # the resident inverse (theta2): gathered whole, and applied to vectors
    V = np.asfortranarray(np.cos(np.outer(np.arange(n), np.arange(1, 4)) * 0.01))
    res["AinvV"] = m.apply_inverse(V)
    res["inv_diag"] = np.diag(m.inverse()).copy()
    res["train_stats"] = m.train_stats(th2)
    _, X2, Z2, _, _ = make_problem(70, p, B, seed=62)
    pr = m.predict(th2, X2, Z2, 0.3, 1.2)
    res["pred_map"], res["pred_var"] = pr["map"], pr["var"]
    # every rank returns the same values: gather rank 1's gradient to compare
    import torch
    t = torch.from_numpy(np.ascontiguousarray(g2))
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    res["g2_all_ranks"] = np.stack([q.numpy() for q in parts])
    if rank == 0:
        np.savez(out, y=y, X=X, Z=Z, sy=np.array([sy]), V=V, X2=X2, Z2=Z2, **res)
    m.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
