"""Host-callback collectives for the sharded model (ace_comm_ops,
ace_model_create_sharded_host): the panel broadcast / all-gather of every
sweep step and the per-evaluation all-reduces go through torch.distributed
on host buffers.  A validation transport -- e.g. gloo between processes that
share one GPU -- for the per-process packing and ownership logic that the
in-process simulated group cannot exercise; RCCL (ace_model_create_sharded)
is the production path.
"""
from __future__ import annotations

import numpy as np

from ._lib import ALLGATHER_FN, ALLREDUCE_FN, BCAST_FN, CommOps


class HostComm:
    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)

        def view(p, count):
            return torch.from_numpy(np.ctypeslib.as_array(p, shape=(count,)))

        def bcast(_user, buf, count, root):
            try:
                if count > 0:
                    dist.broadcast(view(buf, count), src=root, group=group)
                return 0
            except Exception:  # reported to the library as a failed collective
                return 1

        def allgather(_user, send, recv, count):
            try:
                if count > 0:
                    out = view(recv, count * self.world)
                    dist.all_gather(list(out.chunk(self.world)), view(send, count), group=group)
                return 0
            except Exception:
                return 1

        def allreduce(_user, buf, count, op):
            try:
                if count > 0:
                    dist.all_reduce(view(buf, count),
                                    op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX,
                                    group=group)
                return 0
            except Exception:
                return 1

        self._fns = (BCAST_FN(bcast), ALLGATHER_FN(allgather), ALLREDUCE_FN(allreduce))
        self.ops = CommOps(None, *self._fns)
