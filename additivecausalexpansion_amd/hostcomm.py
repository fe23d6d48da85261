"""Host-callback collectives for the sharded model (ace_comm_ops,
ace_model_create_sharded_host): the panel broadcast / all-gather of every
sweep step and the per-evaluation all-reduces go through torch.distributed
on host buffers.  A validation transport -- e.g. gloo between processes that
share one GPU -- for the per-process packing and ownership logic that the
in-process simulated group cannot exercise; RCCL (ace_model_create_sharded)
is the production path.

Failure: a collective that raises returns 1, the library turns that into an
ACE_ERR_HIP status and the rank leaves the sweep.  Its peers then wait in the
matching collective until the process group's timeout or until the failing
process exits (gloo then errors out on the closed connections), so a caller
should end the failing process (tests/hostcomm_worker.py does) and create
the group with a short timeout.  After a failure every later collective of
this HostComm fails at once (`failed` holds the first exception).
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
        self.failed = None

        def guarded(fn):
            def run(*a):
                if self.failed is not None:
                    return 1
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # reported to the library as a failed collective
                    self.failed = e
                    return 1
            return run

        def view(p, count):
            return torch.from_numpy(np.ctypeslib.as_array(p, shape=(count,)))

        @guarded
        def bcast(_user, buf, count, root):
            if count > 0:
                dist.broadcast(view(buf, count), src=root, group=group)

        @guarded
        def allgather(_user, send, recv, count):
            if count > 0:
                out = view(recv, count * self.world)
                dist.all_gather(list(out.chunk(self.world)), view(send, count), group=group)

        @guarded
        def allreduce(_user, buf, count, op):
            if count > 0:
                dist.all_reduce(view(buf, count),
                                op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MAX,
                                group=group)

        self._fns = (BCAST_FN(bcast), ALLGATHER_FN(allgather), ALLREDUCE_FN(allreduce))
        self.ops = CommOps(None, *self._fns)
