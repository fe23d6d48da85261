"""World-size-2 gloo test of bench.py's multi-process path (the driver runs
bench.py under torch.distributed.run with one rank per GPU): rendezvous,
barrier, max-over-ranks timing and the whole-job aggregation.  CPU only."""
import os
import socket
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    dist, r, w, local = bench._dist_init()
    assert (r, w, local) == (rank, world, rank)
    bench._barrier_sync(dist)
    # each rank "processed" its own replica in a different time
    dt = 1.0 + rank
    mx = bench._allreduce_max(dist, dt)
    q.put((rank, mx))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_max_and_barrier():
    torch = pytest.importorskip("torch")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = sorted(q.get(timeout=5) for _ in range(2))
    assert got == [(0, 2.0), (1, 2.0)]  # both ranks see the max over ranks


def test_single_process_path_has_no_collective():
    sys.path.insert(0, ROOT)
    import bench
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    dist, rank, world, local = bench._dist_init()
    assert dist is None and world == 1 and rank == 0
    assert bench._allreduce_max(None, 3.5) == 3.5
