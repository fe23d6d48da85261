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


_GUARD = """
import sys, time, json
sys.path.insert(0, {root!r})
import bench
line = {{"metric": "m", "value": 1.5}}
def leg():
    {body}
sh, failed = bench.run_guarded(line, leg, {timeout})
line["sharded"] = sh
print(json.dumps(line), flush=True)
if failed:
    bench.os._exit(bench.EXIT_SHARDED_FAILED)
"""


@pytest.mark.parametrize("body,timeout,rc,err", [
    ("return {'evals_per_s': 2.0}", 30, 0, None),
    ("raise RuntimeError('rccl')", 30, 3, "RuntimeError: rccl"),
    ("time.sleep(60)", 1.0, 3, "timed out after 1 s"),  # a hung collective
])
def test_sharded_leg_failure_shows_in_exit_status(body, timeout, rc, err):
    """bench.py's sharded leg (N > 1) runs under a watchdog: a leg that
    raises or hangs still gets the headline line printed, and the run then
    exits non-zero (EXIT_SHARDED_FAILED = 3), so a hung collective is visible
    in the driver's rc rather than hidden behind rc 0."""
    import json
    import subprocess
    r = subprocess.run([sys.executable, "-c", _GUARD.format(root=ROOT, body=body, timeout=timeout)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == rc, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.5  # the headline survives
    if err is None:
        assert line["sharded"] == {"evals_per_s": 2.0}
    else:
        assert err in line["sharded"]["error"]
