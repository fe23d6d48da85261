"""Streams and hardware queues (DESIGN §5 "Streams and hardware queues").

The box runs GPU_MAX_HW_QUEUES = 4: a process with more HIP streams than
that has the runtime share hardware queues between streams.  The library's
schedules are correct under any serialisation of their streams in host
order (every cross-stream wait is enqueued after the record it waits for),
uses only non-blocking streams and never the null stream.  These tests run
the sweep + prediction in processes that hold more streams than queues:
  * torch streams with work in flight + two full ace contexts + one
    single-stream context (ACE_STREAMS=1), results bit-identical;
  * the driver's multi-GPU bench configuration at world size 1: bench.py
    --mode sharded under torch.distributed.run, i.e. torch's NCCL process
    group and ace's own RCCL communicator in one process.
Each runs once, in a child bounded by a timeout with faulthandler armed and
the library's bounded sync (ACE_SYNC_TIMEOUT) below it."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import run_child

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

pytestmark = pytest.mark.gpu

_MANY = """
import os, sys, numpy as np
sys.path.insert(0, {root!r})
import torch
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
x = torch.randn(2048, 2048, device="cuda", dtype=torch.float64)
tstreams = [torch.cuda.Stream() for _ in range(3)]
def busy():  # torch work in flight on its own streams while ace runs
    for s in tstreams:
        with torch.cuda.stream(s):
            for _ in range(4):
                y_ = x @ x
ctxs = [A.Context(0), A.Context(0)]
os.environ["ACE_STREAMS"] = "1"
ctxs.append(A.Context(0))
os.environ.pop("ACE_STREAMS")
n, nx = 2300, 700
y, X, Z, th, sy = make_problem(n, 8, 6, seed=41)
_, X2, Z2, _, _ = make_problem(nx, 8, 6, seed=42)
zx = (np.arange(nx) % 2 == 0).astype(float)
models = []
for c in ctxs:
    m = A.DeviceModel({kernel!r}, n, 8, 6, ctx=c)
    m.set_data(y, X, Z, sy)
    models.append(m)
res = [[] for _ in models]
for it in (1, 2):
    for j, m in enumerate(models):  # interleaved across the contexts
        busy()
        g, st, mu = m.para_update(it, th.copy())
        p = m.predict(th + 0.01, X2, Z2, 0.2, 1.4)
        q = m.predict_marginal(th + 0.01, X2, np.asfortranarray(0.5 * Z2), zx, 1.4, 0.9, True)
        res[j].append(np.concatenate([g, st, [mu], p["map"], p["var"], q["map"], q["var"],
                                      np.atleast_1d(q["ate"]["map"]), np.atleast_1d(q["ate"]["var"])]))
torch.cuda.synchronize()
np.save({out!r}, np.stack([np.concatenate(r) for r in res]))
print("streams: torch 3 + null + ace 3 + 3 + 1 =", 3 + 1 + 7)
"""


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
def test_sweep_and_predict_with_more_streams_than_hw_queues(tmp_path, kernel):
    """11 streams against 4 hardware queues: torch streams busy with GEMMs,
    two 3-stream ace contexts and a 1-stream one running para_update +
    predict + predict_marginal interleaved; every context's results equal
    bit for bit (n = 2300: 9 sweep steps, a last 1-step group)."""
    out = str(tmp_path / "many.npy")
    run_child(_MANY.format(root=ROOT, kernel=kernel, out=out), timeout=110)
    r = np.load(out)
    assert np.all(np.isfinite(r))
    assert np.array_equal(r[0], r[1]) and np.array_equal(r[0], r[2])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_sharded_leg_under_torchrun_world1(tmp_path):
    """The process configuration of the driver's `bench.py --gpus N` sharded
    leg at N = 1: torch.distributed.run, torch's NCCL (RCCL) process group
    initialised and used (the unique-id broadcast), then ace's own RCCL
    communicator and its three streams, one C2 sharded evaluation.  Checks
    the JSON line and that the process exits 0 within its limit."""
    env = dict(os.environ, ACE_SYNC_TIMEOUT="150", PYTHONFAULTHANDLER="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--mode", "sharded", "--shard-config", "C2",
           "--steps", "1", "--warmup", "1"]
    try:
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    except subprocess.TimeoutExpired as e:
        raise AssertionError(f"sharded bench hung\n{e.stderr}")
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    sh = line["sharded"]
    assert line["n_gpus"] == 1 and sh["n"] == 16384 and sh["kernel"] == "Matern32"
    assert np.isfinite(line["value"]) and line["value"] > 0
    assert np.all(np.isfinite(sh["last_stats"]))
