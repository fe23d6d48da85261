"""The sharded HIP path in several processes: each rank
is its own process with its own ace_ctx (all on the box's one GPU), and the
panel broadcast / all-gather of every sweep step plus the per-evaluation
all-reduces go through gloo via host-callback collectives
(ace_model_create_sharded_host).  Unlike the in-process simulated group this
exercises the per-process packing, ownership masks, tile lists and the
one-local-rank code paths of ace_shard.cpp -- everything RCCL runs, except
the transport.  Checked against the single-GPU model and the oracle.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from conftest import record_error
from test_gpu import close

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.default_context()
    return pkg


@pytest.fixture(scope="module")
def O():
    from oracle import ace_oracle
    return ace_oracle


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_group(world, out, kind, n, p, B):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), LOCAL_RANK="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "hostcomm_worker.py"),
                                       out, kind, str(n), str(p), str(B)], env=env))
    rcs = []
    for pr in procs:
        try:
            rcs.append(pr.wait(timeout=100))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    return dict(np.load(out))


@pytest.mark.parametrize("world,kind,n,p,B", [(2, "SE", 700, 3, 4), (3, "Matern32", 900, 5, 5),
                                              (2, "Matern32", 2000, 6, 5)])
def test_sharded_processes_match_single_gpu_and_oracle(A, O, tmp_path, world, kind, n, p, B):
    """The head / tail lookahead schedule runs in every rank process: the bulk
    update of group g is in flight while the rank's host exchanges group
    g+1's panels, each panel's head rows (head path) and tail rows + row
    pieces (tail path) in separate blocking exchanges (n = 2000: 8 sweep
    steps, 3 groups).  The processes'
    inverse equals the in-process simulated group's of the same world size
    bit for bit (same kernels, same operand order; only the transport and the
    concurrency differ), the all-reduced sums to the last bits, and the
    single-GPU model and the oracle to rounding."""
    r = _run_group(world, str(tmp_path / "r.npz"), kind, n, p, B)
    y, X, Z, sy = r["y"], r["X"], r["Z"], float(r["sy"][0])
    # the processes ran the head / tail schedule: every step's exchange split
    # into a head broadcast and a tail broadcast (+ all-gather), host callbacks
    from test_shard_gpu import eval_calls
    want = eval_calls(n, world)
    want["groups"] = 0  # RCCL group launches: none over host callbacks
    assert dict(zip(("broadcast", "allgather", "allreduce", "groups"),
                    r["calls_eval1"].tolist())) == want, r["calls_eval1"]
    # every rank returned the same gradient
    for q in range(1, world):
        assert np.array_equal(r["g2_all_ranks"][q], r["g2_all_ranks"][0])
    sim = A.DeviceModel(kind, n, p, B, world=world, rank=0, sharded=True)
    sim.set_data(y, X, Z, sy)
    th1 = r["theta1"].copy()
    th1[1] = 0.0
    gs1, ss1, _ = sim.para_update(1, th1)
    gs2, ss2, _ = sim.para_update(2, r["theta2"].copy())
    # the swept matrix has no reduction in it: bitwise; the gradient sums are
    # all-reduced (gloo's summation order vs the simulated group's rank
    # order, exact for two ranks): to the last bits
    assert np.array_equal(np.diag(sim.inverse()), r["inv_diag"])
    close(gs1, r["g1"], 1e-13, 1e-14)
    close(ss1, r["st1"], 1e-13, 0)
    close(gs2, r["g2"], 1e-13, 1e-14)
    close(ss2, r["st2"], 1e-13, 0)
    if world == 2:
        assert np.array_equal(gs2, r["g2"]) and np.array_equal(ss2, r["st2"])
    sim.close()
    # the oracle at theta2 (also the scale of mu's cancellation below)
    th2 = r["theta2"]
    sym = O.kernmat_SE_symmetric_cpp if kind == "SE" else O.kernmat_Matern32_symmetric_cpp
    grad = O.grad_SE_cpp if kind == "SE" else O.grad_Matern_cpp
    K = sym(X, Z, th2)
    inv = O.invkernel_cpp(K["full"], th2[0])
    # mu = 0.5 (1' A^-1 y) / (1' A^-1 1) sums terms ~1e5 times mu itself here:
    # two inverses that agree to a relative delta give mus that agree to
    # ~delta * that sum, so mu is bounded by the sum, not by mu
    mu_terms = 0.5 * float((np.abs(inv["inv"]) @ np.abs(y)).sum()) / abs(float(inv["inv"].sum()))
    # <= 5x the largest measured (1.7e-16 mu_terms, profiles/r06_error_table.txt)
    mu_tol = 8e-16 * mu_terms
    # the single-GPU model on the same data and thetas
    m = A.DeviceModel(kind, n, p, B)
    m.set_data(y, X, Z, sy)
    th1 = r["theta1"].copy()
    th1[1] = 0.0  # para_update(1) overwrote theta[1] with mu: restart from the input
    g1, st1, mu1 = m.para_update(1, th1)
    # the sharded sweep's operand order differs from the single GPU's (R = Pn,
    # C = W): gradient and stats agree to 1e-9
    record_error("processes theta1[1] (mu): |err| / mu_terms", abs(th1[1] - r["theta1"][1]) / mu_terms, 8e-16)
    assert abs(th1[1] - r["theta1"][1]) <= mu_tol, (th1[1], r["theta1"][1], mu_tol)
    close(np.delete(th1, 1), np.delete(r["theta1"], 1), 1e-9, 1e-12)
    close(g1, r["g1"], 1e-9, 1e-11)
    close(st1, r["st1"], 1e-9, 1e-12)
    record_error("processes mu_post: |err| / mu_terms", abs(mu1 - float(r["mu1"][0])) / mu_terms, 8e-16)
    assert abs(mu1 - float(r["mu1"][0])) <= mu_tol, (mu1, r["mu1"][0], mu_tol)
    g2, st2, _ = m.para_update(2, r["theta2"].copy())
    close(g2, r["g2"], 1e-9, 1e-11)
    close(st2, r["st2"], 1e-9, 1e-12)
    # the sharded sweep forms W with the operands swapped:
    # inverse entries agree to a few 1e-9 of the largest one
    close(m.apply_inverse(r["V"]), r["AinvV"], 1e-7, 1e-8)
    close(np.diag(m.inverse()), r["inv_diag"], 1e-7, 1e-8)
    close(m.train_stats(r["theta2"]), r["train_stats"], 1e-8, 1e-9)
    pr = m.predict(r["theta2"], r["X2"], r["Z2"], 0.3, 1.2)
    close(pr["map"], r["pred_map"], 1e-8, 1e-10)
    close(pr["var"], r["pred_var"], 1e-7, 1e-10)
    # the oracle at theta2 (gradient and stats of para_update)
    st = np.zeros(2)
    g = grad(y, X, Z, K["full"], K["elements"], inv["inv"], inv["eigenval"], th2.copy(), st, B, sy)
    close(r["g2"], g, 1e-6, 1e-9)
    close(r["st2"], st, 1e-6, 1e-9)
