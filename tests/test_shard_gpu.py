"""GPU parity tests of the block-column-sharded model through
the C ABI (ace_model_create_sharded).

On one GPU the G ranks are simulated inside the process (unique_id=None):
every rank has its own local column blocks, panel buffers and tile lists,
and the broadcast / all-gather / all-reduce are device copies with the
RCCL semantics, so the packing, ownership maps and redundant pivot chains
are the ones the multi-process run uses.  A world-size-1 RCCL communicator
runs the real RCCL code path on the single card: dlopen, ncclCommInitRank,
ncclCommSplit, the creation warm-up, and every collective of the sweep --
each step's grouped head broadcast (first communicator, side stream) and
tail broadcast + all-gather (second communicator, second side stream), the
two all-reduces and the interrupt vote per evaluation, the inverse's
all-gather -- counted by ace_model_comm_calls and asserted call for call.
With one rank those collectives move no bytes between GPUs; results are
bitwise equal to the simulated one-rank group, whose collectives are the
identity.

Tolerances as in test_gpu.py: gradients / stats 1e-6 relative (north star),
inverse 1e-9 of its scale."""
import numpy as np

from conftest import run_child
import pytest
from test_gpu import close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def A():
    import additivecausalexpansion_amd as pkg
    pkg.default_context()
    return pkg


@pytest.fixture(scope="module")
def O():
    from oracle import ace_oracle
    return ace_oracle


def _oracle_eval(O, kernel, y, X, Z, th, sy, B, it):
    sym, _, grad = O.KERNELS[kernel]
    t = th.copy()
    Kl = sym(X, Z, t)
    inv = O.invkernel_cpp(Kl["full"], t[0])
    if it == 1:
        t[1] = O.mu_solution_cpp(y, inv["inv"])
    st = np.zeros(2)
    g = grad(y, X, Z, Kl["full"], Kl["elements"], inv["inv"], inv["eigenval"], t, st, B, sy)
    return t, g, st, inv


@pytest.mark.parametrize("kernel", ["SE", "Matern32"])
@pytest.mark.parametrize("world,n,p,B", [(2, 300, 2, 5), (3, 700, 3, 4), (4, 1000, 20, 10),
                                          (8, 1100, 5, 3), (5, 130, 1, 2), (3, 600, 50, 16),
                                          (2, 400, 32, 12)])
def test_sharded_sim_matches_oracle(A, O, kernel, world, n, p, B):
    """world simulated ranks; n not a multiple of 256, ranks owning no pivot
    block (world 8 / 5 at small n), both kernels, iter 1 (mu first) and 2;
    C4- and C3-shaped feature/basis counts (p = 50, B = 16; p = 32, B = 12)."""
    from additivecausalexpansion_amd.synthetic import make_problem
    y, X, Z, th, sy = make_problem(n, p, B, seed=11)
    m = A.DeviceModel(kernel, n, p, B, world=world, rank=0, sharded=True)
    m.set_data(y, X, Z, sy)
    for it in (1, 2):
        t_dev = th.copy()
        g, st, mu_post = m.para_update(it, t_dev)
        t_ref, g_ref, st_ref, inv = _oracle_eval(O, kernel, y, X, Z, th, sy, B, it)
        # mu = 0.5 yK1 / 1K1 (Q4) cancels; y is standardised, so 1e-9 absolute
        assert t_dev[1] == pytest.approx(t_ref[1], rel=1e-6, abs=1e-9)
        close(g, g_ref)
        close(st, st_ref)
        assert mu_post == pytest.approx(O.mu_solution_cpp(y, inv["inv"]), rel=1e-6, abs=1e-9)
        if it == 1:
            close(m.inverse(), inv["inv"], 1e-9, 1e-9)
        th = th + 0.01


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_sim_matches_single_gpu(A, world):
    """Sharded and single-GPU models agree to rounding at a size with 8 pivot
    blocks (several lookahead steps, every rank owning several blocks)."""
    from additivecausalexpansion_amd.synthetic import make_problem
    n, p, B = 2000, 6, 5
    y, X, Z, th, sy = make_problem(n, p, B, seed=5)
    single = A.DeviceModel("Matern32", n, p, B)
    single.set_data(y, X, Z, sy)
    sh = A.DeviceModel("Matern32", n, p, B, world=world, sharded=True)
    sh.set_data(y, X, Z, sy)
    g1, s1, m1 = single.para_update(2, th.copy())
    g2, s2, m2 = sh.para_update(2, th.copy())
    close(g2, g1, 1e-9, 1e-11)
    close(s2, s1, 1e-10, 0)
    assert m2 == pytest.approx(m1, rel=1e-9)
    close(sh.inverse(), single.inverse(), 1e-9, 1e-10)  # operand order differs: rounding


def test_sharded_train_stats_keeps_inverse(A, O):
    from additivecausalexpansion_amd.synthetic import make_problem
    n, p, B = 600, 3, 4
    y, X, Z, th, sy = make_problem(n, p, B, seed=3)
    m = A.DeviceModel("SE", n, p, B, world=3, sharded=True)
    m.set_data(y, X, Z, sy)
    m.para_update(2, th.copy())
    inv1 = m.inverse()
    th2 = th + 0.05
    st = m.train_stats(th2)
    K = O.kernmat_SE_symmetric_cpp(X, Z, th2)["full"]
    inv = O.invkernel_cpp(K, th2[0])
    close(st, O.stats_cpp(y, K, inv["inv"], inv["eigenval"], th2[1], sy))
    assert np.array_equal(m.inverse(), inv1)  # Q6


def eval_calls(n, world):
    """Collectives of one para_update of the head / tail sweep on one rank
    (DESIGN.md §7): per step a head broadcast and a tail broadcast, one
    RCCL group each; an all-gather of row pieces in every step after the
    first; the all-reduces of the AUG rows and of the gradient sums, and the
    interrupt vote."""
    S = -(-n // 256)
    return {"broadcast": 2 * S, "allgather": S - 1, "allreduce": 3, "groups": 2 * S}


def _delta(after, before):
    return {k: after[k] - before[k] for k in after}


@pytest.mark.parametrize("n", [900, 2300])
def test_sharded_rccl_world1_matches_oracle(A, O, n):
    """A real RCCL communicator (world size 1): the multi-process code path
    on one card, with every sweep collective issued (counted call for call)
    and results bitwise equal to the simulated one-rank group's (identity
    collectives).  n = 900: 4 sweep steps in 2 groups; 2300: 9 steps."""
    from additivecausalexpansion_amd.synthetic import make_problem
    uid = A.comm_unique_id()
    assert len(uid) == 128
    p, B = 4, 4
    y, X, Z, th, sy = make_problem(n, p, B, seed=9)
    m = A.DeviceModel("Matern32", n, p, B, world=1, rank=0, unique_id=uid, sharded=True)
    c0 = m.comm_calls()
    # creation: the warm-up's grouped broadcast + all-gather on both
    # communicators and one all-reduce
    assert c0 == {"broadcast": 2, "allgather": 2, "allreduce": 1, "groups": 2}, c0
    m.set_data(y, X, Z, sy)
    t1 = th.copy()
    g, st, mu = m.para_update(1, t1)
    c1 = m.comm_calls()
    assert _delta(c1, c0) == eval_calls(n, 1), (c1, c0)
    t2 = th + 0.01
    g2, st2, _ = m.para_update(2, t2.copy())
    c2 = m.comm_calls()
    assert _delta(c2, c1) == eval_calls(n, 1)
    inv_r = m.inverse()
    assert _delta(m.comm_calls(), c2) == {"broadcast": 0, "allgather": 1, "allreduce": 0, "groups": 0}
    # the simulated one-rank group (collectives are the identity, none issued)
    s = A.DeviceModel("Matern32", n, p, B, world=1, rank=0, sharded=True)
    s.set_data(y, X, Z, sy)
    ts1 = th.copy()
    gs, sts, mus = s.para_update(1, ts1)
    gs2, sts2, _ = s.para_update(2, t2.copy())
    assert s.comm_calls() == {"broadcast": 0, "allgather": 0, "allreduce": 0, "groups": 0}
    assert np.array_equal(g, gs) and np.array_equal(st, sts) and mu == mus
    assert np.array_equal(t1, ts1)
    assert np.array_equal(g2, gs2) and np.array_equal(st2, sts2)
    assert np.array_equal(inv_r, s.inverse())
    s.close()
    _, g_ref, st_ref, inv = _oracle_eval(O, "Matern32", y, X, Z, th, sy, B, 1)
    close(g, g_ref)
    close(st, st_ref)
    m.close()


def test_sharded_large_residual(A):
    """n = 6000 over 4 simulated ranks: ||A A^-1 - I|| and the log-det through
    the stats, vs the single-GPU model (size-independent properties)."""
    from additivecausalexpansion_amd.synthetic import make_problem
    n, p, B = 6000, 8, 6
    y, X, Z, th, sy = make_problem(n, p, B, seed=21)
    sh = A.DeviceModel("SE", n, p, B, world=4, sharded=True)
    sh.set_data(y, X, Z, sy)
    single = A.DeviceModel("SE", n, p, B)
    single.set_data(y, X, Z, sy)
    g2, s2, _ = sh.para_update(2, th.copy())
    g1, s1, _ = single.para_update(2, th.copy())
    close(g2, g1, 1e-8, 1e-10)
    close(s2, s1, 1e-9, 0)
    inv = sh.inverse()
    K = A.kernmat_SE_symmetric_cpp(X, Z, th)["full"]
    K[np.diag_indices(n)] += np.exp(th[0])
    R = K @ inv
    R[np.diag_indices(n)] -= 1.0
    assert np.abs(R).max() < 1e-7


_SCHED = """
import sys, numpy as np
sys.path.insert(0, {root!r})
import additivecausalexpansion_amd as A
from additivecausalexpansion_amd.synthetic import make_problem
y, X, Z, th, sy = make_problem({n}, 6, 5, seed=19)
m = A.DeviceModel("SE", {n}, 6, 5, world={world}, rank=0, sharded=True)
m.set_data(y, X, Z, sy)
g1, s1, _ = m.para_update(1, th.copy())
g2, s2, _ = m.para_update(2, th + 0.02)
np.savez({out!r}, g1=g1, s1=s1, g2=g2, s2=s2, inv=m.inverse())
"""


@pytest.mark.parametrize("world,n", [(1, 2000), (3, 1700), (4, 2300)])
def test_sharded_pair_schedule_is_bitwise_neutral(tmp_path, world, n):
    """The sharded sweep's pair-step lookahead schedule (two steps per bulk
    launch, second side stream, single-step cross on 128-tiles; ACE_PAIR=1,
    default) and the one-step schedule (ACE_PAIR=0) give bit-identical
    results: every tile sees the same MFMA chains in the same order; and so
    does the exchange packing fused into the cross launches (default)
    against separate pack launches (ACE_FUSE_PACK=0), and the pair launches
    on k_update_multi (default) against k_update_pair (ACE_MULTI2=0).  The
    default runs the head / tail schedule (round 5: the single-GPU lists, the
    exchange split into a head broadcast and a tail broadcast + all-gather);
    ACE_SHARD_HEADS=0 the group schedule without the split.  n
    gives 8, 7 (an odd last group) and 9 sweep steps; the simulated group
    runs the lookahead with all ranks on the shared streams."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    variants = {"step": {"ACE_PAIR": "0"}, "pair": {"ACE_FUSE_PACK": "0"}, "fused": {},
                "pair_kernel": {"ACE_MULTI2": "0"}, "groups": {"ACE_SHARD_HEADS": "0"}}
    for v, extra in variants.items():
        out = str(tmp_path / f"s{v}.npz")
        env = dict(os.environ, **extra)
        run_child(_SCHED.format(root=root, n=n, world=world, out=out), env=env, timeout=100)
        outs[v] = np.load(out)
    for v in ("pair", "fused", "groups"):
        for k in ("g1", "s1", "g2", "s2", "inv"):
            assert np.array_equal(outs["step"][k], outs[v][k]), (v, k)
