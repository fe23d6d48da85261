"""CPU tests of the block-column-sharded design
through its numpy model (tests/shard_model.py): ownership invariants, the
simulated rank group, and a real multi-process run over torch.distributed
gloo (world sizes 2 and 3) whose panel broadcast / row-piece all-gather /
aug-vector all-reduce are the collectives the HIP path issues over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import shard_model as SM  # noqa: E402


def _problem(n, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-1, 1, (n, 3))
    d2 = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    K = np.exp(-d2 / 0.8)
    y = rng.normal(size=n)
    return K, -2.0, y


@pytest.mark.parametrize("G", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("n", [1, 300, 1000, 2049])
def test_every_tile_has_exactly_one_owner(G, n):
    npad = -(-n // SM.NB) * SM.NB
    naug = npad + SM.AUG
    for T, ntile in ((SM.UT, naug // SM.UT), (64, npad // 64), (64, -(-n // 64))):
        owned = {}
        for r in range(G):
            for t in SM.own_tiles(ntile, T, G, r):
                assert t not in owned
                owned[t] = r
        assert len(owned) == ntile * (ntile + 1) // 2
    # local column storage covers every block exactly once
    assert sum(SM.ncols_local(naug, G, r) for r in range(G)) == -(-naug // SM.NB) * SM.NB
    # lcol is a bijection of the owned columns onto [0, ncols_local)
    for r in range(G):
        cols = [c for c in range(naug) if SM.owns(c, G, r)]
        loc = [SM.lcol(c, G) for c in cols]
        assert len(set(loc)) == len(loc) and (not loc or max(loc) < SM.ncols_local(naug, G, r))
    # all-gather slots: every block j < k lands in exactly one (rank, slot)
    for k in range(npad // SM.NB):
        m = SM.row_slots(k, G)
        slots = {(j % G, j // G) for j in range(k)}
        assert len(slots) == k and all(q < m for _, q in slots)


def _check(inv, vec, npad, K, sigma, y, piv=None):
    n = K.shape[0]
    A = K + np.exp(sigma) * np.eye(n)
    ref = np.linalg.inv(A)
    scale = np.abs(ref).max()
    assert np.abs(inv - ref).max() < 1e-10 * scale
    u, v = vec[:n], vec[npad:npad + n]
    assert np.allclose(u, ref @ y, rtol=1e-9, atol=1e-10 * scale)
    assert np.allclose(v, ref @ np.ones(n), rtol=1e-9, atol=1e-10 * scale)
    yKy, yK1, oK1 = vec[2 * npad:2 * npad + 3]
    assert yKy == pytest.approx(y @ ref @ y, rel=1e-9)
    assert yK1 == pytest.approx(y @ ref @ np.ones(n), rel=1e-8, abs=1e-9 * scale)
    assert oK1 == pytest.approx(np.ones(n) @ ref @ np.ones(n), rel=1e-9)
    if piv is not None:
        assert np.sum(np.log(piv)) == pytest.approx(np.linalg.slogdet(A)[1], rel=1e-10)


@pytest.mark.parametrize("G", [1, 2, 3, 4])
def test_simulated_group_inverts(G):
    """n = 600: 3 sweep steps, ranks owning 0..2 pivot blocks."""
    K, sigma, y = _problem(600, seed=G)
    ranks, vec, npad = SM.sweep_sim(K, sigma, y, G)
    for R in ranks[1:]:  # the redundant pivot chains agree bit for bit
        assert np.array_equal(R.piv, ranks[0].piv)
    _check(SM.full_inverse(ranks, 600), vec, npad, K, sigma, y, ranks[0].piv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, HERE)
    import torch.distributed as dist

    import shard_model as SMw
    dist.init_process_group("gloo", rank=rank, world_size=world)
    K, sigma, y = _problem(n, seed=7)
    R, vec, npad = SMw.sweep_dist(K, sigma, y, SMw.TorchComm(dist))
    q.put((rank, R.A, R.piv, vec, npad))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_ranks_invert(world):
    """world processes over gloo: broadcast + all-gather per step, all-reduce
    of the aug vector; the ranks' local columns assemble to A^-1."""
    pytest.importorskip("torch")
    import torch.multiprocessing as mp
    n = 700
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted((q.get(timeout=240) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    K, sigma, y = _problem(n, seed=7)
    A, npad = SM.augmented(K, sigma, y)
    ranks = []
    for rank, Aloc, piv, vec, _ in got:
        R = SM.RankState.__new__(SM.RankState)
        R.G, R.r, R.npad, R.naug, R.A, R.piv = world, rank, npad, A.shape[0], Aloc, piv
        ranks.append(R)
        assert np.array_equal(vec, got[0][3])  # every rank holds the same reduced vector
    _check(SM.full_inverse(ranks, n), got[0][3], npad, K, sigma, y, got[0][2])
