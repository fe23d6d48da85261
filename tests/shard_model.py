"""numpy model of the block-column-sharded sweep (additivecausalexpansion_amd/
csrc/ace_shard.cpp + the shard kernels in ace_sweep.hip): the same column
ownership (NB-wide blocks, block j on rank j % G, local block j // G), the
same panel exchange (broadcast of rows >= k0 from the owner of block k,
all-gather of the NB x NB row pieces A[k-block, j-block] of every rank's
blocks j < k, slot (j % G, j // G)), the redundant pivot sweep, W formed
only for the rows a rank consumes, the operand-swapped update
A_IJ += Pn_I W_J^T over the rank's own tiles, and the all-reduce of the
AUG-row vector.  Used by the CPU tests, in one process (SimComm) and across
gloo ranks (TorchComm).  Test infrastructure only."""
from __future__ import annotations

import numpy as np

NB, SUB, UT, AUG = 256, 64, 128, 128


def lcol(c, G):
    return c if G == 1 else (c // NB // G) * NB + c % NB


def owns(c, G, r):
    return G == 1 or (c // NB) % G == r


def ncols_local(naug, G, r):
    nblk = -(-naug // NB)
    return len(range(r, nblk, G)) * NB


def own_tiles(ntile, T, G, r):
    return [(I, J) for I in range(ntile) for J in range(I + 1) if owns(J * T, G, r)]


def row_slots(k, G):
    return -(-k // G)


class SimComm:
    """All G ranks in one process: collectives act on the list of rank states."""

    def __init__(self, G):
        self.G = G


class TorchComm:
    """One rank per process over torch.distributed (gloo on CPU)."""

    def __init__(self, dist):
        self.dist = dist
        self.G = dist.get_world_size()
        self.r = dist.get_rank()

    def bcast(self, arr, root):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        self.dist.broadcast(t, src=root)
        return t.numpy()

    def allgather(self, arr):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        out = [torch.empty_like(t) for _ in range(self.G)]
        self.dist.all_gather(out, t)
        return [o.numpy() for o in out]

    def allreduce(self, arr):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        self.dist.all_reduce(t)
        return t.numpy()


def pivot_block(Dblk):
    """Sweep of the NB x NB pivot block in SUB-column sub-steps (k_pivot +
    k_panel restricted to the pivot rows): returns W_kk = -D^-1 and the
    pivots."""
    nb = Dblk.shape[0]
    W = Dblk.copy()
    piv = np.zeros(nb)
    for s in range(nb // SUB):
        p0 = s * SUB
        D = W[p0:p0 + SUB, p0:p0 + SUB].copy()
        S = W[p0:p0 + SUB, :].copy()
        for t in range(SUB):
            d = D[t, t]
            piv[p0 + t] = d
            rd = 1.0 / d
            col = D[:, t].copy()
            row = D[t, :].copy()
            D -= np.outer(col, row) * rd
            D[:, t] = col * rd
            D[t, :] = row * rd
            D[t, t] = -rd
        for i0 in range(0, nb, SUB):
            sl = slice(i0, i0 + SUB)
            if i0 == p0:
                V = D.copy()
                base = np.zeros((SUB, nb))
            else:
                V = -W[sl, p0:p0 + SUB] @ D
                base = W[sl, :].copy()
            new = base - V @ S
            new[:, p0:p0 + SUB] = V
            W[sl, :] = new
    return W, piv


class RankState:
    def __init__(self, A_full_lower, npad, G, r):
        naug = A_full_lower.shape[0]
        self.G, self.r, self.npad, self.naug = G, r, npad, naug
        self.A = np.zeros((naug, ncols_local(naug, G, r)))
        for j in range(r, -(-naug // NB), G):  # assembly: own column blocks (lower part)
            c0, w = j * NB, min(NB, naug - j * NB)
            self.A[:, lcol(c0, G):lcol(c0, G) + w] = np.tril(A_full_lower)[:, c0:c0 + w]
        self.tiles = own_tiles(naug // UT, UT, G, r)
        self.piv = np.zeros(npad)

    def pack(self, k):
        G, r, k0, naug = self.G, self.r, k * NB, self.naug
        low = None
        if k % G == r:  # k_pack_lower, mirroring the pivot block's upper half
            L = lcol(k0, G)
            low = self.A[k0:, L:L + NB].copy()
            blk = low[:NB, :]
            low[:NB, :] = np.tril(blk) + np.tril(blk, -1).T
        send = np.zeros((max(row_slots(k, G), 1), NB, NB))
        for q, j in enumerate(range(r, k, G)):  # k_pack_rows
            send[q] = self.A[k0:k0 + NB, q * NB:(q + 1) * NB]
        return low, send[:row_slots(k, G)]

    def unpack_chain(self, k, low, recv):
        """k_unpack_panel + pivot chain + k_panel_gemm for the rows r consumes."""
        G, k0, naug = self.G, k * NB, self.naug
        P = np.zeros((naug, NB))
        P[k0:, :] = low
        for j in range(k):  # P[i, c] = A[k0 + c, i] from slot (j % G, j // G)
            P[j * NB:(j + 1) * NB, :] = recv[j % G][j // G].T
        Pn = -P
        Wkk, piv = pivot_block(P[k0:k0 + NB, :])
        self.piv[k0:k0 + NB] = piv
        W = np.full((naug, NB), np.nan)  # rows this rank does not form stay NaN
        for i0 in range(0, naug, SUB):
            if k0 <= i0 < k0 + NB:
                W[i0:i0 + SUB] = Wkk[i0 - k0:i0 - k0 + SUB]
            elif owns(i0, G, self.r) or (owns(k0, G, self.r) and i0 >= k0):
                W[i0:i0 + SUB] = Pn[i0:i0 + SUB] @ Wkk
        return Pn, W

    def update(self, k, Pn, W):
        G, k0 = self.G, k * NB
        kt0, kt1 = k0 // UT, (k0 + NB) // UT
        for I, J in self.tiles:
            R = slice(I * UT, (I + 1) * UT)
            L0 = lcol(J * UT, G)
            C = slice(L0, L0 + UT)
            Ik, Jk = kt0 <= I < kt1, kt0 <= J < kt1
            if Ik and not Jk:
                self.A[R, C] = W[J * UT:(J + 1) * UT, I * UT - k0:I * UT - k0 + UT].T
            elif Ik or Jk:
                self.A[R, C] = W[R, J * UT - k0:J * UT - k0 + UT]
            else:
                self.A[R, C] = self.A[R, C] + Pn[R, :] @ W[J * UT:(J + 1) * UT, :].T

    def aug_vec(self):
        npad, G, r = self.npad, self.G, self.r
        v = np.zeros(2 * npad + 3)
        for j in range(npad):
            if owns(j, G, r):
                v[j] = self.A[npad, lcol(j, G)]
                v[npad + j] = self.A[npad + 1, lcol(j, G)]
        if owns(npad, G, r):
            l = lcol(npad, G)
            v[2 * npad:] = [-self.A[npad, l], -self.A[npad + 1, l], -self.A[npad + 1, l + 1]]
        return v


def augmented(K, sigma, y):
    n = K.shape[0]
    npad = -(-n // NB) * NB
    naug = npad + AUG
    A = np.zeros((naug, naug))
    A[:npad, :npad] = np.eye(npad)
    A[:n, :n] = K + np.exp(sigma) * np.eye(n)
    A[npad, :n] = y
    A[npad + 1, :n] = 1.0
    return A, npad


def sweep_sim(K, sigma, y, G):
    """All G ranks in one process; returns per-rank states and the reduced
    aug vector."""
    A, npad = augmented(K, sigma, y)
    ranks = [RankState(A, npad, G, r) for r in range(G)]
    for k in range(npad // NB):
        packed = [R.pack(k) for R in ranks]
        low = packed[k % G][0]
        recv = [p[1] for p in packed]
        panels = [R.unpack_chain(k, low, recv) for R in ranks]
        for R, (Pn, W) in zip(ranks, panels):
            R.update(k, Pn, W)
    vec = sum(R.aug_vec() for R in ranks)
    return ranks, vec, npad


def sweep_dist(K, sigma, y, comm):
    """This process's rank of a G-rank group over torch.distributed."""
    A, npad = augmented(K, sigma, y)
    R = RankState(A, npad, comm.G, comm.r)
    naug = A.shape[0]
    for k in range(npad // NB):
        low, send = R.pack(k)
        if low is None:
            low = np.zeros((naug - k * NB, NB))
        low = comm.bcast(low, k % comm.G)
        m = row_slots(k, comm.G)
        recv = comm.allgather(send) if m > 0 else [np.zeros((0, NB, NB))] * comm.G
        Pn, W = R.unpack_chain(k, low, recv)
        R.update(k, Pn, W)
    vec = comm.allreduce(R.aug_vec())
    return R, vec, npad


def full_inverse(ranks, n):
    """-A^-1 lower from the ranks' local columns -> symmetric A^-1 (n x n)."""
    naug = ranks[0].naug
    L = np.zeros((naug, naug))
    for R in ranks:
        for j in range(R.r, -(-naug // NB), R.G):
            c0, w = j * NB, min(NB, naug - j * NB)
            L[:, c0:c0 + w] = R.A[:, lcol(c0, R.G):lcol(c0, R.G) + w]
    L = np.tril(L)
    full = L + np.tril(L, -1).T
    return -full[:n, :n]
