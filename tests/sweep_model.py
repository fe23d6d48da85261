"""numpy model of the device sweep (additivecausalexpansion_amd/csrc/ace_sweep.hip)
with the same blocking, storage and AUG-row handling, used by the CPU tests
to validate the algorithm and the kernels' index arithmetic without a GPU.
Test infrastructure only."""
from __future__ import annotations

import numpy as np

NB, SUB, UT, AUG = 256, 64, 128, 128


def sweep_lower(A, npad, nb=NB, sub=SUB, ut=UT):
    """In place on A (naug x naug, only the lower triangle is read), mirroring
    k_gather / k_pivot / k_panel / k_update.  Returns the pivots."""
    naug = A.shape[0]
    piv = np.zeros(npad)
    nT = naug // ut
    for k0 in range(0, npad, nb):
        # gather: symmetric access of lower storage
        rows = np.arange(naug)[:, None]
        cols = (k0 + np.arange(nb))[None, :]
        lo = np.where(rows >= cols, A[rows, cols], A[cols, rows])
        P = lo.copy()
        W = lo.copy()
        for s in range(nb // sub):
            p0 = k0 + s * sub
            D = W[p0:p0 + sub, s * sub:(s + 1) * sub].copy()
            S = W[p0:p0 + sub, :].copy()
            for t in range(sub):
                d = D[t, t]
                piv[p0 + t] = d
                rd = 1.0 / d
                col = D[:, t].copy()
                row = D[t, :].copy()
                D -= np.outer(col, row) * rd
                D[:, t] = col * rd
                D[t, :] = row * rd
                D[t, t] = -rd
            SW = D
            for i0 in range(0, naug, sub):
                sl = slice(i0, i0 + sub)
                if i0 == p0:
                    V = SW.copy()
                    base = np.zeros((sub, nb))
                else:
                    V = -W[sl, s * sub:(s + 1) * sub] @ SW
                    base = W[sl, :].copy()
                new = base - V @ S
                new[:, s * sub:(s + 1) * sub] = V
                W[sl, :] = new
        kt0, kt1 = k0 // ut, (k0 + nb) // ut
        for I in range(nT):
            for J in range(I + 1):
                Ik, Jk = kt0 <= I < kt1, kt0 <= J < kt1
                R = slice(I * ut, (I + 1) * ut)
                C = slice(J * ut, (J + 1) * ut)
                if Ik and not Jk:
                    A[R, C] = W[C, (I * ut - k0):(I * ut - k0) + ut].T
                elif Ik or Jk:
                    A[R, C] = W[R, (J * ut - k0):(J * ut - k0) + ut]
                else:
                    A[R, C] = A[R, C] - W[R, :] @ P[C, :].T
    return piv


def invert_with_aug(K, sigma, y=None, nb=NB, aug=AUG):
    n = K.shape[0]
    npad = -(-n // nb) * nb
    naug = npad + aug
    A = np.zeros((naug, naug))
    A[:npad, :npad] = np.eye(npad)
    A[:n, :n] = K + np.exp(sigma) * np.eye(n)
    if y is not None:
        A[npad, :n] = y
        A[npad + 1, :n] = 1.0
    piv = sweep_lower(A, npad, nb=nb)
    L = np.tril(A)
    Afull = L + np.tril(L, -1).T
    inv = -Afull[:n, :n]
    out = {"inv": inv, "piv": piv, "logdet": float(np.sum(np.log(piv)))}
    if y is not None:
        out.update(u=A[npad, :n], v=A[npad + 1, :n], yKy=-A[npad, npad], yK1=-A[npad + 1, npad],
                   oK1=-A[npad + 1, npad + 1])
    return out
