"""Independent fp64 restatement of one para_update on the GPU with PyTorch --
TEST INFRASTRUCTURE ONLY (the full-size parity tests in
tests/test_fullsize_gpu.py run it in a child process; nothing in the product
path imports it, and it never loads libace_hip.so).

It follows the reference's arithmetic, not the engine's:
  * reduced kernel K = sum_b K_b, kernel length scales at theta[1+b+B(i+1)]
    (Q1), SE K_b = z_r z_c exp(lam_b - r2_b), Matern32
    K_b = z_r z_c (1 + sqrt3 t) exp(lam_b - sqrt3 t), t = sqrt(r2_b)
    (src/kernel_SE_cpp.cpp:82-130, src/kernel_Matern_cpp.cpp:203-235);
  * A = K + e^theta0 I inverted by Cholesky (torch.linalg / rocSOLVER, not
    the engine's Gauss-Jordan sweep); log det = 2 sum log diag L
    (src/kernel_SE_cpp.cpp:137-157 uses eig_sym: same log det);
  * mu_solution 0.5 sum(A^-1 y) / sum(A^-1) at iter 1 (Q4,
    src/utilities_cpp.cpp:6-10);
  * alpha = A^-1 (y - mu), T = A^-1 - alpha alpha^T, gradients
    -0.5 e^theta0 tr T, -0.5 sum T K_b, SE -0.5 e^-theta_j sum T K_b d_i^2,
    Matern -2.25 e^-theta_j sum T K_b d_i^2 / (1 + sqrt(3 r~2_b)) with the
    gradient-indexed scales theta[2+B+b+B i] (Q1, Q2), g1 = sum alpha (SE)
    (src/kernel_SE_cpp.cpp:161-243, src/kernel_Matern_cpp.cpp:340-467);
  * stats: RMSE std_y ||ybar - K alpha|| / sqrt(n) with the EXPLICIT product
    (src/kernel_SE_cpp.cpp:238) and log evidence -0.5 (n log 2 pi + log det
    + y.alpha) (Q3, src/include/ace_kernel_utils.hpp:33-36).
The pair sums run over row chunks; sum_rc M d_i^2 is taken as
sum_r x_ri^2 R_r + sum_c x_ci^2 C_c - 2 sum_r x_ri (M X)_ri (R, C the row /
column sums of M), one GEMM per slice instead of p elementwise passes.

Prediction (mode "predict"): pred_cpp and pred_marginal_cpp with ATE / ATT /
ATU (src/pred_cpp.cpp:8-126) with the inverse at theta_inv (the last
para_update's, Q6: R/kernel_SE_R6.R:37) and the kernels at theta
(R/kernel_SE_R6.R:75-97): tmp = K_xX A^-1, map = mean_y + std_y (tmp (y - mu)
+ mu), var = std_y^2 |diag(K_xx - tmp K_xX^T) + e^theta0|; marginal over
slices 1..B-1 with the derivative basis dZ2, the full nx x nx posterior
matrix for the averaged effects.  Returned beside each variance: the
quadratic form before the sqrt and the size of the terms it cancels.

usage: python tests/torch_ref.py in.npz out.npz
  in:  kernel ("SE"/"Matern32"), y, X, Z, theta, std_y, it
       [mode="predict", theta_inv, X2, Z2, dZ2, zx, mean_y, std_Z]
  out: grad, stats, rmse_identity, logdet, mu, alpha_head
       (predict: map, var, var_q, var_terms, mmap, mvar, mvar_q, mvar_terms,
        avg_map[3], avg_q[3], avg_terms[3])
"""
import math
import sys

import numpy as np
import torch


def para_update(kernel, y, X, Z, theta, std_y, it, dev="cuda", chunk=1024):
    f64 = torch.float64
    n, p = X.shape
    B = Z.shape[1] + 1
    th = np.array(theta, dtype=np.float64)
    Xt = torch.tensor(X, dtype=f64, device=dev)
    yt = torch.tensor(y, dtype=f64, device=dev)
    zt = [None] + [torch.tensor(Z[:, b - 1], dtype=f64, device=dev) for b in range(1, B)]
    wk = torch.tensor([[math.exp(-th[1 + b + B * (i + 1)]) for i in range(p)] for b in range(B)],
                      dtype=f64, device=dev)
    wg = torch.tensor([[math.exp(-th[2 + B + b + B * i]) for i in range(p)] for b in range(B)],
                      dtype=f64, device=dev)
    lam = [float(th[2 + b]) for b in range(B)]
    X2 = Xt * Xt
    s3 = math.sqrt(3.0)

    def r2_rows(r0, r1, w):
        s = X2 @ w
        G = torch.addmm(s[r0:r1, None], Xt[r0:r1] * w, Xt.T, alpha=-2.0)
        G.add_(s[None, :]).clamp_(min=0.0)
        idx = torch.arange(r0, r1, device=dev)
        G[idx - r0, idx] = 0.0  # r == c: no distance
        return G

    def kb_rows(r0, r1, b):
        G = r2_rows(r0, r1, wk[b])
        if kernel == "SE":
            K = G.neg_().add_(lam[b]).exp_()
        else:
            t = G.sqrt_()
            e = torch.exp(lam[b] - s3 * t)
            K = t.mul_(s3).add_(1.0).mul_(e)
        if b > 0:
            K.mul_(zt[b][r0:r1, None]).mul_(zt[b][None, :])
        return K

    # A = K + e^theta0 I, Cholesky, inverse
    A = torch.empty((n, n), dtype=f64, device=dev)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        acc = kb_rows(r0, r1, 0)
        for b in range(1, B):
            acc.add_(kb_rows(r0, r1, b))
        A[r0:r1] = acc
        del acc
    A.diagonal().add_(math.exp(th[0]))
    L, info = torch.linalg.cholesky_ex(A)
    del A
    if int(info) != 0:
        raise RuntimeError(f"not positive definite (info {int(info)})")
    logdet = float(2.0 * torch.log(torch.diagonal(L)).sum())
    Ainv = torch.cholesky_inverse(L)
    del L
    mu = None
    if it == 1:
        mu = float(0.5 * (Ainv @ yt).sum() / Ainv.sum())
        th[1] = mu
    ybar = yt - th[1]
    alpha = Ainv @ ybar
    trT = float(torch.diagonal(Ainv).sum() - (alpha * alpha).sum())
    g_lam = np.zeros(B)
    g_len = np.zeros((B, p))
    Kalpha = torch.zeros(n, dtype=f64, device=dev)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        T = Ainv[r0:r1] - alpha[r0:r1, None] * alpha[None, :]
        for b in range(B):
            K = kb_rows(r0, r1, b)
            Kalpha[r0:r1] += K @ alpha
            M = K.mul_(T)
            g_lam[b] += float(M.sum())
            if kernel == "Matern32":
                F = r2_rows(r0, r1, wg[b]).mul_(3.0).sqrt_().add_(1.0)
                M.div_(F)
                del F
            R = M.sum(1)
            C = M.sum(0)
            MX = M @ Xt
            g = (X2[r0:r1] * R[:, None]).sum(0) + (X2 * C[:, None]).sum(0) \
                - 2.0 * (Xt[r0:r1] * MX).sum(0)
            g_len[b] += g.cpu().numpy()
            del M, R, C, MX
        del T
    P = 2 + B * (p + 1)
    grad = np.zeros(P)
    grad[0] = -0.5 * trT * math.exp(th[0])
    grad[1] = float(alpha.sum()) if kernel == "SE" else 0.0
    for b in range(B):
        grad[2 + b] = -0.5 * g_lam[b]
        for i in range(p):
            j = 2 + B + b + B * i
            fac = -0.5 if kernel == "SE" else -0.25 * 9
            grad[j] = fac * g_len[b, i] * math.exp(-th[j])
    resid = ybar - Kalpha
    rmse = std_y * float(torch.linalg.norm(resid)) / math.sqrt(n)
    rmse_identity = std_y * math.exp(th[0]) * float(torch.linalg.norm(alpha)) / math.sqrt(n)
    ev = -0.5 * (n * math.log(2 * math.pi) + logdet + float(yt @ alpha))
    return {"grad": grad, "stats": np.array([rmse, ev]), "rmse_identity": rmse_identity,
            "logdet": logdet, "mu": np.nan if mu is None else mu,
            "alpha_head": alpha[:64].cpu().numpy()}


def _weights(th, B, p, dev):
    f64 = torch.float64
    wk = torch.tensor([[math.exp(-th[1 + b + B * (i + 1)]) for i in range(p)] for b in range(B)],
                      dtype=f64, device=dev)
    return wk, [float(th[2 + b]) for b in range(B)]


def kernel_sum(kernel, Xa, Za, Xb, Zb, th, b0, b1, same=False, dev="cuda"):
    """sum_{b0 <= b < b1} K_b(Xa, Xb) (src/kernel_SE_cpp.cpp:9-64,
    src/kernel_Matern_cpp.cpp:52-93), z_0 = 1, z_b = Z[:, b-1]."""
    f64 = torch.float64
    p = Xa.shape[1]
    B = Za.shape[1] + 1
    wk, lam = _weights(th, B, p, dev)
    xa = torch.tensor(Xa, dtype=f64, device=dev)
    xb = torch.tensor(Xb, dtype=f64, device=dev)
    s3 = math.sqrt(3.0)
    out = torch.zeros((xa.shape[0], xb.shape[0]), dtype=f64, device=dev)
    for b in range(b0, b1):
        w = wk[b]
        G = torch.addmm(((xa * xa) @ w)[:, None], xa * w, xb.T, alpha=-2.0)
        G.add_(((xb * xb) @ w)[None, :]).clamp_(min=0.0)
        if same:
            G.fill_diagonal_(0.0)
        if kernel == "SE":
            K = G.neg_().add_(lam[b]).exp_()
        else:
            t = G.sqrt_()
            e = torch.exp(lam[b] - s3 * t)
            K = t.mul_(s3).add_(1.0).mul_(e)
        if b > 0:
            K.mul_(torch.tensor(Za[:, b - 1], dtype=f64, device=dev)[:, None])
            K.mul_(torch.tensor(Zb[:, b - 1], dtype=f64, device=dev)[None, :])
        out.add_(K)
        del G, K
    return out


def predict(kernel, y, X, Z, theta_inv, theta, X2, Z2, dZ2, zx, mean_y, std_y, std_Z, dev="cuda"):
    f64 = torch.float64
    n = X.shape[0]
    B = Z.shape[1] + 1
    th = np.array(theta, dtype=np.float64)
    A = kernel_sum(kernel, X, Z, X, Z, theta_inv, 0, B, same=True, dev=dev)
    A.diagonal().add_(math.exp(theta_inv[0]))
    L, info = torch.linalg.cholesky_ex(A)
    del A
    if int(info) != 0:
        raise RuntimeError(f"not positive definite (info {int(info)})")
    Ainv = torch.cholesky_inverse(L)
    del L
    w = torch.tensor(y, dtype=f64, device=dev) - th[1]
    out = {}
    # pred_cpp (src/pred_cpp.cpp:8-34)
    KxX = kernel_sum(kernel, X2, Z2, X, Z, th, 0, B, dev=dev)
    tmp = KxX @ Ainv
    out["map"] = (mean_y + std_y * (tmp @ w + th[1])).cpu().numpy()
    q = (tmp * KxX).sum(1)
    kxx = torch.diagonal(kernel_sum(kernel, X2, Z2, X2, Z2, th, 0, B, same=True, dev=dev))
    d = kxx - q + math.exp(th[0])
    out["var_q"] = d.cpu().numpy()
    out["var"] = (std_y * torch.sqrt(d.abs())).pow(2).cpu().numpy()
    out["var_terms"] = (std_y ** 2 * (kxx.abs() + q.abs() + math.exp(th[0]))).cpu().numpy()
    del KxX, tmp
    # pred_marginal_cpp (src/pred_cpp.cpp:37-126): slices 1..B-1 (or 0 if B == 1)
    b0, b1 = (1, B) if B > 1 else (0, 1)
    KmX = kernel_sum(kernel, X2, dZ2, X, Z, th, b0, b1, dev=dev)
    Kmx = kernel_sum(kernel, X2, dZ2, X2, dZ2, th, b0, b1, same=True, dev=dev)
    tmp = KmX @ Ainv
    yx = std_y * (tmp @ w) / std_Z
    C = tmp @ KmX.T
    post = Kmx - C
    dq = torch.diagonal(post)
    out["mmap"] = yx.cpu().numpy()
    out["mvar_q"] = dq.cpu().numpy()
    out["mvar"] = (std_y * torch.sqrt(dq.abs()) / std_Z).pow(2).cpu().numpy()
    out["mvar_terms"] = ((std_y / std_Z) ** 2 * (torch.diagonal(Kmx).abs() +
                                                 torch.diagonal(C).abs())).cpu().numpy()
    zt = torch.tensor(zx, dtype=f64, device=dev)
    nx = X2.shape[0]
    ntx = float(int(zx.sum()))
    ate = float(yx.mean())
    att = float(yx @ zt) / ntx
    atu = (ate * nx - att * ntx) / (nx - ntx)
    am, aq, at = [ate, att, atu], [], []
    for wv, cnt in ((torch.ones(nx, dtype=f64, device=dev), nx), (zt, ntx),
                    ((zt == 0).to(f64), nx - ntx)):
        aq.append(float(wv @ post @ wv))
        at.append((std_y / cnt) ** 2 * (abs(float(wv @ Kmx @ wv)) + abs(float(wv @ C @ wv))))
    out["avg_map"] = np.array(am)
    out["avg_q"] = np.array(aq)
    out["avg_terms"] = np.array(at)
    return out


def main():
    inp, out = sys.argv[1], sys.argv[2]
    with np.load(inp, allow_pickle=False) as d:
        args = {k: d[k] for k in d.files}
    if "mode" in args and str(args["mode"]) == "predict":
        r = predict(str(args["kernel"]), args["y"], args["X"], args["Z"], args["theta_inv"],
                    args["theta"], args["X2"], args["Z2"], args["dZ2"], args["zx"],
                    float(args["mean_y"]), float(args["std_y"]), float(args["std_Z"]))
        np.savez(out, **r)
        return
    r = para_update(str(args["kernel"]), args["y"], args["X"], args["Z"], args["theta"],
                    float(args["std_y"]), int(args["it"]))
    np.savez(out, **r)


if __name__ == "__main__":
    main()
