"""Vendor-library reference points on the same MI355X (comparison only; the
product path uses none of these): rocBLAS/hipBLASLt fp64 GEMM of the sweep
update's shape, and rocSOLVER potrf + potri (torch.linalg.cholesky +
torch.cholesky_inverse) at C2's n -- the n^3-flop job the Gauss-Jordan sweep
replaces.  Prints one JSON line."""
import json
import sys
import time

import torch


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    out = {"n": n, "device": torch.cuda.get_device_name(0)}
    # GEMM of the update's shape: C (n x n) += P (n x 256) W^T (256 x n)
    P = torch.randn(n, 256, device=dev, dtype=torch.float64, generator=g)
    W = torch.randn(n, 256, device=dev, dtype=torch.float64, generator=g)
    C = torch.randn(n, n, device=dev, dtype=torch.float64, generator=g)
    t = timeit(lambda: C.addmm_(P, W.t()), 5)
    out["gemm_nxn_k256_tflops"] = 2.0 * n * n * 256 / t / 1e12
    # square GEMM (best-case vendor fp64 rate)
    m = 8192
    a = torch.randn(m, m, device=dev, dtype=torch.float64, generator=g)
    b = torch.randn(m, m, device=dev, dtype=torch.float64, generator=g)
    t = timeit(lambda: a @ b, 5)
    out["gemm_8192_tflops"] = 2.0 * m ** 3 / t / 1e12
    del a, b, C
    # potrf + potri on an SPD matrix (n^3 flops together)
    X = torch.rand(n, 20, device=dev, dtype=torch.float64, generator=g)
    K = torch.exp(-torch.cdist(X, X) ** 2 / 2.0) + 0.1 * torch.eye(n, device=dev,
                                                                     dtype=torch.float64)
    tc = timeit(lambda: torch.linalg.cholesky(K), 2)
    L = torch.linalg.cholesky(K)
    ti = timeit(lambda: torch.cholesky_inverse(L), 2)
    out["potrf_ms"] = tc * 1e3
    out["potri_ms"] = ti * 1e3
    out["potrf_potri_ms"] = (tc + ti) * 1e3
    out["potrf_potri_tflops"] = n ** 3 / (tc + ti) / 1e12
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
