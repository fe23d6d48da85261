// ace_symm.hip -- products with the resident inverse (device-resident
// prediction, ace_model_apply_inverse).
//
// After a para_update the swept matrix A holds -A^-1 in its lower triangle
// (single GPU: the whole naug x naug array; sharded: the rank's NB-wide
// column blocks, block-cyclic).  The reference multiplies by the explicit
// inverse in pred_cpp (src/pred_cpp.cpp:19, 69: tmp = K_xX * invK_XX); here
// the product is taken straight from the lower storage:
//
//   Out (n x k) = scale * S V,   S = the symmetric n x n matrix whose lower
//   triangle is stored in A, V = an n x k operand given either directly
//   (col-major, ld ldv) or as the transpose of a k x n col-major matrix
//   (VT: V[p][c] = M[c + p * ldv], the K_xX of prediction, so that
//   Out = S K_xX^T = (K_xX S)^T).
//
// Sharded: each rank adds only the entries of S it stores -- S[q][p] for
// p >= q from its own column blocks p and, mirrored, S[q][p] = A[p][q] for
// q < p from its own column blocks q -- so the sum over ranks of the
// partial products is S V.  A 16-wide k-chunk of the product touches only
// one column block, so a chunk the rank does not own is skipped whole
// (block-uniform: the barriers stay uniform), and each rank does 1/G of the
// MFMA work.
//
// 256 threads, 128 (rows) x 64 (columns) output tile, 4 waves of 32 x 64
// (2 x 4 v_mfma_f64_16x16x4_f64 fragments), BK = 16 k-chunks staged
// through LDS with a register prefetch of the next chunk.
#include <cstdlib>

#include "ace_internal.h"

namespace ace {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int SR = 128, SC = 64, SBK = 16;
constexpr int SLS = SR + 16;  // LDS pitch of the S stage
constexpr int SLV = SC + 16;  // LDS pitch of the V stage

// TRI (single GPU): Out = scale L V with L the STRICTLY lower part of the
// stored matrix (row q, column p < q) -- the k-chunks below the tile's rows
// and the masked diagonal block only, so half of k_symm's MFMA work on
// average and only coalesced column loads (prediction's variance, see
// k_pred_cols_tri).
template <bool VT, bool TRI>
__global__ __launch_bounds__(256) void k_symm(const double *__restrict__ A, int64_t ld, int64_t n,
                                              int G, int rank, const double *__restrict__ V,
                                              int64_t ldv, int64_t k, double scale,
                                              double *__restrict__ out, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) double sS[2][SBK][SLS];
  __shared__ __attribute__((aligned(16))) double sV[2][SBK][SLV];
  const int64_t R0 = (int64_t)blockIdx.y * SR, C0 = (int64_t)blockIdx.x * SC;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const bool rowown = owns_col(R0, G, rank);  // the tile's rows lie in one NB block
  // S staging: lower chunks read 128 consecutive rows of one column (thread:
  // row sm .. sm + 7 of column si), upper chunks 16 consecutive rows of one
  // column of the mirror (thread: column tq of the mirror, rows 8 tj ..)
  const int si = tid >> 4, sm = (tid & 15) * 8;
  const int tq = tid >> 1, tj = (tid & 1) * 8;
  // V staging: 4 doubles per thread
  const int vi = tid >> 4, vc = (tid & 15) * 4;    // VT:  k-row vi, columns vc..vc+3
  const int vci = tid >> 2, vpi = (tid & 3) * 4;   // !VT: column vci, k-rows vpi..vpi+3
  double rs[8], rv[4];
  // chunk class of k-chunk kk: 0 skip, 1 lower (all p < q), 2 upper (all
  // p > q), 3 mixed (the chunk crosses the tile's rows: same NB block)
  auto cls = [&](int64_t kk) -> int {
    if (TRI) return kk + SBK <= R0 ? 1 : (kk < R0 + SR ? 4 : 0);
    if (kk + SBK <= R0) return owns_col(kk, G, rank) ? 1 : 0;
    if (kk >= R0 + SR) return rowown ? 2 : 0;
    return rowown ? 3 : 0;
  };
  auto load = [&](int64_t kk, int c) {
    if (c == 1) {
      const int64_t p = kk + si;
      const double *col = A + lcol(p, G) * ld;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t q = R0 + sm + e;
        rs[e] = (q < n && p < n) ? col[q] : 0.0;
      }
    } else if (c == 2) {
      const int64_t q = R0 + tq;
      const double *col = A + lcol(q, G) * ld;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t p = kk + tj + e;
        rs[e] = (q < n && p < n) ? col[p] : 0.0;
      }
    } else if (c == 4) {  // TRI diagonal block: row q, column p < q only
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t p = kk + si, q = R0 + sm + e;
        rs[e] = (q < n && p < n && q > p) ? A[q + p * ld] : 0.0;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int64_t p = kk + si, q = R0 + sm + e;
        double v = 0.0;
        if (q < n && p < n) v = (q >= p) ? A[q + lcol(p, G) * ld] : A[p + lcol(q, G) * ld];
        rs[e] = v;
      }
    }
    if (!VT) {  // V[p + c ldv]: 4 consecutive p of one column per thread
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t p = kk + vpi + e, c = C0 + vci;
        rv[e] = (p < n && c < k) ? V[p + c * ldv] : 0.0;
      }
    } else {    // V[c + p ldv]: 4 consecutive c of one k-row per thread
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t p = kk + vi, c = C0 + vc + e;
        rv[e] = (p < n && c < k) ? V[c + p * ldv] : 0.0;
      }
    }
  };
  auto store = [&](int buf, int c) {
    if (c == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) sS[buf][tj + e][tq] = rs[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) sS[buf][si][sm + e] = rs[e];
    }
    if (!VT) {
#pragma unroll
      for (int e = 0; e < 4; ++e) sV[buf][vpi + e][vci] = rv[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) sV[buf][vi][vc + e] = rv[e];
    }
  };
  d4 acc[4][2];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) acc[ci][ri] = d4{0.0, 0.0, 0.0, 0.0};
  // the owned chunks, in order; cur / nxt chunk and their classes
  const int64_t kend = TRI ? (n < R0 + SR ? n : R0 + SR) : n;
  int64_t kk = 0;
  int c = 0;
  while (kk < kend && (c = cls(kk)) == 0) kk += SBK;
  if (kk < kend) {
    load(kk, c);
    store(0, c);
  }
  __syncthreads();
  int buf = 0;
  while (kk < kend) {
    int64_t kn = kk + SBK;
    int cn = 0;
    while (kn < kend && (cn = cls(kn)) == 0) kn += SBK;
    if (kn < kend) load(kn, cn);
#pragma unroll
    for (int q4 = 0; q4 < SBK / 4; ++q4) {
      double a[4], b[2];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) a[ci] = sV[buf][4 * q4 + lk][16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) b[ri] = sS[buf][4 * q4 + lk][32 * w + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    if (kn < kend) store(buf ^ 1, cn);
    __syncthreads();
    buf ^= 1;
    kk = kn;
    c = cn;
  }
#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t q = R0 + 32 * w + 16 * ri + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t cc = C0 + 16 * ci + lk + 4 * j;
        if (q < n && cc < k) out[q + cc * ldo] = scale * acc[ci][ri][j];
      }
    }
}

hipError_t launch_symm(const double *A, int64_t ld, int64_t n, int G, int rank, const double *V,
                       int64_t ldv, bool vt, int64_t k, double scale, double *out, int64_t ldo,
                       hipStream_t st) {
  if (n <= 0 || k <= 0) return hipSuccess;
  const dim3 grid((unsigned)((k + SC - 1) / SC), (unsigned)((n + SR - 1) / SR));
  if (vt)
    hipLaunchKernelGGL((k_symm<true, false>), grid, dim3(256), 0, st, A, ld, n, G, rank, V, ldv, k,
                       scale, out, ldo);
  else
    hipLaunchKernelGGL((k_symm<false, false>), grid, dim3(256), 0, st, A, ld, n, G, rank, V, ldv, k,
                       scale, out, ldo);
  return hipGetLastError();
}

// The triangular product on the sweep update's tile machinery (ACE_TRMM_BIG,
// default): 512 threads, 128 x 128 output tiles (8 waves of 64 x 32), BK =
// 16 chunks through double-buffered LDS with a register prefetch.  Row tiles
// are taken bottom-up (blockIdx.y = 0 is the last row tile, the longest k
// range), so the cheap tiles form the launch's tail.
constexpr int TT = 128, TBK = 16, TLD = TT + 16;
__global__ __launch_bounds__(512, 2) void k_trmm_lower(const double *__restrict__ A, int64_t ld,
                                                       int64_t n, const double *__restrict__ V,
                                                       int64_t ldv, int64_t k, double scale,
                                                       double *__restrict__ out, int64_t ldo) {
  __shared__ __attribute__((aligned(16))) double sS[2][TBK][TLD];  // [p][q - R0]
  __shared__ __attribute__((aligned(16))) double sV[2][TBK][TLD];  // [p][c - C0]
  const int64_t nrt = (n + TT - 1) / TT;
  const int64_t R0 = (nrt - 1 - (int64_t)blockIdx.y) * TT, C0 = (int64_t)blockIdx.x * TT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int wr = wv & 1, wc = wv >> 1;  // rows 64 wr.., columns 32 wc..
  const int sp = tid >> 5, sm = (tid & 31) * 4;  // staging: chunk row sp, 4 consecutive entries
  const int64_t kend = n < R0 + TT ? n : R0 + TT;
  double rs[4], rv[4];
  auto load = [&](int64_t kk) {
    const int64_t p = kk + sp;
    const bool diag = kk + TBK > R0;  // the chunk reaches the tile's rows: keep p < q only
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t q = R0 + sm + e, c = C0 + sm + e;
      rs[e] = (p < n && q < n && (!diag || q > p)) ? A[q + p * ld] : 0.0;
      rv[e] = (p < n && c < k) ? V[c + p * ldv] : 0.0;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      sS[buf][sp][sm + e] = rs[e];
      sV[buf][sp][sm + e] = rv[e];
    }
  };
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) acc[ci][ri] = d4{0.0, 0.0, 0.0, 0.0};
  if (kend > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t kk = 0; kk < kend; kk += TBK) {
    const bool more = kk + TBK < kend;
    if (more) load(kk + TBK);
#pragma unroll
    for (int q4 = 0; q4 < TBK / 4; ++q4) {
      double a[2], b[4];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sV[buf][4 * q4 + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) b[ri] = sS[buf][4 * q4 + lk][64 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 4; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t q = R0 + 64 * wr + 16 * ri + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t c = C0 + 32 * wc + 16 * ci + lk + 4 * j;
        if (q < n && c < k) out[q + c * ldo] = scale * acc[ci][ri][j];
      }
    }
}

static bool trmm_big() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_TRMM_BIG");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

hipError_t launch_trmm_lower(const double *A, int64_t ld, int64_t n, const double *V, int64_t ldv,
                             int64_t k, double scale, double *out, int64_t ldo, hipStream_t st) {
  if (n <= 0 || k <= 0) return hipSuccess;
  if (trmm_big()) {
    const dim3 grid((unsigned)((k + TT - 1) / TT), (unsigned)((n + TT - 1) / TT));
    hipLaunchKernelGGL(k_trmm_lower, grid, dim3(512), 0, st, A, ld, n, V, ldv, k, scale, out, ldo);
    return hipGetLastError();
  }
  const dim3 grid((unsigned)((k + SC - 1) / SC), (unsigned)((n + SR - 1) / SR));
  hipLaunchKernelGGL((k_symm<true, true>), grid, dim3(256), 0, st, A, ld, n, 1, 0, V, ldv, k, scale,
                     out, ldo);
  return hipGetLastError();
}

// ---------------------------------------------------------------- prediction sums
// For each test point c < nx (T' = S K_xX^T, n x nx, ld ldt; K = K_xX,
// nx x n, ld ldk):  a[c] = sum_q T'[q][c] w[q]   (tmp (y - mu), src/pred_cpp.cpp:20)
//                   d[c] = sum_q T'[q][c] K[c][q] (diag(tmp K_xX^T), :22)
// One workgroup per test point; T' column reads are contiguous.
__global__ __launch_bounds__(256) void k_pred_cols(const double *__restrict__ T, int64_t ldt,
                                                   const double *__restrict__ K, int64_t ldk,
                                                   int64_t n, const double *__restrict__ w,
                                                   double *__restrict__ a, double *__restrict__ d) {
  __shared__ double sh[2][4];
  const int64_t c = blockIdx.x;
  const double *tc = T + c * ldt;
  double sa = 0.0, sd = 0.0;
  for (int64_t q = threadIdx.x; q < n; q += 256) {
    const double t = tc[q];
    sa = fma(t, w[q], sa);
    sd = fma(t, K[c + q * ldk], sd);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sd += __shfl_xor(sd, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][wv] = sa;
    sh[1][wv] = sd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a[c] = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    d[c] = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
  }
}

hipError_t launch_pred_cols(const double *T, int64_t ldt, const double *K, int64_t ldk, int64_t n,
                            int64_t nx, const double *w, double *a, double *d, hipStream_t st) {
  if (nx <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pred_cols, dim3((unsigned)nx), dim3(256), 0, st, T, ldt, K, ldk, n, w, a,
                     d);
  return hipGetLastError();
}

// Triangular form (single GPU): with S = L + L^T + D (L strictly lower),
// Y = L K^T (n x nx, ld ldt) from launch_trmm_lower and s = S w:
//   a[c] = sum_q K[c][q] s[q]
//   d[c] = (K S K^T)[c][c] = sum_q K[c][q] (2 Y[q][c] + D[q] K[c][q])
__global__ __launch_bounds__(256) void k_pred_cols_tri(const double *__restrict__ Y, int64_t ldt,
                                                       const double *__restrict__ K, int64_t ldk,
                                                       int64_t n, const double *__restrict__ sv,
                                                       const double *__restrict__ D,
                                                       double *__restrict__ a,
                                                       double *__restrict__ d) {
  __shared__ double sh[2][4];
  const int64_t c = blockIdx.x;
  const double *yc = Y + c * ldt;
  double sa = 0.0, sd = 0.0;
  for (int64_t q = threadIdx.x; q < n; q += 256) {
    const double kq = K[c + q * ldk];
    sa = fma(kq, sv[q], sa);
    sd = fma(kq, fma(D[q], kq, 2.0 * yc[q]), sd);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    sa += __shfl_xor(sa, o, 64);
    sd += __shfl_xor(sd, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][wv] = sa;
    sh[1][wv] = sd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a[c] = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    d[c] = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
  }
}

hipError_t launch_pred_cols_tri(const double *Y, int64_t ldt, const double *K, int64_t ldk,
                                int64_t n, int64_t nx, const double *sv, const double *D, double *a,
                                double *d, hipStream_t st) {
  if (nx <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pred_cols_tri, dim3((unsigned)nx), dim3(256), 0, st, Y, ldt, K, ldk, n, sv,
                     D, a, d);
  return hipGetLastError();
}

// D[q] = scale A[q][q] (the diagonal of the stored matrix)
__global__ void k_diag_scaled(const double *__restrict__ A, int64_t ld, int64_t n, double scale,
                              double *__restrict__ D) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n) D[q] = scale * A[q + q * ld];
}

hipError_t launch_diag_scaled(const double *A, int64_t ld, int64_t n, double scale, double *D,
                              hipStream_t st) {
  hipLaunchKernelGGL(k_diag_scaled, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A, ld, n,
                     scale, D);
  return hipGetLastError();
}

// w = y - mu (the reference's y_X - mu, src/pred_cpp.cpp:20, 70)
__global__ void k_center(const double *__restrict__ y, int64_t n, double mu,
                         double *__restrict__ w) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) w[j] = y[j] - mu;
}

hipError_t launch_center(const double *y, int64_t n, double mu, double *w, hipStream_t st) {
  hipLaunchKernelGGL(k_center, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, n, mu, w);
  return hipGetLastError();
}

}  // namespace ace
