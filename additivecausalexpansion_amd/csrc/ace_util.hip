// ace_util.hip -- small device kernels around the hot path: augmented-row
// setup, alpha/mu from the swept corner, deterministic reductions, GEMV,
// a bounds-checked MFMA f64 GEMM for prediction, and prediction row sums.
#include "ace_internal.h"

namespace ace {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for 256 threads (deterministic order).
__device__ __forceinline__ double block_sum256(double v, double *sh) {
  v = wsum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  const double r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  __syncthreads();
  return r;
}

// Block-wide sum for 1024 threads (deterministic order): the latency-bound
// per-evaluation reductions (colsum of the tile partials, final sums with
// n logs) run 4x shorter loops per thread than at 256.
__device__ __forceinline__ double block_sum1024(double v, double *sh) {
  v = wsum(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int q = 0; q < 16; q += 4) r += (sh[q] + sh[q + 1]) + (sh[q + 2] + sh[q + 3]);
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------- AUG rows
// rows npad .. npad+AUG-1 of A: row 0 = y (j < n), row 1 = 1 (j < n), 0 else
__global__ void k_aug_init(double *__restrict__ A, int64_t ld, int64_t npad, int64_t n,
                           const double *__restrict__ y, int G, int rank, int *__restrict__ z0,
                           int n0, int *__restrict__ z1, int n1) {
  const int64_t j = blockIdx.x;  // global column
  const int t = threadIdx.x;     // AUG rows
  if (j == 0) {
    for (int i = t; i < n0; i += AUG) z0[i] = 0;
    for (int i = t; i < n1; i += AUG) z1[i] = 0;
  }
  if (!owns_col(j, G, rank)) return;
  double v = 0.0;
  if (j < n) {
    if (t == 0) v = y ? y[j] : 0.0;  // y == null: the 1 row only
    else if (t == 1) v = 1.0;
  }
  A[(npad + t) + lcol(j, G) * ld] = v;
}

hipError_t launch_aug_init(double *A, int64_t ld, int64_t npad, int64_t n, const double *y,
                           hipStream_t st, int G, int rank, int *z0, int n0, int *z1, int n1) {
  hipLaunchKernelGGL(k_aug_init, dim3((unsigned)ld), dim3(AUG), 0, st, A, ld, npad, n, y, G,
                     rank, z0, n0, z1, n1);
  return hipGetLastError();
}

// Sharded model: the swept AUG rows of the rank's own columns into
// vec = [u (npad) | v (npad) | yKy, yK1, 1K1], zero elsewhere, so that a
// sum over ranks (all-reduce) yields the whole vectors on every rank.
__global__ void k_aug_extract(const double *__restrict__ A, int64_t ld, int64_t npad, int G,
                              int rank, double *__restrict__ vec) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < npad) {
    const bool own = owns_col(j, G, rank);
    const int64_t l = lcol(j, G);
    vec[j] = own ? A[npad + l * ld] : 0.0;
    vec[npad + j] = own ? A[(npad + 1) + l * ld] : 0.0;
  }
  if (j == 0) {
    const bool own = owns_col(npad, G, rank);
    const int64_t l = lcol(npad, G);
    vec[2 * npad + 0] = own ? -A[npad + l * ld] : 0.0;
    vec[2 * npad + 1] = own ? -A[(npad + 1) + l * ld] : 0.0;
    vec[2 * npad + 2] = own ? -A[(npad + 1) + (l + 1) * ld] : 0.0;
  }
}

hipError_t launch_aug_extract(const double *A, int64_t ld, int64_t npad, int G, int rank,
                              double *vec, hipStream_t st) {
  hipLaunchKernelGGL(k_aug_extract, dim3((unsigned)((npad + 255) / 256)), dim3(256), 0, st, A,
                     ld, npad, G, rank, vec);
  return hipGetLastError();
}

// out[0] = sum_j y_j (A^-1 1)_j and out[1] = 1^T A^-1 1 from the swept AUG
// row 1 and corner (one workgroup, fixed order): mu_solution_cpp's
// sum(inv y) and accu(inv) without a pass over the inverse (Q4).
__global__ __launch_bounds__(1024) void k_aug_dot(const double *__restrict__ A, int64_t ld,
                                                  int64_t npad, int64_t n,
                                                  const double *__restrict__ y,
                                                  double *__restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += 1024) s += y[j] * A[(npad + 1) + j * ld];
  s = block_sum1024(s, sh);
  if (threadIdx.x == 0) {
    out[0] = s;
    out[1] = -A[(npad + 1) + (npad + 1) * ld];
  }
}

hipError_t launch_aug_dot(const double *A, int64_t ld, int64_t npad, int64_t n, const double *y,
                          double *out, hipStream_t st) {
  hipLaunchKernelGGL(k_aug_dot, dim3(1), dim3(1024), 0, st, A, ld, npad, n, y, out);
  return hipGetLastError();
}

// alpha / scal from the all-reduced aug vector (same formulas as
// k_alpha_from_aug).
__global__ void k_alpha_from_vec(const double *__restrict__ vec, int64_t npad, int64_t n,
                                 double theta1, int use_mu, double *__restrict__ alpha,
                                 double *__restrict__ scal) {
  const double yKy = vec[2 * npad], yK1 = vec[2 * npad + 1], oK1 = vec[2 * npad + 2];
  const double mu = 0.5 * yK1 / oK1;  // Q4 (src/utilities_cpp.cpp:9)
  const double mu_eff = use_mu ? mu : theta1;
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) alpha[j] = vec[j] - mu_eff * vec[npad + j];
  if (j == 0) {
    scal[0] = yKy;
    scal[1] = yK1;
    scal[2] = oK1;
    scal[3] = mu;
    scal[4] = mu_eff;
  }
}

hipError_t launch_alpha_from_vec(const double *vec, int64_t npad, int64_t n, double theta1,
                                 int use_mu, double *alpha, double *scal, hipStream_t st) {
  hipLaunchKernelGGL(k_alpha_from_vec, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, vec,
                     npad, n, theta1, use_mu, alpha, scal);
  return hipGetLastError();
}

// y += x (in-process all-reduce of the simulated rank group)
__global__ void k_axpy1(const double *__restrict__ x, double *__restrict__ y, int64_t count) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < count) y[j] += x[j];
}

hipError_t launch_add(const double *x, double *y, int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_axpy1, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, x, y,
                     count);
  return hipGetLastError();
}

__global__ void k_alpha_from_aug(const double *__restrict__ A, int64_t ld, int64_t npad,
                                 int64_t n, double theta1, int use_mu,
                                 double *__restrict__ alpha, double *__restrict__ scal,
                                 const double *__restrict__ theta1p) {
  const double yKy = -A[npad + npad * ld];
  const double yK1 = -A[(npad + 1) + npad * ld];
  const double oK1 = -A[(npad + 1) + (npad + 1) * ld];
  const double mu = 0.5 * yK1 / oK1;  // Q4 (src/utilities_cpp.cpp:9)
  const double mu_eff = use_mu ? mu : (theta1p ? *theta1p : theta1);
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) {
    const double u = A[npad + j * ld];
    const double v = A[(npad + 1) + j * ld];
    alpha[j] = u - mu_eff * v;
  }
  if (j == 0) {
    scal[0] = yKy;
    scal[1] = yK1;
    scal[2] = oK1;
    scal[3] = mu;
    scal[4] = mu_eff;
  }
}

hipError_t launch_alpha_from_aug(const double *A, int64_t ld, int64_t npad, int64_t n,
                                 double theta1, int use_mu, double *alpha, double *scal,
                                 hipStream_t st, const double *theta1p) {
  hipLaunchKernelGGL(k_alpha_from_aug, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A,
                     ld, npad, n, theta1, use_mu, alpha, scal, theta1p);
  return hipGetLastError();
}

// ---------------------------------------------------------------- reductions
__global__ __launch_bounds__(1024) void k_colsum(const double *__restrict__ in, int64_t nrows,
                                                 double *__restrict__ out) {
  __shared__ double sh[16];
  const int j = blockIdx.x;
  const double *p = in + (int64_t)j * nrows;
  double s = 0.0;
  for (int64_t t = threadIdx.x; t < nrows; t += 1024) s += p[t];
  s = block_sum1024(s, sh);
  if (threadIdx.x == 0) out[j] = s;
}

hipError_t launch_colsum(const double *in, int64_t nrows, int ncols, double *out,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_colsum, dim3(ncols), dim3(1024), 0, st, in, nrows, out);
  return hipGetLastError();
}

// Sums of the tile-major gradient partials (one row of ncols per tile).
// Pass 1: block (g, ch) sums columns 64 g .. 64 g + 63 over tile chunk ch;
// lane = column, so each wave reads one contiguous 512-B run of a tile row;
// the 4 waves interleave tiles and meet in LDS.  Pass 2: the chunk partials.
// Fixed summation order: bit-identical run to run.
constexpr int TS_CHUNKS = 128;

__global__ __launch_bounds__(256) void k_tile_sums1(const double *__restrict__ part,
                                                    int64_t ntiles, int ncols,
                                                    double *__restrict__ work) {
  __shared__ double sh[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int64_t per = (ntiles + TS_CHUNKS - 1) / TS_CHUNKS;
  const int64_t t0 = (int64_t)blockIdx.y * per;
  const int64_t t1 = t0 + per < ntiles ? t0 + per : ntiles;
  double s = 0.0;
  if (col < ncols)
    for (int64_t t = t0 + wv; t < t1; t += 4) s += part[t * ncols + col];
  sh[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && col < ncols)
    work[(int64_t)blockIdx.y * ncols + col] = (sh[0][lane] + sh[1][lane]) + (sh[2][lane] + sh[3][lane]);
}

__global__ __launch_bounds__(256) void k_tile_sums2(const double *__restrict__ work, int ncols,
                                                    double *__restrict__ out) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= ncols) return;
  double s = 0.0;
  for (int ch = 0; ch < TS_CHUNKS; ++ch) s += work[(int64_t)ch * ncols + col];
  out[col] = s;
}

int64_t tile_sums_work(int ncols) { return (int64_t)TS_CHUNKS * ncols; }

hipError_t launch_tile_sums(const double *part, int64_t ntiles, int ncols, double *work,
                            double *out, hipStream_t st) {
  if (ncols <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_tile_sums1, dim3((unsigned)((ncols + 63) / 64), TS_CHUNKS), dim3(256), 0,
                     st, part, ntiles, ncols, work);
  hipLaunchKernelGGL(k_tile_sums2, dim3((unsigned)((ncols + 255) / 256)), dim3(256), 0, st, work,
                     ncols, out);
  return hipGetLastError();
}

// s = Kfull alpha (explicit, the ABI path) or null: then the fused model's
// identity ybar - Kfull alpha = sig alpha is used -- A = Kfull + sig I is the
// matrix the sweep inverted and alpha = A^-1 ybar, so the residual of
// src/stats_cpp.cpp:25 needs no pass over Kfull.
__global__ __launch_bounds__(1024) void k_final_sums(const double *__restrict__ y,
                                                    const double *__restrict__ mup,
                                                    const double *__restrict__ alpha,
                                                    const double *__restrict__ s, double sig,
                                                    int64_t n, const double *__restrict__ piv,
                                                    int64_t npiv, double *__restrict__ sums,
                                                    const double *__restrict__ sigp,
                                                    const int *__restrict__ flag) {
  __shared__ double sh[16];
  const double mu = *mup;
  if (sigp) sig = *sigp;
  double e2 = 0.0, ya = 0.0, sa = 0.0, ld = 0.0;
  for (int64_t x = threadIdx.x; x < n; x += 1024) {
    const double ybar = y[x] - mu;
    const double e = s ? ybar - s[x] : sig * alpha[x];
    e2 += e * e;
    ya += y[x] * alpha[x];
    sa += alpha[x];
  }
  for (int64_t x = threadIdx.x; x < npiv; x += 1024) ld += log(piv[x]);
  e2 = block_sum1024(e2, sh);
  ya = block_sum1024(ya, sh);
  sa = block_sum1024(sa, sh);
  ld = block_sum1024(ld, sh);
  if (threadIdx.x == 0) {
    sums[0] = e2;
    sums[1] = ya;
    sums[2] = sa;
    sums[3] = ld;
    if (flag) sums[4] = (double)*flag;
  }
}

hipError_t launch_final_sums(const double *y, const double *mu, const double *alpha, const double *s,
                             double sig, int64_t n, const double *piv, int64_t npiv,
                             double *sums, hipStream_t st, const double *sigp, const int *flag) {
  hipLaunchKernelGGL(k_final_sums, dim3(1), dim3(1024), 0, st, y, mu, alpha, s, sig, n, piv, npiv,
                     sums, sigp, flag);
  return hipGetLastError();
}

// ---------------------------------------------------------------- GEMV
__global__ void k_gemv(const double *__restrict__ M, int64_t ld, int64_t m, int64_t k,
                       const double *__restrict__ x, double *__restrict__ y) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  double s = 0.0;
  for (int64_t c = 0; c < k; ++c) s = fma(M[r + c * ld], x[c], s);
  y[r] = s;
}

hipError_t launch_gemv(const double *M, int64_t ld, int64_t m, int64_t k, const double *x,
                       double *y, hipStream_t st) {
  hipLaunchKernelGGL(k_gemv, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, M, ld, m, k,
                     x, y);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_gemv_t(const double *__restrict__ M, int64_t ld,
                                                int64_t m, const double *__restrict__ x,
                                                double *__restrict__ y) {
  __shared__ double sh[4];
  const int64_t c = blockIdx.x;
  double s = 0.0;
  for (int64_t r = threadIdx.x; r < m; r += 256) s = fma(M[r + c * ld], x[r], s);
  s = block_sum256(s, sh);
  if (threadIdx.x == 0) y[c] = s;
}

hipError_t launch_gemv_t(const double *M, int64_t ld, int64_t m, int64_t k, const double *x,
                         double *y, hipStream_t st) {
  hipLaunchKernelGGL(k_gemv_t, dim3((unsigned)k), dim3(256), 0, st, M, ld, m, x, y);
  return hipGetLastError();
}

// ---------------------------------------------------------------- GEMM
// C (m x n) = A (m x k) B (k x n), col-major; 128x128 tiles, 4 waves of
// 4x4 v_mfma_f64_16x16x4_f64 fragments; zero-filled edges.
constexpr int GBK = 16, GLD = 144;

__global__ __launch_bounds__(256) void k_gemm_nn(int64_t m, int64_t n, int64_t k,
                                                 const double *__restrict__ A, int64_t lda,
                                                 const double *__restrict__ B, int64_t ldb,
                                                 double *__restrict__ C, int64_t ldc) {
  __shared__ double sA[GBK][GLD];
  __shared__ double sB[GBK][GLD];
  const int64_t R0 = (int64_t)blockIdx.y * 128, C0 = (int64_t)blockIdx.x * 128;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1, lr = lane & 15, lk = lane >> 4;
  d4 acc[4][4];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) acc[ci][ri] = d4{0.0, 0.0, 0.0, 0.0};
  const int ak = tid >> 4, am = (tid & 15) * 8;  // A stage: row block of 8, one k
  const int bc = tid >> 1, bk = (tid & 1) * 8;   // B stage: one column, 8 k
  for (int64_t k0 = 0; k0 < k; k0 += GBK) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t r = R0 + am + e, kk = k0 + ak;
      sA[ak][am + e] = (r < m && kk < k) ? A[r + kk * lda] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int64_t c = C0 + bc, kk = k0 + bk + e;
      sB[bk + e][bc] = (c < n && kk < k) ? B[kk + c * ldb] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GBK / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) a[ci] = sB[4 * kk + lk][64 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) b[ri] = sA[4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll
        for (int ri = 0; ri < 4; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t c = C0 + 64 * wc + 16 * ci + lk + 4 * j;
        if (r < m && c < n) C[r + c * ldc] = acc[ci][ri][j];
      }
    }
}

hipError_t launch_gemm_nn(int64_t m, int64_t n, int64_t k, const double *A, int64_t lda,
                          const double *B, int64_t ldb, double *C, int64_t ldc,
                          hipStream_t st) {
  dim3 grid((unsigned)((n + 127) / 128), (unsigned)((m + 127) / 128));
  hipLaunchKernelGGL(k_gemm_nn, grid, dim3(256), 0, st, m, n, k, A, lda, B, ldb, C, ldc);
  return hipGetLastError();
}

// ---------------------------------------------------------------- copies
// out (full n x n) = scale * sym(A lower); tile-transposed through LDS.
// G > 1: A is block-cyclic column storage (launch_sym_from_cyclic).
__device__ __forceinline__ int64_t cyc_col(int64_t c, int64_t ld, int G, int64_t slot) {
  return G == 1 ? c * ld : ((c / NB) % G) * slot + lcol(c, G) * ld;
}

__global__ __launch_bounds__(256) void k_sym_from_lower(const double *__restrict__ A,
                                                        int64_t ld, int64_t n, double scale,
                                                        double *__restrict__ out,
                                                        int64_t ldo, int G, int64_t slot) {
  __shared__ double t[64][65];
  const int64_t I = blockIdx.y, J = blockIdx.x;
  const int tid = threadIdx.x;
  if (I >= J) {
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const int64_t r = I * 64 + a, c = J * 64 + b;
      if (r < n && c < n) {
        const double v = (r >= c) ? A[r + cyc_col(c, ld, G, slot)] : A[c + cyc_col(r, ld, G, slot)];
        out[r + c * ldo] = scale * v;
      }
    }
  } else {
    // upper tile (I < J): out[r, c] = A[c, r] with c > r: read tile (J, I) of A
    for (int e = tid; e < 4096; e += 256) {
      const int b = e & 63, a = e >> 6;  // b: row of A (= c), a: col of A (= r)
      const int64_t c = J * 64 + b, r = I * 64 + a;
      t[a][b] = (r < n && c < n) ? A[c + cyc_col(r, ld, G, slot)] : 0.0;
    }
    __syncthreads();
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const int64_t r = I * 64 + a, c = J * 64 + b;
      if (r < n && c < n) out[r + c * ldo] = scale * t[a][b];
    }
  }
}

hipError_t launch_sym_from_lower(const double *A, int64_t ld, int64_t n, double scale,
                                 double *out, int64_t ldo, hipStream_t st) {
  const unsigned nt = (unsigned)((n + 63) / 64);
  hipLaunchKernelGGL(k_sym_from_lower, dim3(nt, nt), dim3(256), 0, st, A, ld, n, scale, out,
                     ldo, 1, (int64_t)0);
  return hipGetLastError();
}

hipError_t launch_sym_from_cyclic(const double *A, int64_t ld, int64_t n, int G,
                                  int64_t slot_elems, double scale, double *out, int64_t ldo,
                                  hipStream_t st) {
  const unsigned nt = (unsigned)((n + 63) / 64);
  hipLaunchKernelGGL(k_sym_from_lower, dim3(nt, nt), dim3(256), 0, st, A, ld, n, scale, out,
                     ldo, G, slot_elems);
  return hipGetLastError();
}

// dst (npad x npad block, ld_dst): src K in [0,m)x[0,n), + diag on its
// diagonal, identity elsewhere (padding).
__global__ void k_copy_add_diag(const double *__restrict__ src, int64_t lds, int64_t m,
                                int64_t n, double diag, double *__restrict__ dst,
                                int64_t ldd, int64_t npad) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (r >= npad) return;
  double v;
  if (r < m && c < n) v = src[r + c * lds] + (r == c ? diag : 0.0);
  else v = (r == c) ? 1.0 : 0.0;
  dst[r + c * ldd] = v;
}

hipError_t launch_prepare_A(const double *src, int64_t n, double diag, double *dst, int64_t ldd,
                            int64_t npad, hipStream_t st) {
  hipLaunchKernelGGL(k_copy_add_diag, dim3((unsigned)((npad + 255) / 256), (unsigned)npad),
                     dim3(256), 0, st, src, n, n, n, diag, dst, ldd, npad);
  return hipGetLastError();
}

__global__ void k_fill(double *p, int64_t count, double v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) p[i] = v;
}

hipError_t launch_fill(double *p, int64_t count, double v, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, p, count,
                     v);
  return hipGetLastError();
}

__global__ void k_log_abs(const double *__restrict__ Z, double *__restrict__ LZ, int64_t count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) LZ[i] = log(fabs(Z[i]));
}

hipError_t launch_log_abs(const double *Z, double *LZ, int64_t count, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_log_abs, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, Z, LZ,
                     count);
  return hipGetLastError();
}

// ---------------------------------------------------------------- prediction
// Kmarg = slice(1) + slice(2) + ... (src/pred_cpp.cpp:55-67), or slice 0 if B == 1
__global__ void k_marginal_sum(const double *__restrict__ cube, int64_t mn, int B,
                               double *__restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= mn) return;
  double s;
  if (B > 1) {
    s = cube[i + mn];
    for (int b = 2; b < B; ++b) s += cube[i + (int64_t)b * mn];
  } else {
    s = cube[i];
  }
  out[i] = s;
}

hipError_t launch_marginal_sum(const double *cube, int64_t m, int64_t n, int B, double *out,
                               hipStream_t st) {
  const int64_t mn = m * n;
  hipLaunchKernelGGL(k_marginal_sum, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, st, cube,
                     mn, B, out);
  return hipGetLastError();
}

__global__ void k_pred_rows(const double *__restrict__ T, const double *__restrict__ K,
                            int64_t ld, int64_t nx, int64_t nX, const double *__restrict__ w,
                            double *__restrict__ a, double *__restrict__ q) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nx) return;
  double sa = 0.0, sq = 0.0;
  for (int64_t c = 0; c < nX; ++c) {
    const double t = T[r + c * ld];
    sa = fma(t, w[c], sa);
    sq = fma(t, K[r + c * ld], sq);
  }
  a[r] = sa;
  q[r] = sq;
}

hipError_t launch_pred_rows(const double *T, const double *K, int64_t ld, int64_t nx,
                            int64_t nX, const double *w, double *a, double *q,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_pred_rows, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, st, T, K, ld,
                     nx, nX, w, a, q);
  return hipGetLastError();
}

// part[j*n + c] = W[c,j] * sum_r M[r,c] W[r,j]   (j = 0..2)
__global__ __launch_bounds__(256) void k_quad3_cols(const double *__restrict__ M, int64_t ld,
                                                    int64_t n, const double *__restrict__ Wt,
                                                    double *__restrict__ part) {
  __shared__ double sh[4];
  const int64_t c = blockIdx.x;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int64_t r = threadIdx.x; r < n; r += 256) {
    const double v = M[r + c * ld];
    s0 = fma(v, Wt[r], s0);
    s1 = fma(v, Wt[r + n], s1);
    s2 = fma(v, Wt[r + 2 * n], s2);
  }
  s0 = block_sum256(s0, sh);
  s1 = block_sum256(s1, sh);
  s2 = block_sum256(s2, sh);
  if (threadIdx.x == 0) {
    part[c] = Wt[c] * s0;
    part[n + c] = Wt[c + n] * s1;
    part[2 * n + c] = Wt[c + 2 * n] * s2;
  }
}

hipError_t launch_quad3(const double *M, int64_t ld, int64_t n, const double *W, double *q,
                        hipStream_t st) {
  // q must have room for 3*n + 3 doubles: partials then the 3 sums
  hipLaunchKernelGGL(k_quad3_cols, dim3((unsigned)n), dim3(256), 0, st, M, ld, n, W, q + 3);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return launch_colsum(q + 3, n, 3, q, st);
}

}  // namespace ace
