// ace_pairs_mm.hip -- pair-tile kernels whose feature loops run on the fp64
// matrix cores (v_mfma_f64_16x16x4_f64), so their register footprint does
// not grow with the covariate count p.
//
// The weighted squared distance of slice b is expanded,
//   r2_b(r,c) = s_b(r) + s_b(c) - 2 sum_i w_bi x_ri x_ci,  s_b(x) = sum_i w_bi x_i^2,
// and the cross term of a 64x64 pair tile is one MFMA GEMM with K = p.
// On gfx950 the fp64 matrix and vector rates are equal (78.6 TF/s each), so
// this is not about raw flops.  The expansion removes the per-pair d_i^2
// vectors (p VGPRs per pair) and the p-long FMA chains.  The per-lane state
// no longer depends on p, so large-p tiles (C3: p = 32, C4: p = 50) keep
// 3-4 waves per SIMD instead of one with scratch spills.  The cancellation
// in the expansion is bounded by eps * (s_b(r) + s_b(c)); r2 is clamped at 0
// and forced to 0 on the diagonal.
//
// Tile ownership (64 x 64 pairs, 256 threads): wave w, lane (lr, lk) owns
// row r = R0 + 16 w + lr and the 16 columns c = C0 + 16 cb + lk + 4 v
// (cb, v in 0..3) -- exactly the fragment layout of the MFMA result
// D = X_J (w_b X_I)^T, so no data moves between the GEMM and the
// elementwise kernel math.
#include "ace_internal.h"

namespace ace {

// Register caps (__launch_bounds__ second argument = waves per SIMD):
// gradient 2 (LDS 2 x 33 KB at p = 64 allows 2 workgroups per CU anyway),
// assembly 3 up to PM = 32 and 2 above (3 would spill at PM = 64).
typedef double d4 __attribute__((ext_vector_type(4)));

#define SQRT3 1.7320508075688772

__device__ __forceinline__ double sgn_mm(double x) {
  return (double)((0.0 < x) - (x < 0.0));
}

// Reference expressions of one slice value (same as ace_pairs.hip kval):
//  SE  (src/kernel_SE_cpp.cpp:96, 119), Matern32 (src/kernel_Matern_cpp.cpp:217-227).
template <int KIND>
__device__ __forceinline__ double kval_mm(int b, double r2, double lam, double zlo, double zhi,
                                          double lzlo, double lzhi) {
  if (KIND == 0) {
    if (b == 0) return exp(lam - r2);
    if (zlo == 0.0 || zhi == 0.0) return 0.0;
    return (sgn_mm(zlo) * sgn_mm(zhi)) * exp(((lam - r2) + lzlo) + lzhi);
  } else {
    const double t = sqrt(r2);
    const double e = (1.0 + SQRT3 * t) * exp(lam - SQRT3 * t);
    if (b == 0) return e;
    if (zlo == 0.0) return 0.0;
    return (e * zlo) * zhi;
  }
}

// Lower 64-tile (I, J) of block t: from the rank's list, or the row-major
// triangle index.
__device__ __forceinline__ void tile_of(const Tile *tiles, int64_t t, int64_t &I, int64_t &J) {
  if (tiles) {
    const Tile tt = tiles[t];
    I = tt.I;
    J = tt.J;
  } else {
    I = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    while (I * (I + 1) / 2 > t) --I;
    J = t - I * (I + 1) / 2;
  }
}

// ---------------------------------------------------------------------------
// Fused assembly (mode 0): lower 64-tiles of A (sigma on the diagonal,
// identity on padding) and of the Kfull copy; same outputs as
// k_assembly<PM, KIND, 0>.
// ---------------------------------------------------------------------------
template <int PM, int KIND>
__global__ __launch_bounds__(256, (PM <= 32 ? 3 : 2)) void k_asm_mm(PairSide S, int B, int ZS, TabView tab,
                                                double sig, double *__restrict__ out, int64_t ld,
                                                double *__restrict__ kcopy,
                                                const Tile *__restrict__ tiles, int G) {
  constexpr int XP = PM + 1;  // odd LDS pitch
  constexpr int KQ = PM / 4;
  __shared__ double sXJ[64 * XP];
  __shared__ double sSc[64];
  __shared__ double sZc[64], sLZc[64];
  __shared__ double sW[PM];
  int64_t I, J;
  tile_of(tiles, blockIdx.x, I, J);
  if (G > 1) {
    const int64_t coff = lcol(J * AT, G) - J * AT;
    out += coff * ld;
    if (kcopy) kcopy += coff * ld;
  }
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int64_t R0 = I * AT, C0 = J * AT, n = S.n;
  const int64_t r = R0 + 16 * w + lr;
  for (int e = tid; e < 64 * PM; e += 256) {
    const int c = e / PM, i = e - c * PM;
    sXJ[c * XP + i] = S.X[(C0 + c) * PM + i];
  }
  double xq[KQ];
#pragma unroll
  for (int kk = 0; kk < KQ; ++kk) xq[kk] = S.X[r * PM + 4 * kk + lk];
  double kf[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) kf[cb][v] = 0.0;

  for (int b = 0; b < B; ++b) {
    __syncthreads();  // previous slice done with sW / sSc (and sXJ staged)
    if (tid < PM) sW[tid] = tab.wk[b * PM + tid];
    if (b > 0 && tid >= 64 && tid < 128) {
      sZc[tid - 64] = S.Z[(C0 + tid - 64) * ZS + b - 1];
      if (KIND == 0) sLZc[tid - 64] = S.LZ[(C0 + tid - 64) * ZS + b - 1];
    }
    __syncthreads();
    if (tid < 64) {
      double s = 0.0;
#pragma unroll 4
      for (int i = 0; i < PM; ++i) {
        const double x = sXJ[tid * XP + i];
        s = fma(x * x, sW[i], s);
      }
      sSc[tid] = s;
    }
    double sr = 0.0;
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) sr = fma(xq[kk] * xq[kk], sW[4 * kk + lk], sr);
    sr += __shfl_xor(sr, 16, 64);
    sr += __shfl_xor(sr, 32, 64);
    d4 acc[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < KQ; ++kk) {
      const double bop = xq[kk] * sW[4 * kk + lk];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(sXJ[(16 * cb + lr) * XP + 4 * kk + lk], bop,
                                                       acc[cb], 0, 0, 0);
    }
    __syncthreads();  // sSc ready
    const double lam = tab.lam[b];
    double zr = 0.0, lzr = 0.0;
    if (b > 0) {
      zr = S.Z[r * ZS + b - 1];
      if (KIND == 0) lzr = S.LZ[r * ZS + b - 1];
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int cl = 16 * cb + lk + 4 * v;
        const int64_t c = C0 + cl;
        double r2 = fmax(fma(-2.0, acc[cb][v], sr + sSc[cl]), 0.0);
        if (c == r) r2 = 0.0;
        double zc = 0.0, lzc = 0.0;
        if (b > 0) {
          zc = sZc[cl];
          if (KIND == 0) lzc = sLZc[cl];
        }
        const double kb = (r < c) ? kval_mm<KIND>(b, r2, lam, zr, zc, lzr, lzc)
                                  : kval_mm<KIND>(b, r2, lam, zc, zr, lzc, lzr);
        kf[cb][v] += kb;
        __builtin_amdgcn_sched_barrier(0);  // one pair at a time: bounded live ranges
      }
  }
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + 16 * cb + lk + 4 * v;
      if (r < n && c < n) {
        out[r + c * ld] = (r == c) ? kf[cb][v] + sig : kf[cb][v];
        if (kcopy) kcopy[r + c * ld] = kf[cb][v];
      } else {
        out[r + c * ld] = (r == c) ? 1.0 : 0.0;  // identity padding
      }
    }
}

// ---------------------------------------------------------------------------
// Fused gradient traces (same outputs as k_grad2): per slice b (descending),
//   GEMM1  G = X_J (w_b X_I)^T        -> r2, K_b, U = T K_b [/ (1 + sqrt(3 r~2_b))]
//   GEMM2  V = U [X_J | 1]            -> for every feature i
//          sum_rc U d_i^2 = sum_r (x_ri^2 R_r - 2 x_ri V_ri) + sum_c x_ci^2 C_c
//          with R_r = V_r,p (row sums) and C_c (column sums, through LDS).
// U never leaves the registers for the GEMMs: the GEMM1 result fragment
// (row r = 16w+lr, column c = 16cb+lk+4v) is exactly GEMM2's A fragment for
// k-step 4cb+v.  The row operand x_r is read from global memory (L1/L2) in
// the k-loop, so no register holds a p-long vector.
// Matern32: r~2_b uses the gradient-indexed weights, which equal slice b+1's
// kernel weights (Q1), so the factor 1 + sqrt3 t of slice b+1 is cached per
// pair; the last slice gets its own GEMM with wg[B-1].
// ---------------------------------------------------------------------------
template <int PM>
__device__ __forceinline__ void gemm1_mm(const double *sXJ, const double *__restrict__ xrow,
                                         const double *sw, int lr, int lk, d4 (&acc)[4]) {
  constexpr int XP = PM + 1;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) acc[cb] = d4{0.0, 0.0, 0.0, 0.0};
  // one k-step of operands in flight (explicit prefetch; the scheduling
  // barrier keeps the compiler from hoisting every load of the loop)
  double an[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) an[cb] = sXJ[(16 * cb + lr) * XP + lk];
  double xn = xrow[lk];
#pragma unroll
  for (int kk = 0; kk < PM / 4; ++kk) {
    double ac[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) ac[cb] = an[cb];
    const double bop = xn * sw[4 * kk + lk];
    if (kk + 1 < PM / 4) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) an[cb] = sXJ[(16 * cb + lr) * XP + 4 * (kk + 1) + lk];
      xn = xrow[4 * (kk + 1) + lk];
    }
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
      acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[cb], bop, acc[cb], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// s_b of the 64 columns (threads 0..63, from LDS) and of the 64 rows
// (threads 64..127, from global X) into sSc / sSr.
template <int PM>
__device__ __forceinline__ void slice_norms(const double *sXJ, const double *__restrict__ X,
                                            int64_t R0, const double *sw, int tid, double *sSc,
                                            double *sSr) {
  constexpr int XP = PM + 1;
  if (tid < 64) {
    double s = 0.0;
    for (int i = 0; i < PM; ++i) {
      const double x = sXJ[tid * XP + i];
      s = fma(x * x, sw[i], s);
    }
    sSc[tid] = s;
  } else if (tid < 128) {
    const double *xr = X + (R0 + tid - 64) * PM;
    double s = 0.0;
    for (int i = 0; i < PM; ++i) {
      const double x = xr[i];
      s = fma(x * x, sw[i], s);
    }
    sSr[tid - 64] = s;
  }
}

__device__ __forceinline__ double rcp_nr_mm(double f) {
  double q = __builtin_amdgcn_rcp(f);
  double e = fma(-f, q, 1.0);
  q = fma(q, e, q);
  e = fma(-f, q, 1.0);
  return fma(q, e, q);
}

template <int PM, int KIND>
__global__ __launch_bounds__(256, 2) void k_grad_mm(PairSide S, int B, int ZS, TabView tab,
                                                 const double *__restrict__ A, int64_t ld,
                                                 double sA, const double *__restrict__ alpha,
                                                 double *__restrict__ gpart,
                                                 double *__restrict__ trpart, int64_t ntiles,
                                                 const Tile *__restrict__ tiles, int G) {
  constexpr int XP = PM + 1;
  constexpr int NV = PM + 1;
  constexpr int NB2 = (PM + 1 + 15) / 16;    // GEMM2 column blocks: [x | 1]
  constexpr int NBR = PM / 16, LRR = PM % 16;  // where R_r lands
  constexpr int UP = 65;                       // sU pitch
  __shared__ double sXJ[64 * XP];
  __shared__ double sU[64 * UP];
  __shared__ double sSc[64], sSr[64], sZc[64], sLZc[64], sC[4][64];
  __shared__ double sW[PM];
  __shared__ double sRed[4][NB2 * 16 + 1];
  const int64_t t = blockIdx.x;
  int64_t I, J;
  tile_of(tiles, t, I, J);
  if (G > 1) A += (lcol(J * AT, G) - J * AT) * ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int64_t R0 = I * AT, C0 = J * AT, n = S.n;
  const int64_t r = R0 + 16 * w + lr;
  const bool rvalid = r < n;
  const double *xrow = S.X + r * PM;
  for (int e = tid; e < 64 * PM; e += 256) {
    const int c = e / PM, i = e - c * PM;
    sXJ[c * XP + i] = S.X[(C0 + c) * PM + i];
  }
  // T = w_rc (sA A[r,c] - alpha_r alpha_c), w = 2 off the diagonal (lower pairs)
  const double ar = rvalid ? alpha[r] : 0.0;
  double tv[4][4];
  double tr = 0.0;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + 16 * cb + lk + 4 * v;
      double x = 0.0;
      if (rvalid && c < n && !(I == J && c > r)) {
        x = sA * A[r + c * ld] - ar * alpha[c];
        if (c == r) tr += x;
        else x *= 2.0;
      }
      tv[cb][v] = x;
    }
  double fc[4][4];  // Matern: 1 + sqrt3 t of slice b+1
  d4 acc[4];
  for (int b = B - 1; b >= 0; --b) {
    const bool last = (b == B - 1);
    if (KIND == 1 && last) {  // Matern, last slice: r~2 with its own weights
      __syncthreads();
      if (tid < PM) sW[tid] = tab.wg[b * PM + tid];
      __syncthreads();
      slice_norms<PM>(sXJ, S.X, R0, sW, tid, sSc, sSr);
      gemm1_mm<PM>(sXJ, xrow, sW, lr, lk, acc);
      __syncthreads();
      const double sr = sSr[16 * w + lr];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int cl = 16 * cb + lk + 4 * v;
          double rt2 = fmax(fma(-2.0, acc[cb][v], sr + sSc[cl]), 0.0);
          if (C0 + cl == r) rt2 = 0.0;
          fc[cb][v] = 1.0 + sqrt(3.0 * rt2);
        }
    }
    __syncthreads();  // previous users of sW / sSc / sSr / sZc / sU / sRed are done
    if (tid < PM) sW[tid] = tab.wk[b * PM + tid];
    if (b > 0 && tid >= 64 && tid < 128) {
      sZc[tid - 64] = S.Z[(C0 + tid - 64) * ZS + b - 1];
      if (KIND == 0) sLZc[tid - 64] = S.LZ[(C0 + tid - 64) * ZS + b - 1];
    }
    __syncthreads();
    slice_norms<PM>(sXJ, S.X, R0, sW, tid, sSc, sSr);
    gemm1_mm<PM>(sXJ, xrow, sW, lr, lk, acc);
    __syncthreads();  // sSc, sSr, sZc ready
    const double sr = sSr[16 * w + lr];
    const double lam = tab.lam[b];
    double zr = 0.0, lzr = 0.0;
    if (b > 0) {
      zr = S.Z[r * ZS + b - 1];
      if (KIND == 0) lzr = S.LZ[r * ZS + b - 1];
    }
    double gl = 0.0;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int cl = 16 * cb + lk + 4 * v;
        const int64_t c = C0 + cl;
        double r2 = fmax(fma(-2.0, acc[cb][v], sr + sSc[cl]), 0.0);
        if (c == r) r2 = 0.0;
        double zc = 0.0, lzc = 0.0;
        if (b > 0) {
          zc = sZc[cl];
          if (KIND == 0) lzc = sLZc[cl];
        }
        const bool rlo = r < c;
        const double zlo = rlo ? zr : zc, zhi = rlo ? zc : zr;
        double kb, f = 1.0;
        if (KIND == 0) {
          kb = kval_mm<0>(b, r2, lam, zlo, zhi, rlo ? lzr : lzc, rlo ? lzc : lzr);
        } else {
          const double tt = sqrt(r2);
          f = 1.0 + SQRT3 * tt;
          const double e = f * exp(lam - SQRT3 * tt);
          kb = (b == 0) ? e : (zlo == 0.0 ? 0.0 : (e * zlo) * zhi);
        }
        const double tk = tv[cb][v] * kb;
        gl += tk;
        double u;
        if (KIND == 0) {
          u = tk;
        } else {
          u = tk * rcp_nr_mm(fc[cb][v]);
          fc[cb][v] = f;
        }
        acc[cb][v] = u;
        sU[(16 * w + lr) * UP + cl] = u;
        __builtin_amdgcn_sched_barrier(0);
      }
    // GEMM2 over the column blocks, the block holding R_r first
    double Rv[4] = {0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < NB2; ++q) {
      const int nb = (q == 0) ? NBR : (q <= NBR ? q - 1 : q);
      const int nn = 16 * nb + lr;
      const double bconst = (nn == PM) ? 1.0 : 0.0;
      const int fo = nn < PM ? nn : 0;
      d4 a2 = d4{0.0, 0.0, 0.0, 0.0};
      double xn = sXJ[lk * XP + fo];
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const double x = xn;
        if (kk + 1 < 16) xn = sXJ[(4 * (kk + 1) + lk) * XP + fo];
        a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[kk >> 2][kk & 3], nn < PM ? x : bconst,
                                                  a2, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // a2[v'] = V[r' = R0 + 16 w + lk + 4 v'][nn]
      if (q == 0) {
#pragma unroll
        for (int v = 0; v < 4; ++v) Rv[v] = __shfl(a2[v], lk * 16 + LRR, 64);
      }
      double part = 0.0;
      if (nn < PM) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const double x = S.X[(R0 + 16 * w + lk + 4 * v) * PM + nn];
          part += fma(x * x, Rv[v], -2.0 * x * a2[v]);
        }
      }
      part += __shfl_xor(part, 16, 64);
      part += __shfl_xor(part, 32, 64);
      if (lk == 0) sRed[w][nn] = part;
    }
    gl += __shfl_xor(gl, 1, 64);
    gl += __shfl_xor(gl, 2, 64);
    gl += __shfl_xor(gl, 4, 64);
    gl += __shfl_xor(gl, 8, 64);
    gl += __shfl_xor(gl, 16, 64);
    gl += __shfl_xor(gl, 32, 64);
    if (lane == 0) sRed[w][NB2 * 16] = gl;
    __syncthreads();  // sU, sRed complete
    {  // column sums of U: thread (quarter q, column c) over 16 rows
      const int c = tid & 63, qq = tid >> 6;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += sU[(16 * qq + k) * UP + c];
      sC[qq][c] = s;
    }
    __syncthreads();
    if (tid < PM) {
      double g = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) g += sRed[q][tid];
      double gc = 0.0;
      for (int c = 0; c < 64; ++c) {
        const double x = sXJ[c * XP + tid];
        gc = fma(x * x, (sC[0][c] + sC[1][c]) + (sC[2][c] + sC[3][c]), gc);
      }
      gpart[((int64_t)b * NV + tid) * ntiles + t] = g + gc;
    } else if (tid == PM) {
      const double g = (sRed[0][NB2 * 16] + sRed[1][NB2 * 16]) + (sRed[2][NB2 * 16] + sRed[3][NB2 * 16]);
      gpart[((int64_t)b * NV + PM) * ntiles + t] = g;
    }
  }
  // trace of T
  tr += __shfl_xor(tr, 1, 64);
  tr += __shfl_xor(tr, 2, 64);
  tr += __shfl_xor(tr, 4, 64);
  tr += __shfl_xor(tr, 8, 64);
  tr += __shfl_xor(tr, 16, 64);
  tr += __shfl_xor(tr, 32, 64);
  __syncthreads();
  if (lane == 0) sSr[w] = tr;
  __syncthreads();
  if (tid == 0) trpart[t] = (sSr[0] + sSr[1]) + (sSr[2] + sSr[3]);
}

template <int PM>
static hipError_t grad_mm_pm(int kind, PairSide S, int B, int ZS, TabView tab, const double *A,
                             int64_t ld, double sA, const double *alpha, double *gpart,
                             double *trpart, hipStream_t st, const Tile *tiles, int64_t ntiles,
                             int G) {
  const int64_t nt = (S.n + AT - 1) / AT;
  const int64_t nblk = tiles ? ntiles : nt * (nt + 1) / 2;
  if (nblk == 0) return hipSuccess;
  if (kind == 0)
    hipLaunchKernelGGL((k_grad_mm<PM, 0>), dim3((unsigned)nblk), dim3(256), 0, st, S, B, ZS, tab,
                       A, ld, sA, alpha, gpart, trpart, nblk, tiles, G);
  else
    hipLaunchKernelGGL((k_grad_mm<PM, 1>), dim3((unsigned)nblk), dim3(256), 0, st, S, B, ZS, tab,
                       A, ld, sA, alpha, gpart, trpart, nblk, tiles, G);
  return hipGetLastError();
}

hipError_t launch_grad_mm(int kind, int PM, PairSide S, int B, int ZS, TabView tab,
                          const double *A, int64_t ld, double sA, const double *alpha,
                          double *gpart, double *trpart, hipStream_t st, const Tile *tiles,
                          int64_t ntiles, int G) {
  switch (PM) {
#define ACE_CASE(P) \
  case P:           \
    return grad_mm_pm<P>(kind, S, B, ZS, tab, A, ld, sA, alpha, gpart, trpart, st, tiles, ntiles, G);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

template <int PM>
static hipError_t asm_mm_pm(int kind, PairSide S, int64_t npad, int B, int ZS, TabView tab,
                            double sig, double *out, int64_t ld, double *kcopy, hipStream_t st,
                            const Tile *tiles, int64_t ntiles, int G) {
  const int64_t nt = npad / AT;
  const int64_t nblk = tiles ? ntiles : nt * (nt + 1) / 2;
  if (nblk == 0) return hipSuccess;
  if (kind == 0)
    hipLaunchKernelGGL((k_asm_mm<PM, 0>), dim3((unsigned)nblk), dim3(256), 0, st, S, B, ZS, tab,
                       sig, out, ld, kcopy, tiles, G);
  else
    hipLaunchKernelGGL((k_asm_mm<PM, 1>), dim3((unsigned)nblk), dim3(256), 0, st, S, B, ZS, tab,
                       sig, out, ld, kcopy, tiles, G);
  return hipGetLastError();
}

hipError_t launch_assembly_mm(int kind, int PM, PairSide S, int64_t npad, int B, int ZS,
                              TabView tab, double sig, double *out, int64_t ld, double *kcopy,
                              hipStream_t st, const Tile *tiles, int64_t ntiles, int G) {
  switch (PM) {
#define ACE_CASE(P) \
  case P: return asm_mm_pm<P>(kind, S, npad, B, ZS, tab, sig, out, ld, kcopy, st, tiles, ntiles, G);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ace
