// ace_pairs.hip -- pair-space kernels of the hot path, written for gfx950.
//
//  * k_assembly : reduced-kernel assembly K = sum_b K_b (a1-a4 of SURVEY §8a)
//  * k_grad     : fused gradient traces -0.5 tr(T dK/dtheta) for every
//                 hyperparameter, plus the Kfull*alpha rows for the RMSE
//                 (a7/a8), without materialising the n x n x B cube.
//
// Both kernels walk 64x64 pair tiles with 256 threads: lane = row r, the
// wave id picks 16 columns c = J*64 + wave + 4m, so every column-side
// operand (x_c, z_c, the per-b weight rows) is wave-uniform and is fetched
// with scalar loads, and every store to the column-major matrix is one
// contiguous 512-B segment per wave.  fp64 VALU bound.
#include <algorithm>
#include <cstdlib>

#include "ace_internal.h"

namespace ace {

#define SQRT3 1.7320508075688772

__device__ __forceinline__ double sgn(double x) {
  return (double)((0.0 < x) - (x < 0.0));
}

// One slice value K_b for a pair, following the reference expressions:
//  SE  (src/kernel_SE_cpp.cpp:96, 119 / 39, 53): slice 0 exp(lam - r2);
//      b>=1: sign(z_lo) sign(z_hi) exp(((lam - r2) + log|z_lo|) + log|z_hi|),
//      0 if either z is exactly 0 (Q7).
//  Matern32 (src/kernel_Matern_cpp.cpp:217-227 / 79-86): t = sqrt(r2),
//      e = (1 + sqrt3 t) exp(lam - sqrt3 t); b>=1: (e z_lo) z_hi, 0 if
//      z_lo == 0 (and, in the cross kernel, if z_hi == 0).
// "lo" is the first operand of the reference's product: the smaller index
// of a symmetric pair (upper-triangle loop), the X1/Z1 side of a cross pair.
template <int KIND, bool CROSS>
__device__ __forceinline__ double kval(int b, double r2, double lam, double zlo,
                                       double zhi, double lzlo, double lzhi) {
  if (KIND == 0) {
    if (b == 0) return exp(lam - r2);
    if (zlo == 0.0 || zhi == 0.0) return 0.0;
    return (sgn(zlo) * sgn(zhi)) * exp(((lam - r2) + lzlo) + lzhi);
  } else {
    const double t = sqrt(r2);
    const double e = (1.0 + SQRT3 * t) * exp(lam - SQRT3 * t);
    if (b == 0) return e;
    if (zlo == 0.0) return 0.0;
    if (CROSS && zhi == 0.0) return 0.0;
    return (e * zlo) * zhi;
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------
// Assembly.  MODE 0: fused (lower tiles of A incl. sigma + identity padding)
//            MODE 1: symmetric full output (+cube), MODE 2: cross (+cube).
// ---------------------------------------------------------------------------
template <int PM, int KIND, int MODE>
__global__ __launch_bounds__(256) void k_assembly(PairSide R, PairSide C, int64_t npad,
                                                  int B, int ZS, TabView tab, double sig,
                                                  double *__restrict__ out, int64_t ld,
                                                  double *__restrict__ cube,
                                                  const Tile *__restrict__ tiles, int G, int b0,
                                                  int b1) {
  int I = blockIdx.y, J = blockIdx.x;
  if (MODE == 0 && tiles) {  // sharded: the rank's own lower tiles, 1-D grid
    const Tile tt = tiles[blockIdx.x];
    I = tt.I;
    J = tt.J;
  }
  if (MODE != 2 && J > I) return;
  if (MODE == 0 && G > 1) {  // local column storage (ace_internal.h lcol)
    const int64_t coff = lcol((int64_t)J * AT, G) - (int64_t)J * AT;
    out += coff * ld;
    if (cube) cube += coff * ld;
  }
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t r = (int64_t)I * AT + lane;
  const int64_t nR = (MODE == 0) ? npad : R.n;
  const int64_t nC = (MODE == 0) ? npad : C.n;
  if (r >= nR) return;
  const bool rvalid = r < R.n;
  double xr[PM];
#pragma unroll
  for (int i = 0; i < PM; ++i) xr[i] = rvalid ? R.X[r * PM + i] : 0.0;
  const int64_t cubeld = (MODE == 2) ? R.n : R.n;  // n (sym) or n1 (cross)
  const int64_t slice = (MODE == 2) ? R.n * C.n : R.n * R.n;

  for (int m = 0; m < AT / 4; ++m) {
    const int64_t c = (int64_t)J * AT + wv + 4 * m;  // wave-uniform
    if (c >= nC) break;
    if (MODE == 1 && I == J && c > r) continue;  // lower half, mirrored below
    const bool cvalid = c < C.n;
    if (!(rvalid && cvalid)) {
      if (MODE == 0) out[r + c * ld] = (r == c) ? 1.0 : 0.0;  // identity padding
      continue;
    }
    double d2[PM];
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      const double d = xr[i] - C.X[c * PM + i];
      d2[i] = d * d;
    }
    const bool rlo = (MODE == 2) || (r < c);  // row is the reference's first operand
    double kf = 0.0;
    for (int b = b0; b < b1; ++b) {  // [0, B), or the marginal slices of prediction
      const double *w = tab.wk + b * PM;
      double r2 = 0.0;
#pragma unroll
      for (int i = 0; i < PM; ++i) r2 = fma(d2[i], w[i], r2);
      double zr = 0.0, zc = 0.0, lzr = 0.0, lzc = 0.0;
      if (b > 0) {
        zr = R.Z[r * ZS + b - 1];
        zc = C.Z[c * ZS + b - 1];
        if (KIND == 0) {
          lzr = R.LZ[r * ZS + b - 1];
          lzc = C.LZ[c * ZS + b - 1];
        }
      }
      const double kb =
          rlo ? kval<KIND, MODE == 2>(b, r2, tab.lam[b], zr, zc, lzr, lzc)
              : kval<KIND, MODE == 2>(b, r2, tab.lam[b], zc, zr, lzc, lzr);
      kf += kb;
      if (MODE != 0 && cube) {
        cube[r + c * cubeld + b * slice] = kb;
        if (MODE == 1 && c != r) cube[c + r * cubeld + b * slice] = kb;
      }
    }
    if (MODE == 0) {
      out[r + c * ld] = (r == c) ? kf + (tab.sig ? *tab.sig : sig) : kf;
      if (cube) cube[r + c * ld] = kf;  // Kfull copy for the RMSE product (the sweep
                                        // overwrites out)
    } else {
      out[r + c * ld] = kf;
      if (MODE == 1 && c != r) out[c + r * ld] = kf;
    }
  }
}

// ---------------------------------------------------------------------------
// Gradient traces.  T = w_rc (sA A[r,c] - alpha_r alpha_c) on lower pairs,
// w = 2 off the diagonal, 1 on it (T and dK are symmetric, so the full-matrix
// trace tr(T dK) = sum_rc T_rc dK_rc, src/include/ace_kernel_utils.hpp:23-26).
// Per b: lambda sum   sum T K_b                       (src/kernel_SE_cpp.cpp:224-227)
//        length sums  sum T K_b d_i^2                 (SE, 161-188)
//                     sum T K_b/(1+sqrt(3 r~2)) d_i^2 (Matern32, kernel_Matern 340-377;
//                     r~2 uses the gradient-indexed weights wg)
// One 64x64 lower tile per workgroup; T stays in registers (16 pairs per
// lane) while the b loop runs outermost with PM+1 running sums.  The per-b
// block reduction goes through LDS in [value][thread] order (conflict-free,
// two levels) instead of 6-step cross-lane shuffles per value.
// ---------------------------------------------------------------------------
// Column-side operands (x_c, z_c, weight rows) are wave-uniform: they are
// read through the constant address space so they land in SGPRs via scalar
// loads instead of 64-lane vector loads of one address.
typedef const __attribute__((address_space(4))) double *cdp;

// Matern32: the gradient-indexed weights of slice b are the kernel weights of
// slice b+1 (wg[b] == wk[b+1] bit for bit, both exp(-theta[2+B+b+B i]) --
// SURVEY Q1), so r~2_b = r2_{b+1}.  The b loop runs downwards and keeps
// r2_{b+1} per pair in registers: one weighted dot product per (pair, b)
// instead of two; only the last slice uses its own wg row.
template <int PM, int KIND, bool CUBE>
__global__ __launch_bounds__(256) void k_grad(PairSide S, int B, int ZS, TabView tab,
                                              const double *__restrict__ A, int64_t ld,
                                              double sA, const double *__restrict__ alpha,
                                              const double *__restrict__ cube,
                                              double *__restrict__ gpart, int64_t ldg,
                                              const Tile *__restrict__ tiles, int G) {
  constexpr int NV = PM + 1;
  constexpr int NM = AT / 4;
  __shared__ double red[NV][64];
  __shared__ double red2[NV][4];
  __shared__ double sT[NM][256];                        // T of each lane's pairs
  __shared__ double sR[(KIND == 1 && !CUBE) ? NM : 1][256];  // r2_{b+1} per pair
  const int64_t t = blockIdx.x;
  int64_t I, J;
  if (tiles) {  // sharded: the rank's own lower tiles
    const Tile tt = tiles[t];
    I = tt.I;
    J = tt.J;
    A += (lcol(J * AT, G) - J * AT) * ld;
  } else {
    I = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    while (I * (I + 1) / 2 > t) --I;
    J = t - I * (I + 1) / 2;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t n = S.n;
  const int64_t r = I * AT + lane;
  const bool rvalid = r < n;
  const int64_t rr = rvalid ? r : 0;
  const int64_t c0 = J * AT + wv;  // columns c0 + 4m (rows of X exist up to a multiple of 64)
  cdp Xc = (cdp)S.X;
  cdp Zc = (cdp)S.Z;
  cdp LZc = (cdp)S.LZ;
  cdp WK = (cdp)tab.wk;
  cdp WG = (cdp)tab.wg;
  cdp LAM = (cdp)tab.lam;

  double xr[PM];
#pragma unroll
  for (int i = 0; i < PM; ++i) xr[i] = S.X[rr * PM + i];
  const double ar = rvalid ? alpha[rr] : 0.0;

  unsigned valid = 0;
  double tr = 0.0;
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int64_t c = c0 + 4 * m;
    const bool v = rvalid && c < n && !(I == J && c > r);
    double tv = 0.0;
    if (v) {
      tv = sA * A[r + c * ld] - ar * alpha[c];
      if (c == r) tr += tv;
      else tv *= 2.0;
      valid |= 1u << m;
    }
    sT[m][tid] = tv;  // each lane only ever reads its own column of sT / sR
  }

  for (int b = B - 1; b >= 0; --b) {
    double g[PM];
#pragma unroll
    for (int i = 0; i < PM; ++i) g[i] = 0.0;
    double gl = 0.0;
    cdp wk = WK + b * PM;
    cdp wg = WG + b * PM;
    const double lam = LAM[b];
    const bool last = (b == B - 1);
    double zr = 0.0, lzr = 0.0;
    if (b > 0) {
      zr = S.Z[rr * ZS + b - 1];
      if (KIND == 0) lzr = S.LZ[rr * ZS + b - 1];
    }
#pragma unroll 1
    for (int m = 0; m < NM; ++m) {
      const int64_t c = c0 + 4 * m;
      double d2[PM];
#pragma unroll
      for (int i = 0; i < PM; ++i) {
        const double d = xr[i] - Xc[c * PM + i];
        d2[i] = d * d;
      }
      double kb, rt2 = 0.0;
      if (CUBE) {
        kb = ((valid >> m) & 1u) ? cube[r + c * n + (int64_t)b * n * n] : 0.0;
        if (KIND == 1) {
#pragma unroll
          for (int i = 0; i < PM; ++i) rt2 = fma(d2[i], wg[i], rt2);
        }
      } else {
        double r2 = 0.0;
#pragma unroll
        for (int i = 0; i < PM; ++i) r2 = fma(d2[i], wk[i], r2);
        double zc = 0.0, lzc = 0.0;
        if (b > 0) {
          zc = Zc[c * ZS + b - 1];
          if (KIND == 0) lzc = LZc[c * ZS + b - 1];
        }
        kb = (r < c) ? kval<KIND, false>(b, r2, lam, zr, zc, lzr, lzc)
                     : kval<KIND, false>(b, r2, lam, zc, zr, lzc, lzr);
        if (KIND == 1) {
          if (last) {
#pragma unroll
            for (int i = 0; i < PM; ++i) rt2 = fma(d2[i], wg[i], rt2);
          } else {
            rt2 = sR[m][tid];
          }
          sR[m][tid] = r2;
        }
      }
      const double tm = sT[m][tid];
      gl = fma(tm, kb, gl);
      double U;
      if (KIND == 0) U = tm * kb;
      else U = tm * (kb / (1.0 + sqrt(3.0 * rt2)));
#pragma unroll
      for (int i = 0; i < PM; ++i) g[i] = fma(U, d2[i], g[i]);
    }
    // block reduction: two xor-shuffle steps fold each wave to 16 lanes, the
    // 64 survivors go to LDS in [value][slot] order, 4 x 16 -> 4 -> 1
#pragma unroll
    for (int i = 0; i < PM; ++i) {
      double v = g[i];
      v += __shfl_xor(v, 32, 64);
      v += __shfl_xor(v, 16, 64);
      if (lane < 16) red[i][wv * 16 + lane] = v;
    }
    {
      double v = gl;
      v += __shfl_xor(v, 32, 64);
      v += __shfl_xor(v, 16, 64);
      if (lane < 16) red[PM][wv * 16 + lane] = v;
    }
    __syncthreads();
    if (tid < NV * 4) {
      const int i = tid % NV, sg = tid / NV;
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 16; ++k) s += red[i][16 * sg + k];
      red2[i][sg] = s;
    }
    __syncthreads();
    if (tid < NV) {
      const double s = (red2[tid][0] + red2[tid][1]) + (red2[tid][2] + red2[tid][3]);
      gpart[t * ldg + (int64_t)b * NV + tid] = s;
    }
  }
  // trace of T (diagonal pairs)
  {
    double v = tr;
    v += __shfl_xor(v, 32, 64);
    v += __shfl_xor(v, 16, 64);
    if (lane < 16) red[0][wv * 16 + lane] = v;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int k = 0; k < 64; ++k) s += red[0][k];
    gpart[t * ldg + (int64_t)B * NV] = s;
  }
}

// ---------------------------------------------------------------------------
// Fused gradient (no cube): slices are taken two at a time so each pair's
// d_i^2 is formed once per two slices, and for Matern32 the factor
// 1 + sqrt(3 r~2_b) is the (1 + sqrt3 t) already formed by slice b+1's kernel
// value (wg[b] == wk[b+1], see above), cached per pair in LDS across passes.
// Per (pair, slice): p FMAs for r2, one sqrt + exp (+ one reciprocal for
// Matern), p FMAs into the running sums.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double rcp_nr(double f) {
  double q = __builtin_amdgcn_rcp(f);
  double e = fma(-f, q, 1.0);
  q = fma(q, e, q);
  e = fma(-f, q, 1.0);
  return fma(q, e, q);
}

// kernel value of slice b plus (Matern) its factor 1 + sqrt3 * sqrt(r2)
template <int KIND>
__device__ __forceinline__ double kval_f(int b, double r2, double lam, double zlo, double zhi,
                                         double lzlo, double lzhi, double &f) {
  if (KIND == 0) {
    f = 1.0;
    return kval<0, false>(b, r2, lam, zlo, zhi, lzlo, lzhi);
  } else {
    const double t = sqrt(r2);
    f = 1.0 + SQRT3 * t;
    const double e = f * exp(lam - SQRT3 * t);
    if (b == 0) return e;
    if (zlo == 0.0) return 0.0;
    return (e * zlo) * zhi;
  }
}

template <int PM>
__device__ __forceinline__ void grad_block_reduce(const double (&g)[PM], double gl,
                                                  double (*red)[64], double (*red2)[4],
                                                  int tid, int lane, int wv,
                                                  double *__restrict__ out, int64_t stride) {
  constexpr int NV = PM + 1;
#pragma unroll
  for (int i = 0; i < PM; ++i) {
    double v = g[i];
    v += __shfl_xor(v, 32, 64);
    v += __shfl_xor(v, 16, 64);
    if (lane < 16) red[i][wv * 16 + lane] = v;
  }
  {
    double v = gl;
    v += __shfl_xor(v, 32, 64);
    v += __shfl_xor(v, 16, 64);
    if (lane < 16) red[PM][wv * 16 + lane] = v;
  }
  __syncthreads();
  if (tid < NV * 4) {
    const int i = tid % NV, sg = tid / NV;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[i][16 * sg + k];
    red2[i][sg] = s;
  }
  __syncthreads();
  if (tid < NV) out[tid * stride] = (red2[tid][0] + red2[tid][1]) + (red2[tid][2] + red2[tid][3]);
}

template <int PM, int KIND>
__global__ __launch_bounds__(256) void k_grad2(PairSide S, int B, int ZS, TabView tab,
                                               const double *__restrict__ A, int64_t ld,
                                               double sA, const double *__restrict__ alpha,
                                               double *__restrict__ gpart, int64_t ldg,
                                               const Tile *__restrict__ tiles, int G) {
  constexpr int NV = PM + 1;
  constexpr int NM = AT / 4;
  __shared__ double red[NV][64];
  __shared__ double red2[NV][4];
  __shared__ double sT[NM][256];                      // T of each lane's pairs
  __shared__ double sF[KIND == 1 ? NM : 1][256];      // Matern: 1 + sqrt3 t of slice b+1
  const int64_t t = blockIdx.x;
  int64_t I, J;
  if (tiles) {  // sharded: the rank's own lower tiles
    const Tile tt = tiles[t];
    I = tt.I;
    J = tt.J;
    A += (lcol(J * AT, G) - J * AT) * ld;
  } else {
    I = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    while (I * (I + 1) / 2 > t) --I;
    J = t - I * (I + 1) / 2;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t n = S.n;
  const int64_t r = I * AT + lane;
  const bool rvalid = r < n;
  const int64_t rr = rvalid ? r : 0;
  const int64_t c0 = J * AT + wv;
  cdp Xc = (cdp)S.X;
  cdp Zc = (cdp)S.Z;
  cdp LZc = (cdp)S.LZ;
  cdp WK = (cdp)tab.wk;
  cdp WG = (cdp)tab.wg;
  cdp LAM = (cdp)tab.lam;

  double xr[PM];
#pragma unroll
  for (int i = 0; i < PM; ++i) xr[i] = S.X[rr * PM + i];
  const double ar = rvalid ? alpha[rr] : 0.0;

  double tr = 0.0;
#pragma unroll
  for (int m = 0; m < NM; ++m) {
    const int64_t c = c0 + 4 * m;
    const bool v = rvalid && c < n && !(I == J && c > r);
    double tv = 0.0;
    if (v) {
      tv = sA * A[r + c * ld] - ar * alpha[c];
      if (c == r) tr += tv;
      else tv *= 2.0;
    }
    sT[m][tid] = tv;  // each lane only reads back its own column of sT / sF
  }

  for (int b1 = B - 1; b1 >= 0; b1 -= 2) {
    const int b0 = b1 - 1;  // may be -1 (odd B): second slice skipped
    const bool two = b0 >= 0;
    double g1[PM], g0[PM];
#pragma unroll
    for (int i = 0; i < PM; ++i) g1[i] = g0[i] = 0.0;
    double gl1 = 0.0, gl0 = 0.0;
    cdp wk1 = WK + b1 * PM;
    cdp wk0 = WK + (two ? b0 : b1) * PM;
    cdp wgl = WG + b1 * PM;  // used only when b1 == B-1 (its r~2 has its own row)
    const double lam1 = LAM[b1], lam0 = LAM[two ? b0 : b1];
    const bool last = (b1 == B - 1);
    double zr1 = 0.0, lzr1 = 0.0, zr0 = 0.0, lzr0 = 0.0;
    if (b1 > 0) {
      zr1 = S.Z[rr * ZS + b1 - 1];
      if (KIND == 0) lzr1 = S.LZ[rr * ZS + b1 - 1];
    }
    if (b0 > 0) {
      zr0 = S.Z[rr * ZS + b0 - 1];
      if (KIND == 0) lzr0 = S.LZ[rr * ZS + b0 - 1];
    }
#pragma unroll 1
    for (int m = 0; m < NM; ++m) {
      const int64_t c = c0 + 4 * m;
      const bool rlo = r < c;
      double d2[PM];
#pragma unroll
      for (int i = 0; i < PM; ++i) {
        const double d = xr[i] - Xc[c * PM + i];
        d2[i] = d * d;
      }
      const double tm = sT[m][tid];
      // slice b1
      double U1, f1;
      {
        double r2 = 0.0;
#pragma unroll
        for (int i = 0; i < PM; ++i) r2 = fma(d2[i], wk1[i], r2);
        double zc = 0.0, lzc = 0.0;
        if (b1 > 0) {
          zc = Zc[c * ZS + b1 - 1];
          if (KIND == 0) lzc = LZc[c * ZS + b1 - 1];
        }
        const double kb = rlo ? kval_f<KIND>(b1, r2, lam1, zr1, zc, lzr1, lzc, f1)
                              : kval_f<KIND>(b1, r2, lam1, zc, zr1, lzc, lzr1, f1);
        gl1 = fma(tm, kb, gl1);
        if (KIND == 0) {
          U1 = tm * kb;
        } else {
          double fn;
          if (last) {
            double rt2 = 0.0;
#pragma unroll
            for (int i = 0; i < PM; ++i) rt2 = fma(d2[i], wgl[i], rt2);
            fn = 1.0 + sqrt(3.0 * rt2);
          } else {
            fn = sF[m][tid];
          }
          U1 = (tm * kb) * rcp_nr(fn);
        }
      }
#pragma unroll
      for (int i = 0; i < PM; ++i) g1[i] = fma(U1, d2[i], g1[i]);
      if (two) {
        double r2 = 0.0;
#pragma unroll
        for (int i = 0; i < PM; ++i) r2 = fma(d2[i], wk0[i], r2);
        double zc = 0.0, lzc = 0.0;
        if (b0 > 0) {
          zc = Zc[c * ZS + b0 - 1];
          if (KIND == 0) lzc = LZc[c * ZS + b0 - 1];
        }
        double f0;
        const double kb = rlo ? kval_f<KIND>(b0, r2, lam0, zr0, zc, lzr0, lzc, f0)
                              : kval_f<KIND>(b0, r2, lam0, zc, zr0, lzc, lzr0, f0);
        gl0 = fma(tm, kb, gl0);
        double U0;
        if (KIND == 0) {
          U0 = tm * kb;
        } else {
          U0 = (tm * kb) * rcp_nr(f1);
          sF[m][tid] = f0;
        }
#pragma unroll
        for (int i = 0; i < PM; ++i) g0[i] = fma(U0, d2[i], g0[i]);
      }
    }
    grad_block_reduce<PM>(g1, gl1, red, red2, tid, lane, wv, gpart + t * ldg + (int64_t)b1 * NV,
                          1);
    if (two)
      grad_block_reduce<PM>(g0, gl0, red, red2, tid, lane, wv, gpart + t * ldg + (int64_t)b0 * NV,
                            1);
  }
  // trace of T (diagonal pairs)
  {
    double v = tr;
    v += __shfl_xor(v, 32, 64);
    v += __shfl_xor(v, 16, 64);
    __syncthreads();
    if (lane < 16) red[0][wv * 16 + lane] = v;
  }
  __syncthreads();
  if (tid == 0) {
    double s = 0.0;
    for (int k = 0; k < 64; ++k) s += red[0][k];
    gpart[t * ldg + (int64_t)B * NV] = s;
  }
}

// ---------------------------------------------------------------------------
// Diagonal of a symmetric kernel matrix over slices [b0, b1): r2 = 0 on the
// diagonal, so K_b(r, r) is the reference expression at r2 = 0 with both z
// operands z_r (kernmat_*_symmetric_cpp's r == c entries; prediction needs
// only diag(K_xx), src/pred_cpp.cpp:22-28, 71-77).
// ---------------------------------------------------------------------------
template <int KIND>
__global__ void k_kdiag(PairSide S, int ZS, TabView tab, int b0, int b1, double *__restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= S.n) return;
  double s = 0.0;
  for (int b = b0; b < b1; ++b) {
    double z = 0.0, lz = 0.0;
    if (b > 0) {
      z = S.Z[r * ZS + b - 1];
      if (KIND == 0) lz = S.LZ[r * ZS + b - 1];
    }
    s += kval<KIND, false>(b, 0.0, tab.lam[b], z, z, lz, lz);
  }
  out[r] = s;
}

hipError_t launch_kdiag(int kind, PairSide S, int ZS, TabView tab, int b0, int b1, double *out,
                        hipStream_t st) {
  if (S.n <= 0) return hipSuccess;
  const dim3 grid((unsigned)((S.n + 255) / 256));
  if (kind == 0) hipLaunchKernelGGL(k_kdiag<0>, grid, dim3(256), 0, st, S, ZS, tab, b0, b1, out);
  else hipLaunchKernelGGL(k_kdiag<1>, grid, dim3(256), 0, st, S, ZS, tab, b0, b1, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Dispatch over the compiled feature-count buckets.
// ---------------------------------------------------------------------------
static const int kBuckets[] = {4, 8, 12, 16, 20, 24, 32, 48, 64};

int pm_bucket(int p) {
  for (int b : kBuckets)
    if (p <= b) return b;
  return -1;
}

int64_t grad_ntiles(int64_t n) {
  const int64_t nt = (n + AT - 1) / AT;
  return nt * (nt + 1) / 2;
}

template <int PM>
static hipError_t asm_pm(int mode, int kind, PairSide R, PairSide C, int64_t npad, int B,
                         int ZS, TabView tab, double sig, double *out, int64_t ld,
                         double *cube, hipStream_t st, const Tile *tiles, int64_t ntiles, int G,
                         int b0, int b1) {
  dim3 blk(256);
  dim3 grid;
  if (mode == 0 && tiles) {
    if (ntiles == 0) return hipSuccess;
    grid = dim3((unsigned)ntiles);
  } else if (mode == 0) {
    const unsigned nt = (unsigned)(npad / AT);
    grid = dim3(nt, nt);
  } else if (mode == 1) {
    const unsigned nt = (unsigned)((R.n + AT - 1) / AT);
    grid = dim3(nt, nt);
  } else {
    grid = dim3((unsigned)((C.n + AT - 1) / AT), (unsigned)((R.n + AT - 1) / AT));
  }
#define ACE_ASM(K, M) \
  hipLaunchKernelGGL((k_assembly<PM, K, M>), grid, blk, 0, st, R, C, npad, B, ZS, tab, sig, out, ld, \
                     cube, tiles, G, b0, b1)
  if (kind == 0) {
    if (mode == 0) ACE_ASM(0, 0);
    else if (mode == 1) ACE_ASM(0, 1);
    else ACE_ASM(0, 2);
  } else {
    if (mode == 0) ACE_ASM(1, 0);
    else if (mode == 1) ACE_ASM(1, 1);
    else ACE_ASM(1, 2);
  }
#undef ACE_ASM
  return hipGetLastError();
}

// Fused-model pair kernels: the MFMA-expansion kernels (ace_pairs_mm.hip)
// for the assembly at every bucket and for the gradient from PM = 32 up; the
// MFMA-expansion kernels (ace_pairs_mm.hip) for fused-model assembly and the
// cube-less gradient at every PM; the all-VALU kernels remain for the ABI
// modes (cube outputs) and when the per-tile staging does not fit in LDS
// (profiles/r01_pairs_ab.txt: C2 p=20 gradient MFMA 7.45 ms vs VALU 9.1 ms,
// assembly 3.4 vs 3.96 ms; C4 p=50 gradient 372 vs 1534 ms).  ACE_PAIRS=valu
// forces the VALU family (diagnostic A/B switch).
bool pairs_use_mm(int PM, bool grad) {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_PAIRS");
    v = !e ? 2 : (e[0] == 'm' ? 1 : (e[0] == 'v' ? 0 : 2));
  }
  (void)grad;
  return v != 0;
}

hipError_t launch_assembly(int mode, int kind, int PM, PairSide R, PairSide C, int64_t npad,
                           int B, int ZS, TabView tab, double sig, double *out, int64_t ld,
                           double *cube, hipStream_t st, const Tile *tiles, int64_t ntiles,
                           int G, int part, int b0, int b1) {
  if (b1 < 0) b1 = B;
  if (mode == 0 && pairs_use_mm(PM, false) && mm_lds_ok(PM, B, kind, false))
    return launch_assembly_mm(kind, PM, R, npad, B, ZS, tab, sig, out, ld, cube, st, tiles,
                              ntiles, G, part);
  if (mode == 2 && !cube && !tiles && pairs_use_mm(PM, false) && cross_mm_lds_ok(PM, B, kind))
    return launch_cross_mm(kind, PM, R, C, B, ZS, tab, b0, b1, out, ld, st);
  if (part == 2) return hipSuccess;  // the all-VALU path assembles everything in part 1
  switch (PM) {
#define ACE_CASE(P) \
  case P:           \
    return asm_pm<P>(mode, kind, R, C, npad, B, ZS, tab, sig, out, ld, cube, st, tiles, ntiles, G, \
                     b0, b1);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

template <int PM>
static hipError_t grad_pm(int kind, PairSide S, int B, int ZS, TabView tab, const double *A,
                          int64_t ld, double sA, const double *alpha, const double *cube,
                          double *gpart, hipStream_t st, const Tile *tiles, int64_t ntiles,
                          int G) {
  const int64_t nsuper = tiles ? ntiles : grad_ntiles(S.n);
  if (nsuper == 0) return hipSuccess;
  const int64_t ldg = grad_part_cols(PM, B);
  dim3 grid((unsigned)nsuper), blk(256);
#define ACE_G(K, CB)                                                                          \
  hipLaunchKernelGGL((k_grad<PM, K, CB>), grid, blk, 0, st, S, B, ZS, tab, A, ld, sA, alpha, \
                     cube, gpart, ldg, tiles, G)
  const bool cb = cube != nullptr;
  if (cb) {
    if (kind == 0) ACE_G(0, true);
    else ACE_G(1, true);
  } else if (kind == 0) {
    hipLaunchKernelGGL((k_grad2<PM, 0>), grid, blk, 0, st, S, B, ZS, tab, A, ld, sA, alpha,
                       gpart, ldg, tiles, G);
  } else {
    hipLaunchKernelGGL((k_grad2<PM, 1>), grid, blk, 0, st, S, B, ZS, tab, A, ld, sA, alpha,
                       gpart, ldg, tiles, G);
  }
#undef ACE_G
  return hipGetLastError();
}

int grad_order_block() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_GRAD_ORDER");
    // 4: gradient HBM reads 1.52 -> 1.21 GB per C2 evaluation against the
    // 1.07 GB lower triangle (the per-tile X / Z staging stays in each XCD's
    // L2), time-neutral (profiles/r02_grad_ab.txt)
    v = e ? std::max(0, atoi(e)) : 4;
  }
  return v;
}

hipError_t launch_grad(int kind, int PM, PairSide S, int B, int ZS, TabView tab,
                       const double *A, int64_t ld, double sA, const double *alpha,
                       const double *cube, double *gpart, hipStream_t st,
                       const Tile *tiles, int64_t ntiles, int G, int64_t ndiag) {
  // The all-VALU gradient kernels keep per-lane p-long arrays and static LDS
  // that outgrow the 64 KB default at PM = 64: above PM = 48 the MFMA kernel
  // always runs, and it recomputes K_b instead of reading a given cube (the
  // cube is kernmat's K_b for the same theta, so the traces are the same).
  const bool valu_ok = PM <= 48;
  if ((!cube || !valu_ok) && (pairs_use_mm(PM, true) || !valu_ok) && mm_lds_ok(PM, B, kind, true))
    return launch_grad_mm(kind, PM, S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles, ntiles,
                          G, ndiag);
  if (!valu_ok) return hipErrorInvalidValue;
  switch (PM) {
#define ACE_CASE(P) \
  case P:           \
    return grad_pm<P>(kind, S, B, ZS, tab, A, ld, sA, alpha, cube, gpart, st, tiles, ntiles, G);
    // no PM = 64 instantiation: the all-VALU gradient's per-lane arrays and
    // static LDS outgrow their budget there (it returned wrong traces); the
    // MFMA kernel above serves every PM > 48
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ace
