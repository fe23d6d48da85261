// ace_sweep.hip -- in-place SPD inversion + log-determinant for gfx950.
//
// The reference inverts A = K + e^sigma I by a symmetric eigendecomposition
// (src/kernel_SE_cpp.cpp:137-157).  Here A is inverted by the blocked
// Gauss-Jordan sweep for SPD matrices (Quintana-Orti, Quintana-Orti, Sun,
// van de Geijn, "A note on parallel matrix inversion", SIAM J. Sci. Comput.
// 22(5), 2001): the same n^3 flops as Cholesky + SPD inverse, but every step
// is one blocked right-looking Cholesky step whose SYRK/GEMM update is
// extended over the already-eliminated rows, so each update launch covers
// the whole (lower) matrix instead of a shrinking trailing block.
//
// Step k (panel = block column k, NB = 256 wide):
//   gather   : P = A[:, k] (symmetric access of the lower storage); W = P
//   4 x sub  : pivot  - eliminate the 64x64 diagonal sub-block in LDS
//                       (scalar sweeps; its pivots are the Cholesky diagonal
//                       squared -> log det), 1 workgroup
//              panel  - apply that elimination to the n x 256 panel W
//   update   : A_ij -= W_i P_j^T on every lower 128x128 tile outside block k
//              (v_mfma_f64_16x16x4_f64, acc initialised from A), and the
//              tiles of block k receive W (the swept panel)
// After the last step the K block of A holds -A^-1.  The AUG rows appended
// below A (y and 1) are swept along: they end holding (A^-1 y)^T, (A^-1 1)^T
// and the corner -[y 1]^T A^-1 [y 1], which give alpha, mu_solution and
// y.alpha with no extra pass over the inverse.
#include "ace_internal.h"

namespace ace {

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- gather
__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ A, int64_t ld,
                                                int64_t k0, double *__restrict__ P,
                                                double *__restrict__ W, int64_t ldp) {
  __shared__ double tile[64][65];
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  const int j0 = blockIdx.y * 64;
  const int64_t col0 = k0 + j0;
  const int tid = threadIdx.x;
  const bool all_lower = i0 >= col0 + 63;
  const bool all_upper = i0 + 63 < col0;
  if (all_lower) {
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const double v = A[(i0 + a) + (col0 + b) * ld];
      P[(i0 + a) + (int64_t)(j0 + b) * ldp] = -v;
      W[(i0 + a) + (int64_t)(j0 + b) * ldp] = v;
    }
  } else if (all_upper) {
    for (int e = tid; e < 4096; e += 256) {
      const int b = e & 63, a = e >> 6;
      tile[a][b] = A[(col0 + b) + (i0 + a) * ld];
    }
    __syncthreads();
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const double v = tile[a][b];
      P[(i0 + a) + (int64_t)(j0 + b) * ldp] = -v;
      W[(i0 + a) + (int64_t)(j0 + b) * ldp] = v;
    }
  } else {
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const int64_t i = i0 + a, c = col0 + b;
      const double v = (i >= c) ? A[i + c * ld] : A[c + i * ld];
      P[i + (int64_t)(j0 + b) * ldp] = -v;
      W[i + (int64_t)(j0 + b) * ldp] = v;
    }
  }
}

// ---------------------------------------------------------------- pivot
// Sweeps the 64x64 sub-block s of the panel's pivot rows in LDS:
//   d = D_tt; D_ij -= D_it D_tj / d; D_it /= d; D_tj /= d; D_tt = -1/d
// -> SW = -D_s^-1.  Also snapshots the 64 pivot rows (all NB columns) into S
// before the panel kernel overwrites them.  Records every pivot d.
__global__ __launch_bounds__(256) void k_pivot(const double *__restrict__ W, int64_t ldp,
                                               int64_t k0, int s, double *__restrict__ SW,
                                               double *__restrict__ S, double *__restrict__ piv,
                                               int *__restrict__ flag) {
  __shared__ double D[SUB][SUB + 1];
  const int64_t p0 = k0 + (int64_t)s * SUB;
  const int tid = threadIdx.x;
  for (int e = tid; e < SUB * SUB; e += 256) {
    const int a = e & 63, b = e >> 6;
    D[a][b] = W[(p0 + a) + (int64_t)(s * SUB + b) * ldp];
  }
  for (int e = tid; e < SUB * NB; e += 256) {
    const int a = e & 63, j = e >> 6;
    S[a + j * SUB] = W[(p0 + a) + (int64_t)j * ldp];
  }
  __syncthreads();
  const int i = tid & 63, jb = tid >> 6;
  for (int t = 0; t < SUB; ++t) {
    const double d = D[t][t];
    const double rd = 1.0 / d;
    const double dit = D[i][t];
    double v[SUB / 4];
#pragma unroll
    for (int q = 0; q < SUB / 4; ++q) {
      const int j = jb + 4 * q;
      const double dtj = D[t][j];
      const double dij = D[i][j];
      double x;
      if (i == t) x = (j == t) ? -rd : dtj * rd;
      else if (j == t) x = dit * rd;
      else x = fma(-(dit * dtj), rd, dij);
      v[q] = x;
    }
    if (tid == 0) {
      piv[p0 + t] = d;
      if (!(d > 0.0) || !isfinite(d)) *flag = 1;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SUB / 4; ++q) D[i][jb + 4 * q] = v[q];
    __syncthreads();
  }
  for (int e = tid; e < SUB * SUB; e += 256) {
    const int a = e & 63, b = e >> 6;
    SW[a + b * SUB] = D[a][b];
  }
}

// ---------------------------------------------------------------- panel
// Applies sub-pivot s to 64 rows of the panel W (Naug x NB):
//   other rows : V = -W[:, s] SW (= W_is D_s^-1); W[:, s] = V;
//                W[:, j] -= V S[:, j]            (j outside s)
//   pivot rows : V = SW;  W[:, s] = SW;  W[:, j] = -SW S[:, j] (= D_s^-1 S)
__global__ __launch_bounds__(256) void k_panel(double *__restrict__ W, int64_t ldp, int64_t k0,
                                               int s, const double *__restrict__ SW,
                                               const double *__restrict__ S) {
  __shared__ double sSW[SUB][SUB + 1];
  __shared__ double sV[SUB][SUB + 1];
  __shared__ double sX[SUB][SUB + 1];
  const int64_t i0 = (int64_t)blockIdx.x * SUB;
  const bool pivrows = (i0 == k0 + (int64_t)s * SUB);
  const int tid = threadIdx.x;
  const int ra = tid & 15, cb = tid >> 4;  // rows ra+16q, cols cb+16q
  for (int e = tid; e < SUB * SUB; e += 256) {
    const int a = e & 63, b = e >> 6;
    sSW[a][b] = SW[a + b * SUB];
    if (!pivrows) sX[a][b] = W[(i0 + a) + (int64_t)(s * SUB + b) * ldp];
  }
  __syncthreads();
  double acc[4][4];
  if (pivrows) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) acc[q][qq] = sSW[ra + 16 * q][cb + 16 * qq];
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) acc[q][qq] = 0.0;
    for (int t = 0; t < SUB; ++t) {
      double xa[4], sb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) xa[q] = sX[ra + 16 * q][t];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sb[qq] = sSW[t][cb + 16 * qq];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) acc[q][qq] = fma(-xa[q], sb[qq], acc[q][qq]);
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      sV[ra + 16 * q][cb + 16 * qq] = acc[q][qq];
      W[(i0 + ra + 16 * q) + (int64_t)(s * SUB + cb + 16 * qq) * ldp] = acc[q][qq];
    }
  __syncthreads();
  for (int cc = 0; cc < NB / SUB; ++cc) {
    if (cc == s) continue;
    for (int e = tid; e < SUB * SUB; e += 256) {
      const int a = e & 63, b = e >> 6;
      sX[a][b] = S[a + (int64_t)(cc * SUB + b) * SUB];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        acc[q][qq] = pivrows ? 0.0
                             : W[(i0 + ra + 16 * q) + (int64_t)(cc * SUB + cb + 16 * qq) * ldp];
    for (int t = 0; t < SUB; ++t) {
      double va[4], sb[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) va[q] = sV[ra + 16 * q][t];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) sb[qq] = sX[t][cb + 16 * qq];
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) acc[q][qq] = fma(-va[q], sb[qq], acc[q][qq]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        W[(i0 + ra + 16 * q) + (int64_t)(cc * SUB + cb + 16 * qq) * ldp] = acc[q][qq];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- update
// One 128x128 lower tile (I, J) of A.  Tiles outside block k:
//   A_IJ += Pn_J-rows x W_I-rows^T over the NB panel columns  (Pn = -P)
// computed as D = Pn W^T + C with the MFMA's D[row=c][col=r] so that the
// 16 lanes of a fragment walk consecutive rows of the column-major A.
// Tiles of block k receive the swept panel W (transposed for the row block).
constexpr int BK = 16;      // panel columns staged per LDS buffer
constexpr int LDL = 144;    // LDS row pitch (doubles): 128 + 16, bank-conflict free
constexpr int NCH = NB / BK;

__global__ __launch_bounds__(256, 2) void k_update(double *__restrict__ A, int64_t ld,
                                                   const double *__restrict__ W,
                                                   const double *__restrict__ Pn, int64_t ldp,
                                                   int64_t k0) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  const int J = blockIdx.x, I = blockIdx.y;
  if (J > I) return;
  const int kt0 = (int)(k0 / UT), kt1 = kt0 + NB / UT;
  const bool Ik = I >= kt0 && I < kt1, Jk = J >= kt0 && J < kt1;
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int tid = threadIdx.x;

  if (Ik || Jk) {
    if (Ik && !Jk) {
      // row block k, columns left of it: A[k0+a, c] = W[c, a]
      double *tileT = &sW[0][0][0];  // 64 x 65 scratch
      for (int sa = 0; sa < 2; ++sa)
        for (int sb = 0; sb < 2; ++sb) {
          __syncthreads();
          for (int e = tid; e < 4096; e += 256) {
            const int c = e & 63, a = e >> 6;
            tileT[a * 65 + c] = W[(C0 + 64 * sb + c) + (R0 - k0 + 64 * sa + a) * ldp];
          }
          __syncthreads();
          for (int e = tid; e < 4096; e += 256) {
            const int a = e & 63, c = e >> 6;
            A[(R0 + 64 * sa + a) + (C0 + 64 * sb + c) * ld] = tileT[a * 65 + c];
          }
        }
    } else {
      // column block k (and the diagonal block): A[r, k0+j] = W[r, j]
      for (int e = tid; e < UT * UT; e += 256) {
        const int a = e & (UT - 1), c = e >> 7;
        A[(R0 + a) + (C0 + c) * ld] = W[(R0 + a) + (C0 - k0 + c) * ldp];
      }
    }
    return;
  }

  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[4][4];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 64 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = A[r + (c + 4 * j) * ld];
    }

  const int sk = tid >> 4, sm = (tid & 15) * 8;
  const double *gW = W + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = Pn + (C0 + sm) + (int64_t)sk * ldp;
  double2 rw[4], rp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    rw[e] = *reinterpret_cast<const double2 *>(gW + 2 * e);
    rp[e] = *reinterpret_cast<const double2 *>(gP + 2 * e);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    *reinterpret_cast<double2 *>(&sW[0][sk][sm + 2 * e]) = rw[e];
    *reinterpret_cast<double2 *>(&sP[0][sk][sm + 2 * e]) = rp[e];
  }
  __syncthreads();

  for (int ch = 0; ch < NCH; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCH) {
      const int64_t off = (int64_t)(ch + 1) * BK * ldp;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        rw[e] = *reinterpret_cast<const double2 *>(gW + off + 2 * e);
        rp[e] = *reinterpret_cast<const double2 *>(gP + off + 2 * e);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[4], b[4];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) a[ci] = sP[cur][4 * kk + lk][64 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) b[ri] = sW[cur][4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 4; ++ci)
#pragma unroll
        for (int ri = 0; ri < 4; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    if (ch + 1 < NCH) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + 2 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + 2 * e]) = rp[e];
      }
    }
    __syncthreads();
  }

#pragma unroll
  for (int ci = 0; ci < 4; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 64 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) A[r + (c + 4 * j) * ld] = acc[ci][ri][j];
    }
}

double sweep_update_flops(int64_t naug) {
  // lower tiles outside the pivot block, 2*UT*UT*NB flops each, summed over steps
  const int64_t nT = naug / UT;
  const int64_t steps = (naug - AUG) / NB;
  const int64_t kt = NB / UT;
  const int64_t tiles_total = nT * (nT + 1) / 2;
  // tiles touching block k: kt rows x (column tiles) ... count exactly per step
  double flops = 0.0;
  for (int64_t k = 0; k < steps; ++k) {
    const int64_t kt0 = k * kt, kt1 = kt0 + kt;
    int64_t touching = 0;
    for (int64_t I = 0; I < nT; ++I) {
      const bool Ik = I >= kt0 && I < kt1;
      if (Ik) touching += I + 1;  // J = 0..I
      else if (I >= kt1) touching += kt;  // J in block k
    }
    flops += (double)(tiles_total - touching) * 2.0 * UT * UT * NB;
  }
  return flops;
}

hipError_t run_sweep(const SweepBufs &b, hipStream_t st, hipEvent_t *ev, int nev,
                     int *nev_used) {
  const int64_t naug = b.ld;
  const unsigned nT = (unsigned)(naug / UT);
  int used = 0;
  for (int64_t k0 = 0; k0 < b.npad; k0 += NB) {
    hipLaunchKernelGGL(k_gather, dim3((unsigned)(naug / 64), NB / 64), dim3(256), 0, st, b.A,
                       b.ld, k0, b.P, b.W, b.ld);
    for (int s = 0; s < NB / SUB; ++s) {
      hipLaunchKernelGGL(k_pivot, dim3(1), dim3(256), 0, st, b.W, b.ld, k0, s, b.SW, b.S,
                         b.piv, b.flag);
      hipLaunchKernelGGL(k_panel, dim3((unsigned)(naug / SUB)), dim3(256), 0, st, b.W, b.ld,
                         k0, s, b.SW, b.S);
    }
    if (ev && used + 2 <= nev) (void)hipEventRecord(ev[used], st);
    hipLaunchKernelGGL(k_update, dim3(nT, nT), dim3(256), 0, st, b.A, b.ld, b.W, b.P, b.ld,
                       k0);
    if (ev && used + 2 <= nev) {
      (void)hipEventRecord(ev[used + 1], st);
      used += 2;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (nev_used) *nev_used = used;
  return hipSuccess;
}

}  // namespace ace
