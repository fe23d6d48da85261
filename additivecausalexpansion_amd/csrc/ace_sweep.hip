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

#include <functional>
#include <map>

#include "ace_wgtime.h"

namespace ace {

typedef double d4 __attribute__((ext_vector_type(4)));

// The lookahead chain kernels (k_pivot, k_panel: one to four workgroups of
// latency-bound work) share CUs with the MFMA-heavy update tiles of the main
// stream.  Raising their waves' issue priority lets them win the SIMD
// arbitration instead of getting a 1/5 share of the issue slots.
// (Priority 3 on them and on the head-path gather k_update_q: C1 -0.06 ms
// on one box, +0.01 on another, C2 +0.15 ms -- not kept,
// profiles/r05_v19_ab_prio.txt.)
#define CHAIN_PRIO() __builtin_amdgcn_s_setprio(1)

// ---------------------------------------------------------------- pivot
// Sweeps the 64x64 sub-block s of the panel's pivot rows:
//   d = D_tt; D_ij -= D_it D_tj / d; D_it /= d; D_tj /= d; D_tt = -1/d
// -> SW = -D_s^-1 (exactly symmetric: every product is formed as a*b with
// a = D_it = D_ti).  Layout: lane = row i, wave w of NW keeps columns
// CW w .. CW w + CW - 1 (CW = 64 / NW) in registers; per pivot the owning
// wave publishes column t and lane t of every wave publishes its part of
// row t through double-buffered LDS vectors, so there is one barrier per
// pivot.  More waves = fewer dependent VALU operations per wave per pivot
// (the chain's critical path); the arithmetic per element is the same for
// every NW.  D_s is read from the pivot-row snapshot S (written by k_gather
// / the previous panel update); every pivot d (Cholesky diagonal squared)
// is recorded.
template <int NW>
struct PivotLds {
  __attribute__((aligned(16))) double colb[2][SUB];
  __attribute__((aligned(16))) double rowb[2][SUB];
  double pv[SUB];
};

// the sub-sweep itself: v = this lane's row, columns CW w .. CW w + CW - 1
template <int NW>
__device__ __forceinline__ void pivot_sweep(double (&v)[SUB / NW], PivotLds<NW> &L, int tid) {
  constexpr int CW = SUB / NW;
  static_assert(CW % 2 == 0, "double2 row publishing");
  const int lane = tid & 63, w = tid >> 6;
  // no global memory traffic inside the loop: every __syncthreads() is then
  // a bare s_barrier (a pending global store would add a vmcnt(0) wait)
#pragma unroll 1
  for (int tw = 0; tw < NW; ++tw) {
#pragma unroll
    for (int tq = 0; tq < CW; ++tq) {
      const int t = CW * tw + tq;
      const int buf = tq & 1;
      if (w == tw) L.colb[buf][lane] = v[tq];
      if (lane == t) {
#pragma unroll
        for (int q = 0; q < CW; q += 2)
          *reinterpret_cast<double2 *>(&L.rowb[buf][CW * w + q]) = double2{v[q], v[q + 1]};
      }
      __syncthreads();
      const double d = L.rowb[buf][t];
      // 1/d by v_rcp_f64 + two Newton steps (<= 1 ulp): five dependent fp64
      // operations on the chain's critical path instead of the eleven of
      // the IEEE division sequence
      double rd = __builtin_amdgcn_rcp(d);
      double re = fma(-d, rd, 1.0);
      rd = fma(rd, re, rd);
      re = fma(-d, rd, 1.0);
      rd = fma(rd, re, rd);
      const double dit = L.colb[buf][lane];
      double rt[CW];
#pragma unroll
      for (int q = 0; q < CW; q += 2) {
        const double2 x = *reinterpret_cast<const double2 *>(&L.rowb[buf][CW * w + q]);
        rt[q] = x.x;
        rt[q + 1] = x.y;
      }
#pragma unroll
      for (int q = 0; q < CW; ++q) {
        const int j = CW * w + q;
        const double dtj = rt[q];
        double x;
        if (lane == t) x = (j == t) ? -rd : dtj * rd;
        else if (j == t) x = dit * rd;
        else x = fma(-(dit * dtj), rd, v[q]);
        v[q] = x;
      }
      if (tid == 0) L.pv[t] = d;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------- blocked pivot
// The same 64x64 sweep as pivot_sweep<4> (same register layout in and out,
// pivots into pv[]), blocked by 16 (ACE_PIVOT_BLK=1, default): the sweep
// operator composes, so sweeping pivots 0..63 one by one equals four block
// sweeps of the 16x16 diagonal blocks, each
//   M_ss <- S = -D^-1 (D = M_ss),  M_sc <- D^-1 M_sc = -S M_sc,
//   M_rc <- M_rc - M_rs D^-1 M_sc = M_rc + M_rs (S M_sc)   (r, c != s).
// The 16 scalar pivots of M_ss run in ONE wave with no barrier and no LDS:
// lane (r, g) = (lane & 15, lane >> 4) holds M(r, 4g .. 4g+3); pivot t's
// row comes by a 64-bit DPP row_newbcast:t (lane t of every 16-lane row
// holds row t's part of that row's columns) and its column by a
// permlane16/32 swap pair that replicates row t/4 (the lanes holding
// column t) into all four rows.  Every wave sweeps M_ss redundantly, so S
// is in every wave's registers as the MFMA A operand (the k index of a
// 16x16x4 step permuted to 4g + e, which needs no data movement); wave w !=
// s then forms Un = S M_sw (4 MFMAs), writes M_sw = -Un (and its mirror
// M_ws), and for c >= w, c != s updates M_cw += M_cs Un (4 MFMAs each, k
// permuted to g + 4e so that Un's accumulator layout is the B operand as it
// stands) and mirrors it: every off-diagonal block is formed once and
// mirrored, every diagonal block from its lower triangle, so M stays exactly
// symmetric as the scalar sweep keeps it.  Per 16 pivots ~35 VALU + 4
// permlane + 5 DPP instructions per wave instead of 16 barriers and 64
// columns of updates per row: the latency of the pivot chain's 64x64 sweep
// (k_pivot 35 us alone, 93 us under the bulk update) is what this cuts.
// M: the 64x64 matrix in LDS (pitch P, even, 16-B aligned rows).
#ifndef ACE_PIVOT_BLK
#define ACE_PIVOT_BLK 1
#endif
#ifndef ACE_BULK_RESERVE_N
#define ACE_BULK_RESERVE_N 8192
#endif
#ifndef ACE_PGEMM_HEADQ
#define ACE_PGEMM_HEADQ 1
#endif

// broadcast lane T of every 16-lane row to the row (64-bit DPP)
template <int T>
__device__ __forceinline__ double row_bcast(double x) {
  long v = __builtin_bit_cast(long, x);
  // bound_ctrl set with full masks: every lane is written from a valid source
  // lane, so the old value is dead and needs no zero-initialising move
  long b = __builtin_amdgcn_update_dpp((long)0, v, 0x150 + T, 0xf, 0xf, true);  // v_mov_b64_dpp
  return __builtin_bit_cast(double, b);
}

// replicate 16-lane row G of x into all four rows, on the LDS crossbar: two
// ds_bpermute (no LDS memory) instead of four v_permlane16/32_swap and the
// operand copies they need (x stays live) -- the pivot sweep's column fetch,
// C1 3.74 -> 3.65 ms (profiles/r05_v13_ab_pivot.txt)
template <int G>
__device__ __forceinline__ double rep_row_bp(double x, int lane) {
  const int addr = ((lane & 15) | (G << 4)) << 2;
  const unsigned long v = __builtin_bit_cast(unsigned long, x);
  const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(addr, (int)(unsigned)(v >> 32));
  return __builtin_bit_cast(double, ((unsigned long)hi << 32) | lo);
}

// one scalar pivot t of the 16x16 block in the one-wave layout (see above);
// the pivot d goes to pv[T] from one lane (rec: wave 0).  Measured variants
// (C1, profiles/r05_v12_ab_c1.txt, r05_v13_ab_pivot.txt; all bit-identical):
// column t+1 fetched before the update (its replication off the pivot chain)
// with permlanes, +5 instructions per pivot: +0.07 ms; with ds_bpermute: as
// this form; one FMA per element for the pivot row and the rest (row t with
// c' = -1, x' = 0; 33 instead of 39 instructions per pivot): as this form.
template <int T>
__device__ __forceinline__ void blk_pivot(double (&x)[4], int r, int g, double &dk) {
  constexpr int TG = T >> 2, TE = T & 3;
  const double c = rep_row_bp<TG>(x[TE], r | (g << 4));  // M(r, t)
  double rw[4];                          // M(t, 4g + e)
#pragma unroll
  for (int e = 0; e < 4; ++e) rw[e] = row_bcast<T>(x[e]);
  const double d = row_bcast<T>(c);      // M(t, t)
  double rd = __builtin_amdgcn_rcp(d);  // + two Newton steps, as in pivot_sweep
  double re = fma(-d, rd, 1.0);
  rd = fma(rd, re, rd);
  re = fma(-d, rd, 1.0);
  rd = fma(rd, re, rd);
  // branch-free (selects): row t gets M(t, j) / d, column t M(i, t) / d,
  // the pivot -1/d, the rest M(i, j) - M(i, t) M(t, j) / d
  const bool isrow = r == T;
  const double cd = c * rd;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bool jt = (4 * g + e) == T;  // lane-uniform per row: g is the row index
    const double vn = fma(-(c * rw[e]), rd, x[e]);
    const double vr = rw[e] * rd;
    x[e] = jt ? (isrow ? -rd : cd) : (isrow ? vr : vn);
  }
  dk = r == T ? d : dk;  // lane r keeps pivot r's value (stored once per block)
}

template <int P>
__device__ __forceinline__ double2 lds_ld2(const double *p) {
  if constexpr (P % 2 == 0) return *reinterpret_cast<const double2 *>(p);
  else return double2{p[0], p[1]};
}
template <int P>
__device__ __forceinline__ void lds_st2(double *p, double a, double b) {
  if constexpr (P % 2 == 0) *reinterpret_cast<double2 *>(p) = double2{a, b};
  else { p[0] = a; p[1] = b; }
}

template <int P>
__device__ __forceinline__ void pivot_sweep_blk(double (&v)[SUB / 4], double (*M)[P], double *pv,
                                                int tid) {
  const int lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, g = lane >> 4;
#pragma unroll
  for (int q = 0; q < SUB / 4; q += 2)
    lds_st2<P>(&M[lane][16 * w + q], v[q], v[q + 1]);
  __syncthreads();
#pragma unroll 1
  for (int s = 0; s < 4; ++s) {
    const int s0 = 16 * s;
    double x[4];
    {
      const double2 a = lds_ld2<P>(&M[s0 + r][s0 + 4 * g]);
      const double2 b = lds_ld2<P>(&M[s0 + r][s0 + 4 * g + 2]);
      x[0] = a.x; x[1] = a.y; x[2] = b.x; x[3] = b.y;
    }
    {
      double dk = 0.0;
#define BP(T) blk_pivot<T>(x, r, g, dk)
      BP(0);  BP(1);  BP(2);  BP(3);  BP(4);  BP(5);  BP(6);  BP(7);
      BP(8);  BP(9);  BP(10); BP(11); BP(12); BP(13); BP(14); BP(15);
#undef BP
      if (w == 0 && g == 0) pv[s0 + r] = dk;  // read after the barriers below
    }
    // this sub-step's block update, computed from the old values before the
    // barrier (reads), stored after it (writes of blocks other waves read)
    const bool upd = w != s;
    d4 un = d4{0.0, 0.0, 0.0, 0.0};  // Un(g + 4jj, r) = (S M_sw)(g + 4jj, r)
    d4 res[4];                        // M_cw(g + 4jj, r) + (M_cs Un)(g + 4jj, r)
    if (upd) {
      {
        // B operand: M_sw(4g + e, r) = M_ws(r, 4g + e)
        const double2 a = lds_ld2<P>(&M[16 * w + r][s0 + 4 * g]);
        const double2 b = lds_ld2<P>(&M[16 * w + r][s0 + 4 * g + 2]);
        un = __builtin_amdgcn_mfma_f64_16x16x4f64(x[0], a.x, un, 0, 0, 0);
        un = __builtin_amdgcn_mfma_f64_16x16x4f64(x[1], a.y, un, 0, 0, 0);
        un = __builtin_amdgcn_mfma_f64_16x16x4f64(x[2], b.x, un, 0, 0, 0);
        un = __builtin_amdgcn_mfma_f64_16x16x4f64(x[3], b.y, un, 0, 0, 0);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < w || c == s) continue;
        d4 acc;
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = M[16 * c + g + 4 * e][16 * w + r];  // C: M_cw
#pragma unroll
        for (int e = 0; e < 4; ++e)  // A: M_cs(r, g + 4e); B: Un's layout as it stands
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(M[16 * c + r][s0 + g + 4 * e], un[e], acc, 0,
                                                     0, 0);
        res[c] = acc;
      }
    }
    __syncthreads();
    if (!upd) {  // the sweeping block itself: S
      lds_st2<P>(&M[s0 + r][s0 + 4 * g], x[0], x[1]);
      lds_st2<P>(&M[s0 + r][s0 + 4 * g + 2], x[2], x[3]);
    } else {
      // M_sw = -Un and its mirror M_ws
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        M[s0 + g + 4 * jj][16 * w + r] = -un[jj];
        M[16 * w + r][s0 + g + 4 * jj] = -un[jj];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c < w || c == s) continue;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int a = g + 4 * jj;  // res[c][jj] = M_cw(a, r)
          if (c != w || a >= r) {
            M[16 * c + a][16 * w + r] = res[c][jj];
            M[16 * w + r][16 * c + a] = res[c][jj];
          }
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < SUB / 4; q += 2) {
    const double2 a = lds_ld2<P>(&M[lane][16 * w + q]);
    v[q] = a.x;
    v[q + 1] = a.y;
  }
}

// pivots (and the non-PD flag) and SW = -D^-1 out
template <int NW>
__device__ __forceinline__ void pivot_store(const double (&v)[SUB / NW], const double *pv,
                                            int tid, double *__restrict__ SW,
                                            double *__restrict__ piv, int64_t p0,
                                            int *__restrict__ flag) {
  constexpr int CW = SUB / NW;
  const int lane = tid & 63, w = tid >> 6;
  if (tid < SUB) {
    const double d = pv[tid];
    piv[p0 + tid] = d;
    if (!(d > 0.0) || !isfinite(d)) *flag = 1;
  }
#pragma unroll
  for (int q = 0; q < CW; ++q) SW[lane + (CW * w + q) * SUB] = v[q];
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void k_pivot(const double *__restrict__ S, int s,
                                                   double *__restrict__ SW,
                                                   double *__restrict__ piv, int64_t p0,
                                                   int *__restrict__ flag) {
  ACE_WGT(1, true);
  CHAIN_PRIO();
  constexpr int CW = SUB / NW;
  __shared__ PivotLds<NW> L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double v[CW];
#pragma unroll
  for (int q = 0; q < CW; ++q) v[q] = S[lane + (s * SUB + CW * w + q) * SUB];
  ACE_WGT_MARK(0);
  if constexpr (ACE_PIVOT_BLK && NW == 4) {
    __shared__ double M[SUB][SUB + 2];
    pivot_sweep_blk<SUB + 2>(v, M, L.pv, tid);
  } else {
    pivot_sweep<NW>(v, L, tid);
  }
  ACE_WGT_MARK(1);
  pivot_store<NW>(v, L.pv, tid, SW, piv, p0, flag);
}

static void launch_pivot(const double *S, int s, double *SW, double *piv, int64_t p0, int *flag,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_pivot<4>, dim3(1), dim3(256), 0, st, S, s, SW, piv, p0, flag);
}

// ---------------------------------------------------------------- gather
// P = -A[:, k] for every row; W = A[:, k] only on the pivot rows (k_panel
// sweeps them; k_panel_gemm forms every other row of W from P).
__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ A, int64_t ld,
                                                int64_t k0, double *__restrict__ P,
                                                double *__restrict__ W, int64_t ldp,
                                                double *__restrict__ S0) {
  __shared__ double tile[64][65];
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  const int j0 = blockIdx.y * 64;
  const int64_t col0 = k0 + j0;
  const int tid = threadIdx.x;
  const bool all_lower = i0 >= col0 + 63;
  const bool all_upper = i0 + 63 < col0;
  const bool piv = i0 >= k0 && i0 < k0 + NB;  // pivot rows: W needed
  if (all_lower) {
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const double v = A[(i0 + a) + (col0 + b) * ld];
      P[(i0 + a) + (int64_t)(j0 + b) * ldp] = -v;
      if (piv) W[(i0 + a) + (int64_t)(j0 + b) * ldp] = v;
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
      if (piv) W[(i0 + a) + (int64_t)(j0 + b) * ldp] = v;
    }
  } else {
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const int64_t i = i0 + a, c = col0 + b;
      const double v = (i >= c) ? A[i + c * ld] : A[c + i * ld];
      P[i + (int64_t)(j0 + b) * ldp] = -v;
      if (piv) W[i + (int64_t)(j0 + b) * ldp] = v;
    }
  }
  if (i0 == k0) {  // pivot rows of sub-block 0: snapshot for k_pivot / k_panel
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      S0[a + (int64_t)(j0 + b) * SUB] = W[(i0 + a) + (int64_t)(j0 + b) * ldp];
    }
  }
}

// ---------------------------------------------------------------- panel
// Applies sub-pivot s to 64 rows of the panel W (Naug x NB), on MFMA:
//   other rows : V = -W[:, s] SW (= W_is D_s^-1); W[:, s] = V;
//                W[:, j] -= V S[:, j]            (j outside s)
//   pivot rows : V = SW;  W[:, s] = SW;  W[:, j] = -SW S[:, j] (= D_s^-1 S)
// Wave w owns rows 16w..16w+15.  Phase 1 forms Vn^T = -V^T = SW W_is^T
// (SW is symmetric) so that its accumulator fragments are directly the B
// operands of phase 2's D = S_chunk^T Vn^T + W_chunk^T (no LDS round trip).
// LDS pitch for sSW: 64 + 16 doubles, conflict-free fragment reads
// (ACE_PLD=72: the split kernel's LDS fits 72 KB, the hole one finished
// bulk-update workgroup leaves -- A/B switch)
#ifndef ACE_PLD
#define ACE_PLD 80
#endif
constexpr int PLD = ACE_PLD;
constexpr int SLD = 66;  // LDS pitch for the transposed S chunk (c-major)

__global__ __launch_bounds__(256) void k_panel(double *__restrict__ W, int64_t ldp, int64_t k0,
                                               int s, const double *__restrict__ SW,
                                               const double *__restrict__ S,
                                               double *__restrict__ Snext, int64_t row0) {
  CHAIN_PRIO();
  __shared__ double sSW[SUB][PLD];  // sSW[b][a] = SW(a, b)
  __shared__ double sSt[SUB][SLD];  // sSt[c][t] = S(t, 64 cc + c)
  const int64_t i0 = row0 + (int64_t)blockIdx.x * SUB;
  const bool pivrows = (i0 == k0 + (int64_t)s * SUB);
  const bool nextrows = (s + 1 < NB / SUB) && (i0 == k0 + (int64_t)(s + 1) * SUB);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  for (int e = tid; e < SUB * SUB; e += 256) {
    const int a = e & 63, b = e >> 6;
    sSW[b][a] = SW[a + b * SUB];
  }
  __syncthreads();
  const int64_t row = i0 + 16 * w + lr;
  const int srow = 16 * w + lr;  // row within the block (for Snext)
  d4 acc1[4];
  if (pivrows) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc1[ct][j] = -sSW[16 * ct + lk + 4 * j][16 * w + lr];
  } else {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc1[ct] = d4{0.0, 0.0, 0.0, 0.0};
    double bw[SUB / 4];  // all 16 B fragments in flight at once
#pragma unroll
    for (int kk = 0; kk < SUB / 4; ++kk) bw[kk] = W[row + (int64_t)(s * SUB + 4 * kk + lk) * ldp];
#pragma unroll
    for (int kk = 0; kk < SUB / 4; ++kk) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc1[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(sSW[4 * kk + lk][16 * ct + lr], bw[kk],
                                                        acc1[ct], 0, 0, 0);
    }
  }
  // acc1[ct][j] = Vn[i = row][t' = 16 ct + lk + 4 j];  W[:, s] = V = -Vn
#pragma unroll
  for (int ct = 0; ct < 4; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = s * SUB + 16 * ct + lk + 4 * j;
      W[row + (int64_t)col * ldp] = -acc1[ct][j];
      if (nextrows) Snext[srow + col * SUB] = -acc1[ct][j];
    }
  for (int cc = 0; cc < NB / SUB; ++cc) {
    if (cc == s) continue;
    // issue this chunk's accumulator loads before the staging barrier
    d4 accs[4];
#pragma unroll
    for (int ctc = 0; ctc < 4; ++ctc)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        accs[ctc][j] = pivrows ? 0.0 : W[row + (int64_t)(cc * SUB + 16 * ctc + lk + 4 * j) * ldp];
    __syncthreads();
    for (int e = tid; e < SUB * SUB; e += 256) {
      const int t = e & 63, c = e >> 6;
      sSt[c][t] = S[t + (cc * SUB + c) * SUB];
    }
    __syncthreads();
#pragma unroll
    for (int ctc = 0; ctc < 4; ++ctc) {
      d4 acc = accs[ctc];
#pragma unroll
      for (int kk = 0; kk < SUB / 4; ++kk)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sSt[16 * ctc + lr][4 * kk + lk],
                                                   acc1[kk >> 2][kk & 3], acc, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = cc * SUB + 16 * ctc + lk + 4 * j;
        W[row + (int64_t)col * ldp] = acc[j];
        if (nextrows) Snext[srow + col * SUB] = acc[j];
      }
    }
  }
}

// ---------------------------------------------------------------- split panel
// k_panel's arithmetic with the column chunks spread over workgroups:
// workgroup (g, cc) updates rows g (64) of the pivot block in chunk cc (64
// columns) only -- (NB/SUB)^2 small workgroups instead of NB/SUB that each
// walk every chunk.  Under the bulk update a chain workgroup runs on a CU it
// shares with an update workgroup, so the chain's latency is its
// per-workgroup work (profiles/r02_chain_ab.txt).  Phase 1 (Vn for the
// rows) is recomputed by each workgroup of the row group, so its input
// W[:, s] must not change during sub-step s:
//   * sub-step s >= 1 reads it from X[s & 1], the copy of chunk s that the
//     chunk-s workgroups of sub-step s-1 wrote beside W;
//   * sub-step 0 reads W[:, 0] (the gathered panel) and writes its chunk 0
//     (V) to V0 instead of W; sub-step 1 takes chunk 0's accumulator there.
// X[0], X[1] and V0 are NB x SUB (row within the pivot block, column within
// the chunk) after SW[0], SW[1] in the SW buffer.  The workgroup holding the
// next diagonal block D_{s+1} (g = cc = s + 1) then runs the k_pivot
// sub-sweep of sub-step s+1 on it (into SWn = the other SW buffer), which
// saves one launch -- and its wait for a free CU slot under the bulk update
// -- per sub-step.  Every element sees k_panel's / k_pivot's operations in
// their order: bit-identical.
template <class Mark>
__device__ __forceinline__ void panel_split_step(
    double *__restrict__ W, int64_t ldp, int64_t k0, int s, const double *__restrict__ SW,
    const double *__restrict__ S, double *__restrict__ Snext, double *__restrict__ Xb,
    double *__restrict__ SWn, double *__restrict__ piv, int *__restrict__ flag,
    double (&sSW)[SUB][PLD], double (&sSt)[SUB][SLD], PivotLds<4> &PL, int g, int cc,
    const Mark &mark) {
  // sSW[b][a] = SW(a, b); sSt[c][t] = S(t, 64 cc + c)
  constexpr int NS = NB / SUB;
  constexpr int64_t CH = (int64_t)NB * SUB;  // one chunk buffer
  double *const V0 = Xb + 2 * CH;
  const bool pivrows = g == s;
  const bool nextrows = s + 1 < NS && g == s + 1;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int srow = 16 * w + lr;     // row within the row group (and Snext)
  const int brow = g * SUB + srow;  // row within the pivot block
  const int64_t row = k0 + brow;
  d4 accs[4];
  if (cc != s && !pivrows) {
    const bool fromv = s == 1 && cc == 0;
    const double *src = fromv ? V0 + brow : W + row + (int64_t)(cc * SUB) * ldp;
    const int64_t lds = fromv ? NB : ldp;
#pragma unroll
    for (int ctc = 0; ctc < 4; ++ctc)
#pragma unroll
      for (int j = 0; j < 4; ++j) accs[ctc][j] = src[(int64_t)(16 * ctc + lk + 4 * j) * lds];
  } else {
#pragma unroll
    for (int ctc = 0; ctc < 4; ++ctc) accs[ctc] = d4{0.0, 0.0, 0.0, 0.0};
  }
  // Every global load of the prologue is issued before the first LDS store:
  // the inputs are the previous chain launch's outputs, so this is one
  // memory round trip instead of one per staging-loop turn (C1 marks: 9.2 us
  // from entry to the staged operands, profiles/r05_v3_wgt_c1.txt)
  double bw[SUB / 4];
  if (!pivrows) {
    const double *src = s == 0 ? W + row : Xb + (int64_t)(s & 1) * CH + brow;
    const int64_t lds = s == 0 ? ldp : NB;
#pragma unroll
    for (int kk = 0; kk < SUB / 4; ++kk) bw[kk] = src[(int64_t)(4 * kk + lk) * lds];
  }
  {
    constexpr int NQ = SUB * SUB / 512;  // double2 per thread and matrix
    double2 tw[NQ], ts[NQ];
    const double *Sc = S + (int64_t)cc * SUB * SUB;  // S(a, 64 cc + b) = Sc[a + 64 b]
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = 2 * (tid + 256 * q);
      tw[q] = *reinterpret_cast<const double2 *>(SW + e);
      if (cc != s) ts[q] = *reinterpret_cast<const double2 *>(Sc + e);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = 2 * (tid + 256 * q), a = e & 63, b = e >> 6;
      sSW[b][a] = tw[q].x;
      sSW[b][a + 1] = tw[q].y;
      if (cc != s) {
        sSt[b][a] = ts[q].x;
        sSt[b][a + 1] = ts[q].y;
      }
    }
  }
  __syncthreads();
  mark(0);
  d4 acc1[4];
  if (pivrows) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc1[ct][j] = -sSW[16 * ct + lk + 4 * j][16 * w + lr];
  } else {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc1[ct] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < SUB / 4; ++kk) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc1[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(sSW[4 * kk + lk][16 * ct + lr], bw[kk],
                                                        acc1[ct], 0, 0, 0);
    }
  }
  if (cc == s) {
    // acc1[ct][j] = Vn[row][16 ct + lk + 4 j]; chunk s = V = -Vn
    double *dst = s == 0 ? V0 + brow : W + row + (int64_t)(s * SUB) * ldp;
    const int64_t ldd = s == 0 ? NB : ldp;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 16 * ct + lk + 4 * j;
        dst[(int64_t)c * ldd] = -acc1[ct][j];
        if (nextrows) Snext[srow + (s * SUB + c) * SUB] = -acc1[ct][j];
      }
    return;
  }
  // chunk s+1 is the next sub-step's phase-1 input: copy it to X[(s+1) & 1]
  double *const xnext = cc == s + 1 ? Xb + (int64_t)((s + 1) & 1) * CH + brow : nullptr;
  const bool fusepiv = nextrows && cc == s + 1;  // this workgroup holds D_{s+1}
#pragma unroll
  for (int ctc = 0; ctc < 4; ++ctc) {
    d4 &acc = accs[ctc];
#pragma unroll
    for (int kk = 0; kk < SUB / 4; ++kk)
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sSt[16 * ctc + lr][4 * kk + lk],
                                                 acc1[kk >> 2][kk & 3], acc, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * ctc + lk + 4 * j;
      const int col = cc * SUB + c;
      W[row + (int64_t)col * ldp] = acc[j];
      if (nextrows) Snext[srow + col * SUB] = acc[j];
      if (xnext) xnext[(int64_t)c * NB] = acc[j];
    }
  }
  mark(1);
  if (!fusepiv) return;
  // D_{s+1}: accs[ctc][j] = D(srow, 16 ctc + lk + 4 j) -> lane = row layout
  __syncthreads();  // every wave is done with sSW (phase 1)
#pragma unroll
  for (int ctc = 0; ctc < 4; ++ctc)
#pragma unroll
    for (int j = 0; j < 4; ++j) sSW[16 * ctc + lk + 4 * j][srow] = accs[ctc][j];
  __syncthreads();
  double v[SUB / 4];
#pragma unroll
  for (int q = 0; q < SUB / 4; ++q) v[q] = sSW[16 * w + q][lane];
#if ACE_PIVOT_BLK
  mark(2);
  pivot_sweep_blk<SLD>(v, sSt, PL.pv, tid);  // sSt is free (the update phase is done)
#else
  mark(2);
  pivot_sweep<4>(v, PL, tid);
#endif
  mark(3);
  pivot_store<4>(v, PL.pv, tid, SWn, piv, k0 + (int64_t)(s + 1) * SUB, flag);
}


__global__ __launch_bounds__(256) void k_panel_split(double *__restrict__ W, int64_t ldp,
                                                     int64_t k0, int s,
                                                     const double *__restrict__ SW,
                                                     const double *__restrict__ S,
                                                     double *__restrict__ Snext,
                                                     double *__restrict__ Xb,
                                                     double *__restrict__ SWn,
                                                     double *__restrict__ piv,
                                                     int *__restrict__ flag) {
  ACE_WGT(2, true);
  CHAIN_PRIO();
  __shared__ double sSW[SUB][PLD];
  __shared__ double sSt[SUB][SLD];
  __shared__ PivotLds<4> PL;
  auto mark = [&](int i) { (void)i; ACE_WGT_MARK(i); };
  panel_split_step(W, ldp, k0, s, SW, S, Snext, Xb, SWn, piv, flag, sSW, sSt, PL, (int)blockIdx.x,
                   (int)blockIdx.y, mark);
}

// The four sub-steps of the split panel sweep in ONE launch (ACE_CHAIN_FUSE,
// small n): the same 16 workgroups run sub-step s = 0 .. 3, each the
// workgroup (g, cc) of k_panel_split's grid, with a grid barrier between the
// sub-steps instead of a launch boundary -- every workgroup keeps its CU slot
// across the chain, and the next sub-step's workgroups do not wait for a
// dispatch.  Every workgroup does exactly k_panel_split's work in the same
// order: bit-identical.  The barrier: each workgroup drains its stores,
// releases them at agent scope (they cross the XCDs' L2s) and adds 1 to
// ctr[0]; sub-step s + 1 starts when ctr[0] reaches 16 (s + 1) and the
// workgroup has acquired.  The 16 workgroups need not be resident at once
// to make progress: a waiting one only spins (s_sleep) while the others are
// dispatched as other launches' workgroups leave.  Bounded: a wait over 0.5 s
// sets *flag = 2 (read like a non-positive pivot: the evaluation reports NaN)
// and goes on, so every wave reaches the exit.  ctr[0] (barrier) and ctr[1]
// (exits) start at zero: the last workgroup out resets both for the next
// sweep's launch on this panel slot (by then every other workgroup has
// passed every barrier).
__device__ __forceinline__ void chain_barrier(int *ctr, int target, int *flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > 50000000ull) {  // 100 MHz counter: 0.5 s
        __hip_atomic_store(flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ __launch_bounds__(256, 2) void k_panel_split4(double *__restrict__ W, int64_t ldp,
                                                      int64_t k0, double *__restrict__ SW,
                                                      double *__restrict__ S0,
                                                      double *__restrict__ S1,
                                                      double *__restrict__ piv,
                                                      int *__restrict__ flag, int *ctr) {
  ACE_WGT(2, true);
  CHAIN_PRIO();
  __shared__ double sSW[SUB][PLD];
  __shared__ double sSt[SUB][SLD];
  __shared__ PivotLds<4> PL;
  auto mark = [&](int i) { (void)i; ACE_WGT_MARK(i); };
  static_assert(NB / SUB == 4, "four sub-steps");
  double *const Xb = SW + 2 * SUB * SUB, *const SW1 = SW + SUB * SUB;
  const int g = (int)blockIdx.x, cc = (int)blockIdx.y;
  const int nwg = (int)(gridDim.x * gridDim.y);
  // each sub-step inlined with its s a constant (ping-pong buffers as
  // panel_chain's launches): every copy keeps k_panel_split's registers,
  // where one loop over a runtime s held 363 (no co-residency beside the
  // bulk update's 128-register waves)
  panel_split_step(W, ldp, k0, 0, SW, S0, S1, Xb, SW1, piv, flag, sSW, sSt, PL, g, cc, mark);
  chain_barrier(ctr, nwg, flag);
  panel_split_step(W, ldp, k0, 1, SW1, S1, S0, Xb, SW, piv, flag, sSW, sSt, PL, g, cc, mark);
  chain_barrier(ctr, 2 * nwg, flag);
  panel_split_step(W, ldp, k0, 2, SW, S0, S1, Xb, SW1, piv, flag, sSW, sSt, PL, g, cc, mark);
  chain_barrier(ctr, 3 * nwg, flag);
  panel_split_step(W, ldp, k0, 3, SW1, S1, S0, Xb, SW, piv, flag, sSW, sSt, PL, g, cc, mark);
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(ctr + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1) {
    __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ctr + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- panel GEMM
// After the four sub-sweeps restricted to the pivot rows, W[k0:k0+NB, :]
// holds W_kk = -D^-1 (symmetric).  Every other row of the panel is then one
// GEMM:  W_i = A_ik D^-1 = Pn_i W_kk  (Pn = -P).  Computed transposed,
// Out^T[c][i] = sum_k W_kk[c][k] Pn[i][k], so that fragment lanes walk
// consecutive rows of W.  64 rows x NB columns per 512-thread workgroup,
// 8 waves = 4 row strips x 2 column halves, 8 MFMA fragments each.
constexpr int GBKP = 8;            // k per LDS stage
constexpr int GLB = NB + 16;       // pitch of the W_kk stage  [k][c]
constexpr int GLA = SUB + 16;      // pitch of the Pn stage    [k][i]

// Sharded model (G > 1): rank r forms W only for the rows it consumes -- the
// rows of its own column blocks (operand of its update tiles) and, on the
// owner of block k, every row >= k0 (written back into column block k).
__global__ __launch_bounds__(512) void k_panel_gemm(double *__restrict__ W,
                                                    const double *__restrict__ Pn, int64_t ldp,
                                                    int64_t k0, int G, int r) {
  __shared__ __attribute__((aligned(16))) double sB[2][GBKP][GLB];
  __shared__ __attribute__((aligned(16))) double sA[2][GBKP][GLA];
  const int64_t i0 = (int64_t)blockIdx.x * SUB;
  if (i0 >= k0 && i0 < k0 + NB) return;  // pivot rows are already final
  if (G > 1 && !owns_col(i0, G, r) && !(owns_col(k0, G, r) && i0 >= k0)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv & 3, wc = wv >> 2;
  const int lr = lane & 15, lk = lane >> 4;
  constexpr int CT = NB / 2 / 16;  // c-tiles per wave
  d4 acc[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) acc[ct] = d4{0.0, 0.0, 0.0, 0.0};
  // staging maps: B: 8 k x NB c  (NB/128 double2 per thread); A: 8 k x 64 i (1 per thread)
  const int bk = tid >> 6, bc = (tid & 63) * (NB / 64);
  const int ak = tid >> 6, ai = tid & 63;
  constexpr int NBQ = NB / 128;  // double2 per thread for the B stage
  double2 rb[NBQ];
  double ra;
  auto load = [&](int kc) {
#pragma unroll
    for (int e = 0; e < NBQ; ++e)
      rb[e] = *reinterpret_cast<const double2 *>(W + (k0 + bc + 2 * e) + (int64_t)(kc + bk) * ldp);
    ra = Pn[(i0 + ai) + (int64_t)(kc + ak) * ldp];
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < NBQ; ++e) *reinterpret_cast<double2 *>(&sB[buf][bk][bc + 2 * e]) = rb[e];
    sA[buf][ak][ai] = ra;
  };
  load(0);
  store(0);
  __syncthreads();
  constexpr int NCHP = NB / GBKP;
  for (int ch = 0; ch < NCHP; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCHP) load((ch + 1) * GBKP);
#pragma unroll
    for (int kk = 0; kk < GBKP / 4; ++kk) {
      const double b = sA[cur][4 * kk + lk][16 * wi + lr];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f64_16x16x4f64(
            sB[cur][4 * kk + lk][(NB / 2) * wc + 16 * ct + lr], b, acc[ct], 0, 0, 0);
    }
    if (ch + 1 < NCHP) store(cur ^ 1);
    __syncthreads();
  }
  const int64_t row = i0 + 16 * wi + lr;
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      W[row + (int64_t)((NB / 2) * wc + 16 * ct + lk + 4 * j) * ldp] = acc[ct][j];
}

// ---------------------------------------------------------------- update
// One 128x128 lower tile (I, J) of A per 512-thread workgroup.  Tiles
// outside block k:  A_IJ += R_I C_J^T over the NB panel columns, computed
// as D = C R^T + acc with the MFMA's D[row=c][col=r] so that the 16 lanes of
// a fragment walk consecutive rows of the column-major A.  The product is
// -P_I D^-1 P_J^T for either operand order: single GPU R = W (swept panel,
// every row) and C = Pn (= -P); sharded R = Pn (every rank holds the whole
// gathered panel) and C = W (formed only for the rank's own column rows).
// 8 waves, each a 64(r) x 32(c) block of 4x2 v_mfma_f64_16x16x4_f64
// fragments: 32 accumulator doubles per lane, so 4 waves fit per SIMD
// (61 TF/s vs 46 TF/s for 4 waves of 64x64 -- the latency of the LDS
// fragment reads is hidden by the other waves, tools/bench_update.hip).
// Tiles of block k receive the swept panel Wk (transposed for the row
// block).  Column tile J is stored at local column lcol(J*UT, G).
#ifndef ACE_BK
#define ACE_BK 16
#endif
constexpr int BK = ACE_BK;  // panel columns staged per LDS buffer
constexpr int LDL = 144;    // LDS row pitch (doubles): 128 + 16, bank-conflict free
constexpr int NCH = NB / BK;
constexpr int UTHREADS = 512;
// Panel staging (the update / panel-GEMM kernels): each thread moves two
// double2 of a BK x width chunk row, the two halves of the row (sm and sm +
// width / 2, sm = 2 (lane % (width / 4))), so each ds_write_b128 lane group
// of 8 covers 128 contiguous bytes -- all 32 write banks -- instead of 8
// lanes 32 bytes apart (2-way conflicts, MI355X_MICROARCH.md LDS table; the
// round-4 change, -0.3 ms per C2 evaluation, bit-identical).
constexpr int SM128 = 2, SH128 = 64;
constexpr int SM64 = 2, SH64 = 32;
static_assert(BK == 16, "staging maps 512 threads x 4 doubles onto a 128 x 16 chunk");

// A tiles are read and written once per sweep step, by whichever XCD runs
// the tile: nontemporal loads and stores leave the XCD L2s to the re-read
// panels (profiles/r01_pairs_ab.txt: plain 85.3, write-through stores 85.0,
// nontemporal stores 84.5, nontemporal loads + stores 84.3 ms/eval).
__device__ __forceinline__ void st_a(double *p, double v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ double ld_a(const double *p) { return __builtin_nontemporal_load(p); }

// Gather fused into a lookahead cross launch (ACE_XGATHER): the cross tiles
// of block kg are exactly the lower tiles holding column block kg of the
// symmetric matrix, so the launch that writes them can also write what
// k_gather would read back from them -- P = -A[:, kg], W = A[:, kg] on the
// pivot rows, the sub-block-0 snapshot S0 -- from the values it stores: the
// same doubles, one chain launch less per panel.  k0 < 0: no gather.
struct GatherOut {
  double *P, *W, *S0;
  int64_t k0, ldp;
  // pack mode (sharded, low != null, G > 1): also write what shard_pack
  // would read back for the exchange of step k0 / NB -- the owner's column
  // block rows >= k0 into low (ld h, the pivot block's upper part mirrored)
  // and the rank's row pieces A[k-block, j-block], j < k, into send (slot =
  // local block index).  P / W / S0 (when set) receive the panel rows the
  // rank owns, so that shard_unpack_chain only fills the rows of other ranks.
  double *low = nullptr, *send = nullptr;
  int64_t h = 0;
  int G = 1;
  // head / tail exchange of the sharded head schedule: low holds only the
  // column rows from k0 + lr0 on (ld h): the head part [k0, hend) with lr0 = 0,
  // the tail part [hend, naug) with lr0 = hend - k0
  int64_t lr0 = 0;
};
static inline GatherOut no_gather() { return GatherOut{nullptr, nullptr, nullptr, -1, 0}; }
static inline GatherOut pack_out(double *low, double *send, double *P, double *W, double *S0,
                                 int64_t k0, int64_t naug, int G) {
  GatherOut g{P, W, S0, k0, naug};
  if (G > 1) {
    g.low = low;
    g.send = send;
  }
  g.h = naug - k0;
  g.G = G;
  return g;
}

// the value v stored at lower position (r, c) of A (r >= c; entries above
// the diagonal of a diagonal tile are not part of the lower storage)
__device__ __forceinline__ void gput(const GatherOut &g, int64_t r, int64_t c, double v) {
  if (r < c) return;
  const int64_t cc = c - g.k0, rr = r - g.k0;
  if (g.low) {  // pack mode (k_pack_lower / k_pack_rows layouts)
    if ((uint64_t)cc < (uint64_t)NB) {  // column block k: rows >= k0 (r >= c >= k0)
      g.low[(rr - g.lr0) + cc * g.h] = v;
      if ((uint64_t)rr < (uint64_t)NB && r != c) g.low[cc + rr * g.h] = v;  // mirror
    } else if ((uint64_t)rr < (uint64_t)NB) {  // row block k, an own column c < k0
      g.send[(lcol(c, g.G) / NB) * NB * NB + rr + (c % NB) * NB] = v;
    }
  }
  if (!g.P) return;
  if ((uint64_t)cc < (uint64_t)NB) {  // column block kg: row r of the panel
    g.P[r + cc * g.ldp] = -v;
    if ((uint64_t)rr < (uint64_t)NB) {
      g.W[r + cc * g.ldp] = v;
      if (rr < SUB) g.S0[rr + cc * SUB] = v;
    }
  }
  if ((uint64_t)rr < (uint64_t)NB && r != c) {  // row block kg: row c of the panel (symmetry)
    g.P[c + rr * g.ldp] = -v;
    if ((uint64_t)cc < (uint64_t)NB) {
      g.W[c + rr * g.ldp] = v;
      if (cc < SUB) g.S0[cc + rr * SUB] = v;
    }
  }
}

// the AUG row block's dead rows (16 .. 127: zero padding, not computed):
// k_gather copies them too.  L0: the local column of C0 (sharded).
__device__ __forceinline__ void gput_aug_dead(const GatherOut &g, const double *A, int64_t ld,
                                              int64_t R0, int64_t C0, int tid, int nthr,
                                              int64_t L0 = -1) {
  const int64_t cc0 = C0 - g.k0;
  if ((uint64_t)cc0 >= (uint64_t)NB) return;
  const int64_t lc0 = L0 >= 0 ? L0 : C0;
  for (int e = tid; e < (UT - 16) * UT; e += nthr) {
    const int a = 16 + e % (UT - 16), c = e / (UT - 16);
    const double v = A[(R0 + a) + (lc0 + c) * ld];
    if (g.low) g.low[(R0 + a - g.k0 - g.lr0) + (cc0 + c) * g.h] = v;
    if (g.P) g.P[(R0 + a) + (cc0 + c) * g.ldp] = -v;
  }
}

// Every lower tile except the "cross" of block kx (tiles with I or J in
// block kx, updated earlier by k_update_x for the lookahead; kx < 0: none).
// tiles == nullptr: all lower tiles, 1-D grid in row-major order; otherwise
// the rank's own tiles from the list.
__global__ __launch_bounds__(UTHREADS, 2) void k_update(double *__restrict__ A, int64_t ld,
                                                        const double *__restrict__ Rop,
                                                        const double *__restrict__ Cop,
                                                        const double *__restrict__ Wk,
                                                        int64_t ldp, int64_t k0, int kx,
                                                        const Tile *__restrict__ tiles, int G,
                                                        GatherOut go) {
  ACE_WGT(6, gridDim.x < 4096 || blockIdx.x % 32 == 0);
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  constexpr int KT = NB / UT;
  int I, J;
  if (tiles) {
    const Tile tt = tiles[blockIdx.x];
    I = tt.I;
    J = tt.J;
    if (I < 0) return;  // padding of the XCD order
  } else {
    const int t = blockIdx.x;
    int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    while (i * (i + 1) / 2 > t) --i;
    I = i;
    J = t - i * (i + 1) / 2;
  }
  if (kx >= 0 && ((I >= kx * KT && I < (kx + 1) * KT) || (J >= kx * KT && J < (kx + 1) * KT)))
    return;
  const int kt0 = (int)(k0 / UT), kt1 = kt0 + KT;
  const bool Ik = I >= kt0 && I < kt1, Jk = J >= kt0 && J < kt1;
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int64_t L0 = lcol(C0, G);
  const int tid = threadIdx.x;

  if (Ik || Jk) {
    if (Ik && !Jk) {
      // row block k, columns left of it: A[k0+a, c] = Wk[c, a]
      double *tileT = &sW[0][0][0];  // 64 x 65 scratch
      for (int sa = 0; sa < 2; ++sa)
        for (int sb = 0; sb < 2; ++sb) {
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int c = e & 63, a = e >> 6;
            tileT[a * 65 + c] = Wk[(C0 + 64 * sb + c) + (R0 - k0 + 64 * sa + a) * ldp];
          }
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int a = e & 63, c = e >> 6;
            const double v = tileT[a * 65 + c];
            A[(R0 + 64 * sa + a) + (L0 + 64 * sb + c) * ld] = v;
            if (go.k0 >= 0) gput(go, R0 + 64 * sa + a, C0 + 64 * sb + c, v);
          }
        }
    } else {
      // column block k (and the diagonal block): A[r, k0+j] = Wk[r, j]
      for (int e = tid; e < UT * UT; e += UTHREADS) {
        const int a = e & (UT - 1), c = e >> 7;
        const double v = Wk[(R0 + a) + (C0 - k0 + c) * ldp];
        A[(R0 + a) + (L0 + c) * ld] = v;
        if (go.k0 >= 0) gput(go, R0 + a, C0 + c, v);
      }
    }
    return;
  }

  const int lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  if (R0 >= ld - AUG) {
    // tile of the AUG row block: only its first 16 rows (y, 1 and zero
    // padding) are live, the rest stay zero.  Wave wv does the 16 x 16 block
    // of columns 16 wv.. straight from the panels (same k order as below, so
    // the same results), 1/8 of a full tile's MFMAs.
    d4 acc;
    const int64_t r = R0 + lr;
    const int64_t c = L0 + 16 * wv + lk;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = ld_a(&A[r + (c + 4 * j) * ld]);
    const double *gr = Rop + R0 + lr + (int64_t)lk * ldp;
    const double *gc = Cop + C0 + 16 * wv + lr + (int64_t)lk * ldp;
    double an = gc[0], bn = gr[0];
    for (int kk = 0; kk < NB / 4; ++kk) {
      const double a = an, bb = bn;
      if (kk + 1 < NB / 4) {
        an = gc[(int64_t)(4 * (kk + 1)) * ldp];
        bn = gr[(int64_t)(4 * (kk + 1)) * ldp];
      }
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st_a(&A[r + (c + 4 * j) * ld], acc[j]);
    if (go.k0 >= 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) gput(go, r, C0 + 16 * wv + lk + 4 * j, acc[j]);
      gput_aug_dead(go, A, ld, R0, C0, tid, UTHREADS, L0);
    }
    return;
  }
  // staging: each thread moves 4 doubles of each operand per chunk (issued
  // before the C tile, so chunk 0 reaches LDS without waiting for C)
  const int sk = tid >> 5, sm = (tid & 31) * SM128;  // 2nd half at sm + SH128
  // scalar panel bases + 32-bit element offsets (as k_update_multi)
  const int roff = (int)((R0 + sm) + (int64_t)sk * ldp), coff = (int)((C0 + sm) + (int64_t)sk * ldp);
  double2 rw[2], rp[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    rw[e] = *reinterpret_cast<const double2 *>(Rop + roff + SH128 * e);
    rp[e] = *reinterpret_cast<const double2 *>(Cop + coff + SH128 * e);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the C-tile loads behind them
  const int wr = wv & 1, wc = wv >> 1;  // rows 64*wr.., cols 32*wc..
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = ld_a(&A[r + (c + 4 * j) * ld]);
    }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    *reinterpret_cast<double2 *>(&sW[0][sk][sm + SH128 * e]) = rw[e];
    *reinterpret_cast<double2 *>(&sP[0][sk][sm + SH128 * e]) = rp[e];
  }
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCH) {
      const int64_t off = (int64_t)(ch + 1) * BK * ldp;
      const double *nw = Rop + off, *np = Cop + off;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        rw[e] = *reinterpret_cast<const double2 *>(nw + roff + SH128 * e);
        rp[e] = *reinterpret_cast<const double2 *>(np + coff + SH128 * e);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[4];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) b[ri] = sW[cur][4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 4; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    if (ch + 1 < NCH) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + SH128 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + SH128 * e]) = rp[e];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) st_a(&A[r + (c + 4 * j) * ld], acc[ci][ri][j]);
    }
  if (go.k0 >= 0) {
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          gput(go, R0 + 64 * wr + 16 * ri + lr, C0 + 32 * wc + 16 * ci + lk + 4 * j, acc[ci][ri][j]);
  }
}

// Panel GEMM on the update kernel's 128 x 128 tiles (ACE_PGEMM_TILES, the
// default): W_I,J = Pn_I W_kk[:, J] for the two 128-column halves J of the
// panel, K = NB.  Same operand roles, k order and zero start as
// k_panel_gemm, so bit-identical to it, but each workgroup runs the bulk
// update's pipelined 8-wave tile: under the bulk update k_panel_gemm's 64-row
// strips held 258 update-sized CU slots for ~185 us per panel (skipping it
// took 6 ms off a C2 evaluation, profiles/r02_chain_ab.txt).
__global__ __launch_bounds__(UTHREADS, 2) void k_panel_gemm_t(double *__restrict__ W,
                                                              const double *__restrict__ Pn,
                                                              int64_t ldp, int64_t k0, int G,
                                                              int r, int rt0 = 0,
                                                              int rs0 = 1 << 30, int rs1 = 1 << 30) {
  ACE_WGT(3, true);
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];  // Pn rows of the tile
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];  // W_kk rows c
  // row tile rt0 + blockIdx.x, skipping row tiles [rs0, rs1) (the head/tail
  // split of run_sweep_heads; default: every row tile)
  int rt = rt0 + (int)blockIdx.x;
  if (rt >= rs0) rt += rs1 - rs0;
  const int64_t R0 = (int64_t)rt * UT, C0 = (int64_t)blockIdx.y * UT;
  if (R0 >= k0 && R0 < k0 + NB) return;  // pivot rows are already final
  if (G > 1 && !owns_col(R0, G, r) && !(owns_col(k0, G, r) && R0 >= k0)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int sk = tid >> 5, sm = (tid & 31) * SM128;  // 2nd half at sm + SH128
  const double *gW = Pn + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = W + (k0 + C0 + sm) + (int64_t)sk * ldp;  // W_kk(c, k) = W[k0 + c, k]
  // One chunk of loads in flight, in 108 VGPRs (two workgroups per CU).  A
  // two-deep pipeline (round 5) needed 132 VGPRs: under a bulk launch of
  // 128-VGPR waves it waited for two of them to leave a SIMD, C2 +4.4 ms
  // (profiles/r05_v3_ab_c2.txt); the head launches use k_panel_gemm_q.
  const int wr = wv & 1, wc = wv >> 1;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) acc[ci][ri] = d4{0.0, 0.0, 0.0, 0.0};
  // the two register sets as named values (arrays passed to helpers ended
  // up in scratch)
  double2 w00, w01, p00, p01;
#define PG_LOAD(W0, W1, P0, P1, CH)                                               \
  do {                                                                            \
    const int64_t off_ = (int64_t)(CH) * BK * ldp;                                \
    W0 = *reinterpret_cast<const double2 *>(gW + off_);                           \
    W1 = *reinterpret_cast<const double2 *>(gW + off_ + SH128);                   \
    P0 = *reinterpret_cast<const double2 *>(gP + off_);                           \
    P1 = *reinterpret_cast<const double2 *>(gP + off_ + SH128);                   \
  } while (0)
#define PG_STAGE(W0, W1, P0, P1, BUF)                                             \
  do {                                                                            \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm]) = W0;                          \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm + SH128]) = W1;                  \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm]) = P0;                          \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm + SH128]) = P1;                  \
  } while (0)
  auto mma = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[4];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) b[ri] = sW[cur][4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 4; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
  };
  {
    PG_LOAD(w00, w01, p00, p01, 0);
    PG_STAGE(w00, w01, p00, p01, 0);
    __syncthreads();
    ACE_WGT_MARK(0);
    for (int ch = 0; ch < NCH; ++ch) {
      const int cur = ch & 1;
      if (ch + 1 < NCH) PG_LOAD(w00, w01, p00, p01, ch + 1);
      mma(cur);
      if (ch + 1 < NCH) PG_STAGE(w00, w01, p00, p01, cur ^ 1);
      __syncthreads();
    }
  }
#undef PG_LOAD
#undef PG_STAGE
  ACE_WGT_MARK(1);
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t rr = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) W[rr + (c + 4 * j) * ldp] = acc[ci][ri][j];
    }
}

// Two sweep steps per launch: A_IJ += W_a,I Pn_a,J^T + W_b,I Pn_b,J^T with
// panels a (block [ka0, ka0 + NB)) and b = a + 1 (the next block), K = 2 NB
// per tile -- every accumulator runs the same MFMA chain over the same k
// order as two k_update launches (acc stored / reloaded in fp64 between
// them), so the results are bit-identical, while the C tile is read and
// written once per two steps.  Tiles of block b take W_b (k_update's copy);
// tiles of block a take W_a (what step a left there) and then only panel b's
// product; tiles with I or J in blocks [kx0, kx1) (the lookahead cross,
// updated on the side stream) are skipped.  Sharded (G > 1 or wcol): A's
// columns are block-cyclic (lcol) and the operands swapped (R = Pn, C = W).
__device__ __forceinline__ void update_pair_tile(
    int I, int J, double (&sW)[2][BK][LDL], double (&sP)[2][BK][LDL], double *__restrict__ A,
    int64_t ld, const double *__restrict__ Ra, const double *__restrict__ Ca,
    const double *__restrict__ Rb, const double *__restrict__ Cb, int64_t ldp, int64_t ka0,
    const GatherOut &go, int G, bool wcol) {
  constexpr int KT = NB / UT;
  const int64_t kb0 = ka0 + NB;
  const int ta0 = (int)(ka0 / UT), tb0 = ta0 + KT;
  const bool Ia = I >= ta0 && I < tb0, Ja = J >= ta0 && J < tb0;
  const bool Ib = I >= tb0 && I < tb0 + KT, Jb = J >= tb0 && J < tb0 + KT;
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int64_t L0 = lcol(C0, G);  // A's local column of the tile (sharded: block-cyclic)
  const int tid = threadIdx.x;
  // single GPU: R = W, C = Pn; sharded (wcol): R = Pn, C = W (own columns)
  const double *Wa = wcol ? Ca : Ra, *Wb = wcol ? Cb : Rb;

  if (Ib || Jb) {  // block b holds W_b after the pair
    if (Ib && !Jb) {
      double *tileT = &sW[0][0][0];  // 64 x 65 scratch
      for (int sa = 0; sa < 2; ++sa)
        for (int sb = 0; sb < 2; ++sb) {
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int c = e & 63, a = e >> 6;
            tileT[a * 65 + c] = Wb[(C0 + 64 * sb + c) + (R0 - kb0 + 64 * sa + a) * ldp];
          }
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int a = e & 63, c = e >> 6;
            const double v = tileT[a * 65 + c];
            A[(R0 + 64 * sa + a) + (L0 + 64 * sb + c) * ld] = v;
            if (go.k0 >= 0) gput(go, R0 + 64 * sa + a, C0 + 64 * sb + c, v);
          }
        }
    } else {
      for (int e = tid; e < UT * UT; e += UTHREADS) {
        const int a = e & (UT - 1), c = e >> 7;
        const double v = Wb[(R0 + a) + (C0 - kb0 + c) * ldp];
        A[(R0 + a) + (L0 + c) * ld] = v;
        if (go.k0 >= 0) gput(go, R0 + a, C0 + c, v);
      }
    }
    return;
  }
  // block a (not b): the tile starts from W_a and gets panel b only
  const bool from_w = Ia || Ja;
  // W_a at (row r, column c) of such a tile: column block a (and the
  // diagonal block) W_a[r, c - ka0]; row block a W_a[c, r - ka0] (transposed)
  const int64_t wrs = Ja ? 1 : ldp, wcs = Ja ? ldp : 1;  // strides of r, c
  const double *wab = Ja ? Wa - ka0 * ldp : Wa - ka0 * ldp;  // (r, c) -> wab[r wrs + c wcs]

  const int lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  if (R0 >= ld - AUG) {  // AUG row block: 16 live rows (as k_update)
    d4 acc;
    const int64_t r = R0 + lr;
    const int64_t c = C0 + 16 * wv + lk, lc = L0 + 16 * wv + lk;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[j] = from_w ? wab[r * wrs + (c + 4 * j) * wcs] : ld_a(&A[r + (lc + 4 * j) * ld]);
    for (int pnl = from_w ? 1 : 0; pnl < 2; ++pnl) {
      const double *gr = (pnl ? Rb : Ra) + R0 + lr + (int64_t)lk * ldp;
      const double *gc = (pnl ? Cb : Ca) + C0 + 16 * wv + lr + (int64_t)lk * ldp;
      double an = gc[0], bn = gr[0];
      for (int kk = 0; kk < NB / 4; ++kk) {
        const double a = an, bb = bn;
        if (kk + 1 < NB / 4) {
          an = gc[(int64_t)(4 * (kk + 1)) * ldp];
          bn = gr[(int64_t)(4 * (kk + 1)) * ldp];
        }
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st_a(&A[r + (lc + 4 * j) * ld], acc[j]);
    if (go.k0 >= 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) gput(go, r, c + 4 * j, acc[j]);
      gput_aug_dead(go, A, ld, R0, C0, tid, UTHREADS, L0);
    }
    return;
  }
  const int sk = tid >> 5, sm = (tid & 31) * 4;  // (the split mapping costs this kernel 12 VGPRs)
  // 32-bit element offsets from the (scalar) panel bases: the loads take a
  // scalar base + vector offset (no 64-bit address VGPRs; -1 ms per C2
  // evaluation, profiles/r03_v4_group_ab.txt)
  const int roff = (int)((R0 + sm) + (int64_t)sk * ldp), coff = (int)((C0 + sm) + (int64_t)sk * ldp);
  double2 rw0, rw1, rp0, rp1;
  {
    const double *w = (from_w ? Rb : Ra) + roff, *pp = (from_w ? Cb : Ca) + coff;
    rw0 = *reinterpret_cast<const double2 *>(w);
    rw1 = *reinterpret_cast<const double2 *>(w + 2);
    rp0 = *reinterpret_cast<const double2 *>(pp);
    rp1 = *reinterpret_cast<const double2 *>(pp + 2);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the C-tile loads behind them
  const int wr = wv & 1, wc = wv >> 1;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk, lc = L0 + 32 * wc + 16 * ci + lk;
      if (from_w) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ci][ri][j] = wab[r * wrs + (c + 4 * j) * wcs];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ci][ri][j] = ld_a(&A[r + (lc + 4 * j) * ld]);
      }
    }
  *reinterpret_cast<double2 *>(&sW[0][sk][sm]) = rw0;
  *reinterpret_cast<double2 *>(&sW[0][sk][sm + 2]) = rw1;
  *reinterpret_cast<double2 *>(&sP[0][sk][sm]) = rp0;
  *reinterpret_cast<double2 *>(&sP[0][sk][sm + 2]) = rp1;
  __syncthreads();
  // chunk ch of segment seg (0: panel a, 1: panel b) uses LDS buffer ch & 1
  // (NCH is even, so the parity runs on across the two segments)
  for (int seg = from_w ? 1 : 0; seg < 2; ++seg) {
    const double *sw = seg ? Rb : Ra, *sp = seg ? Cb : Ca;
    for (int ch = 0; ch < NCH; ++ch) {
      const int cur = ch & 1;
      const bool more = ch + 1 < NCH || seg == 0;
      if (more) {
        const double *nw = (ch + 1 < NCH ? sw + (int64_t)(ch + 1) * BK * ldp : Rb) + roff;
        const double *np = (ch + 1 < NCH ? sp + (int64_t)(ch + 1) * BK * ldp : Cb) + coff;
        rw0 = *reinterpret_cast<const double2 *>(nw);
        rw1 = *reinterpret_cast<const double2 *>(nw + 2);
        rp0 = *reinterpret_cast<const double2 *>(np);
        rp1 = *reinterpret_cast<const double2 *>(np + 2);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[2], b[4];
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
        for (int ri = 0; ri < 4; ++ri) b[ri] = sW[cur][4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
        for (int ci = 0; ci < 2; ++ci)
#pragma unroll
          for (int ri = 0; ri < 4; ++ri)
            acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
      }
      if (more) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm]) = rw0;
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + 2]) = rw1;
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm]) = rp0;
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + 2]) = rp1;
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t lc = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) st_a(&A[r + (lc + 4 * j) * ld], acc[ci][ri][j]);
    }
  if (go.k0 >= 0) {
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          gput(go, R0 + 64 * wr + 16 * ri + lr, C0 + 32 * wc + 16 * ci + lk + 4 * j, acc[ci][ri][j]);
  }
}

// Two sweep steps per launch on a tile list (skip rule [kx0, kx1), gather
// go on every tile).
__global__ __launch_bounds__(UTHREADS, 2) void k_update_pair(
    double *__restrict__ A, int64_t ld, const double *__restrict__ Ra,
    const double *__restrict__ Ca, const double *__restrict__ Rb, const double *__restrict__ Cb,
    int64_t ldp, int64_t ka0, int kx0, int kx1, const Tile *__restrict__ tiles, GatherOut go,
    int G, int wcol) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  constexpr int KT = NB / UT;
  int I, J;
  if (tiles) {
    const Tile tt = tiles[blockIdx.x];
    I = tt.I;
    J = tt.J;
    if (I < 0) return;  // padding of the XCD order
  } else {
    const int t = blockIdx.x;
    int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    while (i * (i + 1) / 2 > t) --i;
    I = i;
    J = t - i * (i + 1) / 2;
  }
  if (kx0 >= 0 && ((I >= kx0 * KT && I < kx1 * KT) || (J >= kx0 * KT && J < kx1 * KT))) return;
  update_pair_tile(I, J, sW, sP, A, ld, Ra, Ca, Rb, Cb, ldp, ka0, go, G, wcol != 0);
}

// Z sweep steps per launch (sweep_group() = 3 or 4; k_update_pair is Z = 2):
// npan panels j = 0 .. npan-1 of blocks ka0 / NB + j, operands R[j] = W_j,
// C[j] = Pn_j (single GPU), K = npan NB per tile.  A tile whose row or
// column lies in one of those blocks is overwritten by the step of the
// latest such block jm: it starts from W_jm and takes only panels jm+1 ..
// npan-1 (jm = npan-1: a copy of W_jm); any other tile takes every panel.
// Each accumulator runs the single-step schedule's MFMA chain in the same k
// order (fp64 in registers between panels), so the results are
// bit-identical to npan k_update launches.
struct PanelSet {
  const double *R[4];
  const double *C[4];
};
// panel j's pointer (j wave-uniform: scalar selects, no indexed kernarg)
__device__ __forceinline__ const double *psel(const double *const (&p)[4], int j) {
  return j == 0 ? p[0] : j == 1 ? p[1] : j == 2 ? p[2] : p[3];
}

// SH (sharded): A holds the rank's block-cyclic columns (tile column C0 at
// local column lcol(C0, G)) and the operands are swapped, R = Pn, C = W (W
// is only computed for the rows the rank consumes, its own columns).
template <bool SH, bool OPQ = false>
__device__ __forceinline__ void update_multi_tile(int I, int J, double (&sW)[2][BK][LDL],
                                                  double (&sP)[2][BK][LDL], double *__restrict__ A,
                                                  int64_t ld, const PanelSet &ps, int npan,
                                                  int64_t ldp, int64_t ka0, const GatherOut &go,
                                                  int G) {
  constexpr int KT = NB / UT;
  const int ta0 = (int)(ka0 / UT);
  const int di = I - ta0, dj = J - ta0;
  const int bi = (di >= 0 && di < npan * KT) ? di / KT : -1;
  const int bj = (dj >= 0 && dj < npan * KT) ? dj / KT : -1;
  const int jm = bi > bj ? bi : bj;  // the latest group block holding the tile
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int64_t L0 = SH ? lcol(C0, G) : C0;  // A's local column of the tile
  int tid = threadIdx.x;
  // OPQ (the persistent loop of k_update_multi_r): the lane index opaque per
  // tile, so the compiler does not hoist every lane-derived address out of
  // the tile loop (162 VGPRs, one workgroup per CU, without it)
  if (OPQ) __asm__ volatile("" : "+v"(tid));
  const double *const(&WS)[4] = SH ? ps.C : ps.R;  // the W operands

  if (jm == npan - 1) {  // the last block: W of the last step
    const double *Wl = psel(WS, jm);
    const int64_t kl0 = ka0 + (int64_t)jm * NB;
    if (bi == jm && bj != jm) {
      double *tileT = &sW[0][0][0];  // 64 x 65 scratch
      for (int sa = 0; sa < 2; ++sa)
        for (int sb = 0; sb < 2; ++sb) {
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int c = e & 63, a = e >> 6;
            tileT[a * 65 + c] = Wl[(C0 + 64 * sb + c) + (R0 - kl0 + 64 * sa + a) * ldp];
          }
          __syncthreads();
          for (int e = tid; e < 4096; e += UTHREADS) {
            const int a = e & 63, c = e >> 6;
            const double v = tileT[a * 65 + c];
            A[(R0 + 64 * sa + a) + (L0 + 64 * sb + c) * ld] = v;
            if (go.k0 >= 0) gput(go, R0 + 64 * sa + a, C0 + 64 * sb + c, v);
          }
        }
    } else {
      for (int e = tid; e < UT * UT; e += UTHREADS) {
        const int a = e & (UT - 1), c = e >> 7;
        const double v = Wl[(R0 + a) + (C0 - kl0 + c) * ldp];
        A[(R0 + a) + (L0 + c) * ld] = v;
        if (go.k0 >= 0) gput(go, R0 + a, C0 + c, v);
      }
    }
    return;
  }
  const bool from_w = jm >= 0;
  const int seg0 = from_w ? jm + 1 : 0;
  // W_jm at (row r, column c): column block jm (and its diagonal block)
  // W_jm[r, c - kj0], row block jm W_jm[c, r - kj0] (transposed)
  const bool jin = bj == jm;
  const int64_t wrs = jin ? 1 : ldp, wcs = jin ? ldp : 1;
  const double *wab = from_w ? psel(WS, jm) - (ka0 + (int64_t)jm * NB) * ldp : nullptr;

  const int lane = tid & 63, wv = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  if (R0 >= ld - AUG) {  // AUG row block: 16 live rows (as k_update)
    d4 acc;
    const int64_t r = R0 + lr;
    const int64_t c = C0 + 16 * wv + lk, lc = L0 + 16 * wv + lk;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      acc[j] = from_w ? wab[r * wrs + (c + 4 * j) * wcs] : ld_a(&A[r + (lc + 4 * j) * ld]);
    for (int pnl = seg0; pnl < npan; ++pnl) {
      const double *gr = psel(ps.R, pnl) + R0 + lr + (int64_t)lk * ldp;
      const double *gc = psel(ps.C, pnl) + C0 + 16 * wv + lr + (int64_t)lk * ldp;
      double an = gc[0], bn = gr[0];
      for (int kk = 0; kk < NB / 4; ++kk) {
        const double a = an, bb = bn;
        if (kk + 1 < NB / 4) {
          an = gc[(int64_t)(4 * (kk + 1)) * ldp];
          bn = gr[(int64_t)(4 * (kk + 1)) * ldp];
        }
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bb, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) st_a(&A[r + (lc + 4 * j) * ld], acc[j]);
    if (go.k0 >= 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) gput(go, r, c + 4 * j, acc[j]);
      gput_aug_dead(go, A, ld, R0, C0, tid, UTHREADS, L0);
    }
    return;
  }
  // (the sharded form keeps the 4-consecutive mapping: the split one costs
  // it 8 VGPRs and a wave per SIMD)
  constexpr int SMU = SH ? 4 : SM128, SHU = SH ? 2 : SH128;
  const int sk = tid >> 5, sm = (tid & 31) * SMU;  // 2nd half at sm + SHU
  // 32-bit element offsets from the (scalar) panel bases: the loads take a
  // scalar base + vector offset, so the segment pointers cost no VGPRs
  const int roff = (int)((R0 + sm) + (int64_t)sk * ldp), coff = (int)((C0 + sm) + (int64_t)sk * ldp);
  double2 rw0, rw1, rp0, rp1;
  {
    const double *w = psel(ps.R, seg0) + roff, *pp = psel(ps.C, seg0) + coff;
    rw0 = *reinterpret_cast<const double2 *>(w);
    rw1 = *reinterpret_cast<const double2 *>(w + SHU);
    rp0 = *reinterpret_cast<const double2 *>(pp);
    rp1 = *reinterpret_cast<const double2 *>(pp + SHU);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the C-tile loads behind them
  const int wr = wv & 1, wc = wv >> 1;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk, lc = L0 + 32 * wc + 16 * ci + lk;
      if (from_w) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ci][ri][j] = wab[r * wrs + (c + 4 * j) * wcs];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[ci][ri][j] = ld_a(&A[r + (lc + 4 * j) * ld]);
      }
    }
  *reinterpret_cast<double2 *>(&sW[0][sk][sm]) = rw0;
  *reinterpret_cast<double2 *>(&sW[0][sk][sm + SHU]) = rw1;
  *reinterpret_cast<double2 *>(&sP[0][sk][sm]) = rp0;
  *reinterpret_cast<double2 *>(&sP[0][sk][sm + SHU]) = rp1;
  __syncthreads();
  // chunk ch of every segment uses LDS buffer ch & 1 (NCH is even, so the
  // parity runs on across segments)
  for (int seg = seg0; seg < npan; ++seg) {
    const double *sw = psel(ps.R, seg), *sp = psel(ps.C, seg);
    const bool last = seg + 1 == npan;
    const double *nxw = last ? sw : psel(ps.R, seg + 1);
    const double *nxp = last ? sp : psel(ps.C, seg + 1);
    for (int ch = 0; ch < NCH; ++ch) {
      const int cur = ch & 1;
      const bool more = ch + 1 < NCH || !last;
      if (more) {
        const double *nw = (ch + 1 < NCH ? sw + (int64_t)(ch + 1) * BK * ldp : nxw) + roff;
        const double *np = (ch + 1 < NCH ? sp + (int64_t)(ch + 1) * BK * ldp : nxp) + coff;
        rw0 = *reinterpret_cast<const double2 *>(nw);
        rw1 = *reinterpret_cast<const double2 *>(nw + SHU);
        rp0 = *reinterpret_cast<const double2 *>(np);
        rp1 = *reinterpret_cast<const double2 *>(np + SHU);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double a[2], b[4];
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
        for (int ri = 0; ri < 4; ++ri) b[ri] = sW[cur][4 * kk + lk][64 * wr + 16 * ri + lr];
#pragma unroll
        for (int ci = 0; ci < 2; ++ci)
#pragma unroll
          for (int ri = 0; ri < 4; ++ri)
            acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
      }
      if (more) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm]) = rw0;
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + SHU]) = rw1;
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm]) = rp0;
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + SHU]) = rp1;
      }
      __syncthreads();
    }
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t lc = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) st_a(&A[r + (lc + 4 * j) * ld], acc[ci][ri][j]);
    }
  if (go.k0 >= 0) {
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          gput(go, R0 + 64 * wr + 16 * ri + lr, C0 + 32 * wc + 16 * ci + lk + 4 * j, acc[ci][ri][j]);
  }
}

// npan (1 .. 4) steps in one launch on a tile list (null: every lower tile,
// row-major grid), skipping the tiles with I or J in blocks [kx0, kx1).
template <bool SH>
__global__ __launch_bounds__(UTHREADS, 2) void k_update_multi(double *__restrict__ A, int64_t ld,
                                                              PanelSet ps, int npan, int64_t ldp,
                                                              int64_t ka0, int kx0, int kx1,
                                                              const Tile *__restrict__ tiles,
                                                              GatherOut go, int G) {
  ACE_WGT(5, gridDim.x < 4096 || blockIdx.x % 32 == 0);
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  constexpr int KT = NB / UT;
  int I, J;
  if (tiles) {
    const Tile tt = tiles[blockIdx.x];
    I = tt.I;
    J = tt.J;
    if (I < 0) return;  // padding of the XCD order
  } else {
    const int t = blockIdx.x;
    int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    while (i * (i + 1) / 2 > t) --i;
    I = i;
    J = t - i * (i + 1) / 2;
  }
  if (kx0 >= 0 && ((I >= kx0 * KT && I < kx1 * KT) || (J >= kx0 * KT && J < kx1 * KT))) return;
  update_multi_tile<SH>(I, J, sW, sP, A, ld, ps, npan, ldp, ka0, go, G);
}

// CUs of the current device, read once per device (the persistent queue's
// grid: two workgroups per CU; 256 on MI355X, fewer on a harvested part)
static int device_cu_count() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// Small n (run_sweep_heads with b.breserve > 0): the bulk launch as a
// persistent work queue that leaves `reserve` CUs of every shader engine to
// the panel chains.  At n = 4096 a bulk launch is short beside the chains,
// but while it runs it holds every CU slot (two 512-thread workgroups of
// 128 VGPRs per CU), so each chain launch issued meanwhile waited for its end
// (C1 trace: a 33-us k_update_q took 171 us; a plain launch split into
// smaller grids only serialised the bulk, profiles/r05_v3_ab_c1_bulkcap.txt).
// The reservation protocol is k_asm_mm_q's: the first workgroups to land on
// the first `reserve` CUs of an engine claim them and leave (at most a
// quarter of the grid per reserved CU), everyone else takes tiles from
// queue[0] until the list is done -- every workgroup reaches the exit.  Each
// tile is k_update_multi's (bit-identical).  queue: [next, leavers, 2 x 32
// CU claims].
template <bool SH>
__global__ __launch_bounds__(UTHREADS, 2) void k_update_multi_r(double *__restrict__ A, int64_t ld,
                                                                PanelSet ps, int npan, int64_t ldp,
                                                                int64_t ka0, int kx0, int kx1,
                                                                const Tile *__restrict__ tiles,
                                                                int64_t ntiles,
                                                                int *__restrict__ queue,
                                                                int reserve, GatherOut go) {
  ACE_WGT(5, gridDim.x < 4096 || blockIdx.x % 32 == 0);
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  __shared__ int next;
  constexpr int KT = NB / UT;
  if (reserve > 0) {
    if (threadIdx.x == 0) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);        // HW_REG_HW_ID
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7;  // HW_REG_XCC_ID
      const unsigned se = (hw >> 13) & 3;
      const int key = (int)((hw >> 8) & 0xff) + 1;  // cu [11:8], sh [12], se [15:13]
      int mine = 0;
      for (int r = 0; r < reserve && !mine; ++r) {
        const int old = atomicCAS(queue + 2 + 2 * (4 * xcc + se) + r, 0, key);
        mine = old == 0 || old == key;
      }
      next = mine ? (atomicAdd(queue + 1, 1) < (int)gridDim.x * reserve / 4) : 0;
    }
    __syncthreads();
    if (next) return;  // the whole workgroup (one CU)
    __syncthreads();
  }
  for (;;) {
    if (threadIdx.x == 0) next = atomicAdd(queue, 1);
    __syncthreads();  // also: every wave is done with the previous tile's LDS
    const int64_t idx = next;
    __syncthreads();
    if (idx >= ntiles) break;
    const Tile tt = tiles[idx];
    const int I = tt.I, J = tt.J;
    if (I < 0) continue;  // padding of the XCD order
    if (kx0 >= 0 && ((I >= kx0 * KT && I < kx1 * KT) || (J >= kx0 * KT && J < kx1 * KT))) continue;
    update_multi_tile<SH, true>(I, J, sW, sP, A, ld, ps, npan, ldp, ka0, go, 1);
  }
}

// CUs per shader engine a small-n bulk launch leaves to the panel chains
// (k_update_multi_r): ACE_BULK_RESERVE (0 .. 2) overrides; default 1 up to
// n = ACE_BULK_RESERVE_N, none above (there the bulk launches are the
// critical path and need every CU).
bool q_first(int64_t naug) {
  static int v = -2;
  if (v == -2) {
    const char *e = getenv("ACE_QFIRST");
    v = e ? (atoi(e) != 0) : -1;
  }
  if (v >= 0) return v != 0;
  return naug <= ACE_BULK_RESERVE_N + AUG;
}

int bulk_reserve(int64_t naug) {
  static int v = -2;
  if (v == -2) {
    const char *e = getenv("ACE_BULK_RESERVE");
    v = e ? std::max(0, std::min(2, atoi(e))) : -1;
  }
  if (v >= 0) return v;
  return naug <= ACE_BULK_RESERVE_N + AUG ? 1 : 0;
}


// Lookahead update: only the tiles with I or J in block kx (the next panel).
// About 2 n/128 tiles -- one workgroup per CU at 128 x 128 -- so it uses
// 64 x 64 tiles (4 waves of 32 x 32) for 4x the workgroups; same math and
// write-back rule as k_update.  Sharded: rank r keeps the tiles whose
// column block it owns.
constexpr int XT = 64;
constexpr int XL = XT + 8;  // LDS pitch
__global__ __launch_bounds__(256) void k_update_x(double *__restrict__ A, int64_t ld,
                                                  const double *__restrict__ Rop,
                                                  const double *__restrict__ Cop,
                                                  const double *__restrict__ Wk, int64_t ldp,
                                                  int64_t k0, int kx, int G, int rank) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][XL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][XL];
  constexpr int KX = NB / XT;  // 64-tiles per block
  int I, J;
  const int y = blockIdx.y;
  if (y < KX) {
    I = kx * KX + y;
    J = blockIdx.x;
    if (J > I) return;
  } else {
    J = kx * KX + (y - KX);
    I = blockIdx.x;
    if (I < (kx + 1) * KX) return;
  }
  const int64_t R0 = (int64_t)I * XT, C0 = (int64_t)J * XT;
  if (!owns_col(C0, G, rank)) return;
  if (R0 >= ld - AUG + XT) return;  // AUG rows 64..127: zero padding, stays zero
  const int64_t L0 = lcol(C0, G);
  const int kt0 = (int)(k0 / XT), kt1 = kt0 + KX;
  const bool Ik = I >= kt0 && I < kt1, Jk = J >= kt0 && J < kt1;
  const int tid = threadIdx.x;
  if (Ik || Jk) {
    if (Ik && !Jk) {
      double *tileT = &sW[0][0][0];  // 64 x 65 scratch (fits in sW)
      for (int e = tid; e < 4096; e += 256) {
        const int c = e & 63, a = e >> 6;
        tileT[a * 65 + c] = Wk[(C0 + c) + (R0 - k0 + a) * ldp];
      }
      __syncthreads();
      for (int e = tid; e < 4096; e += 256) {
        const int a = e & 63, c = e >> 6;
        A[(R0 + a) + (L0 + c) * ld] = tileT[a * 65 + c];
      }
    } else {
      for (int e = tid; e < XT * XT; e += 256) {
        const int a = e & (XT - 1), c = e >> 6;
        A[(R0 + a) + (L0 + c) * ld] = Wk[(R0 + a) + (C0 - k0 + c) * ldp];
      }
    }
    return;
  }
  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 32*wr.., cols 32*wc..
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[2][2];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t r = R0 + 32 * wr + 16 * ri + lr;
      const int64_t c = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = A[r + (c + 4 * j) * ld];
    }
  // staging: 256 threads x (4 doubles of each operand) per 64 x 16 chunk
  const int sk = tid >> 4, sm = (tid & 15) * SM64;  // 2nd half at sm + SH64
  const double *gW = Rop + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = Cop + (C0 + sm) + (int64_t)sk * ldp;
  double2 rw[2], rp[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    rw[e] = *reinterpret_cast<const double2 *>(gW + SH64 * e);
    rp[e] = *reinterpret_cast<const double2 *>(gP + SH64 * e);
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    *reinterpret_cast<double2 *>(&sW[0][sk][sm + SH64 * e]) = rw[e];
    *reinterpret_cast<double2 *>(&sP[0][sk][sm + SH64 * e]) = rp[e];
  }
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCH) {
      const int64_t off = (int64_t)(ch + 1) * BK * ldp;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        rw[e] = *reinterpret_cast<const double2 *>(gW + off + SH64 * e);
        rp[e] = *reinterpret_cast<const double2 *>(gP + off + SH64 * e);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[2];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) b[ri] = sW[cur][4 * kk + lk][32 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
    if (ch + 1 < NCH) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + SH64 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + SH64 * e]) = rp[e];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t r = R0 + 32 * wr + 16 * ri + lr;
      const int64_t c = L0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) A[r + (c + 4 * j) * ld] = acc[ci][ri][j];
    }
}

// Latency-critical lookahead updates of the head path (run_sweep_heads): npan
// panels from ps on a list of 128-tiles none of which lies in a panel's
// block (so no copies), as 64 x 64 quarters (blockIdx.x = 4 t + quarter;
// the upper quarter of a diagonal tile too, as k_update computes it) with
// k_update_x's 4-wave MFMA chain per panel and the accumulators kept across
// panels: per element the same chain as k_update / k_update_multi, a quarter
// of a 128-tile's work per workgroup.  go: the gather fused into the launch.
__global__ __launch_bounds__(256, 4) void k_update_q(double *__restrict__ A, int64_t ld, PanelSet ps,
                                                  int npan, int64_t ldp,
                                                  const Tile *__restrict__ tiles, GatherOut go,
                                                  double *__restrict__ pivSW,
                                                  double *__restrict__ piv,
                                                  int *__restrict__ flag) {
  ACE_WGT(4, true);
  // sW and sP in one buffer: the fused pivot below reuses it as its matrix
  __shared__ __attribute__((aligned(16))) double sbuf[2][2][BK][XL];
  static_assert(sizeof(sbuf) >= SUB * (SUB + 2) * sizeof(double), "pivot matrix fits the staging");
  double (*sW)[BK][XL] = sbuf[0];
  double (*sP)[BK][XL] = sbuf[1];
  const Tile tt = tiles[blockIdx.x >> 2];
  if (tt.I < 0) return;  // padding of the XCD order
  const int q = blockIdx.x & 3;
  const int64_t R0 = (int64_t)tt.I * UT + XT * (q & 1), C0 = (int64_t)tt.J * UT + XT * (q >> 1);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 32*wr.., cols 32*wc..
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[2][2];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t r = R0 + 32 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = A[r + (c + 4 * j) * ld];
    }
  const int sk = tid >> 4, sm = (tid & 15) * SM64;  // 2nd half at sm + SH64
  // The npan panels' NCH chunks as one sequence with two chunks of loads in
  // flight (round 5): chunk t is loaded into one of two register sets two
  // chunks before it is staged, so its latency overlaps two chunks' MFMAs.
  // A head-path launch is latency-bound (C1 trace: 33 us per one-panel
  // launch); the MFMA chain and its k order are unchanged: bit-identical.
  // Staging registers as named values (an array here was kept in scratch).
  double2 w00, w01, p00, p01, w10, w11, p10, p11;
  const int T = npan * NCH;
#define UQ_LOAD(W0, W1, P0, P1, TT)                                               \
  do {                                                                            \
    const int pj_ = (TT) / NCH, ch_ = (TT) - pj_ * NCH;                           \
    const int64_t off_ = (int64_t)ch_ * BK * ldp;                                 \
    const double *gW_ = psel(ps.R, pj_) + (R0 + sm) + (int64_t)sk * ldp + off_;   \
    const double *gP_ = psel(ps.C, pj_) + (C0 + sm) + (int64_t)sk * ldp + off_;   \
    W0 = *reinterpret_cast<const double2 *>(gW_);                                 \
    W1 = *reinterpret_cast<const double2 *>(gW_ + SH64);                          \
    P0 = *reinterpret_cast<const double2 *>(gP_);                                 \
    P1 = *reinterpret_cast<const double2 *>(gP_ + SH64);                          \
  } while (0)
#define UQ_STAGE(W0, W1, P0, P1, BUF)                                             \
  do {                                                                            \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm]) = W0;                          \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm + SH64]) = W1;                   \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm]) = P0;                          \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm + SH64]) = P1;                   \
  } while (0)
  auto mma = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[2];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) b[ri] = sW[cur][4 * kk + lk][32 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
  };
  static_assert(NCH % 2 == 0 && NCH >= 4, "two chunks per pipeline turn");
  UQ_LOAD(w00, w01, p00, p01, 0);
  UQ_STAGE(w00, w01, p00, p01, 0);
  UQ_LOAD(w10, w11, p10, p11, 1);
  UQ_LOAD(w00, w01, p00, p01, 2);
  __syncthreads();
#pragma unroll 1
  for (int t = 0; t < T; t += 2) {
    mma(0);
    UQ_STAGE(w10, w11, p10, p11, 1);
    if (t + 3 < T) UQ_LOAD(w10, w11, p10, p11, t + 3);
    __syncthreads();
    mma(1);
    if (t + 2 < T) {
      UQ_STAGE(w00, w01, p00, p01, 0);
      if (t + 4 < T) UQ_LOAD(w00, w01, p00, p01, t + 4);
    }
    __syncthreads();
  }
#undef UQ_LOAD
#undef UQ_STAGE
  ACE_WGT_MARK(0);
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t r = R0 + 32 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double v = acc[ci][ri][j];
        A[r + (c + 4 * j) * ld] = v;
        if (go.k0 >= 0) gput(go, r, c + 4 * j, v);
      }
    }
  // pivSW: this launch gathers a panel, and the quarter holding that panel's
  // first 64 x 64 diagonal block D_0 also runs its sub-sweep (k_pivot's,
  // into pivSW / piv / flag) -- the input is the lower values just stored,
  // mirrored, i.e. exactly the S0 snapshot k_pivot would read: bit-identical,
  // one head-path launch less per panel
  if (pivSW && go.k0 >= 0 && R0 == go.k0 && C0 == go.k0) {
    __shared__ double pv[SUB];
    double(*M)[SUB + 2] = reinterpret_cast<double(*)[SUB + 2]>(&sbuf[0][0][0][0]);
    // (the chunk loop ended with a barrier: the staging buffers are free)
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) {
        const int a = 32 * wr + 16 * ri + lr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = 32 * wc + 16 * ci + lk + 4 * j;
          if (a >= c) {
            M[a][c] = acc[ci][ri][j];
            M[c][a] = acc[ci][ri][j];
          }
        }
      }
    __syncthreads();
    double v[SUB / 4];
#pragma unroll
    for (int q = 0; q < SUB / 4; ++q) v[q] = M[lane][16 * wv + q];
    ACE_WGT_MARK(1);
    pivot_sweep_blk<SUB + 2>(v, M, pv, tid);
    ACE_WGT_MARK(2);
    pivot_store<4>(v, pv, tid, pivSW, piv, go.k0, flag);
  }
}

// k_update_q with every 64 x 64 quarter split into four 32 x 32 pieces,
// one per 256-thread workgroup (each wave one 16 x 16 MFMA block), for the
// latency-critical head launches of small n (ACE_QSPLIT): four times the
// workgroups, a quarter of each one's K loop.  Every element's MFMA chain
// (operands, k order, accumulator start) is k_update_q's: bit-identical.
// The quarter holding D_0 of a gathered panel is finished by its last
// piece: each piece stores (and gathers) its part, releases it at agent
// scope and counts into *qctr; the piece that counts last acquires, reads
// D_0 back from the gathered snapshot S0 -- the values k_update_q's fused
// sweep reads from its registers -- runs the sub-sweep and resets *qctr.
// No workgroup waits for another.
__global__ __launch_bounds__(256, 4) void k_update_q4(double *__restrict__ A, int64_t ld, PanelSet ps,
                                                   int npan, int64_t ldp,
                                                   const Tile *__restrict__ tiles, GatherOut go,
                                                   double *__restrict__ pivSW,
                                                   double *__restrict__ piv,
                                                   int *__restrict__ flag, int *__restrict__ qctr) {
  ACE_WGT(4, true);
  constexpr int QT = XT / 2;        // 32: the piece
  constexpr int QL = QT + 8;        // LDS pitch
  __shared__ __attribute__((aligned(16))) double sbuf[SUB * (SUB + 2)];  // staging, then D_0
  static_assert(2 * 2 * BK * QL <= SUB * (SUB + 2), "staging fits");
  double (*sW)[BK][QL] = reinterpret_cast<double (*)[BK][QL]>(sbuf);
  double (*sP)[BK][QL] = reinterpret_cast<double (*)[BK][QL]>(sbuf + 2 * BK * QL);
  __shared__ int last;
  const Tile tt = tiles[blockIdx.x >> 4];
  if (tt.I < 0) return;  // padding of the XCD order
  const int q = (blockIdx.x >> 2) & 3, pc = blockIdx.x & 3;
  const int64_t Rq = (int64_t)tt.I * UT + XT * (q & 1), Cq = (int64_t)tt.J * UT + XT * (q >> 1);
  const int64_t R0 = Rq + QT * (pc & 1), C0 = Cq + QT * (pc >> 1);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 16*wr.., cols 16*wc.. of the piece
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc;
  {
    const int64_t r = R0 + 16 * wr + lr;
    const int64_t c = C0 + 16 * wc + lk;
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = A[r + (c + 4 * j) * ld];
  }
  const int sk = tid >> 4, sm = (tid & 15) * 2;  // one double2 of each operand per chunk
  double2 w0, p0, w1, p1;
  const int T = npan * NCH;
#define UQ4_LOAD(W, P, TT)                                                         \
  do {                                                                             \
    const int pj_ = (TT) / NCH, ch_ = (TT) - pj_ * NCH;                            \
    const int64_t off_ = (int64_t)ch_ * BK * ldp;                                  \
    W = *reinterpret_cast<const double2 *>(psel(ps.R, pj_) + (R0 + sm) + (int64_t)sk * ldp + off_); \
    P = *reinterpret_cast<const double2 *>(psel(ps.C, pj_) + (C0 + sm) + (int64_t)sk * ldp + off_); \
  } while (0)
#define UQ4_STAGE(W, P, BUF)                                                       \
  do {                                                                             \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm]) = W;                            \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm]) = P;                            \
  } while (0)
  auto mma = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const double a = sP[cur][4 * kk + lk][16 * wc + lr];
      const double b = sW[cur][4 * kk + lk][16 * wr + lr];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
  };
  static_assert(NCH % 2 == 0 && NCH >= 4, "two chunks per pipeline turn");
  UQ4_LOAD(w0, p0, 0);
  UQ4_STAGE(w0, p0, 0);
  UQ4_LOAD(w1, p1, 1);
  UQ4_LOAD(w0, p0, 2);
  __syncthreads();
#pragma unroll 1
  for (int t = 0; t < T; t += 2) {
    mma(0);
    UQ4_STAGE(w1, p1, 1);
    if (t + 3 < T) UQ4_LOAD(w1, p1, t + 3);
    __syncthreads();
    mma(1);
    if (t + 2 < T) {
      UQ4_STAGE(w0, p0, 0);
      if (t + 4 < T) UQ4_LOAD(w0, p0, t + 4);
    }
    __syncthreads();
  }
#undef UQ4_LOAD
#undef UQ4_STAGE
  ACE_WGT_MARK(0);
  {
    const int64_t r = R0 + 16 * wr + lr;
    const int64_t c = C0 + 16 * wc + lk;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      A[r + (c + 4 * j) * ld] = acc[j];
      if (go.k0 >= 0) gput(go, r, c + 4 * j, acc[j]);
    }
  }
  if (!(pivSW && go.k0 >= 0 && Rq == go.k0 && Cq == go.k0)) return;
  // the D_0 quarter: the last of its four pieces runs the sub-sweep
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    last = __hip_atomic_fetch_add(qctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(qctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (!last) return;
  __shared__ double pv[SUB];
  double(*M)[SUB + 2] = reinterpret_cast<double(*)[SUB + 2]>(sbuf);
  double v[SUB / 4];
  // D_0 = S0[0:64, 0:64] (row a, column c at a + c SUB), as k_pivot reads it
#pragma unroll
  for (int qq = 0; qq < SUB / 4; ++qq)
    v[qq] = __hip_atomic_load(go.S0 + lane + (16 * wv + qq) * SUB, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
  ACE_WGT_MARK(1);
  pivot_sweep_blk<SUB + 2>(v, M, pv, tid);
  ACE_WGT_MARK(2);
  pivot_store<4>(v, pv, tid, pivSW, piv, go.k0, flag);
}

// The head path's panel GEMM (run_sweep_heads) on 64 x 64 quarters of the
// 128-tiles: W_I,J = Pn_I W_kk[:, J] as k_panel_gemm_t, a quarter of its work
// per 256-thread workgroup.  The head launches hold few tiles (the rows of
// the next group's blocks) and k_panel_gemm_t's 8.4 MFLOP per workgroup is a
// CU's MFMA peak for ~27 us (C1 marks: K loop 32 us); quartered, four times
// the CUs share it.  Operand roles (A from W_kk, B from Pn), k order and the
// zero start are k_panel_gemm_t's: bit-identical.  Grid: (64-row blocks of
// row tiles [rt0, rt1), NB / 64 column blocks); k_update_q's two-deep load
// pipeline.
__global__ __launch_bounds__(256, 4) void k_panel_gemm_q(double *__restrict__ W,
                                                       const double *__restrict__ Pn,
                                                       int64_t ldp, int64_t k0, int rt0) {
  ACE_WGT(3, true);
  __shared__ __attribute__((aligned(16))) double sW[2][BK][XL];  // Pn rows of the quarter
  __shared__ __attribute__((aligned(16))) double sP[2][BK][XL];  // W_kk rows c
  const int64_t R0 = (int64_t)rt0 * UT + (int64_t)blockIdx.x * XT, C0 = (int64_t)blockIdx.y * XT;
  if (R0 >= k0 && R0 < k0 + NB) return;  // pivot rows are already final
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 32*wr.., cols 32*wc..
  const int lr = lane & 15, lk = lane >> 4;
  const int sk = tid >> 4, sm = (tid & 15) * SM64;  // 2nd half at sm + SH64
  const double *gW = Pn + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = W + (k0 + C0 + sm) + (int64_t)sk * ldp;  // W_kk(c, k) = W[k0 + c, k]
  d4 acc[2][2];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) acc[ci][ri] = d4{0.0, 0.0, 0.0, 0.0};
  double2 w00, w01, p00, p01, w10, w11, p10, p11;
#define PQ_LOAD(W0, W1, P0, P1, CH)                                               \
  do {                                                                            \
    const int64_t off_ = (int64_t)(CH) * BK * ldp;                                \
    W0 = *reinterpret_cast<const double2 *>(gW + off_);                           \
    W1 = *reinterpret_cast<const double2 *>(gW + off_ + SH64);                    \
    P0 = *reinterpret_cast<const double2 *>(gP + off_);                           \
    P1 = *reinterpret_cast<const double2 *>(gP + off_ + SH64);                    \
  } while (0)
#define PQ_STAGE(W0, W1, P0, P1, BUF)                                             \
  do {                                                                            \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm]) = W0;                          \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm + SH64]) = W1;                   \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm]) = P0;                          \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm + SH64]) = P1;                   \
  } while (0)
  auto mma = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[2], b[2];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) a[ci] = sP[cur][4 * kk + lk][32 * wc + 16 * ci + lr];
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) b[ri] = sW[cur][4 * kk + lk][32 * wr + 16 * ri + lr];
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
          acc[ci][ri] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ci], b[ri], acc[ci][ri], 0, 0, 0);
    }
  };
  static_assert(NCH % 2 == 0 && NCH >= 4, "two chunks per pipeline turn");
  PQ_LOAD(w00, w01, p00, p01, 0);
  PQ_STAGE(w00, w01, p00, p01, 0);
  PQ_LOAD(w10, w11, p10, p11, 1);
  PQ_LOAD(w00, w01, p00, p01, 2);
  __syncthreads();
  ACE_WGT_MARK(0);
#pragma unroll 1
  for (int ch = 0; ch < NCH; ch += 2) {
    mma(0);
    PQ_STAGE(w10, w11, p10, p11, 1);
    if (ch + 3 < NCH) PQ_LOAD(w10, w11, p10, p11, ch + 3);
    __syncthreads();
    mma(1);
    if (ch + 2 < NCH) {
      PQ_STAGE(w00, w01, p00, p01, 0);
      if (ch + 4 < NCH) PQ_LOAD(w00, w01, p00, p01, ch + 4);
    }
    __syncthreads();
  }
#undef PQ_LOAD
#undef PQ_STAGE
  ACE_WGT_MARK(1);
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int64_t rr = R0 + 32 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) W[rr + (c + 4 * j) * ldp] = acc[ci][ri][j];
    }
}

// k_panel_gemm_q on 32 x 32 pieces (ACE_QSPLIT, small n): each wave one
// 16 x 16 MFMA block, four times the workgroups; every element's chain is
// k_panel_gemm_q's (bit-identical).  Grid: (2 x 64-row blocks, 2 NB / 64).
__global__ __launch_bounds__(256, 4) void k_panel_gemm_q4(double *__restrict__ W,
                                                        const double *__restrict__ Pn,
                                                        int64_t ldp, int64_t k0, int rt0) {
  ACE_WGT(3, true);
  constexpr int QT = XT / 2, QL = QT + 8;
  __shared__ __attribute__((aligned(16))) double sW[2][BK][QL];  // Pn rows of the piece
  __shared__ __attribute__((aligned(16))) double sP[2][BK][QL];  // W_kk rows c
  const int64_t R0 = (int64_t)rt0 * UT + (int64_t)blockIdx.x * QT, C0 = (int64_t)blockIdx.y * QT;
  if (R0 >= k0 && R0 < k0 + NB) return;  // pivot rows are already final
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 16*wr.., cols 16*wc..
  const int lr = lane & 15, lk = lane >> 4;
  const int sk = tid >> 4, sm = (tid & 15) * 2;
  const double *gW = Pn + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = W + (k0 + C0 + sm) + (int64_t)sk * ldp;  // W_kk(c, k) = W[k0 + c, k]
  d4 acc = d4{0.0, 0.0, 0.0, 0.0};
  double2 w0, p0, w1, p1;
#define PQ4_LOAD(WW, PP, CH)                                                        \
  do {                                                                              \
    const int64_t off_ = (int64_t)(CH) * BK * ldp;                                  \
    WW = *reinterpret_cast<const double2 *>(gW + off_);                             \
    PP = *reinterpret_cast<const double2 *>(gP + off_);                             \
  } while (0)
#define PQ4_STAGE(WW, PP, BUF)                                                      \
  do {                                                                              \
    *reinterpret_cast<double2 *>(&sW[BUF][sk][sm]) = WW;                            \
    *reinterpret_cast<double2 *>(&sP[BUF][sk][sm]) = PP;                            \
  } while (0)
  auto mma = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const double a = sP[cur][4 * kk + lk][16 * wc + lr];
      const double b = sW[cur][4 * kk + lk][16 * wr + lr];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
  };
  PQ4_LOAD(w0, p0, 0);
  PQ4_STAGE(w0, p0, 0);
  PQ4_LOAD(w1, p1, 1);
  PQ4_LOAD(w0, p0, 2);
  __syncthreads();
  ACE_WGT_MARK(0);
#pragma unroll 1
  for (int ch = 0; ch < NCH; ch += 2) {
    mma(0);
    PQ4_STAGE(w1, p1, 1);
    if (ch + 3 < NCH) PQ4_LOAD(w1, p1, ch + 3);
    __syncthreads();
    mma(1);
    if (ch + 2 < NCH) {
      PQ4_STAGE(w0, p0, 0);
      if (ch + 4 < NCH) PQ4_LOAD(w0, p0, ch + 4);
    }
    __syncthreads();
  }
#undef PQ4_LOAD
#undef PQ4_STAGE
  ACE_WGT_MARK(1);
  const int64_t rr = R0 + 16 * wr + lr;
  const int64_t c = C0 + 16 * wc + lk;
#pragma unroll
  for (int j = 0; j < 4; ++j) W[rr + (c + 4 * j) * ldp] = acc[j];
}

// ---------------------------------------------------------------- sharded panel
// Packing for the panel exchange of step k (sharded model).  The owner of
// block k sends rows [k0, naug) of its column block (contiguous, ld naug-k0)
// by broadcast; every rank sends the NB x NB pieces A[k-block, j-block] of
// its own blocks j < k (slot q = j / G) by all-gather.
// (i_base, lr0, h): rows from i_base on, into low at row offset lr0 (the
// head / tail parts of the head schedule; default: every row >= k0)
__global__ __launch_bounds__(256) void k_pack_lower(const double *__restrict__ A, int64_t ld,
                                                    int G, int64_t k0, int64_t naug,
                                                    double *__restrict__ low, int64_t i_base = -1,
                                                    int64_t lr0 = 0, int64_t hh = -1) {
  const int64_t i0 = (i_base < 0 ? k0 : i_base) + (int64_t)blockIdx.x * 64;
  const int j0 = blockIdx.y * 64;
  const int64_t L = lcol(k0, G);
  const int64_t h = hh < 0 ? naug - k0 : hh;
  low -= lr0;  // row (i - k0) of the column lands at (i - k0 - lr0)
  if (i0 >= k0 + NB || i0 >= k0 + j0 + 64) {  // entirely on / below the diagonal
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      low[(i0 - k0 + a) + (int64_t)(j0 + b) * h] = A[(i0 + a) + (L + j0 + b) * ld];
    }
  } else {
    // pivot block: only its lower triangle is stored, mirror the rest
    // (both indices lie in block k, so the column map is L + offset)
    for (int e = threadIdx.x; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const int ia = (int)(i0 - k0) + a, cb = j0 + b;
      low[ia + (int64_t)cb * h] =
          ia >= cb ? A[(k0 + ia) + (L + cb) * ld] : A[(k0 + cb) + (L + ia) * ld];
    }
  }
}

__global__ __launch_bounds__(256) void k_pack_rows(const double *__restrict__ A, int64_t ld,
                                                   int64_t k0, double *__restrict__ send) {
  const int q = blockIdx.z;  // local block q = global block r + q G (< k)
  const int a0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  double *dst = send + (int64_t)q * NB * NB;
  for (int e = threadIdx.x; e < 4096; e += 256) {
    const int a = e & 63, c = e >> 6;
    dst[(a0 + a) + (c0 + c) * NB] = A[(k0 + a0 + a) + ((int64_t)q * NB + c0 + c) * ld];
  }
}

// Rebuilds panel k on every rank: Pn = -P for every row, W = P on the pivot
// rows, S0 = pivot rows of sub-block 0 (k_pivot's input).  Rows >= k0 come
// from the broadcast block, rows i < k0 (block j = i / NB) from all-gather
// slot (j % G, j / G), transposed: P[i, c] = A[k0 + c, i].  skip_own: the
// rows of rank r's own blocks are already in place (packing cross launch).
// (i_base, lr0, hh): rows from i_base on, low holding the column rows from
// k0 + lr0 on with ld hh (the head / tail parts of the head schedule;
// default: every row, low = rows >= k0)
__global__ __launch_bounds__(256) void k_unpack_panel(const double *__restrict__ low,
                                                      const double *__restrict__ recv, int m,
                                                      int G, int64_t k0, int64_t naug,
                                                      double *__restrict__ Pn,
                                                      double *__restrict__ W, int64_t ldp,
                                                      double *__restrict__ S0, int skip_own,
                                                      int r, int64_t i_base = 0, int64_t lr0 = 0,
                                                      int64_t hh = -1) {
  __shared__ double tile[64][65];
  const int64_t i0 = i_base + (int64_t)blockIdx.x * 64;
  const int j0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  if (skip_own) {  // rows the rank's own (packing) cross launch wrote
    const int64_t kb = k0 / NB;
    if (i0 >= k0 ? kb % G == r : (i0 / NB) % G == r) return;
  }
  if (i0 >= k0) {
    const int64_t h = hh < 0 ? naug - k0 : hh;
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      const double v = low[(i0 - k0 - lr0 + a) + (int64_t)(j0 + b) * h];
      Pn[(i0 + a) + (int64_t)(j0 + b) * ldp] = -v;
      if (i0 < k0 + NB) W[(i0 + a) + (int64_t)(j0 + b) * ldp] = v;
      if (i0 == k0) S0[a + (int64_t)(j0 + b) * SUB] = v;
    }
  } else {
    const int64_t j = i0 / NB;
    const int rr0 = (int)(i0 % NB);
    const double *src = recv + ((j % G) * (int64_t)m + j / G) * NB * NB;
    for (int e = tid; e < 4096; e += 256) {
      const int b = e & 63, a = e >> 6;  // b: panel column (contiguous in src)
      tile[a][b] = src[(j0 + b) + (int64_t)(rr0 + a) * NB];
    }
    __syncthreads();
    for (int e = tid; e < 4096; e += 256) {
      const int a = e & 63, b = e >> 6;
      Pn[(i0 + a) + (int64_t)(j0 + b) * ldp] = -tile[a][b];
    }
  }
}

// Pivot block sweep (4 x 64-column sub-sweeps, pivots -> piv / flag) and the
// panel GEMM for the rows rank r consumes.  W's pivot rows and S[0] must
// hold the panel's pivot rows.
// ACE_CHAIN=0 selects the row-group k_panel (A/B switch; k_panel_split is
// the default and bit-identical).
static bool panel_split() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_CHAIN");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// ACE_CHAIN_FUSE=1 (default): at small n (the bulk-reserve schedule) each
// panel's four split sub-steps run as one k_panel_split4 launch
// (bit-identical; C1 3.60 -> 3.52 ms, profiles/r06_chain_fuse_ab.txt); 0: four
// k_panel_split launches
static bool chain_fuse() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_CHAIN_FUSE");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// ACE_PGEMM_TILES=0 selects the 64-row k_panel_gemm (A/B switch; the tile
// form k_panel_gemm_t is the default and bit-identical)
static bool pgemm_tiles() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_PGEMM_TILES");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// ACE_DIAG_SKIP (compile-time, timing diagnostics only -- the results are
// wrong): bit 1 skips the pivot sub-sweeps and panel updates, bit 2 the panel
// GEMM
#ifndef ACE_DIAG_SKIP
#define ACE_DIAG_SKIP 0
#endif
// pivot0: sub-block 0 was already swept (by the k_update_q launch that
// gathered the panel); fuse_ctr (small n, ACE_CHAIN_FUSE): the four split
// sub-steps in one k_panel_split4 launch, its grid barrier on *fuse_ctr
static void panel_chain(const double *Pn, double *W, int64_t ld, int64_t k0, double *SW,
                        double *const S[2], double *piv, int *flag, int G, int r,
                        hipStream_t st, bool pivot0 = false, bool no_gemm = false,
                        int *fuse_ctr = nullptr, unsigned xlds = 0) {
  const bool split = panel_split();
  double *const SWb[2] = {SW, SW + SUB * SUB};  // ping-pong by sub-step
  if (split && fuse_ctr && !(ACE_DIAG_SKIP & 1)) {
    if (!pivot0) launch_pivot(S[0], 0, SWb[0], piv, k0, flag, st);
    if (xlds) {
      static unsigned set = 0;
      if (set != xlds && hipFuncSetAttribute((const void *)k_panel_split4,
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)xlds) == hipSuccess)
        set = xlds;
    }
    hipLaunchKernelGGL(k_panel_split4, dim3(NB / SUB, NB / SUB), dim3(256), xlds, st, W, ld, k0, SW,
                       S[0], S[1], piv, flag, fuse_ctr);
  }
  for (int s = 0; s < ((ACE_DIAG_SKIP & 1) || (split && fuse_ctr) ? 0 : NB / SUB); ++s) {
    if (!split || (s == 0 && !pivot0))
      launch_pivot(S[s & 1], s, SWb[s & 1], piv, k0 + (int64_t)s * SUB, flag, st);
    if (split)
      hipLaunchKernelGGL(k_panel_split, dim3(NB / SUB, NB / SUB), dim3(256), 0, st, W, ld, k0, s,
                         SWb[s & 1], S[s & 1], S[(s + 1) & 1], SW + 2 * SUB * SUB,
                         SWb[(s + 1) & 1], piv, flag);
    else
      hipLaunchKernelGGL(k_panel, dim3(NB / SUB), dim3(256), 0, st, W, ld, k0, s, SWb[s & 1],
                         S[s & 1], S[(s + 1) & 1], k0);
  }
  if ((ACE_DIAG_SKIP & 2) || no_gemm) return;
  if (pgemm_tiles())
    hipLaunchKernelGGL(k_panel_gemm_t, dim3((unsigned)(ld / UT), NB / UT), dim3(UTHREADS), 0, st,
                       W, Pn, ld, k0, G, r, 0, 1 << 30, 1 << 30);
  else
    hipLaunchKernelGGL(k_panel_gemm, dim3((unsigned)(ld / SUB)), dim3(512), 0, st, W, Pn, ld, k0,
                       G, r);
}

// ACE_XGATHER: pair steps fuse each panel's gather into the lookahead cross
// launch that writes its column block (GatherOut; default 1)
static bool xgather() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_XGATHER");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// gathered: P, W and S[0] of this panel were written by the cross launch
static hipError_t panel_sweep(const SweepBufs &b, int buf, int64_t k0, hipStream_t st,
                              bool gathered = false) {
  const int64_t naug = b.ld;
  if (!gathered)
    hipLaunchKernelGGL(k_gather, dim3((unsigned)(naug / 64), NB / 64), dim3(256), 0, st, b.A, b.ld,
                       k0, b.P[buf], b.W[buf], b.ld, b.S[0]);
  // sweep the NB x NB pivot block in place, then every other panel row:
  // W_i = Pn_i W_kk
  panel_chain(b.P[buf], b.W[buf], b.ld, k0, b.SW, b.S, b.piv, b.flag, 1, 0, st);
  return hipGetLastError();
}

// GEMM tiles of one k_update launch, in full-tile units: a tile of the AUG
// row block computes 16 of its 128 rows.
double update_gemm_tiles(int64_t naug, int64_t k0, int kx, bool look) {
  const int64_t nT = naug / UT, KT = NB / UT, kt0 = k0 / UT, kt1 = kt0 + KT;
  double cnt = 0.0;
  for (int64_t I = 0; I < nT; ++I)
    for (int64_t J = 0; J <= I; ++J) {
      const bool inx = kx >= 0 && ((I >= kx * KT && I < (kx + 1) * KT) ||
                                   (J >= kx * KT && J < (kx + 1) * KT));
      if (inx != look) continue;
      const bool Ik = I >= kt0 && I < kt1, Jk = J >= kt0 && J < kt1;
      if (!(Ik || Jk)) cnt += (I == nT - 1) ? 16.0 / UT : 1.0;
    }
  return cnt;
}

double sweep_flops(int64_t naug, int64_t npad) {
  thread_local int64_t cn = -1, cp = -1;
  thread_local double cf = 0.0;
  if (naug == cn && npad == cp) return cf;
  double f = 0.0;
  for (int64_t k0 = 0; k0 < npad; k0 += NB)
    f += update_gemm_tiles(naug, k0, -1, false) * 2.0 * UT * UT * NB +
         2.0 * (double)(naug - NB) * NB * NB;
  cn = naug;
  cp = npad;
  cf = f;
  return f;
}

int update_order_block() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_UPD_ORDER");
    // 2 with two steps per launch (K = 512 panels per tile): 78.7-78.9 ms
    // per C2 evaluation against 79.1-79.2 at 4, 79.6-79.7 at 3, 81.1-81.2
    // at 8, 79.1-79.5 at 1 and at 0 (row-major); profiles/r02_chain_ab.txt
    v = e ? std::max(0, atoi(e)) : 2;
  }
  return v;
}

bool cross_update_on_tiles() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_XUPD");
    // 1: -0.2 ms per C2 evaluation against k_update_x (same box, 2 rounds:
    // 81.03 / 81.26 vs 81.25 / 81.49 ms); bit-identical
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

std::vector<Tile> cross_update_tiles(int64_t naug, int steps, std::vector<int64_t> &off) {
  const int64_t nT = naug / UT;
  constexpr int KT = NB / UT;
  std::vector<Tile> all;
  off.assign(1, 0);
  for (int k = 0; k + 1 < steps; ++k) {
    const int64_t x0 = (int64_t)(k + 1) * KT, x1 = x0 + KT;
    std::vector<Tile> t;
    for (int64_t I = 0; I < nT; ++I)
      for (int64_t J = 0; J <= I; ++J)
        if ((I >= x0 && I < x1) || (J >= x0 && J < x1)) t.push_back(Tile{(int)I, (int)J});
    const int S = update_order_block();
    const std::vector<Tile> o = S > 0 ? xcd_update_order(t, S) : t;
    all.insert(all.end(), o.begin(), o.end());
    off.push_back((int64_t)all.size());
  }
  return all;
}

// ACE_TAIL_SORT=1 (default): per group, the bulk tile order with each XCD's
// cheap tiles (copies, block a, the AUG row, skipped lookahead tiles) last;
// -0.15 ms per C2 evaluation once the side chain is off the critical path
// (profiles/r02_chain_ab.txt)
bool tail_sort() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_TAIL_SORT");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

std::vector<Tile> pair_bulk_orders(int64_t naug, int steps, int64_t *len, int G, int r, int Z) {
  const int64_t nT = naug / UT;
  constexpr int KT = NB / UT;
  const int ng = (steps + Z - 1) / Z;
  const std::vector<Tile> base = own_tiles(nT, UT, G, r);
  const int S = std::max(1, update_order_block());
  std::vector<Tile> all;
  std::vector<std::vector<Tile>> lists;
  *len = 0;
  for (int g = 0; g < ng; ++g) {
    const int z = std::min(Z, steps - Z * g);
    const int64_t ta0 = (int64_t)Z * g * KT;
    const bool more = g + 1 < ng;
    const int64_t x0 = more ? (int64_t)Z * (g + 1) * KT : -1;
    const int64_t x1 = more ? (int64_t)std::min(Z * (g + 1) + Z, steps) * KT : -1;
    // segments the tile runs: every panel, or those after its latest group
    // block (a copy for the last one)
    auto cost = [&](const Tile &t) -> double {
      const int64_t I = t.I, J = t.J;
      if (more && ((I >= x0 && I < x1) || (J >= x0 && J < x1))) return 0.0;  // skipped
      const int64_t di = I - ta0, dj = J - ta0;
      const int bi = (di >= 0 && di < z * KT) ? (int)(di / KT) : -1;
      const int bj = (dj >= 0 && dj < z * KT) ? (int)(dj / KT) : -1;
      const int jm = std::max(bi, bj);
      if (jm == z - 1) return 0.05;  // copy
      const double rows = (I == nT - 1) ? 16.0 / UT : 1.0;
      return rows * (jm >= 0 ? z - 1 - jm : z);
    };
    lists.push_back(bulk_curve() ? curve_update_order(base, cost) : xcd_update_order(base, S, cost));
    *len = std::max<int64_t>(*len, (int64_t)lists.back().size());
  }
  // one length for every group (padding: whole rows of 8, so the XCD dealing
  // of each list stands)
  for (auto &o : lists) {
    o.resize((size_t)*len, Tile{-1, -1});
    all.insert(all.end(), o.begin(), o.end());
  }
  return all;
}

int sweep_group() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_GROUP");
    // 4 with the head / tail lookahead (run_sweep_heads, default): 75.9
    // against 76.6 ms per C2 evaluation at 2 (same box, 4 runs each,
    // profiles/r03_v5_heads_ab.txt)
    v = e ? std::min(4, std::max(2, atoi(e))) : 4;
  }
  return v;
}

// Z for a model of naug rows: ACE_GROUP when set, else 3 up to n =
// ACE_BULK_RESERVE_N (the chain-bound sizes: C1 3.90 -> 3.75 ms against Z = 4,
// 3.87 at Z = 2 -- a shorter last bulk launch and an earlier first one,
// profiles/r05_v11_ab_c1_group.txt), 4 above
int sweep_group_n(int64_t naug) {
  if (getenv("ACE_GROUP")) return sweep_group();
  return naug <= ACE_BULK_RESERVE_N + AUG ? 3 : 4;
}

bool pair_steps() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_PAIR");
    // 1: 81.4 -> 79.5 ms per C2 evaluation (profiles/r02_chain_ab.txt)
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// ACE_SIDE2: pair steps run the second block's lookahead cross on a second
// side stream, concurrently with the first block's panel chain (default 1)
static bool side2_on() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_SIDE2");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

std::vector<Tile> pair_cross_tiles(int64_t naug, int steps, std::vector<int64_t> &off, int Z) {
  const int64_t nT = naug / UT;
  constexpr int KT = NB / UT;
  const int ng = (steps + Z - 1) / Z;
  const int S = update_order_block();
  std::vector<Tile> all;
  off.assign(3, 0);  // group 0 has no cross lists
  auto in_blk = [&](int64_t t, int blk) { return t >= (int64_t)blk * KT && t < (int64_t)(blk + 1) * KT; };
  for (int g = 1; g < ng; ++g) {
    const int b0 = Z * g, b1 = std::min(Z * g + Z, steps);  // the group's blocks [b0, b1)
    std::vector<Tile> ta, tb;
    for (int64_t I = 0; I < nT; ++I)
      for (int64_t J = 0; J <= I; ++J) {
        if (in_blk(I, b0) || in_blk(J, b0)) {
          ta.push_back(Tile{(int)I, (int)J});
          continue;
        }
        for (int bb = b0 + 1; bb < b1; ++bb)
          if (in_blk(I, bb) || in_blk(J, bb)) {
            tb.push_back(Tile{(int)I, (int)J});
            break;
          }
      }
    for (auto *t : {&ta, &tb}) {
      const std::vector<Tile> o = S > 0 ? xcd_update_order(*t, S) : *t;
      all.insert(all.end(), o.begin(), o.end());
      off.push_back((int64_t)all.size());
    }
  }
  return all;
}

// Head / tail split of the group schedule's lookahead (run_sweep_heads).
// Group G (blocks [kb, kb + z)), lists at off[G 2Z + m] (m = 0, 1 unused for G = 0):
//   m = 0          Q: the lower tiles with I and J in the group's blocks
//   m = 1          the rest of the group's cross (I or J in the group, not in Q)
//   m = 2 + i      Q_{i+1}: the tiles of Q with J in block kb + i + 1 or later
//                  (panel kb + i is applied to them as soon as it is final), i < z - 1
//   m = z + j      T_j: the tiles with I or J in block kb + j minus the head
//                  H_j = {J in block kb + j, I in blocks [kb + j, kb + z)}, 1 <= j < z
// Every list is XCD-dealt like the cross lists.
std::vector<Tile> group_head_tiles(int64_t naug, int steps, int Z, std::vector<int64_t> &off) {
  const int64_t nT = naug / UT;
  constexpr int KT = NB / UT;
  const int ng = (steps + Z - 1) / Z;
  const int S = update_order_block();
  std::vector<Tile> all;
  off.assign((size_t)ng * 2 * Z + 1, 0);
  auto blk = [&](int64_t t) { return (int)(t / KT); };
  for (int G = 0; G < ng; ++G) {
    const int kb = Z * G, z = std::min(Z, steps - kb);
    std::vector<std::vector<Tile>> L((size_t)2 * Z);
    {  // (group 0 uses only m >= 2)
      for (int64_t I = 0; I < nT; ++I)
        for (int64_t J = 0; J <= I; ++J) {
          const int bi = blk(I) - kb, bj = blk(J) - kb;  // relative blocks
          const bool ii = bi >= 0 && bi < z, ij = bj >= 0 && bj < z;
          const Tile t{(int)I, (int)J};
          if (ii && ij) {
            L[0].push_back(t);
            for (int i = 0; i + 1 < z; ++i)
              if (bj >= i + 1) L[(size_t)(2 + i)].push_back(t);
          } else if (ii || ij) {
            L[1].push_back(t);
          }
          for (int j = 1; j < z; ++j) {
            if (bi != j && bj != j) continue;
            const bool head = bj == j && bi >= j && bi < z;
            if (!head) L[(size_t)(z + j)].push_back(t);
          }
        }
    }
    for (int m = 0; m < 2 * Z; ++m) {
      const std::vector<Tile> o = S > 0 ? xcd_update_order(L[(size_t)m], S) : L[(size_t)m];
      all.insert(all.end(), o.begin(), o.end());
      off[(size_t)G * 2 * Z + m + 1] = (int64_t)all.size();
    }
  }
  return all;
}

// GEMM tiles of one launch of npan steps from block ka0 / NB (k_update_multi's
// rule) over every lower tile outside blocks [kx0, kx1), in units of one full
// tile x NB (a tile of the AUG row block computes 16 of 128 rows).
double update_gemm_tiles_group(int64_t naug, int64_t ka0, int npan, int kx0, int kx1) {
  const int64_t nT = naug / UT;
  constexpr int KT = NB / UT;
  const int64_t ta0 = ka0 / UT;
  double cnt = 0.0;
  for (int64_t I = 0; I < nT; ++I)
    for (int64_t J = 0; J <= I; ++J) {
      if (kx0 >= 0 && ((I >= kx0 * KT && I < kx1 * KT) || (J >= kx0 * KT && J < kx1 * KT)))
        continue;
      const int64_t di = I - ta0, dj = J - ta0;
      const int bi = (di >= 0 && di < npan * KT) ? (int)(di / KT) : -1;
      const int bj = (dj >= 0 && dj < npan * KT) ? (int)(dj / KT) : -1;
      const int jm = std::max(bi, bj);
      if (jm == npan - 1) continue;
      cnt += ((I == nT - 1) ? 16.0 / UT : 1.0) * (jm >= 0 ? npan - 1 - jm : npan);
    }
  return cnt;
}

std::vector<Tile> own_tiles(int64_t ntile, int T, int G, int r) {
  std::vector<Tile> t;
  for (int64_t I = 0; I < ntile; ++I)
    for (int64_t J = 0; J <= I; ++J)
      if (owns_col(J * T, G, r)) t.push_back(Tile{(int)I, (int)J});
  return t;
}

std::vector<Tile> xcd_update_order(const std::vector<Tile> &tl, int S,
                                   const std::function<double(const Tile &)> &cost) {
  // super-blocks (I / S, J / S) in row-major order; each goes whole to the
  // XCD with the fewest tiles so far, so an XCD's in-flight tiles share few
  // row / column panel blocks in its L2 (about -1 % per update launch at C2
  // against every-eighth-tile dealing, profiles/r01_pairs_ab.txt)
  constexpr int X = 8;
  std::vector<std::vector<Tile>> q(X);
  std::map<std::pair<int, int>, std::vector<Tile>> sb;
  for (const Tile &t : tl) sb[{t.I / S, t.J / S}].push_back(t);
  for (auto &kv : sb) {
    int x = 0;
    for (int i = 1; i < X; ++i)
      if (q[i].size() < q[x].size()) x = i;
    q[x].insert(q[x].end(), kv.second.begin(), kv.second.end());
  }
  if (cost)  // each XCD's dearest tiles first: its launch tail is the cheap ones
    for (auto &v : q)
      std::stable_sort(v.begin(), v.end(),
                       [&](const Tile &a, const Tile &b) { return cost(a) > cost(b); });
  size_t len = 0;
  for (auto &v : q) len = std::max(len, v.size());
  std::vector<Tile> out(len * X, Tile{-1, -1});
  for (int x = 0; x < X; ++x)
    for (size_t i = 0; i < q[x].size(); ++i) out[i * X + x] = q[x][i];
  return out;
}

// Index of (x, y) along the Hilbert curve of an n x n grid (n a power of 2)
static int64_t hilbert_index(int64_t n, int64_t x, int64_t y) {
  int64_t d = 0;
  for (int64_t s = n / 2; s > 0; s /= 2) {
    const int64_t rx = (x & s) ? 1 : 0, ry = (y & s) ? 1 : 0;
    d += s * s * ((3 * rx) ^ ry);
    if (ry == 0) {
      if (rx == 1) {
        x = n - 1 - x;
        y = n - 1 - y;
      }
      std::swap(x, y);
    }
  }
  return d;
}

bool bulk_curve() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_BULK_CURVE");
    v = e ? (atoi(e) != 0) : 0;
  }
  return v != 0;
}

std::vector<Tile> curve_update_order(const std::vector<Tile> &tl,
                                     const std::function<double(const Tile &)> &cost) {
  // The tiles along a Hilbert curve over the tile grid, cut into 8 pieces of
  // equal estimated work, one per XCD: an XCD's ~64 tiles in flight are
  // neighbours on the curve, a compact patch whose row and column panel
  // blocks its L2 shares (the S x S super-blocks of xcd_update_order are
  // dealt round-robin, so an XCD's in-flight tiles span ~16 super-columns)
  constexpr int X = 8;
  int64_t n = 1, m = 0;
  for (const Tile &t : tl) m = std::max<int64_t>(m, std::max(t.I, t.J) + 1);
  while (n < m) n *= 2;
  std::vector<std::pair<int64_t, size_t>> key(tl.size());
  for (size_t i = 0; i < tl.size(); ++i) key[i] = {hilbert_index(n, tl[i].J, tl[i].I), i};
  std::sort(key.begin(), key.end());
  // work estimate: the cost (segments) plus a launch-slot overhead
  auto wt = [&](const Tile &t) { return (cost ? cost(t) : 1.0) + 0.02; };
  double total = 0.0;
  for (const Tile &t : tl) total += wt(t);
  std::vector<std::vector<Tile>> q(X);
  double acc = 0.0;
  for (const auto &kv : key) {
    const Tile &t = tl[kv.second];
    const int x = std::min(X - 1, (int)(acc / total * X));
    q[x].push_back(t);
    acc += wt(t);
  }
  if (cost)  // each XCD's dearest tiles first (stable: curve order within a class)
    for (auto &v : q)
      std::stable_sort(v.begin(), v.end(),
                       [&](const Tile &a, const Tile &b) { return cost(a) > cost(b); });
  size_t len = 0;
  for (auto &v : q) len = std::max(len, v.size());
  std::vector<Tile> out(len * X, Tile{-1, -1});
  for (int x = 0; x < X; ++x)
    for (size_t i = 0; i < q[x].size(); ++i) out[i * X + x] = q[x][i];
  return out;
}

// Two-panel launches on k_update_multi (default; ACE_MULTI2=0: k_update_pair)
static bool multi2_on() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_MULTI2");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// Z = b.Z sweep steps per bulk launch (Z = 2 is the round-2 pair form).
// Group g = steps Z g .. Z g + z_g - 1 (the last one may be shorter), panels
// in slots k % 2Z.
//   side:  wait(bulk g-1 done) -> cross of group g+1's first block kb with
//          group g's panels (gathers panel kb) -> its chain; side2
//          meanwhile: the cross of the group's other blocks (not in kb) with
//          group g's panels.  Then for j = 1 .. z-1: the cross of block
//          kb + j with panels kb .. kb + j - 1 (gathers panel kb + j) -> its
//          chain.  -> ready(g+1)
//   main:  wait(ready g) -> the bulk launch of group g's panels over every
//          tile outside group g+1's cross.
// Launches of 1 / 2 panels run k_update / k_update_pair, 3 / 4 k_update_multi;
// every element sees the single-step schedule's MFMA chains in the same
// order, so the result is bit-identical to it (tests/test_gpu.py).
static hipError_t run_sweep_groups(const SweepBufs &b, hipStream_t st, const SweepSync *sy,
                                   const SweepTiming *tm) {
  const int64_t naug = b.ld;
  const unsigned nT = (unsigned)(naug / UT);
  const int steps = (int)(b.npad / NB);
  const int Z = b.Z;
  const int ng = (steps + Z - 1) / Z;
  const bool two = sy && sy->side && sy->nev >= 2 * steps + 1;
  hipStream_t side = two ? sy->side : st;
  const bool two2 = two && side2_on() && sy->side2 && sy->nev >= 4 * steps + 4;
  hipStream_t side2 = two2 ? sy->side2 : side;
  auto zsize = [&](int g) { return std::min(Z, steps - Z * g); };
  auto slot = [&](int k) { return k % (2 * Z); };
  auto E1 = [&](int g) { return sy->ev[2 * steps + 1 + 2 * g]; };
  auto E2 = [&](int g) { return sy->ev[2 * steps + 2 + 2 * g]; };
  const bool xg = xgather();
  auto gout = [&](int k) {
    return xg ? GatherOut{b.P[slot(k)], b.W[slot(k)], b.S[0], (int64_t)k * NB, b.ld} : no_gather();
  };
  // npan steps from block kb on a tile list (null: the row-major grid of nt
  // tiles), skipping blocks [kx0, kx1).  Two panels run k_update_multi too
  // (77.1 against 78.1 ms per C2 evaluation with k_update_pair, same box, 3
  // rounds, profiles/r03_v4_group_ab.txt); ACE_MULTI2=0 selects k_update_pair
  const bool multi2 = multi2_on();
  auto upd = [&](int npan, int kb, int kx0, int kx1, const Tile *tl, int64_t nt, GatherOut go,
                 hipStream_t s_) {
    if (nt <= 0) return;
    const int64_t ka0 = (int64_t)kb * NB;
    if (npan == 1) {  // (only ever without a skip range)
      hipLaunchKernelGGL(k_update, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A, b.ld,
                         b.W[slot(kb)], b.P[slot(kb)], b.W[slot(kb)], b.ld, ka0, -1, tl, 1, go);
    } else if (npan == 2 && !multi2) {
      hipLaunchKernelGGL(k_update_pair, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A, b.ld,
                         b.W[slot(kb)], b.P[slot(kb)], b.W[slot(kb + 1)], b.P[slot(kb + 1)], b.ld,
                         ka0, kx0, kx1, tl, go, 1, 0);
    } else {
      PanelSet ps;
      for (int j = 0; j < 4; ++j) {
        ps.R[j] = j < npan ? b.W[slot(kb + j)] : nullptr;
        ps.C[j] = j < npan ? b.P[slot(kb + j)] : nullptr;
      }
      hipLaunchKernelGGL(k_update_multi<false>, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A,
                         b.ld, ps, npan, b.ld, ka0, kx0, kx1, tl, go, 1);
    }
  };
  // blocks kb + 1 .. kb + z - 1 of a group from its own panels, each followed
  // by its chain (on `side`)
  auto inner = [&](int kb, int z) -> hipError_t {
    for (int j = 1; j < z; ++j) {
      const int k = kb + j - 1;  // xoff list k: the tiles with I or J in block k + 1
      const int64_t x0 = b.xoff[k], nx = b.xoff[k + 1] - x0;
      upd(j, kb, -1, -1, b.xtiles + x0, nx, gout(kb + j), side);
      const hipError_t r = panel_sweep(b, slot(kb + j), (int64_t)(kb + j) * NB, side, xg);
      if (r != hipSuccess) return r;
    }
    return hipSuccess;
  };
  hipError_t e;
  if (two) {
    if (!sy->ready_recorded) {
      e = hipEventRecord(sy->ev[2 * steps], st);  // inputs ready
      if (e != hipSuccess) return e;
    }
    if ((e = hipStreamWaitEvent(side, sy->ev[2 * steps], 0)) != hipSuccess) return e;
  }
  // group 0: its first panel is gathered by its chain (nothing wrote it yet)
  if ((e = panel_sweep(b, slot(0), 0, side)) != hipSuccess) return e;
  if ((e = inner(0, zsize(0))) != hipSuccess) return e;
  if (two && (e = hipEventRecord(sy->ev[0], side)) != hipSuccess) return e;
  int used = 0;
  for (int g = 0; g < ng; ++g) {
    const int kg = Z * g;
    const bool more = g + 1 < ng;
    const int kb = Z * (g + 1), zb = more ? zsize(g + 1) : 0;
    if (two && (e = hipStreamWaitEvent(st, sy->ev[2 * g], 0)) != hipSuccess) return e;
    if (more) {
      if (two) {
        if ((e = hipEventRecord(sy->ev[2 * g + 1], st)) != hipSuccess) return e;  // bulk g-1 done
        if ((e = hipStreamWaitEvent(side, sy->ev[2 * g + 1], 0)) != hipSuccess) return e;
      }
      const int64_t pa = b.poff[2 * (g + 1)], na = b.poff[2 * (g + 1) + 1] - pa;
      const int64_t pb = b.poff[2 * (g + 1) + 1], nb = b.poff[2 * (g + 1) + 2] - pb;
      if (nb > 0 && two2) {
        if ((e = hipEventRecord(E1(g + 1), side)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(side2, E1(g + 1), 0)) != hipSuccess) return e;
      }
      upd(zsize(g), kg, -1, -1, b.ptiles + pa, na, gout(kb), side);
      if (nb > 0) {
        upd(zsize(g), kg, -1, -1, b.ptiles + pb, nb, no_gather(), side2);
        if (two2 && (e = hipEventRecord(E2(g + 1), side2)) != hipSuccess) return e;
      }
      if ((e = panel_sweep(b, slot(kb), (int64_t)kb * NB, side, xg)) != hipSuccess) return e;
      if (nb > 0 && two2 && (e = hipStreamWaitEvent(side, E2(g + 1), 0)) != hipSuccess) return e;
      if ((e = inner(kb, zb)) != hipSuccess) return e;
      if (two && (e = hipEventRecord(sy->ev[2 * (g + 1)], side)) != hipSuccess) return e;
    }
    const bool timed = tm && tm->ev && used + 2 <= tm->nev;
    if (timed) (void)hipEventRecord(tm->ev[used], st);
    const int64_t grid = b.gorder ? b.glen : (b.order ? b.norder : (int64_t)nT * (nT + 1) / 2);
    const Tile *ord = b.gorder ? b.gorder + (int64_t)g * b.glen : b.order;
    const int kx0 = more ? kb : -1, kx1 = more ? kb + zb : -1;
    upd(zsize(g), kg, kx0, kx1, ord, grid, no_gather(), st);
    if (timed) {
      (void)hipEventRecord(tm->ev[used + 1], st);
      if (tm->flops)
        tm->flops[used / 2] =
            update_gemm_tiles_group(naug, (int64_t)kg * NB, zsize(g), kx0, kx1) * 2.0 * UT * UT * NB;
      used += 2;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (tm && tm->used) *tm->used = used;
  return hipSuccess;
}

// ACE_HEADS=1: the group schedule with its lookahead split into a head path
// and a tail path (run_sweep_heads)
bool heads_on() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_HEADS");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

// The group schedule with the lookahead split by what the next chain needs
// (lists from group_head_tiles; group g+1 = blocks [kb, kb + z)):
//   side (head path, the critical one): group g's panels on Q (gathers panel
//     kb's head rows) -> for each panel k = kb + j: pivot + sub-steps ->
//     panel GEMM of the rows in blocks (k, kb + z) -> panel k on Q_{j+1}
//     (gathers panel k + 1's head rows) -> ...  -> ready(g+1)
//   side2 (tail path): group g's panels on the rest of the cross -> for each
//     panel k: [after k's sub-steps] the panel GEMM of the other rows ->
//     [after k's head GEMM] T_{j+1}: panels kb .. k on block k + 1's cross
//     minus its head -> ... -> ready2(g+1)
//   main:  wait(ready g, ready2 g) -> the bulk launch of group g.
// Every tile sees the same panels in the same order with the same per-launch
// rule as run_sweep_groups, so the result is bit-identical to it; the head
// path is a chain of small launches (Q: z(z KT + 1) KT / 2 tiles) instead of
// whole block-column crosses.
static hipError_t run_sweep_heads(const SweepBufs &b, hipStream_t st, const SweepSync *sy,
                                  const SweepTiming *tm) {
  const int64_t naug = b.ld;
  const unsigned nT = (unsigned)(naug / UT);
  constexpr int KT = NB / UT;
  const int steps = (int)(b.npad / NB);
  const int Z = b.Z;
  const int ng = (steps + Z - 1) / Z;
  hipStream_t side = sy->side, side2 = sy->side2;
  auto zsize = [&](int g) { return std::min(Z, steps - Z * g); };
  auto slot = [&](int k) { return k % (2 * Z); };
  auto E2 = [&](int g) { return sy->ev[2 * steps + 2 + 2 * g]; };     // ready2(g)
  auto Egh = [&](int k) { return sy->ev[3 * steps + 3 + 2 * k]; };    // panel k's head GEMM done
  auto Esp = [&](int k) { return sy->ev[3 * steps + 4 + 2 * k]; };    // panel k's sub-steps done
  // bulk launch g done: the next-but-one group's Q waits for it on the side
  // stream directly (with the tail path's E2), not through the main stream's
  // combined event -- one cross-stream hop instead of two before each Q, the
  // GPU's idle gap at every C1 group boundary 28 -> 10 us, bitwise equal
  // (profiles/r05_v14_qdirect.txt)
  // (events 5 steps + 3 .. + 7 belong to assemble_and_sweep)
  const bool qdirect = sy->nev >= 6 * steps + 9;
  auto Eb = [&](int g) { return sy->ev[5 * steps + 9 + g]; };  // g = -1: the main stream's
                                                                // work before the sweep
  auto gout = [&](int k) {
    return GatherOut{b.P[slot(k)], b.W[slot(k)], b.S[0], (int64_t)k * NB, b.ld};
  };
  auto list = [&](int G, int m, const Tile *&p, int64_t &n) {
    const int64_t i = (int64_t)G * 2 * Z + m;
    p = b.htiles + b.hoff[i];
    n = b.hoff[i + 1] - b.hoff[i];
  };
  const bool multi2 = multi2_on();
  auto upd = [&](int npan, int kb, int kx0, int kx1, const Tile *tl, int64_t nt, GatherOut go,
                 hipStream_t s_) {
    if (nt <= 0) return;
    const int64_t ka0 = (int64_t)kb * NB;
    if (npan == 1) {
      hipLaunchKernelGGL(k_update, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A, b.ld,
                         b.W[slot(kb)], b.P[slot(kb)], b.W[slot(kb)], b.ld, ka0, -1, tl, 1, go);
    } else if (npan == 2 && !multi2) {
      hipLaunchKernelGGL(k_update_pair, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A, b.ld,
                         b.W[slot(kb)], b.P[slot(kb)], b.W[slot(kb + 1)], b.P[slot(kb + 1)], b.ld,
                         ka0, kx0, kx1, tl, go, 1, 0);
    } else {
      PanelSet ps;
      for (int j = 0; j < 4; ++j) {
        ps.R[j] = j < npan ? b.W[slot(kb + j)] : nullptr;
        ps.C[j] = j < npan ? b.P[slot(kb + j)] : nullptr;
      }
      hipLaunchKernelGGL(k_update_multi<false>, dim3((unsigned)nt), dim3(UTHREADS), 0, s_, b.A,
                         b.ld, ps, npan, b.ld, ka0, kx0, kx1, tl, go, 1);
    }
  };
  // head-path launches on Q lists: 64 x 64 quarters (k_update_q, ACE_HEADQ=1,
  // default) or the 128-tile kernels
  static const bool hq = [] {
    const char *e = getenv("ACE_HEADQ");
    return !(e && atoi(e) == 0);
  }();
  // panels k >= 1 are gathered by k_update_q launches, which sweep their D_0
  // (the blocked pivot only: the same code as k_pivot's, bit-identical)
  const bool fused_pivot = hq && ACE_PIVOT_BLK;
  // Small n (with the bulk queue): the latency-critical launches on 32 x 32
  // pieces (k_update_q4 / k_panel_gemm_q4, bit-identical): every Q launch,
  // the head panel GEMMs and each group's last tail panel GEMM -- C1 3.59 ->
  // 3.41 ms (profiles/r06_qsplit_ab.txt).  ACE_QSPLIT: 1 (default) all of
  // them, 3 the Q launches only, 2 the group-boundary Q only, 0 none.  One
  // D_0 counter per panel after the chain counters (zero when allocated,
  // reset by the last piece).
  static const int qsplit = [] {
    const char *e = getenv("ACE_QSPLIT");
    return e ? atoi(e) : 1;
  }();
  int *const qctr = (qsplit > 0 && b.bq && b.breserve > 0)
                        ? b.bq + (int64_t)((steps + Z - 1) / Z) * BQ_INTS + 2 * steps
                        : nullptr;
  auto qupd = [&](int npan, int kb, const Tile *tl, int64_t nt, GatherOut go, hipStream_t s_,
                  bool boundary = false) {
    if (nt <= 0) return;
    if (!hq) {
      upd(npan, kb, -1, -1, tl, nt, go, s_);
      return;
    }
    PanelSet ps;
    for (int j = 0; j < 4; ++j) {
      ps.R[j] = j < npan ? b.W[slot(kb + j)] : nullptr;
      ps.C[j] = j < npan ? b.P[slot(kb + j)] : nullptr;
    }
    // a launch that gathers a panel also sweeps its D_0 (k_update_q's fused
    // pivot): that panel's chain then starts at sub-step 0's panel update
    const bool fp = fused_pivot && go.k0 >= 0;
    if (qctr && (qsplit != 2 || boundary))  // small n: 32 x 32 pieces (k_update_q4)
      hipLaunchKernelGGL(k_update_q4, dim3((unsigned)(16 * nt)), dim3(256), 0, s_, b.A, b.ld, ps,
                         npan, b.ld, tl, go, fp ? b.SW : nullptr, fp ? b.piv : nullptr,
                         fp ? b.flag : nullptr, qctr + (go.k0 >= 0 ? go.k0 / NB : 0));
    else
      hipLaunchKernelGGL(k_update_q, dim3((unsigned)(4 * nt)), dim3(256), 0, s_, b.A, b.ld, ps, npan,
                         b.ld, tl, go, fp ? b.SW : nullptr, fp ? b.piv : nullptr,
                         fp ? b.flag : nullptr);
  };
  // panel k's GEMM W_i = Pn_i W_kk over row tiles [r0, r1) (head) or all the
  // others (tail); the kernel itself skips the pivot block's rows
  auto pgemm = [&](int k, int r0, int r1, bool head, hipStream_t s_, bool last = false) {
    const int n = head ? r1 - r0 : (int)nT - (r1 - r0);
    if (n <= 0) return;
    if (!head && last && qctr && qsplit == 1) {
      // the group's last tail GEMM is on the path to the next group's Q: on
      // 32 x 32 pieces (k_panel_gemm_q's chain, k_panel_gemm_t's result), the
      // rows before and after the head
      if (r0 > 0)
        hipLaunchKernelGGL(k_panel_gemm_q4, dim3((unsigned)(2 * r0 * (UT / XT)), 2 * (NB / XT)),
                           dim3(256), 0, s_, b.W[slot(k)], b.P[slot(k)], b.ld, (int64_t)k * NB, 0);
      if ((int)nT > r1)
        hipLaunchKernelGGL(k_panel_gemm_q4, dim3((unsigned)(2 * ((int)nT - r1) * (UT / XT)), 2 * (NB / XT)),
                           dim3(256), 0, s_, b.W[slot(k)], b.P[slot(k)], b.ld, (int64_t)k * NB, r1);
      return;
    }
    if (head && ACE_PGEMM_HEADQ && qctr && qsplit == 1)
      hipLaunchKernelGGL(k_panel_gemm_q4, dim3((unsigned)(2 * n * (UT / XT)), 2 * (NB / XT)), dim3(256),
                         0, s_, b.W[slot(k)], b.P[slot(k)], b.ld, (int64_t)k * NB, r0);
    else if (head && ACE_PGEMM_HEADQ)
      hipLaunchKernelGGL(k_panel_gemm_q, dim3((unsigned)(n * (UT / XT)), NB / XT), dim3(256), 0, s_,
                         b.W[slot(k)], b.P[slot(k)], b.ld, (int64_t)k * NB, r0);
    else
      hipLaunchKernelGGL(k_panel_gemm_t, dim3((unsigned)n, NB / UT), dim3(UTHREADS), 0, s_,
                         b.W[slot(k)], b.P[slot(k)], b.ld, (int64_t)k * NB, 1, 0, head ? r0 : 0,
                         head ? 1 << 30 : r0, head ? 1 << 30 : r1);
  };
  // small n: each panel's four split sub-steps in one launch (k_panel_split4),
  // its barrier counter after the bulk queues
  int *const fctr = (b.bq && b.breserve > 0 && chain_fuse()) ? b.bq + (int64_t)ng * BQ_INTS : nullptr;
  // Small n: each fused chain launch with 13 KB of extra LDS, so that no
  // bulk / cross / tail workgroup (73.7 KB) fits beside a chain workgroup
  // (77.3 KB): the chain runs alone on its 16 CUs instead of sharing each
  // with an MFMA-bound workgroup (2x slower).  With the head launches on
  // 32 x 32 pieces (ACE_QSPLIT) C1 3.34 -> 3.10 ms (profiles/r06_chain_xlds_ab.txt;
  // before them only the contention moved, r06_c1_chain_isolation_ab.txt).
  // Placement only: bit-identical.  ACE_CHAIN_XLDS=B overrides the bytes (0:
  // off), ACE_CHAIN_XLDS_J the panel mask within a group (default all),
  // ACE_CHAIN_XLDS_G0=0 leaves group 0's chains (beside the assembly) as they were.
  static const unsigned xlds = [] {
    const char *e = getenv("ACE_CHAIN_XLDS");
    return e ? (unsigned)std::max(0, atoi(e)) : 13312u;
  }();
  static const int xlds_j = [] {
    const char *e = getenv("ACE_CHAIN_XLDS_J");
    return e ? atoi(e) : -1;
  }();
  static const bool xlds_g0 = [] {
    const char *e = getenv("ACE_CHAIN_XLDS_G0");
    return !(e && atoi(e) == 0);
  }();
  auto chain = [&](int k, hipStream_t s_) {  // [pivot +] sub-steps of panel k (gathered)
    const int j = k % Z, G = k / Z;
    panel_chain(b.P[slot(k)], b.W[slot(k)], b.ld, (int64_t)k * NB, b.SW, b.S, b.piv, b.flag, 1, 0,
                s_, fused_pivot && k > 0, true, fctr ? fctr + 2 * k : nullptr,
                (fctr && qctr && (G > 0 || xlds_g0) && ((xlds_j >> j) & 1)) ? xlds : 0u);
  };
  hipError_t e;
  if (b.bq && b.breserve > 0 &&
      (e = hipMemsetAsync(b.bq, 0, (size_t)ng * BQ_INTS * sizeof(int), st)) != hipSuccess)
    return e;  // the bulk queues (k_update_multi_r), before any bulk launch
  if (!sy->ready_recorded) {
    e = hipEventRecord(sy->ev[2 * steps], st);  // inputs ready
    if (e != hipSuccess) return e;
  }
  if ((e = hipStreamWaitEvent(side, sy->ev[2 * steps], 0)) != hipSuccess) return e;
  // group G's lookahead: group G-1's panels on Q (side) and on the rest of
  // the group's cross (side2), then each panel's chain, head / tail GEMMs
  // and the next head / tail updates.  Group 0 has no previous panels: its
  // first panel is gathered by k_gather.  (A non-fused split kernel -- k_pivot
  // for every sub-step, 112 registers, 73 KB of LDS -- did not get group 0's
  // chains beside the assembly's second part: neutral,
  // profiles/r03_v5_heads_ab.txt.)
  // Small n (ACE_QFIRST, default up to n = ACE_BULK_RESERVE_N): at a group
  // boundary the next group's Q launch (its head square, K = Z NB) runs
  // alone -- the rest of the cross (side2) and the bulk launch (main) wait
  // for it.  There the chain is the critical path and the bulk is short; Q
  // beside both took 163 us instead of ~40 (C1 trace, profiles/r05_v4_*).
  const bool qfirst = q_first(naug);
  auto Eq = [&](int G) { return sy->ev[2 * steps + 1 + 2 * G]; };  // group G's Q done
  // ACE_TAIL_LAST=1 (default): group G >= 1's last tail panel GEMM on the head stream
  // after the tail path's last T update (Et(G), an event slot the direct-wait
  // schedule leaves free); the next group's Q then follows it in stream order
  // and waits for the tail path through Et(G) instead of E2(G)
  static const bool tail_last_on = [] {
    const char *e = getenv("ACE_TAIL_LAST");
    return !(e && atoi(e) == 0);
  }();
  // (small n: the chain-bound schedule with the bulk queue)
  auto tlast = [&](int G) {
    return tail_last_on && qdirect && b.bq && b.breserve > 0 && zsize(G) >= 2 &&
           !(G == 0 && sy->tail_split);
  };
  auto Et = [&](int G) { return sy->ev[2 * G + 1]; };
  hipEvent_t const Ef = sy->ev[2 * steps - 1];  // group 0's tail path + filler (odd: free too)
  // group G's first head launch (k_gather / Q); the rest by produce(G)
  auto produce_q = [&](int G) -> hipError_t {
    const int kb = Z * G;
    if (G == 0) {
      hipLaunchKernelGGL(k_gather, dim3((unsigned)(naug / 64), NB / 64), dim3(256), 0, side, b.A,
                         b.ld, (int64_t)0, b.P[slot(0)], b.W[slot(0)], b.ld, b.S[0]);
    } else {
      const Tile *tl;
      int64_t nt;
      list(G, 0, tl, nt);
      qupd(zsize(G - 1), Z * (G - 1), tl, nt, gout(kb), side, true);  // Q
    }
    return qfirst ? hipEventRecord(Eq(G), side) : hipSuccess;
  };
  auto produce = [&](int G) -> hipError_t {
    const int kb = Z * G, zb = zsize(G);
    const Tile *tl;
    int64_t nt;
    if (G > 0) {
      if (qfirst) {
        const hipError_t q = hipStreamWaitEvent(side2, Eq(G), 0);
        if (q != hipSuccess) return q;
      }
      list(G, 1, tl, nt);
      upd(zsize(G - 1), Z * (G - 1), -1, -1, tl, nt, gout(kb), side2);  // the rest of the cross
    }
    hipError_t r;
    const int hend = (kb + zb) * KT;  // head rows end (row tiles)
    // the head path (side) needs nothing of the tail path (side2): group 0's
    // tail may wait for the whole head path (sy->tail_split) -- on the CUs
    // the assembly leaves free the two would otherwise share them step by step
    const bool split = G == 0 && sy->tail_split;
    const bool tl_ = tlast(G);
    auto head = [&](int j) -> hipError_t {
      const int k = kb + j;
      chain(k, side);
      hipError_t q;
      // (the tail path waits for Esp(k) unless its last GEMM moved here, for
      // Egh(k) only before a T launch: no marker packet nobody waits for)
      const bool lastj = j + 1 == zb;
      if (!(tl_ && lastj) && (q = hipEventRecord(Esp(k), side)) != hipSuccess) return q;
      pgemm(k, (k + 1) * KT, hend, true, side);
      if ((!lastj || !tl_) && (q = hipEventRecord(Egh(k), side)) != hipSuccess) return q;
      if (tl_ && j + 1 == zb) {  // the last tail GEMM here, after the tail path's T_{zb-1}
        if ((q = hipStreamWaitEvent(side, Et(G), 0)) != hipSuccess) return q;
        pgemm(k, (k + 1) * KT, hend, false, side, true);
      }
      if (j + 1 < zb) {
        list(G, 2 + j, tl, nt);
        qupd(1, k, tl, nt, gout(k + 1), side);  // panel k on Q_{j+1}
      }
      return hipSuccess;
    };
    auto tail = [&](int j) -> hipError_t {
      const int k = kb + j;
      hipError_t q;
      if (tl_ && j + 1 == zb) return hipSuccess;  // on the head stream (above)
      if ((q = hipStreamWaitEvent(side2, Esp(k), 0)) != hipSuccess) return q;
      pgemm(k, (k + 1) * KT, hend, false, side2, j + 1 == zb);
      if (j + 1 < zb) {
        if ((q = hipStreamWaitEvent(side2, Egh(k), 0)) != hipSuccess) return q;
        list(G, zb + j + 1, tl, nt);
        upd(j + 1, kb, -1, -1, tl, nt, gout(k + 1), side2);  // T_{j+1}
        if (tl_ && j + 2 == zb && (q = hipEventRecord(Et(G), side2)) != hipSuccess) return q;
      }
      return hipSuccess;
    };
    for (int j = 0; j < zb; ++j) {
      if ((r = head(j)) != hipSuccess) return r;
      if (!split && (r = tail(j)) != hipSuccess) return r;
    }
    if ((r = hipEventRecord(sy->ev[2 * G], side)) != hipSuccess) return r;
    if (split) {
      if ((r = hipStreamWaitEvent(side2, sy->ev[2 * G], 0)) != hipSuccess) return r;
      for (int j = 0; j < zb; ++j)
        if ((r = tail(j)) != hipSuccess) return r;
    }
    if (G == 0 && sy->fill && (r = sy->fill(sy->fill_arg, side2)) != hipSuccess) return r;
    // (group 0: the next Q also needs the assembly's filler launch: Ef)
    if (G == 0 && sy->fill && tl_ && (r = hipEventRecord(Ef, side2)) != hipSuccess) return r;
    // (qdirect: E2(G) also stands for the head path, so that the main stream
    // waits for one event before each bulk launch)
    if (qdirect && !split && (r = hipStreamWaitEvent(side2, sy->ev[2 * G], 0)) != hipSuccess)
      return r;
    return hipEventRecord(E2(G), side2);
  };
  if ((e = hipStreamWaitEvent(side2, sy->tail_after ? sy->tail_after : sy->ev[2 * steps], 0)) !=
      hipSuccess)
    return e;
  if ((e = produce_q(0)) != hipSuccess || (e = produce(0)) != hipSuccess) return e;
  if (qdirect && (e = hipEventRecord(Eb(-1), st)) != hipSuccess) return e;
  int used = 0;
  for (int g = 0; g < ng; ++g) {
    const int kg = Z * g;
    const bool more = g + 1 < ng;
    const int kb = Z * (g + 1), zb = more ? zsize(g + 1) : 0;
    if (!qdirect && (e = hipStreamWaitEvent(st, sy->ev[2 * g], 0)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(st, E2(g), 0)) != hipSuccess) return e;
    if (more) {
      // Q(g+1) needs the tail path of g and bulk g-1 (A's square, the panel
      // slots it gathers into); at g = 0 the main stream's assembly instead.
      // The side2 path of g+1 needs the same (its own tail path in order, the
      // head path through E2).  Without qdirect both wait for ev[2g+1], the
      // main stream's record after all three.
      if (qdirect) {
        if ((e = hipStreamWaitEvent(side, !tlast(g) ? E2(g) : (g == 0 && sy->fill) ? Ef : Et(g), 0)) !=
            hipSuccess)
          return e;
        if ((e = hipStreamWaitEvent(side, Eb(g - 1), 0)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(side2, Eb(g - 1), 0)) != hipSuccess) return e;
      } else {
        if ((e = hipEventRecord(sy->ev[2 * g + 1], st)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(side, sy->ev[2 * g + 1], 0)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(side2, sy->ev[2 * g + 1], 0)) != hipSuccess) return e;
      }
      if ((e = produce_q(g + 1)) != hipSuccess) return e;
      if (qfirst && (e = hipStreamWaitEvent(st, Eq(g + 1), 0)) != hipSuccess) return e;
    }
    // (the bulk launch is enqueued before the rest of group g+1's lookahead:
    // at small n the host's enqueue of ~40 launches, not the device, used to
    // hold it back by ~0.5 ms; the device order is the same either way)
    const bool timed = tm && tm->ev && used + 2 <= tm->nev;
    if (timed) (void)hipEventRecord(tm->ev[used], st);
    const int64_t grid = b.gorder ? b.glen : (b.order ? b.norder : (int64_t)nT * (nT + 1) / 2);
    const Tile *ord = b.gorder ? b.gorder + (int64_t)g * b.glen : b.order;
    const int kx0 = more ? kb : -1, kx1 = more ? kb + zb : -1;
    if (b.bq && b.breserve > 0 && ord && zsize(g) > 2) {
      PanelSet ps;
      for (int j = 0; j < 4; ++j) {
        ps.R[j] = j < zsize(g) ? b.W[slot(kg + j)] : nullptr;
        ps.C[j] = j < zsize(g) ? b.P[slot(kg + j)] : nullptr;
      }
      // one workgroup per launch slot: two per CU (k_update_multi_r's occupancy)
      hipLaunchKernelGGL(k_update_multi_r<false>, dim3(2 * device_cu_count()), dim3(UTHREADS), 0, st, b.A, b.ld,
                         ps, zsize(g), b.ld, (int64_t)kg * NB, kx0, kx1, ord, grid,
                         b.bq + (int64_t)g * BQ_INTS, b.breserve, no_gather());
    } else {
      upd(zsize(g), kg, kx0, kx1, ord, grid, no_gather(), st);
    }
    if (timed) {
      (void)hipEventRecord(tm->ev[used + 1], st);
      if (tm->flops)
        tm->flops[used / 2] =
            update_gemm_tiles_group(naug, (int64_t)kg * NB, zsize(g), kx0, kx1) * 2.0 * UT * UT * NB;
      used += 2;
    }
    if (qdirect && g + 2 < ng && (e = hipEventRecord(Eb(g), st)) != hipSuccess) return e;  // Q(g+2)
    if (more && (e = produce(g + 1)) != hipSuccess) return e;
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (tm && tm->used) *tm->used = used;
  return hipSuccess;
}

hipError_t run_sweep(const SweepBufs &b, hipStream_t st, const SweepSync *sy,
                     const SweepTiming *tm) {
  if (pair_steps() && b.ptiles && b.xtiles && b.P[2 * b.Z - 1] && b.npad / NB >= 2) {
    // the group schedules (Z steps per bulk launch): head / tail lookahead
    // (default) or the round-3 group lookahead (ACE_HEADS=0)
    if (b.htiles && heads_on() && sy && sy->side && sy->side2 &&
        sy->nev >= 5 * (int)(b.npad / NB) + 3)
      return run_sweep_heads(b, st, sy, tm);
    return run_sweep_groups(b, st, sy, tm);
  }
  const int64_t naug = b.ld;
  const unsigned nT = (unsigned)(naug / UT);
  const int steps = (int)(b.npad / NB);
  // ACE_LOOKAHEAD=0: one stream, no lookahead (diagnostic: the chain
  // kernels then run alone, uncontended)
  static const int look = [] {
    const char *e = getenv("ACE_LOOKAHEAD");
    return e ? atoi(e) : 1;
  }();
  const bool two = look && sy && sy->side && sy->nev >= 2 * steps + 1;
  hipStream_t side = two ? sy->side : st;
  int used = 0;
  hipError_t e;
  if (two) {
    if (!sy->ready_recorded) {
      e = hipEventRecord(sy->ev[2 * steps], st);  // inputs ready
      if (e != hipSuccess) return e;
    }
    e = hipStreamWaitEvent(side, sy->ev[2 * steps], 0);
    if (e != hipSuccess) return e;
  }
  e = panel_sweep(b, 0, 0, side);
  if (e != hipSuccess) return e;
  if (two) {
    e = hipEventRecord(sy->ev[0], side);
    if (e != hipSuccess) return e;
  }
  for (int k = 0; k < steps; ++k) {
    const int buf = k & 1;
    const int64_t k0 = (int64_t)k * NB;
    const bool more = k + 1 < steps;
    if (two) {
      e = hipStreamWaitEvent(st, sy->ev[2 * k], 0);  // panel k done
      if (e != hipSuccess) return e;
    }
    if (more) {
      if (two) {
        e = hipEventRecord(sy->ev[2 * k + 1], st);  // bulk update k-1 done
        if (e != hipSuccess) return e;
        e = hipStreamWaitEvent(side, sy->ev[2 * k + 1], 0);
        if (e != hipSuccess) return e;
      }
      if (b.xtiles) {  // the cross of block k+1 on k_update's 128-tiles
        const int64_t x0 = b.xoff[k], nx = b.xoff[k + 1] - x0;
        hipLaunchKernelGGL(k_update, dim3((unsigned)nx), dim3(UTHREADS), 0, side, b.A, b.ld,
                           b.W[buf], b.P[buf], b.W[buf], b.ld, k0, -1, b.xtiles + x0, 1,
                           no_gather());
      } else {
        hipLaunchKernelGGL(k_update_x, dim3((unsigned)(naug / XT), 2 * (NB / XT)), dim3(256), 0,
                           side, b.A, b.ld, b.W[buf], b.P[buf], b.W[buf], b.ld, k0, k + 1, 1, 0);
      }
      e = panel_sweep(b, buf ^ 1, k0 + NB, side);
      if (e != hipSuccess) return e;
      if (two) {
        e = hipEventRecord(sy->ev[2 * (k + 1)], side);
        if (e != hipSuccess) return e;
      }
    }
    const bool timed = tm && tm->ev && used + 2 <= tm->nev;
    if (timed) (void)hipEventRecord(tm->ev[used], st);
    hipLaunchKernelGGL(k_update, dim3(b.order ? (unsigned)b.norder : nT * (nT + 1) / 2),
                       dim3(UTHREADS), 0, st, b.A, b.ld, b.W[buf], b.P[buf], b.W[buf], b.ld, k0,
                       more ? k + 1 : -1, b.order, 1, no_gather());
    if (timed) {
      (void)hipEventRecord(tm->ev[used + 1], st);
      if (tm->flops) tm->flops[used / 2] =
          update_gemm_tiles(naug, k0, more ? k + 1 : -1, false) * 2.0 * UT * UT * NB;
      used += 2;
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (tm && tm->used) *tm->used = used;
  return hipSuccess;
}

// ---- sharded step pieces (driven by ace_shard.cpp) --------------------------
int shard_row_slots(int k, int G) { return (k + G - 1) / G; }

// Rank r's all-gather operand of step k lies in place in recv (slot r), so
// the collective needs no local copy (and none at all for one rank).
static double *send_of(const ShardSweep &b, int k) {
  return b.recv + (int64_t)b.r * shard_row_slots(k, b.G) * NB * NB;
}

hipError_t shard_pack(const ShardSweep &b, int k, hipStream_t st) {
  const int64_t k0 = (int64_t)k * NB, naug = b.ld;
  if (k % b.G == b.r)
    hipLaunchKernelGGL(k_pack_lower, dim3((unsigned)((naug - k0) / 64), NB / 64), dim3(256), 0,
                       st, b.A, b.ld, b.G, k0, naug, b.low);
  const int own = k > b.r ? (k - b.r + b.G - 1) / b.G : 0;  // own blocks j < k
  if (own > 0)
    hipLaunchKernelGGL(k_pack_rows, dim3(NB / 64, NB / 64, (unsigned)own), dim3(256), 0, st, b.A,
                       b.ld, k0, send_of(b, k));
  return hipGetLastError();
}

hipError_t shard_unpack_chain(const ShardSweep &b, int k, int buf, hipStream_t st, bool own_done) {
  const int64_t k0 = (int64_t)k * NB, naug = b.ld;
  if (!(own_done && b.G == 1))
    hipLaunchKernelGGL(k_unpack_panel, dim3((unsigned)(naug / 64), NB / 64), dim3(256), 0, st,
                       b.low, b.recv, shard_row_slots(k, b.G), b.G, k0, naug, b.P[buf], b.W[buf],
                       b.ld, b.S[0], own_done ? 1 : 0, b.r);
  panel_chain(b.P[buf], b.W[buf], b.ld, k0, b.SW, b.S, b.piv, b.flag, b.G, b.r, st);
  return hipGetLastError();
}

hipError_t shard_update_cross(const ShardSweep &b, int k, int buf, hipStream_t st) {
  const int64_t naug = b.ld;
  hipLaunchKernelGGL(k_update_x, dim3((unsigned)(naug / XT), 2 * (NB / XT)), dim3(256), 0, st,
                     b.A, b.ld, b.P[buf], b.W[buf], b.W[buf], b.ld, (int64_t)k * NB, k + 1, b.G,
                     b.r);
  return hipGetLastError();
}

hipError_t shard_update_group(const ShardSweep &b, int kb, int npan, int nslot, int kx0, int kx1,
                              const Tile *tiles, int64_t nt, hipStream_t st, int kpack,
                              double *lowp, int64_t lr0, int64_t hh) {
  const int sp = kpack >= 0 ? kpack % nslot : 0;
  GatherOut go = kpack >= 0 ? pack_out(lowp ? lowp : b.low, send_of(b, kpack), b.P[sp], b.W[sp],
                                       b.S[0], (int64_t)kpack * NB, b.ld, b.G)
                            : no_gather();
  if (kpack >= 0 && hh >= 0) {  // the head or the tail part of the column (head schedule)
    go.lr0 = lr0;
    go.h = hh;
  }
  if (nt <= 0) return hipGetLastError();
  if (npan == 1) {  // (only ever without a skip range)
    const int s0 = kb % nslot;
    hipLaunchKernelGGL(k_update, dim3((unsigned)nt), dim3(UTHREADS), 0, st, b.A, b.ld, b.P[s0],
                       b.W[s0], b.W[s0], b.ld, (int64_t)kb * NB, -1, tiles, b.G, go);
    return hipGetLastError();
  }
  PanelSet ps;
  for (int j = 0; j < 4; ++j) {
    ps.R[j] = j < npan ? b.P[(kb + j) % nslot] : nullptr;
    ps.C[j] = j < npan ? b.W[(kb + j) % nslot] : nullptr;
  }
  hipLaunchKernelGGL(k_update_multi<true>, dim3((unsigned)nt), dim3(UTHREADS), 0, st, b.A, b.ld, ps,
                     npan, b.ld, (int64_t)kb * NB, kx0, kx1, tiles, go, b.G);
  return hipGetLastError();
}

// ---- the sharded head schedule's pieces (run_sweep_sharded_heads) ---------
// Owner of block k: column rows [i_lo, i_hi) (>= k0) of its block into low
// (row offset lr0, ld hh); with rows: also every rank's row pieces A[k, j < k]
// into its all-gather slot (panel 0 / the unfused path).
hipError_t shard_pack_part(const ShardSweep &b, int k, int64_t i_lo, int64_t i_hi, double *low,
                           int64_t lr0, int64_t hh, bool rows, hipStream_t st) {
  const int64_t k0 = (int64_t)k * NB, naug = b.ld;
  if (k % b.G == b.r && i_hi > i_lo)
    hipLaunchKernelGGL(k_pack_lower, dim3((unsigned)((i_hi - i_lo) / 64), NB / 64), dim3(256), 0, st,
                       b.A, b.ld, b.G, k0, naug, low, i_lo, lr0, hh);
  const int own = k > b.r ? (k - b.r + b.G - 1) / b.G : 0;
  if (rows && own > 0)
    hipLaunchKernelGGL(k_pack_rows, dim3(NB / 64, NB / 64, (unsigned)own), dim3(256), 0, st, b.A,
                       b.ld, k0, send_of(b, k));
  return hipGetLastError();
}

// Rows [i_lo, i_hi) of panel k (slot buf): from low (rows >= k0: offset lr0,
// ld hh) or from the gathered row pieces (rows < k0); own_done: the rank's
// own rows were written by its packing launch (skipped; none to do at G = 1).
hipError_t shard_unpack_part(const ShardSweep &b, int k, int buf, int64_t i_lo, int64_t i_hi,
                             const double *low, int64_t lr0, int64_t hh, bool own_done,
                             hipStream_t st) {
  if (i_hi <= i_lo || (own_done && b.G == 1)) return hipSuccess;
  const int64_t k0 = (int64_t)k * NB;
  hipLaunchKernelGGL(k_unpack_panel, dim3((unsigned)((i_hi - i_lo) / 64), NB / 64), dim3(256), 0,
                     st, low, b.recv, shard_row_slots(k, b.G), b.G, k0, b.ld, b.P[buf], b.W[buf],
                     b.ld, b.S[0], own_done ? 1 : 0, b.r, i_lo, lr0, hh);
  return hipGetLastError();
}

// Panel k's pivot sub-steps (k_pivot + the split sub-steps), no panel GEMM.
hipError_t shard_chain(const ShardSweep &b, int k, int buf, hipStream_t st) {
  panel_chain(b.P[buf], b.W[buf], b.ld, (int64_t)k * NB, b.SW, b.S, b.piv, b.flag, b.G, b.r, st,
              false, true);
  return hipGetLastError();
}

// Panel k's GEMM W_i = Pn_i W_kk over the rank's rows (k_panel_gemm_t's
// ownership rule) in row tiles [rt_lo, rt_hi) (head) or outside them (tail).
hipError_t shard_pgemm(const ShardSweep &b, int k, int buf, int rt_lo, int rt_hi, bool head,
                       hipStream_t st) {
  const int nT = (int)(b.ld / UT);
  const int n = head ? rt_hi - rt_lo : nT - (rt_hi - rt_lo);
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_panel_gemm_t, dim3((unsigned)n, NB / UT), dim3(UTHREADS), 0, st, b.W[buf],
                     b.P[buf], b.ld, (int64_t)k * NB, b.G, b.r, head ? rt_lo : 0,
                     head ? 1 << 30 : rt_lo, head ? 1 << 30 : rt_hi);
  return hipGetLastError();
}

hipError_t shard_update_main(const ShardSweep &b, int k, int buf, int kx, hipStream_t st) {
  if (b.ntiles > 0)
    hipLaunchKernelGGL(k_update, dim3((unsigned)b.ntiles), dim3(UTHREADS), 0, st, b.A, b.ld,
                       b.P[buf], b.W[buf], b.W[buf], b.ld, (int64_t)k * NB, kx, b.tiles, b.G,
                       no_gather());
  return hipGetLastError();
}

}  // namespace ace

#ifdef ACE_DIAG_WGTIME
// Diagnostic builds: this translation unit's workgroup records (ace_wgtime.h)
extern "C" long long ace_diag_wgtime(void *dst, long long cap, int reset) {
  return ace::wgt_read(dst, cap, reset);
}
#endif
