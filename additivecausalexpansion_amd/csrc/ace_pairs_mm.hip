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
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "ace_internal.h"
#include "ace_wgtime.h"

namespace ace {

// Register caps (__launch_bounds__ second argument = waves per SIMD):
// gradient 2 (LDS 2 x 33 KB at p = 64 allows 2 workgroups per CU anyway),
// assembly 3 up to PM = 32 and 2 above (3 would spill at PM = 64).
typedef double d4 __attribute__((ext_vector_type(4)));

// Pairs per scheduling group in the elementwise loops (a sched_barrier after
// every ACE_MM_PG pairs bounds live ranges; 0 = no barriers).
#ifndef ACE_MM_PG
#define ACE_MM_PG 2
#endif
// Waves per SIMD the 512-thread gradient kernel is compiled for (register cap).
#ifndef ACE_MM_GRAD_WPE
#define ACE_MM_GRAD_WPE 4
#endif
// Most GEMM2 column blocks accumulated per pass of its k-loop (QG2: the
// 512-thread form, whose register cap allowed one).
#ifndef ACE_MM_QG
#define ACE_MM_QG 4
#endif
#ifndef ACE_MM_QG2
#define ACE_MM_QG2 1
#endif
// GEMM2's last column block when PM is not a multiple of 16 (p = 20: 4 live
// features of 16): on v_mfma_f64_4x4x4_4b_f64 (ACE_GRAD_TAIL4=1, default),
// one 4-feature group per instruction at 17 cycles instead of a 16-wide
// block at 64 (profiles/r04_probe_mfma_f64.txt: 4 blocks of 4x4x4, A lane
// 16k + 4m + i, B lane 16k + 4m + j, D lane 16i + 4m + j for block m).  The
// GEMM1 result fragment is its A operand as it stands: lane (lr = 4m + i,
// lk = k) holds U[row lr][column 4kk + k] for k-step kk.
#ifndef ACE_GRAD_TAIL4
#define ACE_GRAD_TAIL4 1
#endif
#define MM_PAIR_FENCE(cb, v) \
  if (ACE_MM_PG > 0 && ((4 * (cb) + (v) + 1) % (ACE_MM_PG > 0 ? ACE_MM_PG : 1)) == 0) \
    __builtin_amdgcn_sched_barrier(0)

#define SQRT3 1.7320508075688772

// Lane-dependent select of two registers as two v_cndmask_b32 (no array
// indexing the compiler could lower to a scratch gather).
__device__ __forceinline__ double sel_f64(bool c, double a, double b) {
  const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  const unsigned lo = c ? (unsigned)ua : (unsigned)ub;
  const unsigned hi = c ? (unsigned)(ua >> 32) : (unsigned)(ub >> 32);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double sgn_mm(double x) {
  return (double)((0.0 < x) - (x < 0.0));
}

// exp(x) without the library's special-case handling: every argument here is
// lam - r2 (+ log|z| terms) or lam - sqrt3 t, finite and bounded above by the
// amplitude parameter.  x = (32 m + j) ln2/32 + r, |r| <= ln2/64:
// exp(x) = 2^m * 2^(j/32) * p(r), p the degree-6 Taylor polynomial
// (truncation < 4e-18), 2^(j/32) from a 32-entry LDS table (correctly
// rounded by the host's pow).  Arguments below about -745 give 0 like exp()
// (v_cvt_i32_f64 saturates, so even huge negative ones); never called with
// -inf (the SE path selects 0 for z = 0 before its log|z| terms matter).
__device__ const double kExp2Tab[32] = {
    1,
    1.0218971486541166,
    1.0442737824274138,
    1.0671404006768237,
    1.0905077326652577,
    1.1143867425958924,
    1.1387886347566916,
    1.1637248587775775,
    1.189207115002721,
    1.215247359980469,
    1.241857812073484,
    1.2690509571917332,
    1.2968395546510096,
    1.3252366431597413,
    1.3542555469368927,
    1.383909881963832,
    1.4142135623730951,
    1.4451808069770467,
    1.4768261459394993,
    1.5091644275934228,
    1.5422108254079407,
    1.5759808451078865,
    1.6104903319492543,
    1.6457554781539649,
    1.681792830507429,
    1.7186192981224779,
    1.7562521603732995,
    1.7947090750031072,
    1.8340080864093424,
    1.8741676341103,
    1.9152065613971474,
    1.9571441241754002};

__device__ __forceinline__ double exp_tb(double x, const double *tab) {
  const double kf = __builtin_rint(x * 46.16624130844683);  // 32 / ln2
  double r = fma(-kf, 0.02166084938653512, x);               // (ln2 / 32) hi
  r = fma(-kf, 5.9631716539705866e-12, r);                   // (ln2 / 32) lo
  const int ki = (int)kf;
  double q = 1.0 / 720.0;
  q = fma(q, r, 1.0 / 120.0);
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q * tab[ki & 31], ki >> 5);
}

// exp_tb with a degree-5 polynomial (truncation < 2.3e-15 relative) for the
// gradient's trace factors (the assembly keeps exp_tb: K enters the inverse)
__device__ __forceinline__ double exp_tb5(double x, const double *tab) {
  const double kf = __builtin_rint(x * 46.16624130844683);
  double r = fma(-kf, 0.02166084938653512, x);
  r = fma(-kf, 5.9631716539705866e-12, r);
  const int ki = (int)kf;
  double q = 1.0 / 120.0;
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q * tab[ki & 31], ki >> 5);
}

// 2^(j/128), j = 0..127, correctly rounded (Python Decimal at 60 digits)
__device__ const double kExp2Tab128[128] = {
    1.0, 1.0054299011128027, 1.0108892860517005, 1.016378314910953,
    1.0218971486541166, 1.0274459491187637, 1.0330248790212284, 1.0386341019613787,
    1.0442737824274138, 1.0499440858006872, 1.0556451783605572, 1.061377227289262,
    1.0671404006768237, 1.0729348675259756, 1.0787607977571199, 1.0846183622133092,
    1.0905077326652577, 1.0964290818163769, 1.102382583307841, 1.1083684117236787,
    1.1143867425958924, 1.1204377524096067, 1.1265216186082418, 1.1326385195987192,
    1.1387886347566916, 1.1449721444318042, 1.1511892299529827, 1.1574400736337511,
    1.1637248587775775, 1.1700437696832502, 1.1763969916502812, 1.182784710984341,
    1.189207115002721, 1.1956643920398273, 1.202156731452703, 1.2086843236265816,
    1.215247359980469, 1.2218460329727576, 1.22848053610687, 1.2351510639369334,
    1.241857812073484, 1.2486009771892048, 1.255380757024691, 1.2621973503942507,
    1.2690509571917332, 1.275941778396392, 1.2828700160787783, 1.2898358734066657,
    1.2968395546510096, 1.3038812651919358, 1.3109612115247644, 1.318079601266064,
    1.3252366431597413, 1.3324325470831615, 1.339667524053303, 1.3469417862329458,
    1.3542555469368927, 1.3616090206382248, 1.3690024229745905, 1.3764359707545302,
    1.383909881963832, 1.3914243757719262, 1.3989796725383112, 1.4065759938190154,
    1.4142135623730951, 1.4218926021691656, 1.42961333839197, 1.4373759974489824,
    1.4451808069770467, 1.4530279958490526, 1.460917794180647, 1.4688504333369818,
    1.4768261459394993, 1.4848451658727524, 1.4929077282912648, 1.5010140696264256,
    1.5091644275934228, 1.5173590411982147, 1.5255981507445384, 1.533881997840956,
    1.5422108254079407, 1.550584877685, 1.559004400237837, 1.567469639965553,
    1.5759808451078865, 1.5845382652524937, 1.593142151342267, 1.6017927556826934,
    1.6104903319492543, 1.6192351351948637, 1.6280274218573478, 1.6368674497669644,
    1.645755478153965, 1.6546917676561943, 1.6636765803267364, 1.6727101796415966,
    1.681792830507429, 1.6909247992693053, 1.7001063537185235, 1.709337763100463,
    1.718619298122478, 1.7279512309618377, 1.7373338352737062, 1.746767386199169,
    1.7562521603732995, 1.7657884359332727, 1.7753764925265212, 1.785016611318935,
    1.7947090750031072, 1.804454167806624, 1.8142521755003989, 1.8241033854070534,
    1.8340080864093424, 1.843966568958626, 1.8539791250833855, 1.864046048397789,
    1.8741676341103, 1.8843441790323345, 1.8945759815869656, 1.9048633418176741,
    1.9152065613971474, 1.925605943636125, 1.9360617934922943, 1.9465744175792332,
    1.9571441241754002, 1.9677712232331759, 1.978456026387951, 1.9891988469672663,
};
// exp for the gradient's trace factors (ACE_GRAD_EXP=2): the 128-entry
// table, |r| <= ln2/256, degree-4 Taylor (truncation < 1.3e-15 relative, the
// degree-5 / 32-entry form's class) -- one FMA fewer per pair than exp_tb5.
// The split of ln2/128 is exp_tb's ln2/32 split divided by 4 (exact).
__device__ __forceinline__ double exp_tb128(double x, const double *tab) {
  const double kf = __builtin_rint(x * 184.66496523378732);  // 128 / ln2
  double r = fma(-kf, 0.02166084938653512 * 0.25, x);          // (ln2 / 128) hi
  r = fma(-kf, 5.9631716539705866e-12 * 0.25, r);              // (ln2 / 128) lo
  const int ki = (int)kf;
  double q = 1.0 / 24.0;
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q * tab[ki & 127], ki >> 7);
}

// Table-free form for the gradient's trace factors (ACE_GRAD_EXP=1):
// x = m ln2 + r, |r| <= ln2/2, exp(r) by a degree-10 polynomial with the
// first three Taylor coefficients pinned and the rest fitted on Chebyshev
// nodes against an extended-precision exp (3.9e-16 relative over the
// interval), so the per-pair chain has no LDS lookup.
#ifndef ACE_GRAD_EXP
#define ACE_GRAD_EXP 0
#endif
__device__ __forceinline__ double exp_pl(double x) {
  const double kf = __builtin_rint(x * 1.4426950408889634);  // 1 / ln2
  double r = fma(-kf, 0.6931471805599453, x);                 // ln2 hi
  r = fma(-kf, 2.3190468138462996e-17, r);                    // ln2 lo
  double q = 2.7545674171354605e-07;
  q = fma(q, r, 2.763525742080496e-06);
  q = fma(q, r, 2.4801715258403783e-05);
  q = fma(q, r, 0.0001984118454548405);
  q = fma(q, r, 0.001388888875659234);
  q = fma(q, r, 0.008333333371438512);
  q = fma(q, r, 0.04166666666704061);
  q = fma(q, r, 0.1666666666661009);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q, (int)kf);
}
__device__ __forceinline__ double exp_grad(double x, const double *tab) {
  return ACE_GRAD_EXP == 2 ? exp_tb128(x, tab) : ACE_GRAD_EXP ? exp_pl(x) : exp_tb5(x, tab);
}
// degree-11 form of exp_pl (7e-18 relative over the interval) for the
// assembly (ACE_ASM_EXP=1): K enters the inverse
#ifndef ACE_ASM_EXP
#define ACE_ASM_EXP 2
#endif
__device__ __forceinline__ double exp_pl11(double x) {
  const double kf = __builtin_rint(x * 1.4426950408889634);
  double r = fma(-kf, 0.6931471805599453, x);
  r = fma(-kf, 2.3190468138462996e-17, r);
  double q = 2.491759739472051e-08;
  q = fma(q, r, 2.762544312686786e-07);
  q = fma(q, r, 2.75578396598084e-06);
  q = fma(q, r, 2.480150797092874e-05);
  q = fma(q, r, 0.00019841269233459403);
  q = fma(q, r, 0.0013888888927429829);
  q = fma(q, r, 0.008333333333614103);
  q = fma(q, r, 0.04166666666660212);
  q = fma(q, r, 0.16666666666666238);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q, (int)kf);
}
// 2^(j/64), j = 0..63, correctly rounded (Python Decimal at 60 digits)
__device__ const double kExp2Tab64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951,
};
// exp for the assembly (ACE_ASM_EXP=2, default): the 64-entry table, |r| <=
// ln2/128, degree-5 Taylor (truncation < 3.6e-17 relative, below half an ulp
// like exp_tb's degree 6) -- one FMA fewer per pair and slice than exp_tb
__device__ __forceinline__ double exp_tb64(double x, const double *tab) {
  const double kf = __builtin_rint(x * 92.33248261689366);  // 64 / ln2
  double r = fma(-kf, 0.02166084938653512 * 0.5, x);          // (ln2 / 64) hi
  r = fma(-kf, 5.9631716539705866e-12 * 0.5, r);              // (ln2 / 64) lo
  const int ki = (int)kf;
  double q = 1.0 / 120.0;
  q = fma(q, r, 1.0 / 24.0);
  q = fma(q, r, 1.0 / 6.0);
  q = fma(q, r, 0.5);
  q = fma(q, r, 1.0);
  q = fma(q, r, 1.0);
  return __builtin_amdgcn_ldexp(q * tab[ki & 63], ki >> 6);
}
__device__ __forceinline__ double exp_asm(double x, const double *tab) {
  return ACE_ASM_EXP == 2 ? exp_tb64(x, tab) : ACE_ASM_EXP ? exp_pl11(x) : exp_tb(x, tab);
}


// sqrt(x), x >= 0 and normal or 0 (r2 values): hardware rsq (~2^-24
// relative), one Goldschmidt step and one correction -- 0 ulp against the
// correctly rounded sqrt over 4M samples (tools/probe_trans.hip; the
// library adds a second correction and denormal rescaling).  x = 0 gives 0
// (the estimate is taken at max(x, 1e-300)).
__device__ __forceinline__ double sqrt_pk(double x) {
  const double y = __builtin_amdgcn_rsq(fmax(x, 1e-300));
  double s = x * y;
  double h = 0.5 * y;
  const double e = fma(-h, s, 0.5);
  s = fma(s, e, s);
  h = fma(h, e, h);
  const double d = fma(-s, s, x);
  return fma(d, h, s);
}

// sqrt_pk for x >= 1e-300 (the assembly clamps Matern r2 there: t = 1e-150
// gives the same 1 + sqrt3 t = 1 and exponential as t = 0 in double), without
// the clamp inside
__device__ __forceinline__ double sqrt_pk_pos(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y;
  double h = 0.5 * y;
  const double e = fma(-h, s, 0.5);
  s = fma(s, e, s);
  h = fma(h, e, h);
  const double d = fma(-s, s, x);
  return fma(d, h, s);
}

// sqrt(x) for the gradient's trace factors, x >= 1e-300: hardware rsq and
// one Goldschmidt step, ~4e-15 relative -- far inside the gradient's
// tolerance, and 3 of sqrt_pk's 9 operations fewer on the per-pair chain.
// (The assembly keeps sqrt_pk: K enters the inverse.)
__device__ __forceinline__ double sqrt_gs(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  const double s = x * y;
  const double h = 0.5 * y;
  return fma(s, fma(-h, s, 0.5), s);
}

// One slice value, the reference expressions (same as ace_pairs.hip kval):
//  SE  (src/kernel_SE_cpp.cpp:96, 119), Matern32 (src/kernel_Matern_cpp.cpp:217-227).
// Without a slice test: the loops run slice 0 with z = 1 and log|z| = 0 (an
// LDS row of ones / zeros), which gives the basis slice's value bit for bit
// (x * 1, x + 0 and 1 * 1 * x are exact).  Every pair of a slice then stays
// in one basic block (round 5: with a b == 0 branch each pair was its own
// block -- k_cross_mm at 168 VGPRs with 62 spills for Matern at PM = 20, the
// assembly tiles one block per pair).  z = 0: SE selects the reference's 0
// (log|0| = -inf makes the exponential NaN), Matern's product is 0.
template <int KIND>
__device__ __forceinline__ double kval_nb(double r2, double lam, double zlo, double zhi,
                                          double lzlo, double lzhi, const double *etab) {
  if (KIND == 0) {
    const double kz = (sgn_mm(zlo) * sgn_mm(zhi)) * exp_asm(((lam - r2) + lzlo) + lzhi, etab);
    return sel_f64(zlo == 0.0 || zhi == 0.0, 0.0, kz);
  } else {
    const double t = sqrt_pk_pos(r2);
    const double e = (1.0 + SQRT3 * t) * exp_asm(lam - SQRT3 * t, etab);
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
// Per-tile staging shared by both kernels (dynamic LDS, doubles):
//   XJ  [64][XP]      column-side covariates (gradient, PM % 16 != 0: [x | x^2])
//   XI  [64][PM+1]    row-side covariates (gradient, PM <= 32: GEMM2 epilogue)
//   Z   [B-1][64]     column-side basis values (slices 1..B-1)
//   LZ  [B-1][64]     log|z| (SE only)
//   Nc  [NS][64]      column norms s_b(x_c) = sum_i w_bi x_ci^2
//   Nr  [NS][64]      row norms s_b(x_r)
//   W   [NS][PM]      slice weights
//   Red               gradient partials of the four waves
// NS = B slice norms with the kernel weights (+ 1 with the gradient weights
// of slice B-1 for the Matern gradient).  Staged once per tile, so the slice
// loops read only LDS and registers, apart from the row values z_r, whose
// load is issued ahead of each slice's GEMM1.
// ---------------------------------------------------------------------------
// LDS pitch of the staged column covariates XJ: the dense PM + 1 (a padded
// pitch without GEMM1's 2-way ds_read_b64 conflicts measured neutral at C2,
// profiles/r03_grad_ab.txt: the kernels are bound by the fp64 dependency
// chains, not by LDS)
__host__ __device__ constexpr int xj_pitch(int PM) { return PM + 1; }

struct MmLayout {
  int etab, xj, xi, z, lz, nc, nr, w, red, red_slices, total;
};

// Gradient partials: one buffer per slice (no barrier inside the slice
// loop) when that fits in 40 KB, else two buffers and a barrier per slice.
// Per slice: [NWV][PM + 1] (x part of every feature, sum T K) and the
// column sums of U of the four row blocks, [4][64].
__host__ __device__ inline MmLayout mm_layout(int PM, int B, int KIND, bool grad, int nwave = 4) {
  MmLayout o;
  const int NS = (grad && KIND == 1) ? B + 1 : B;
  int off = 0;
  o.etab = off;
  off += (grad && ACE_GRAD_EXP == 2) ? 128 : (!grad && ACE_ASM_EXP == 2) ? 64 : 32;
  o.xj = off;
  off += 64 * xj_pitch(PM);
  o.xi = off;
  if (grad && PM <= 32) off += 64 * (PM + 1);
  o.z = off;  // row 0: slice 0's unit basis factors, rows 1..B-1: Z
  off += B * 64;
  o.lz = off;
  if (KIND == 0) off += B * 64;
  o.nc = off;
  off += NS * 64;
  o.nr = off;
  off += NS * 64;
  o.w = off;
  off += NS * PM;
  o.red = off;
  o.red_slices = 0;
  if (grad) {
    const int per = nwave * (PM + 1) + 4 * 64;
    o.red_slices = (B * per * 8 <= 40 * 1024) ? B : 2;
    off += o.red_slices * per + nwave;
  }
  o.total = off;
  return o;
}

struct MmLds {
  double *E, *XJ, *XI, *Z, *LZ, *Nc, *Nr, *W, *Red;
  int red_slices;
};

template <int PM, int KIND, bool GRAD, int NT = 256>
__device__ __forceinline__ MmLds mm_stage(double *lds, PairSide S, int B, int ZS,
                                          const double *__restrict__ wk,
                                          const double *__restrict__ wlast, int64_t R0,
                                          int64_t C0, int tid,
                                          const double *__restrict__ norms = nullptr,
                                          int64_t ldn = 0) {
  constexpr int XP = xj_pitch(PM);
  const MmLayout o = mm_layout(PM, B, KIND, GRAD, NT / 64);
  const int NS = (GRAD && KIND == 1) ? B + 1 : B;
  constexpr bool XI = GRAD && PM <= 32;
  MmLds L;
  L.E = lds + o.etab;
  L.XJ = lds + o.xj;
  L.XI = lds + o.xi;
  L.Z = lds + o.z + 64;  // slice b's row at L.Z + (b - 1) * 64, b = 0 included
  L.LZ = lds + o.lz + 64;
  L.Nc = lds + o.nc;
  L.Nr = lds + o.nr;
  L.W = lds + o.w;
  L.Red = lds + o.red;
  L.red_slices = o.red_slices;
  for (int e = tid; e < 64 * PM; e += NT) {
    const int c = e / PM, i = e - c * PM;
    const double x = S.X[(C0 + c) * PM + i];
    L.XJ[c * XP + i] = x;
    if (XI) L.XI[c * (PM + 1) + i] = S.X[(R0 + c) * PM + i];
  }
  for (int e = tid; e < (B - 1) * 64; e += NT) {
    const int bb = e >> 6, c = e & 63;
    L.Z[e] = S.Z[(C0 + c) * ZS + bb];
    if (KIND == 0) L.LZ[e] = S.LZ[(C0 + c) * ZS + bb];
  }
  if (tid < 64) {  // slice 0: z = 1, log|z| = 0 (products and sums exact)
    L.Z[tid - 64] = 1.0;
    if (KIND == 0) L.LZ[tid - 64] = 0.0;
  }
  if (GRAD && ACE_GRAD_EXP == 2) {
    for (int e = tid; e < 128; e += NT) L.E[e] = kExp2Tab128[e];
  } else if (!GRAD && ACE_ASM_EXP == 2) {
    if (tid < 64) L.E[tid] = kExp2Tab64[tid];
  } else if (tid < 32) {
    L.E[tid] = kExp2Tab[tid];
  }
  for (int e = tid; e < NS * PM; e += NT) L.W[e] = (e < B * PM) ? wk[e] : wlast[e - B * PM];
  __syncthreads();
  // norms: from the per-evaluation table (launch_slice_norms, the same
  // arithmetic once per point instead of once per tile: bit-identical), or
  // task = (side, slice, point), same accumulation order as the per-slice
  // loops they replace (i ascending, fma(x^2, w, s)).  (Round 5: issuing
  // every staging load before the first LDS store, as in k_panel_split's
  // prologue, measured 2.47 -> 2.53 ms for the assembly at C2 and left the
  // gradient tiles' prologue at 13 us -- there the tile's other workgroup
  // keeps the CU's issue busy, the latency is not exposed; not kept.)
  if (norms) {
    for (int e = tid; e < 2 * NS * 64; e += NT) {
      const int side = e / (NS * 64), rem = e - side * NS * 64;
      const int sl = rem >> 6, pt = rem & 63;
      (side == 0 ? L.Nc : L.Nr)[rem] = norms[sl * ldn + (side == 0 ? C0 : R0) + pt];
    }
  } else
  for (int e = tid; e < 2 * NS * 64; e += NT) {
    const int side = e / (NS * 64), rem = e - side * NS * 64;
    const int sl = rem >> 6, pt = rem & 63;
    const double *w = L.W + sl * PM;
    double s = 0.0;
    if (side == 0) {
#pragma unroll 4
      for (int i = 0; i < PM; ++i) {
        const double x = L.XJ[pt * XP + i];
        s = fma(x * x, w[i], s);
      }
      L.Nc[rem] = s;
    } else {
      const double *xr = XI ? L.XI + pt * (PM + 1) : S.X + (R0 + pt) * PM;
#pragma unroll 4
      for (int i = 0; i < PM; ++i) {
        const double x = xr[i];
        s = fma(x * x, w[i], s);
      }
      L.Nr[rem] = s;
    }
  }
  __syncthreads();
  return L;
}

// Row operand of GEMM1 for one lane: x_r[4 kk + lk], kept in registers up to
// PM = 32 and read from L1/L2 above.
template <int PM, bool FROM_PTR = false>
struct RowX {
  static constexpr bool REG = PM <= 32 && !FROM_PTR;
  double q[REG ? PM / 4 : 1];
  const double *g;
  __device__ __forceinline__ void load(const double *xrow, int lk) {
    g = xrow;
    if (REG) {
#pragma unroll
      for (int kk = 0; kk < PM / 4; ++kk) q[kk] = xrow[4 * kk + lk];
    }
  }
  __device__ __forceinline__ double at(int kk, int lk) const {
    return REG ? q[kk] : g[4 * kk + lk];
  }
};

// GEMM1: acc[cb][v] = sum_i w_i x_ci x_ri for the lane's 4 CB pairs
// (row r = 16 w + lr, column c = cbase + 16 cb + lk + 4 v); w in LDS.
template <int XP, int CB = 4, int PM, bool FP>
__device__ __forceinline__ void gemm1_mm(const double *sXJ, const RowX<PM, FP> &xr, const double *w,
                                         int lr, int lk, d4 (&acc)[CB], int cbase = 0) {
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) acc[cb] = d4{0.0, 0.0, 0.0, 0.0};
  const double *xj = sXJ + (cbase + lr) * XP + lk;
  double an[CB];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb) an[cb] = xj[16 * cb * XP];
  double bn = xr.at(0, lk) * w[lk];
#pragma unroll
  for (int kk = 0; kk < PM / 4; ++kk) {
    double ac[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) ac[cb] = an[cb];
    const double bop = bn;
    if (kk + 1 < PM / 4) {
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) an[cb] = xj[16 * cb * XP + 4 * (kk + 1)];
      bn = xr.at(kk + 1, lk) * w[4 * (kk + 1) + lk];
    }
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
      acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[cb], bop, acc[cb], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Slice norms of every point once per evaluation (TabView::norms): the
// per-tile staging's loop, i ascending with fma(x^2, w, s), so every tile
// reads the values it would have computed.
__global__ __launch_bounds__(256) void k_slice_norms(const double *__restrict__ X, int PM,
                                                     int64_t np, int B, int NS,
                                                     const double *__restrict__ wk,
                                                     const double *__restrict__ wlast,
                                                     double *__restrict__ norms) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)NS * np) return;
  const int b = (int)(e / np);
  const int64_t pt = e - (int64_t)b * np;
  const double *w = b < B ? wk + (int64_t)b * PM : wlast;
  const double *x = X + pt * PM;
  double s = 0.0;
  for (int i = 0; i < PM; ++i) {
    const double v = x[i];
    s = fma(v * v, w[i], s);
  }
  norms[e] = s;
}

hipError_t launch_slice_norms(const double *X, int PM, int64_t np, int B, int NS,
                              const double *wk, const double *wlast, double *norms,
                              hipStream_t st) {
  const int64_t tot = (int64_t)NS * np;
  if (tot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_slice_norms, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, X, PM,
                     np, B, NS, wk, wlast, norms);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused assembly (mode 0): lower 64-tiles of A (sigma on the diagonal,
// identity on padding) and of the Kfull copy; same outputs as
// k_assembly<PM, KIND, 0>.
// ---------------------------------------------------------------------------
// tile columns of the assembly's first part (model_pipeline): the first
// sweep group's panels' columns (sweep_group() blocks), at most all of them
static int asm_first_cols(int nt) {
  const int jb = sweep_group_n((int64_t)nt * AT + AUG) * NB / AT;
  return jb < nt ? jb : nt;
}

// Column blocks per wave of the assembly: ACE_ASM_CB = 4 (256 threads, 16
// pairs per lane) or 2 (512 threads, wave w: rows 16 (w & 3).., columns
// 32 (w >> 2)..; 8 pairs per lane), the gradient kernel's layout.
#ifndef ACE_ASM_CB
#define ACE_ASM_CB 4
#endif
constexpr int ASM_NT = 64 * 4 * (4 / ACE_ASM_CB);
// One lower 64-tile (I, J) of the assembly (k_asm_mm, k_asm_mm_q)
template <int PM, int KIND, bool LOWER = false>
__device__ __forceinline__ void asm_mm_tile(double *lds, PairSide S, int B, int ZS, const TabView &tab,
                                            double sg, double *__restrict__ out, int64_t ld,
                                            double *__restrict__ kcopy, int64_t I, int64_t J,
                                            int G) {
  if (G > 1) {
    const int64_t coff = lcol(J * AT, G) - J * AT;
    out += coff * ld;
    if (kcopy) kcopy += coff * ld;
  }
  constexpr int CB = ACE_ASM_CB;
  int tid = threadIdx.x;
  // LOWER (the persistent loop): the lane's indices opaque per tile, so the
  // compiler does not hoist every lane-derived address out of the tile loop
  if (LOWER) __asm__ volatile("" : "+v"(tid));
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int wr = w & 3, cbase = 16 * CB * (w >> 2);
  const int64_t R0 = I * AT, C0 = J * AT, n = S.n;
  const int rl = 16 * wr + lr;
  const int64_t r = R0 + rl;
  constexpr int XP = xj_pitch(PM);
  const MmLds L = mm_stage<PM, KIND, false, ASM_NT>(lds, S, B, ZS, tab.wk, tab.wk, R0, C0, tid,
                                                    tab.norms, tab.ldn);
  RowX<PM> xr;
  xr.load(S.X + r * PM, lk);
  double kf[CB][4];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) kf[cb][v] = 0.0;
  // diagonal tiles (I == J) need the r == c and r < c tests; below the
  // diagonal r > c for every pair
  auto slices = [&](auto diag) {
    constexpr bool DG = decltype(diag)::value;
    for (int b = 0; b < B; ++b) {
      // issued ahead of GEMM1, which hides the latency; slice 0 as z = 1,
      // log|z| = 0 (L.Z / L.LZ row -1), so the pairs need no slice test
      double zr = 1.0, lzr = 0.0;
      if (b > 0) {
        zr = S.Z[r * ZS + b - 1];
        if (KIND == 0) lzr = S.LZ[r * ZS + b - 1];
      }
      d4 acc[CB];
      gemm1_mm<XP, CB>(L.XJ, xr, L.W + b * PM, lr, lk, acc, cbase);
      const double sr = L.Nr[b * 64 + rl];
      const double *nc = L.Nc + b * 64 + cbase;
      const double lam = tab.lam[b];
  #pragma unroll
      for (int cb = 0; cb < CB; ++cb)
  #pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int cl = 16 * cb + lk + 4 * v;
          const int64_t c = C0 + cbase + cl;
          // Matern: r2 >= 1e-300 (sqrt_pk_pos's domain; the same K as 0)
          constexpr double R2MIN = KIND == 1 ? 1e-300 : 0.0;
          double r2 = fmax(fma(-2.0, acc[cb][v], sr + nc[cl]), R2MIN);
          if (DG && c == r) r2 = R2MIN;
          const double zc = L.Z[(b - 1) * 64 + cbase + cl];
          const double lzc = KIND == 0 ? L.LZ[(b - 1) * 64 + cbase + cl] : 0.0;
          const double kb = (DG && r < c) ? kval_nb<KIND>(r2, lam, zr, zc, lzr, lzc, L.E)
                                          : kval_nb<KIND>(r2, lam, zc, zr, lzc, lzr, L.E);
          kf[cb][v] += kb;
          MM_PAIR_FENCE(cb, v);
        }
    }
  };
  if (!LOWER && I == J) slices(std::true_type{});  // LOWER: strictly lower tiles only
  else slices(std::false_type{});
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + cbase + 16 * cb + lk + 4 * v;
      if (r < n && c < n) {
        out[r + c * ld] = (r == c) ? kf[cb][v] + sg : kf[cb][v];
        if (kcopy) kcopy[r + c * ld] = kf[cb][v];
      } else {
        out[r + c * ld] = (r == c) ? 1.0 : 0.0;  // identity padding
      }
    }
}

template <int PM, int KIND>
__global__ __launch_bounds__(ASM_NT, (ACE_ASM_CB == 2 ? 4 : PM <= 32 ? 3 : 2)) void k_asm_mm(PairSide S, int B, int ZS, TabView tab,
                                                double sig, double *__restrict__ out, int64_t ld,
                                                double *__restrict__ kcopy,
                                                const Tile *__restrict__ tiles, int G, int part,
                                                int nt, int JB) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const double sg = tab.sig ? *tab.sig : sig;  // exp(theta[0]) on the diagonal
  int64_t I, J;
  // part 1: the tiles of the first sweep group's panels' columns (J < JB =
  // Z NB / AT, column by column) -- what that group's pivot chains and
  // lookahead crosses need; part 2: the rest (the lower triangle of tiles >=
  // JB); 0: every lower tile / the list
  if (tiles || part == 0) {
    tile_of(tiles, blockIdx.x, I, J);
  } else if (part == 3) {  // the diagonal tiles of part 2 (beside k_asm_mm_q)
    I = J = JB + (int64_t)blockIdx.x;
  } else if (part == 1) {
    int64_t idx = blockIdx.x;
    J = 0;
    while (idx >= nt - J) {
      idx -= nt - J;
      ++J;
    }
    I = J + idx;
  } else {
    tile_of(nullptr, blockIdx.x, I, J);
    I += JB;
    J += JB;
  }
  asm_mm_tile<PM, KIND>(lds, S, B, ZS, tab, sg, out, ld, kcopy, I, J, G);
}

// ---------------------------------------------------------------------------
// Cross assembly on the MFMA r2 expansion (kernmat_*_cpp without a cube,
// src/kernel_SE_cpp.cpp:9-64, src/kernel_Matern_cpp.cpp:52-93; prediction's
// K_xX): tile (I, J) of the R.n x C.n block, rows from R (the reference's
// first operand X1: test points), columns from C (X2: training points),
// slices [b0, b1).  The symmetric tile's arithmetic (asm_mm_tile) with two
// point sets: per slice r2 = s_b(r) + s_b(c) - 2 sum_i w_bi x_ri x_ci, the
// cross term one GEMM1 (K = PM) on v_mfma_f64_16x16x4f64, K_b per pair on
// the VALU in the GEMM's fragment layout; both sides' slice norms computed
// per tile (i ascending, fma(x^2, w, s), as k_slice_norms).  Out of range
// rows / columns are staged as zeros and never written.  Replaces
// k_assembly<PM, KIND, 2> (lane = row, p FMAs per pair and slice on the
// VALU: 10.8 TF/s at n = 16384, nx = 4096).
// ---------------------------------------------------------------------------
template <int PM, int KIND>
__global__ __launch_bounds__(256, PM <= 32 ? 4 : 2) void k_cross_mm(PairSide R, PairSide C, int B,
                                                                   int ZS, TabView tab, int b0,
                                                                   int b1,
                                                                   double *__restrict__ out,
                                                                   int64_t ld) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  constexpr int XP = xj_pitch(PM);
  const int64_t J = blockIdx.x, I = blockIdx.y;
  const int64_t R0 = I * AT, C0 = J * AT;
  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const MmLayout o = mm_layout(PM, B, KIND, false);
  double *const E = lds + o.etab, *const XJ = lds + o.xj, *const Zc = lds + o.z + 64,
               *const LZc = lds + o.lz + 64, *const Nc = lds + o.nc, *const Nr = lds + o.nr,
               *const W = lds + o.w, *const XI = lds + o.total;
  // both sides' points staged (coalesced): the row side's slice norms are
  // then LDS loops too, not PM dependent global loads per thread
  for (int e = tid; e < 64 * PM; e += 256) {
    const int c = e / PM, i = e - c * PM;
    XJ[c * XP + i] = (C0 + c < C.n) ? C.X[(C0 + c) * PM + i] : 0.0;
    XI[c * XP + i] = (R0 + c < R.n) ? R.X[(R0 + c) * PM + i] : 0.0;
  }
  for (int e = tid; e < (B - 1) * 64; e += 256) {
    const int bb = e >> 6, c = e & 63;
    const bool ok = C0 + c < C.n;
    Zc[e] = ok ? C.Z[(C0 + c) * ZS + bb] : 0.0;
    if (KIND == 0) LZc[e] = ok ? C.LZ[(C0 + c) * ZS + bb] : 0.0;
  }
  if (tid < 64) {  // slice 0: z = 1, log|z| = 0
    Zc[tid - 64] = 1.0;
    if (KIND == 0) LZc[tid - 64] = 0.0;
    if (ACE_ASM_EXP == 2) E[tid] = kExp2Tab64[tid];
    else if (tid < 32) E[tid] = kExp2Tab[tid];
  }
  for (int e = tid; e < B * PM; e += 256) W[e] = tab.wk[e];
  __syncthreads();
  for (int e = tid; e < 2 * B * 64; e += 256) {
    const int side = e / (B * 64), rem = e - side * B * 64;
    const int sl = rem >> 6, pt = rem & 63;
    const double *wv = W + sl * PM;
    double s = 0.0;
    if (side == 0) {
#pragma unroll 4
      for (int i = 0; i < PM; ++i) {
        const double x = XJ[pt * XP + i];
        s = fma(x * x, wv[i], s);
      }
      Nc[rem] = s;
    } else {
#pragma unroll 4
      for (int i = 0; i < PM; ++i) {
        const double x = XI[pt * XP + i];
        s = fma(x * x, wv[i], s);
      }
      Nr[rem] = s;
    }
  }
  __syncthreads();
  const int rl = 16 * w + lr;
  const int64_t r = R0 + rl;
  const bool rok = r < R.n;
  RowX<PM> xr;
  xr.load(XI + rl * XP, lk);
  double kf[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) kf[cb][v] = 0.0;
  for (int b = b0; b < b1; ++b) {
    // slice 0 as z = 1, log|z| = 0 (Zc / LZc row -1 holds them): no per-pair
    // slice test (kval_nb)
    double zr = 1.0, lzr = 0.0;
    if (b > 0) {
      zr = rok ? R.Z[r * ZS + b - 1] : 0.0;
      if (KIND == 0) lzr = rok ? R.LZ[r * ZS + b - 1] : 0.0;
    }
    d4 acc[4];
    gemm1_mm<XP, 4>(XJ, xr, W + b * PM, lr, lk, acc, 0);
    const double sr = Nr[b * 64 + rl];
    const double *nc = Nc + b * 64;
    const double *zcol = Zc + (b - 1) * 64, *lzcol = LZc + (b - 1) * 64;
    const double lam = tab.lam[b];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int cl = 16 * cb + lk + 4 * v;
        constexpr double R2MIN = KIND == 1 ? 1e-300 : 0.0;
        const double r2 = fmax(fma(-2.0, acc[cb][v], sr + nc[cl]), R2MIN);
        const double zc = zcol[cl];
        const double lzc = KIND == 0 ? lzcol[cl] : 0.0;
        kf[cb][v] += kval_nb<KIND>(r2, lam, zr, zc, lzr, lzc, E);
        MM_PAIR_FENCE(cb, v);
      }
  }
  if (!rok) return;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + 16 * cb + lk + 4 * v;
      if (c < C.n) out[r + c * ld] = kf[cb][v];
    }
}

// The assembly's second part as a persistent work queue (ACE_ASM_PERSIST):
// one workgroup per launch slot takes tiles of part 2 from a device counter
// (its strictly lower tiles; the diagonal ones run as a plain grid first)
// until none are left, and the workgroups that land on a reserved CU -- the
// first `reserve` CUs of every shader engine to receive one (HW_REG_HW_ID /
// HW_REG_XCC_ID, tools/probe_hwid.hip) -- leave at once.  Those CUs then stay
// free for the first sweep group's head path (side stream), which gets no
// slot beside a full assembly grid: the CU reservation of
// round 3's masked stream, without a fourth stream.  Every workgroup reaches
// the exit (the counter runs past nblk); the tiles are those of part 2, each
// assembled exactly as by k_asm_mm (bit-identical).
template <int PM, int KIND>
__global__ __launch_bounds__(ASM_NT, (ACE_ASM_CB == 2 ? 4 : PM <= 24 ? 4 : PM <= 32 ? 3 : 2)) void k_asm_mm_q(
    PairSide S, int B, int ZS, TabView tab, double sig, double *__restrict__ out, int64_t ld,
    int *__restrict__ queue, int64_t nblk, int JB, int reserve) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  __shared__ int next;
  if (reserve > 0) {
    // at most reserve / 4 of the workgroups leave (queue[1] counts them;
    // twice the reserved slots): a misread CU id can cost speed, never tiles
    if (threadIdx.x == 0) {
      // the first `reserve` CUs of each shader engine that a workgroup lands
      // on claim the engine's slots queue[2 + 2 (4 xcc + se) + r] (CU id + 1):
      // workgroups are handed to the engines in turn and wait for a CU of
      // their own engine, so every engine keeps one, whichever are harvested
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
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
  const double sg = tab.sig ? *tab.sig : sig;
  for (;;) {
    if (threadIdx.x == 0) next = atomicAdd(queue, 1);
    __syncthreads();  // also: every wave is done with the previous tile's LDS
    const int64_t idx = next;
    __syncthreads();
    if (idx >= nblk) break;
    int64_t I, J;
    tile_of(nullptr, idx, I, J);
    asm_mm_tile<PM, KIND, true>(lds, S, B, ZS, tab, sg, out, ld, nullptr, I + JB + 1, J + JB, 1);
  }
}

// ---------------------------------------------------------------------------
// Fused gradient traces (same outputs as k_grad2): per slice b (descending),
//   GEMM1  G = X_J (w_b X_I)^T          -> r2, K_b, U = T K_b [/ (1 + sqrt(3 r~2_b))]
//   GEMM2  V = U X_J                    -> for every feature i
//          sum_rc U d_i^2 = sum_r x_ri^2 R_r + sum_c x_ci^2 C_c - 2 sum_r x_ri V_ri
//          with R_r / C_c the row / column sums of U (lane exchanges, below).
// U never leaves the registers: the GEMM1 result fragment (row r = 16w+lr,
// column c = 16cb+lk+4v) is exactly GEMM2's A fragment for k-step 4cb+v.
// The waves' per-slice partials meet in LDS; with one buffer per slice the
// slice loop has no workgroup barrier at all.
// Matern32: r~2_b uses the gradient-indexed weights, which equal slice b+1's
// kernel weights (Q1), so the factor 1 + sqrt3 t of slice b+1 is cached per
// pair; the last slice gets its own GEMM with wg[B-1].
// ---------------------------------------------------------------------------
// 1/f for f >= 1: v_rcp_f64 (~2^-24 relative) and one Newton step, <= 11
// ulp (tools/probe_trans.hip) -- ample for a factor of the trace sums.
__device__ __forceinline__ double rcp_nr_mm(double f) {
  const double q = __builtin_amdgcn_rcp(f);
  const double e = fma(-f, q, 1.0);
  return fma(q, e, q);
}

// Lane exchanges of the gradient's slice loop without the LDS crossbar: xor
// 1 / 2 / 4 / 8 inside a 16-lane row by DPP moves (xor 4 = row_half_mirror,
// then the quad reversal; xor 8 = row_ror 8), and the xor-16 / xor-32 sums
// by gfx950's v_permlane16/32_swap.  Each lane gets the same partner value
// as __shfl_xor (ds_bpermute), and a + b is commutative, so the sums are
// bit-identical to the ds_bpermute form they replaced (round 2).
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
}
// v of lane (this lane xor m), m = 1, 2, 4, 8
__device__ __forceinline__ double xor_row(double v, int m) {
  if (m == 1) return dpp64<0xB1>(v);          // quad_perm [1,0,3,2]
  if (m == 2) return dpp64<0x4E>(v);          // quad_perm [2,3,0,1]
  if (m == 4) return dpp64<0x1B>(dpp64<0x141>(v));  // xor 7, then xor 3
  return dpp64<0x128>(v);                     // row_ror 8
}
__device__ __forceinline__ double pair_sum(int a_lo, int a_hi, int b_lo, int b_hi) {
  const double a = __longlong_as_double((long long)(((unsigned long long)(unsigned)a_hi << 32) | (unsigned)a_lo));
  const double b = __longlong_as_double((long long)(((unsigned long long)(unsigned)b_hi << 32) | (unsigned)b_lo));
  return a + b;
}
// v + v(lane xor 16), v + v(lane xor 32), in every lane
__device__ __forceinline__ double add_xor16(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = (int)(unsigned)u, hi = (int)(unsigned)(u >> 32);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return pair_sum(l[0], h[0], l[1], h[1]);
}
__device__ __forceinline__ double add_xor32(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const int lo = (int)(unsigned)u, hi = (int)(unsigned)(u >> 32);
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return pair_sum(l[0], h[0], l[1], h[1]);
}

// CB = column blocks (16 wide) per wave.  CB = 4: 256 threads, every wave
// holds 16 rows x 64 columns (16 pairs per lane, 2 workgroups per CU).
// CB = 2: 512 threads, wave w holds rows 16 (w & 3).., columns 32 (w >> 2)..
// (8 pairs per lane): half the per-lane state, so twice the waves per SIMD
// hide the fp64 latencies.
//
// Per slice, with U the T-weighted derivative factors of the wave's pairs:
//   sum_rc U d_i^2 = sum_r x_ri^2 R_r + sum_c x_ci^2 C_c - 2 sum_r x_ri V_ri,
//   V = U X_J (GEMM2, ceil(PM/16) column blocks), R_r / C_c the row / column
//   sums of U.  R_r: in-lane sums + 2 shuffles.  C_c: a reduce-scatter over
//   the 16 lanes of a row group (log2 16 shuffle levels), the four row
//   blocks' sums meet in LDS and sum_c x_ci^2 C_c is formed once per slice.
template <int PM, int KIND, int CB, bool PS, bool DG>
__global__ __launch_bounds__(64 * 4 * (4 / CB), (CB == 2 ? ACE_MM_GRAD_WPE : 2)) void k_grad_mm(
    PairSide S, int B, int ZS, TabView tab, const double *__restrict__ A, int64_t ld, double sA,
    const double *__restrict__ alpha, double *__restrict__ gpart, int64_t ldg,
    const Tile *__restrict__ tiles, int G, int64_t t0) {
  ACE_WGT(7 + (DG ? 1 : 0), true);
  constexpr int NT = 64 * 4 * (4 / CB);      // threads
  constexpr int NWV = NT / 64;               // waves
  constexpr int XP = xj_pitch(PM);
  constexpr bool XIL = PM <= 32;             // row covariates staged in LDS
  constexpr int NV = PM + 1;
  constexpr int NQ = (PM + 15) / 16;         // GEMM2 16-wide column blocks
  // the last block's PM % 16 features on 4x4x4 MFMAs (NT4 groups of 4); not
  // in the Matern two-buffer form (large B), where it would spill at 128 VGPRs
  constexpr bool TAIL4 = ACE_GRAD_TAIL4 && (PM % 16) != 0 && (PS || KIND == 0);
  constexpr int NT4 = TAIL4 ? (PM % 16) / 4 : 0;
  constexpr int NQF = TAIL4 ? NQ - 1 : NQ;   // blocks on v_mfma_f64_16x16x4f64
  // GEMM2 column blocks per pass of its k-loop (one at CB = 2: register cap)
  constexpr int QG0 = CB == 2 ? (NQF < ACE_MM_QG2 ? NQF : ACE_MM_QG2) : (NQF < ACE_MM_QG ? NQF : ACE_MM_QG);
  constexpr int QG = QG0 > 0 ? QG0 : 1;  // (NQF = 0: the loop below does not run)
  constexpr int RS = PM + 1;                 // partial row: [x part | T K]
  constexpr int PER = NWV * RS + 4 * 64;     // per-slice partials (+ column sums)
  constexpr int NKK = 4 * CB;                // GEMM2 k-steps (the wave's columns / 4)
  constexpr int NVAL = 4 * CB;               // pairs per lane
  extern __shared__ __attribute__((aligned(16))) double lds[];
  // DG: diagonal tiles (the r == c and r < c tests), else strictly lower
  // tiles (r > c for every pair).  Partial slot t = t0 + block; the tile is
  // tiles[t] (a list with its diagonal tiles first) or, without a list,
  // (block, block) / the block-th strictly lower tile.
  const int64_t t = t0 + blockIdx.x;
  int64_t I, J;
  if (tiles) {
    I = tiles[t].I;
    J = tiles[t].J;
    if (I < 0) {  // padding of an XCD-dealt list: an all-zero partial row
      for (int64_t e = threadIdx.x; e < ldg; e += NT) gpart[t * ldg + e] = 0.0;
      return;
    }
  } else if (DG) {
    I = J = blockIdx.x;
  } else {
    tile_of(nullptr, blockIdx.x, I, J);  // row-major triangle incl. diagonal, shifted:
    ++I;                                 // (I, J) with J <= I  ->  (I + 1, J), J < I + 1
  }
  if (G > 1) A += (lcol(J * AT, G) - J * AT) * ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int wr = w & 3;                      // row block of the wave
  const int cbase = 16 * CB * (w >> 2);      // first column of the wave
  const int64_t R0 = I * AT, C0 = J * AT, n = S.n;
  const int rl = 16 * wr + lr;
  const int64_t r = R0 + rl;
  const bool rvalid = r < n;
  const double *wlast = (KIND == 1) ? tab.wg + (B - 1) * PM : tab.wk;
  // the tile's A and alpha values are loaded before the staging, so their
  // latency overlaps the staging loads and barriers
  double av[CB][4], alc[CB][4];
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + cbase + 16 * cb + lk + 4 * v;
      const bool ok = rvalid && c < n && !(I == J && c > r);
      av[cb][v] = ok ? A[r + c * ld] : 0.0;
      alc[cb][v] = ok ? alpha[c] : 0.0;
    }
  const double ar = rvalid ? alpha[r] : 0.0;
  const MmLds L = mm_stage<PM, KIND, true, NT>(lds, S, B, ZS, tab.wk, wlast, R0, C0, tid,
                                               tab.norms, tab.ldn);
  ACE_WGT_MARK(0);
  // T = w_rc (sA A[r,c] - alpha_r alpha_c), w = 2 off the diagonal (lower pairs)
  double tv[CB][4];
  double tr = 0.0;
#pragma unroll
  for (int cb = 0; cb < CB; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int64_t c = C0 + cbase + 16 * cb + lk + 4 * v;
      double x = 0.0;
      if (rvalid && c < n && !(I == J && c > r)) {
        x = sA * av[cb][v] - ar * alc[cb][v];
        if (c == r) tr += x;
        else x *= 2.0;
      }
      tv[cb][v] = x;
    }
  RowX<PM, XIL> xr;  // x_r from the staged rows when they are in LDS
  xr.load(XIL ? L.XI + rl * (PM + 1) : S.X + r * PM, lk);
  // tail (TAIL4): this lane's output element of group t is row 16 wr + 4 m4
  // + i4, feature 16 NQF + 4 t + j4; its covariate is the same every slice
  const int i4 = lane >> 4, m4 = (lane >> 2) & 3, j4 = lane & 3;
  double x4[NT4 > 0 ? NT4 : 1];
  if (TAIL4) {
    const int rr = 16 * wr + 4 * m4 + i4;
#pragma unroll
    for (int t4 = 0; t4 < NT4; ++t4) {
      const int nn = 16 * NQF + 4 * t4 + j4;
      x4[t4] = XIL ? L.XI[rr * (PM + 1) + nn] : (R0 + rr < n ? S.X[(R0 + rr) * PM + nn] : 0.0);
    }
  }
  double fc[CB][4];  // Matern: 1 + sqrt3 t of slice b+1
  d4 acc[CB];
  if (KIND == 1) {  // Matern, last slice: r~2 with its own weights
    gemm1_mm<XP, CB>(L.XJ, xr, L.W + B * PM, lr, lk, acc, cbase);
    const double sr = L.Nr[B * 64 + rl];
    const double *nc = L.Nc + B * 64 + cbase;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int cl = 16 * cb + lk + 4 * v;
        double rt2 = fmax(fma(-2.0, acc[cb][v], sr + nc[cl]), 0.0);
        if (DG && C0 + cbase + cl == r) rt2 = 0.0;
        fc[cb][v] = 1.0 + sqrt_pk(3.0 * rt2);
      }
  }
  // gpart[b][i] of this tile from slice b's partials: the waves' x parts,
  // sum_c x_ci^2 C_c, and (i == PM) the waves' sums of T K
  // summed: cc[c] already holds the four row blocks' column sums
  // (cc[c] + cc[64 + c]) + (cc[128 + c] + cc[192 + c]) (summed once per slice)
  auto finish = [&](int b, const double *red, int i, bool summed = false) {
    double g = 0.0;
    if (i < PM) {
#pragma unroll
      for (int q = 0; q < NWV; ++q) g += red[q * RS + i];
      const double *cc = red + NWV * RS;
      double gc = 0.0;
      if (summed) {
        for (int c = 0; c < 64; ++c) {
          const double x = L.XJ[c * XP + i];
          gc = fma(x * x, cc[c], gc);
        }
      } else {
        for (int c = 0; c < 64; ++c) {
          const double x = L.XJ[c * XP + i];
          gc = fma(x * x, (cc[c] + cc[64 + c]) + (cc[128 + c] + cc[192 + c]), gc);
        }
      }
      g += gc;
    } else {
#pragma unroll
      for (int q = 0; q < NWV; ++q) g += red[q * RS + PM];
    }
    gpart[t * ldg + (int64_t)b * NV + i] = g;
  };
  // PS: one partial buffer per slice (the host checked L.red_slices == B)
  constexpr bool per_slice = PS;
  // Slice 0 runs the basis-slice code with z = 1 and log|z| = 0 (an LDS row
  // of ones / zeros; exact), so no per-pair code tests b: a lane's pairs are
  // one straight-line block the scheduler can interleave (a b == 0 test made
  // every pair its own basic block, running its dependent fp64 chain alone)
  // ACE_DIAG_GRAD (timing diagnostics only, results wrong): 1 runs no slice,
  // 2 only the last slice; bits 4 / 8 / 16 / 32 drop the sqrt / exp /
  // reciprocal / GEMM2 of the Matern slice loop; bit 64 the per-slice
  // partials' combination after the loop (column-sum combine + feature dots)
#ifndef ACE_DIAG_GRAD
#define ACE_DIAG_GRAD 0
#endif
  const int bstop = (ACE_DIAG_GRAD & 3) == 1 ? B : (ACE_DIAG_GRAD & 3) == 2 ? B - 1 : 0;
#pragma unroll 1
  for (int b = B - 1; b >= bstop; --b) {
    double *red = L.Red + (per_slice ? b : (b & 1)) * PER;
    double zr = 1.0, lzr = 0.0;  // issued ahead of GEMM1, which hides the latency
    if (b > 0) {
      zr = S.Z[r * ZS + b - 1];
      if (KIND == 0) lzr = S.LZ[r * ZS + b - 1];
    }
    // waves raise their priority while issuing the two GEMM chains
    __builtin_amdgcn_s_setprio(2);
    gemm1_mm<XP, CB>(L.XJ, xr, L.W + b * PM, lr, lk, acc, cbase);
    __builtin_amdgcn_s_setprio(0);
    const double sr = L.Nr[b * 64 + rl];
    const double *nc = L.Nc + b * 64 + cbase;
    const double *zcol = L.Z + (b - 1) * 64 + cbase;
    const double *lzcol = L.LZ + (b - 1) * 64 + cbase;
    const double lam = tab.lam[b];
    double gl = 0.0, rs = 0.0;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int cl = 16 * cb + lk + 4 * v;
        const int64_t c = C0 + cbase + cl;
        // Matern: r2 >= 1e-300 (sqrt_gs's domain); 1e-300 and 0 give the
        // same f = 1 and exponential in double
        constexpr double R2MIN = KIND == 1 ? 1e-300 : 0.0;
        double r2 = fmax(fma(-2.0, acc[cb][v], sr + nc[cl]), R2MIN);
        if (DG && c == r) r2 = R2MIN;
        const double zc = zcol[cl];
        const double lzc = KIND == 0 ? lzcol[cl] : 0.0;
        const bool rlo = DG && r < c;
        const double zlo = rlo ? zr : zc, zhi = rlo ? zc : zr;
        double kb, f = 1.0;
        if (KIND == 0) {
          // log|0| = -inf makes the exponential NaN: a select (not a branch)
          // puts the reference's 0 there
          const double kz = (sgn_mm(zlo) * sgn_mm(zhi)) *
                            exp_grad(((lam - r2) + (rlo ? lzr : lzc)) + (rlo ? lzc : lzr), L.E);
          kb = sel_f64(zlo == 0.0 || zhi == 0.0, 0.0, kz);
        } else {
          const double tt = (ACE_DIAG_GRAD & 4) ? r2 : sqrt_gs(r2);
          f = 1.0 + SQRT3 * tt;
          const double e = (ACE_DIAG_GRAD & 8) ? f * (lam - SQRT3 * tt) : f * exp_grad(lam - SQRT3 * tt, L.E);
          // z = 0 gives a zero product (of either sign: it only enters sums)
          kb = (e * zlo) * zhi;
        }
        const double tk = tv[cb][v] * kb;
        gl += tk;
        double u;
        if (KIND == 0) {
          u = tk;
        } else {
          u = (ACE_DIAG_GRAD & 16) ? tk * fc[cb][v] : tk * rcp_nr_mm(fc[cb][v]);
          fc[cb][v] = f;
        }
        acc[cb][v] = u;
        rs += u;
        MM_PAIR_FENCE(cb, v);
      }
    // R_r: row sums of U over the wave's columns (lanes of one lr hold the 4 quarters)
    rs = add_xor16(rs);
    rs = add_xor32(rs);
    double Rv[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) Rv[v] = __shfl(rs, lk + 4 * v, 64);  // row 16 wr + lk + 4v
    __builtin_amdgcn_s_setprio(2);
    // GEMM2: V = U X_J, QG column blocks per pass of the k-loop
#pragma unroll
    for (int q0 = 0; q0 < ((ACE_DIAG_GRAD & 32) ? 0 : NQF); q0 += QG) {
      d4 a2[QG];
#pragma unroll
      for (int j = 0; j < QG; ++j) a2[j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const double *xc = L.XJ + (cbase + 4 * kk + lk) * XP;
#pragma unroll
        for (int j = 0; j < QG; ++j) {
          const int nn = 16 * (q0 + j) + lr;
          if (q0 + j < NQF)
            a2[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[kk >> 2][kk & 3],
                                                         nn < PM ? xc[nn] : 0.0, a2[j], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // a2[j][v] = V[row 16 wr + lk + 4 v][feature 16 (q0 + j) + lr]
#pragma unroll
      for (int j = 0; j < QG; ++j) {
        if (q0 + j >= NQF) continue;
        const int nn = 16 * (q0 + j) + lr;
        double part = 0.0;
        if (nn < PM) {
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int rr = 16 * wr + lk + 4 * v;
            const double x = XIL ? L.XI[rr * (PM + 1) + nn] : S.X[(R0 + rr) * PM + nn];
            part += fma(x * x, Rv[v], -2.0 * x * a2[j][v]);
          }
        }
        part = add_xor16(part);
        part = add_xor32(part);
        if (lk == 0 && nn < PM) red[w * RS + nn] = part;
      }
    }
    if (TAIL4 && !(ACE_DIAG_GRAD & 32)) {
      // V[row 4 m4 + i4][feature 16 NQF + 4 t + j4] = sum_c U X_J over the
      // wave's columns: 4x4x4 MFMAs, k-step kk = columns 4 kk .. 4 kk + 3
      double a4[NT4 > 0 ? NT4 : 1];
#pragma unroll
      for (int t4 = 0; t4 < NT4; ++t4) a4[t4] = 0.0;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const double *xc = L.XJ + (cbase + 4 * kk + i4) * XP + 16 * NQF + j4;
#pragma unroll
        for (int t4 = 0; t4 < NT4; ++t4)
          a4[t4] = __builtin_amdgcn_mfma_f64_4x4x4f64(acc[kk >> 2][kk & 3], xc[4 * t4], a4[t4], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      // R of row 4 m4 + i4 (rs holds row lr's sum in every lane of that lr)
      const double R4 = __shfl(rs, 4 * m4 + i4, 64);
#pragma unroll
      for (int t4 = 0; t4 < NT4; ++t4) {
        const double x = x4[t4];
        double part = fma(x * x, R4, -2.0 * x * a4[t4]);
        part = add_xor16(part);   // over i4
        part = add_xor32(part);
        part += xor_row(part, 4);  // over m4
        part += xor_row(part, 8);
        if (lane < 4) red[w * RS + 16 * NQF + 4 * t4 + j4] = part;
      }
    }
    __builtin_amdgcn_s_setprio(0);
    // C_c: column sums of U over the wave's 16 rows, reduce-scatter over lr
    {
      // (after GEMM2: U's registers are free again)
      double cv[NVAL];
#pragma unroll
      for (int k = 0; k < NVAL; ++k) cv[k] = acc[k >> 2][k & 3];
      int kk0 = 0, cnt = NVAL;
#pragma unroll
      for (int m = 8; m >= 1; m >>= 1) {
        if (cnt > 1) {
          const int h = cnt / 2;
          const bool up = (lr & m) != 0;
#pragma unroll
          for (int j = 0; j < h; ++j) {
            // both halves into named values first: selecting between the
            // array elements themselves (a lane-dependent index) made the
            // compiler spill cv to scratch and gather it back per lane
            const double lo = cv[j], hi = cv[j + h];
            const double mine = sel_f64(up, hi, lo);
            const double other = sel_f64(up, lo, hi);
            cv[j] = mine + xor_row(other, m);
          }
          if (up) kk0 += h;
          cnt = h;
        } else {
          cv[0] += xor_row(cv[0], m);
        }
      }
      if ((lr & (16 / NVAL - 1)) == 0)
        red[NWV * RS + wr * 64 + cbase + 16 * (kk0 >> 2) + lk + 4 * (kk0 & 3)] = cv[0];
    }
    gl += xor_row(gl, 1);
    gl += xor_row(gl, 2);
    gl += xor_row(gl, 4);
    gl += xor_row(gl, 8);
    gl = add_xor16(gl);
    gl = add_xor32(gl);
    if (lane == 0) red[w * RS + PM] = gl;
    if (!per_slice) {
      __syncthreads();  // the waves' partials of slice b are in red
      if (tid <= PM) finish(b, red, tid);
    }
  }
  ACE_WGT_MARK(1);
  // trace of T
  tr += xor_row(tr, 1);
  tr += xor_row(tr, 2);
  tr += xor_row(tr, 4);
  tr += xor_row(tr, 8);
  tr = add_xor16(tr);
  tr = add_xor32(tr);
  double *str = L.Red + L.red_slices * PER;
  if (lane == 0) str[w] = tr;
  __syncthreads();
  if (per_slice && !(ACE_DIAG_GRAD & 64)) {  // all slices' partials at once
    // each slice's four row-block column sums added once (same expression,
    // so bit-identical), not once per feature
    for (int e = tid; e < B * 64; e += NT) {
      double *cc = L.Red + (e >> 6) * PER + NWV * RS;
      const int c = e & 63;
      cc[c] = (cc[c] + cc[64 + c]) + (cc[128 + c] + cc[192 + c]);
    }
    __syncthreads();
    for (int e = tid; e < B * NV; e += NT) {
      const int bb = e / NV, i = e - bb * NV;
      finish(bb, L.Red + bb * PER, i, true);
    }
  }
  if (tid == 0) {
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < NWV; ++q) s += str[q];
    gpart[t * ldg + (int64_t)B * NV] = s;
  }
}

// Column blocks per wave of the gradient kernel: CB = 2 (512 threads, 8
// pairs per lane, 4 waves per SIMD) wherever it fits 128 VGPRs without
// spilling -- every SE case and Matern up to PM = 32 -- else CB = 4.
// ACE_MM_GRAD_CB=4 forces the 256-thread form (A/B switch).
#ifndef ACE_MM_GRAD_CB
#define ACE_MM_GRAD_CB 2
#endif
__host__ __device__ constexpr int grad_cb(int PM, int kind) {
  return (ACE_MM_GRAD_CB == 2 && (kind == 0 || PM <= 32)) ? 2 : 4;
}

template <int PM, int KIND, bool PS, bool DG>
static hipError_t grad_mm_launch_ps(PairSide S, int B, int ZS, TabView tab, const double *A,
                                    int64_t ld, double sA, const double *alpha, double *gpart,
                                    hipStream_t st, const Tile *tiles, int64_t nblk, int G,
                                    size_t lds, int64_t t0) {
  constexpr int CB = grad_cb(PM, KIND);
  constexpr int NT = 64 * 4 * (4 / CB);
  if (nblk == 0) return hipSuccess;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute((const void *)k_grad_mm<PM, KIND, CB, PS, DG>,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((k_grad_mm<PM, KIND, CB, PS, DG>), dim3((unsigned)nblk), dim3(NT), lds, st,
                     S, B, ZS, tab, A, ld, sA, alpha, gpart, (int64_t)grad_part_cols(PM, B), tiles,
                     G, t0);
  return hipGetLastError();
}

// Two launches: the diagonal tiles (with the r == c / r < c tests) and the
// strictly lower ones.  Without a list: slots [0, nt) diagonal, [nt, ...)
// strictly lower.  With a list: its first ndiag entries are the diagonal
// tiles (ndiag < 0: not partitioned -> one launch of the general form).
template <int PM, int KIND, bool PS>
static hipError_t grad_mm_launch_dg(PairSide S, int B, int ZS, TabView tab, const double *A,
                                    int64_t ld, double sA, const double *alpha, double *gpart,
                                    hipStream_t st, const Tile *tiles, int64_t nslot,
                                    int64_t ndiag, int G, size_t lds) {
  if (tiles && ndiag < 0)
    return grad_mm_launch_ps<PM, KIND, PS, true>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles,
                                                 nslot, G, lds, 0);
  // strictly lower tiles first: the diagonal launch (one tile per CU) is
  // then a short tail instead of sharing the machine with the side stream's
  // Kfull * alpha pass at the start of the gradient phase
  const int64_t nd = tiles ? ndiag : (S.n + AT - 1) / AT;
  hipError_t e = grad_mm_launch_ps<PM, KIND, PS, false>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st,
                                                        tiles, nslot - nd, G, lds, nd);
  if (e != hipSuccess) return e;
  return grad_mm_launch_ps<PM, KIND, PS, true>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles,
                                               nd, G, lds, 0);
}

template <int PM, int KIND>
static hipError_t grad_mm_launch(PairSide S, int B, int ZS, TabView tab, const double *A,
                                 int64_t ld, double sA, const double *alpha, double *gpart,
                                 hipStream_t st, const Tile *tiles, int64_t nslot, int64_t ndiag,
                                 int G) {
  constexpr int CB = grad_cb(PM, KIND);
  constexpr int NT = 64 * 4 * (4 / CB);
  const MmLayout o = mm_layout(PM, B, KIND, true, NT / 64);
  const size_t lds = (size_t)o.total * sizeof(double);
  return o.red_slices == B
             ? grad_mm_launch_dg<PM, KIND, true>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles,
                                                 nslot, ndiag, G, lds)
             : grad_mm_launch_dg<PM, KIND, false>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st,
                                                  tiles, nslot, ndiag, G, lds);
}

template <int PM>
static hipError_t grad_mm_pm(int kind, PairSide S, int B, int ZS, TabView tab, const double *A,
                             int64_t ld, double sA, const double *alpha, double *gpart,
                             hipStream_t st, const Tile *tiles, int64_t ntiles, int64_t ndiag,
                             int G) {
  const int64_t nt = (S.n + AT - 1) / AT;
  const int64_t nslot = tiles ? ntiles : nt * (nt + 1) / 2;
  if (nslot == 0) return hipSuccess;
  return kind == 0 ? grad_mm_launch<PM, 0>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles,
                                           nslot, ndiag, G)
                   : grad_mm_launch<PM, 1>(S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles,
                                           nslot, ndiag, G);
}

// Whether the per-tile staging of the MFMA kernels fits the 160 KB of LDS
// a gfx950 workgroup can use (up to 80 KB two workgroups share a CU; above
// it one, at large B and p).  Every supported shape (B <= 32, p <= 64)
// fits: the largest, SE at PM = 64 and B = 32, stages 127 KB.
bool mm_lds_ok(int PM, int B, int kind, bool grad) {
  const int nwave = grad ? 4 * (4 / grad_cb(PM, kind)) : 4;
  return (int64_t)mm_layout(PM, B, kind == 0 ? 0 : 1, grad, nwave).total *
             (int64_t)sizeof(double) <=
         160 * 1024;
}

hipError_t launch_grad_mm(int kind, int PM, PairSide S, int B, int ZS, TabView tab,
                          const double *A, int64_t ld, double sA, const double *alpha,
                          double *gpart, hipStream_t st, const Tile *tiles, int64_t ntiles, int G,
                          int64_t ndiag) {
  switch (PM) {
#define ACE_CASE(P) \
  case P:           \
    return grad_mm_pm<P>(kind, S, B, ZS, tab, A, ld, sA, alpha, gpart, st, tiles, ntiles, ndiag, G);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

template <int PM>
static hipError_t asm_mm_pm(int kind, PairSide S, int64_t npad, int B, int ZS, TabView tab,
                            double sig, double *out, int64_t ld, double *kcopy, hipStream_t st,
                            const Tile *tiles, int64_t ntiles, int G, int part) {
  const int64_t nt = npad / AT, JB = asm_first_cols((int)nt);
  if (tiles) part = 0;
  const int64_t nblk = tiles ? ntiles
                       : part == 1 ? JB * nt - JB * (JB - 1) / 2
                       : part == 2 ? (nt - JB) * (nt - JB + 1) / 2
                       : part == 3 ? nt - JB
                                   : nt * (nt + 1) / 2;
  if (nblk == 0) return hipSuccess;
  const size_t lds = (size_t)mm_layout(PM, B, kind == 0 ? 0 : 1, false).total * sizeof(double);
  if (lds > 65536) {
    const void *f = kind == 0 ? (const void *)k_asm_mm<PM, 0> : (const void *)k_asm_mm<PM, 1>;
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if (kind == 0)
    hipLaunchKernelGGL((k_asm_mm<PM, 0>), dim3((unsigned)nblk), dim3(ASM_NT), lds, st, S, B, ZS,
                       tab, sig, out, ld, kcopy, tiles, G, part, (int)nt, (int)JB);
  else
    hipLaunchKernelGGL((k_asm_mm<PM, 1>), dim3((unsigned)nblk), dim3(ASM_NT), lds, st, S, B, ZS,
                       tab, sig, out, ld, kcopy, tiles, G, part, (int)nt, (int)JB);
  return hipGetLastError();
}

template <int PM>
static hipError_t asm_mm_persist_pm(int kind, PairSide S, int64_t npad, int B, int ZS, TabView tab,
                                    double sig, double *out, int64_t ld, hipStream_t st, int *queue,
                                    int reserve, int slots, bool fill) {
  const int64_t nt = npad / AT, JB = asm_first_cols((int)nt);
  const int64_t nblk = (nt - JB) * (nt - JB - 1) / 2;  // strictly lower tiles of part 2
  if (nt - JB <= 0) return hipSuccess;
  const size_t lds = (size_t)mm_layout(PM, B, kind == 0 ? 0 : 1, false).total * sizeof(double);
  if (lds > 65536) {
    const void *f = kind == 0 ? (const void *)k_asm_mm_q<PM, 0> : (const void *)k_asm_mm_q<PM, 1>;
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  // part 2's diagonal tiles (the r == c / r < c path) as a plain grid first;
  // a filler launch (fill: `slots` more workgroups on another stream, none
  // reserved) only joins the queue of the running one
  hipError_t e = fill ? hipSuccess
                      : asm_mm_pm<PM>(kind, S, npad, B, ZS, tab, sig, out, ld, nullptr, st, nullptr, 0, 1, 3);
  if (e != hipSuccess || nblk == 0) return e;
  if (fill) reserve = 0;
  if (kind == 0)
    hipLaunchKernelGGL((k_asm_mm_q<PM, 0>), dim3((unsigned)slots), dim3(ASM_NT), lds, st, S, B, ZS,
                       tab, sig, out, ld, queue, nblk, (int)JB, reserve);
  else
    hipLaunchKernelGGL((k_asm_mm_q<PM, 1>), dim3((unsigned)slots), dim3(ASM_NT), lds, st, S, B, ZS,
                       tab, sig, out, ld, queue, nblk, (int)JB, reserve);
  return hipGetLastError();
}

// Workgroup slots of k_asm_mm_q (occupancy x CUs), 0 if unknown; cached per
// (device, kind, B): the queries cost host time every evaluation otherwise
template <int PM>
static int asm_mm_slots(int kind, int B) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  static std::mutex mu;
  static std::map<std::tuple<int, int, int>, int> cache;
  const auto key = std::make_tuple(dev, kind, B);
  {
    std::lock_guard<std::mutex> g(mu);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const size_t lds = (size_t)mm_layout(PM, B, kind == 0 ? 0 : 1, false).total * sizeof(double);
  const void *f = kind == 0 ? (const void *)k_asm_mm_q<PM, 0> : (const void *)k_asm_mm_q<PM, 1>;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, f, ASM_NT, lds) != hipSuccess) return 0;
  // never more than the register file holds (the occupancy API can report
  // one workgroup per CU too many, MI355X_MICROARCH.md): a workgroup that does
  // not fit at launch would be dispatched later into a reserved CU's slot
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, f) == hipSuccess && fa.numRegs > 0) {
    const int alloc = (fa.numRegs + 7) / 8 * 8;
    const int waves = std::min(8, 512 / alloc);  // per SIMD
    per = std::min(per, waves * 4 / (ASM_NT / 64));
  }
  std::lock_guard<std::mutex> g(mu);
  cache[key] = per * ncu;
  return per * ncu;
}

int assembly_persist_per_cu(int kind, int PM, int B) {
  int dev = 0, ncu = 0;  // (an attribute read: cheap, unlike the occupancy query)
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
    return 0;
  switch (PM) {
#define ACE_CASE(P) \
  case P: return asm_mm_slots<P>(kind, B) / ncu;
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return 0;
  }
}

#ifdef ACE_DIAG_WGTIME
}  // namespace ace
extern "C" long long ace_diag_wgtime_pairs(void *dst, long long cap, int reset) {
  return ace::wgt_read(dst, cap, reset);
}
namespace ace {
#endif

hipError_t launch_assembly_persist(int kind, int PM, PairSide S, int64_t npad, int B, int ZS,
                                   TabView tab, double sig, double *out, int64_t ld,
                                   hipStream_t st, int *queue, int reserve, int fill) {
  switch (PM) {
#define ACE_CASE(P)                                                                          \
  case P: {                                                                                  \
    const int slots = fill > 0 ? fill : asm_mm_slots<P>(kind, B);                            \
    if (slots <= 0) return hipErrorInvalidValue;                                             \
    return asm_mm_persist_pm<P>(kind, S, npad, B, ZS, tab, sig, out, ld, st, queue, reserve, \
                                slots, fill > 0);                                            \
  }
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

// k_cross_mm's LDS: the assembly's layout plus the row side's points
static size_t cross_mm_lds(int PM, int B, int kind) {
  return (size_t)(mm_layout(PM, B, kind == 0 ? 0 : 1, false).total + 64 * xj_pitch(PM)) *
         sizeof(double);
}
bool cross_mm_lds_ok(int PM, int B, int kind) { return cross_mm_lds(PM, B, kind) <= 160 * 1024; }

template <int PM>
static hipError_t cross_mm_pm(int kind, PairSide R, PairSide C, int B, int ZS, TabView tab, int b0,
                              int b1, double *out, int64_t ld, hipStream_t st) {
  if (R.n <= 0 || C.n <= 0 || b1 <= b0) return hipSuccess;
  const size_t lds = cross_mm_lds(PM, B, kind);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const void *f = kind == 0 ? (const void *)k_cross_mm<PM, 0> : (const void *)k_cross_mm<PM, 1>;
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  const dim3 grid((unsigned)((C.n + AT - 1) / AT), (unsigned)((R.n + AT - 1) / AT));
  if (kind == 0)
    hipLaunchKernelGGL((k_cross_mm<PM, 0>), grid, dim3(256), lds, st, R, C, B, ZS, tab, b0, b1, out, ld);
  else
    hipLaunchKernelGGL((k_cross_mm<PM, 1>), grid, dim3(256), lds, st, R, C, B, ZS, tab, b0, b1, out, ld);
  return hipGetLastError();
}

hipError_t launch_cross_mm(int kind, int PM, PairSide R, PairSide C, int B, int ZS, TabView tab,
                           int b0, int b1, double *out, int64_t ld, hipStream_t st) {
  switch (PM) {
#define ACE_CASE(P) \
  case P: return cross_mm_pm<P>(kind, R, C, B, ZS, tab, b0, b1, out, ld, st);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_assembly_mm(int kind, int PM, PairSide S, int64_t npad, int B, int ZS,
                              TabView tab, double sig, double *out, int64_t ld, double *kcopy,
                              hipStream_t st, const Tile *tiles, int64_t ntiles, int G, int part) {
  switch (PM) {
#define ACE_CASE(P) \
  case P:           \
    return asm_mm_pm<P>(kind, S, npad, B, ZS, tab, sig, out, ld, kcopy, st, tiles, ntiles, G, part);
    ACE_CASE(4) ACE_CASE(8) ACE_CASE(12) ACE_CASE(16) ACE_CASE(20) ACE_CASE(24)
    ACE_CASE(32) ACE_CASE(48) ACE_CASE(64)
#undef ACE_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace ace
