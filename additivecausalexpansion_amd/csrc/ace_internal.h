// ace_internal.h -- shared declarations between the HIP kernels
// (ace_kernels.hip, ace_sweep.hip) and the host orchestration (ace_api.cpp).
#pragma once
#include <functional>
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ace {

// Sweep (Gauss-Jordan SPD inversion) blocking; see DESIGN.md §3.
#ifndef ACE_NB
#define ACE_NB 256
#endif
constexpr int NB = ACE_NB;  // outer pivot block = panel width
constexpr int SUB = 64;    // inner pivot block, eliminated inside LDS
constexpr int UT = 128;    // update tile (MFMA f64 16x16x4, 4 waves x 64x64)
constexpr int AUG = 128;   // augmented right-hand-side rows (y, 1) appended to A
constexpr int AT = 64;     // assembly / gradient pair tile
constexpr int PMAX = 64;   // largest supported covariate count p
constexpr int BMAX = 32;   // largest supported component count B

// Feature-count buckets the pair kernels are compiled for.
int pm_bucket(int p);  // smallest compiled bucket >= p, or -1

// ---- column sharding ---------------------------------------------------------
// The sharded model (ace_shard.cpp) distributes A by NB-wide column blocks,
// block-cyclic over G ranks: block j lives on rank j % G, as local block
// j / G of a naug-row, column-major local array (same ld, same row index).
// Every kernel that touches A maps a global column through lcol(); G == 1 is
// the identity, which is the single-GPU layout.
__host__ __device__ __forceinline__ int64_t lcol(int64_t c, int G) {
  return G == 1 ? c : (c / NB / G) * NB + c % NB;
}
__host__ __device__ __forceinline__ bool owns_col(int64_t c, int G, int r) {
  return G == 1 || (c / NB) % G == r;
}
// A pair / update tile (row tile I, column tile J) of a per-rank tile list.
struct Tile {
  int I, J;
};

// Per-theta tables, b-major: wk[b*PM+i] = exp(-theta[1+b+B*(i+1)]) (kernel
// index, Q1), wg[b*PM+i] = exp(-theta[2+B+b+B*i]) (gradient index),
// lam[b] = theta[2+b].  Total 2*B*PM + B doubles.
struct TabView {
  const double *wk, *wg, *lam;
  // device exp(theta[0]) (the device-fused training loop's theta lives in
  // HBM); null: the kernels' host `sig` argument
  const double *sig = nullptr;
  // slice norms s_b(x_p) = sum_i w_bi x_pi^2 of every point, norms[b ldn + p]
  // (launch_slice_norms: b < B the kernel weights, b = B the Matern
  // gradient's last-slice weights); null: each pair tile computes its own
  const double *norms = nullptr;
  int64_t ldn = 0;
};

// Row-side / column-side operand of a pair kernel (row-major, padded).
struct PairSide {
  const double *X;   // nrows x PM
  const double *Z;   // nrows x ZS   (basis columns 1..B-1)
  const double *LZ;  // nrows x ZS   log|z| (SE only; may be null for Matern)
  int64_t n;         // valid rows
};

// ---- assembly --------------------------------------------------------------
// mode 0: fused eval -- lower 64-tiles of the n_pad x n_pad block of A (ld),
//         value K + sig on the diagonal, identity on padding rows/cols; if
//         cube is non-null it receives the lower Kfull (same ld).
// mode 1: symmetric ABI output -- full n x n Kfull (ld = n) + optional cube.
// mode 2: cross ABI output -- n1 x n2 Kfull + optional cube.
// part (mode 0 without a tile list): 0 all tiles, 1 the first two panels'
// columns (J < 2 NB/AT), 2 the rest -- 1 then 2 lets the sweep's first
// group of pivot chains (and the cross of block 1) run while part 2 runs.
// b0 / b1 (modes 1 and 2, no cube): sum only slices [b0, b1) -- the
// marginal kernels of prediction (src/pred_cpp.cpp:55-67); b1 < 0 means B.
hipError_t launch_assembly(int mode, int kind, int PM, PairSide rows,
                           PairSide cols, int64_t npad, int B, int ZS,
                           TabView tab, double sig, double *out, int64_t ld,
                           double *cube, hipStream_t st, const Tile *tiles = nullptr,
                           int64_t ntiles = 0, int G = 1, int part = 0, int b0 = 0,
                           int b1 = -1);
// out[r] = sum over b in [b0, b1) of K_b(r, r) (symmetric kernel diagonal)
hipError_t launch_kdiag(int kind, PairSide S, int ZS, TabView tab, int b0, int b1, double *out,
                        hipStream_t st);

// MFMA-expansion variant of mode 0 (ace_pairs_mm.hip)
hipError_t launch_assembly_mm(int kind, int PM, PairSide S, int64_t npad, int B, int ZS,
                              TabView tab, double sig, double *out, int64_t ld,
                              double *kcopy, hipStream_t st, const Tile *tiles,
                              int64_t ntiles, int G, int part = 0);
// the assembly's second part (part 2 of mode 0) as a persistent work queue
// that leaves `reserve` CU ids of shader engine 0 of every XCD free (queue:
// two device ints, reset here on the stream)
hipError_t launch_assembly_persist(int kind, int PM, PairSide S, int64_t npad, int B, int ZS,
                                   TabView tab, double sig, double *out, int64_t ld,
                                   hipStream_t st, int *queue, int reserve, int fill = 0);
// workgroup slots of one CU for the persistent assembly (0 if unknown)
int assembly_persist_per_cu(int kind, int PM, int B);
bool pairs_use_mm(int PM, bool grad);
bool mm_lds_ok(int PM, int B, int kind, bool grad);
bool cross_mm_lds_ok(int PM, int B, int kind);
// mode 2 without a cube on the MFMA r2 expansion (k_cross_mm): R.n x C.n, ld
hipError_t launch_cross_mm(int kind, int PM, PairSide R, PairSide C, int B, int ZS, TabView tab,
                           int b0, int b1, double *out, int64_t ld, hipStream_t st);
hipError_t launch_grad_mm(int kind, int PM, PairSide S, int B, int ZS, TabView tab,
                          const double *A, int64_t ld, double sA, const double *alpha,
                          double *gpart, hipStream_t st, const Tile *tiles, int64_t ntiles, int G,
                          int64_t ndiag);

// ---- gradient --------------------------------------------------------------
// T = sA * A[r,c] - alpha_r alpha_c over the lower 64x64 tiles of [0,n)
// (grad_ntiles(n) of them).
// gpart: tile-major partial sums, one contiguous row of grad_part_cols(PM, B)
//        doubles per tile: [b*(PM+1) + i] (i < PM: length-scale sums,
//        i == PM: lambda sums), then [B*(PM+1)] the trace of T.  Each tile's
//        workgroup writes one contiguous run (launch_tile_sums reduces).
// cube (if non-null, ld n): K_b read from the cube instead of recomputed.
// tiles: the rank's list; ndiag >= 0 says its first ndiag entries are the
// diagonal tiles (lets the MFMA kernel run them separately).
__host__ __device__ constexpr int grad_part_cols(int PM, int B) { return B * (PM + 1) + 1; }
hipError_t launch_grad(int kind, int PM, PairSide side, int B, int ZS,
                       TabView tab, const double *A, int64_t ld, double sA,
                       const double *alpha, const double *cube, double *gpart, hipStream_t st,
                       const Tile *tiles = nullptr, int64_t ntiles = 0, int G = 1,
                       int64_t ndiag = -1);
int64_t grad_ntiles(int64_t n);
// super-block size of the fused model's XCD-dealt gradient tile order (0:
// row-major grid); ACE_GRAD_ORDER=S overrides (A/B switch)
int grad_order_block();
// out[j] = sum_t part[t * ncols + j], j < ncols (deterministic order); work
// needs tile_sums_work(ncols) doubles.
hipError_t launch_tile_sums(const double *part, int64_t ntiles, int ncols, double *work,
                            double *out, hipStream_t st);
int64_t tile_sums_work(int ncols);

// ---- sweep -----------------------------------------------------------------
// doubles of the SW buffer: SW[2] (SUB x SUB, ping-pong by sub-step), then
// k_panel_split's three NB x SUB chunk buffers
constexpr int64_t SW_DOUBLES = 2 * (int64_t)SUB * SUB + 3 * (int64_t)NB * SUB;
struct SweepBufs {
  double *A;      // Naug x Naug, col-major, ld = Naug, lower triangle used
  int64_t ld;     // Naug
  int64_t npad;   // multiple of NB
  double *P[8];   // Naug x NB : -panel (negated copy), slot k & 1 (k % 2Z with Z steps per group)
  double *W[8];   // Naug x NB : panel being swept, same slots; [2] .. null unless used
  int Z = 2;      // steps per bulk launch (sweep_group()); the lists below follow it
  double *SW;     // SW_DOUBLES: 2 SUB x SUB sub-pivot inverses + split-panel chunks
  double *S[2];   // SUB x NB col-major: pivot rows before their sub-sweep (ping-pong)
  double *piv;    // npad pivots
  int *flag;      // set to 1 on a non-positive / non-finite pivot
  const Tile *order = nullptr;  // k_update tile order (xcd_update_order), or row-major
  int64_t norder = 0;
  // lookahead cross update on k_update's 128-tiles (cross_update_tiles):
  // device list of every step's cross tiles, host offsets (steps + 1); null:
  // k_update_x on 64-tiles
  const Tile *xtiles = nullptr;
  const int64_t *xoff = nullptr;
  // two sweep steps per bulk launch (pair_steps()): every group's lookahead
  // cross tiles (pair_cross_tiles), host offsets per group
  const Tile *ptiles = nullptr;
  const int64_t *poff = nullptr;
  const Tile *gorder = nullptr;  // per-group bulk orders (tail_sort), glen each
  const Tile *htiles = nullptr;  // group_head_tiles lists (run_sweep_heads), offsets hoff
  const int64_t *hoff = nullptr;
  int64_t glen = 0;
  // small n: per group a bulk work queue of BQ_INTS ints (k_update_multi_r,
  // zeroed per sweep) and the CUs per shader engine it leaves to the chains
  int *bq = nullptr;
  int breserve = 0;
};
constexpr int BQ_INTS = 2 + 64;
int bulk_reserve(int64_t naug);
bool q_first(int64_t naug);
// Two sweep steps per bulk update launch (k_update_pair, K = 2 NB per tile;
// default): ACE_PAIR=0 selects one step per launch (A/B switch).
bool pair_steps();
// Lookahead cross tiles of group g = steps 2g, 2g + 1, for g = 1 ..
// ngroups-1 (each list dealt to the XCDs): [off[2g], off[2g+1]) the lower
// 128-tiles with I or J in block 2g, [off[2g+1], off[2g+2]) those with I or
// J in block 2g + 1 and not in block 2g (empty for a one-step group).
// Z steps per group (sweep_group()): off[2g] .. off[2g+1] the tiles with I
// or J in the group's first block, off[2g+1] .. off[2g+2] those in its other
// blocks and not in the first.
std::vector<Tile> pair_cross_tiles(int64_t naug, int steps, std::vector<int64_t> &off,
                                   int Z = 2);
// Head / tail lists of the group schedule's lookahead (run_sweep_heads):
// 2Z lists per group at off[G 2Z + m] (see ace_sweep.hip).  heads_on():
// ACE_HEADS switch.
std::vector<Tile> group_head_tiles(int64_t naug, int steps, int Z, std::vector<int64_t> &off);
bool heads_on();
// Steps per bulk launch: 2 (k_update_pair, default), ACE_GROUP=3 or 4 selects
// k_update_multi groups (run_sweep_groups).
int sweep_group();
int sweep_group_n(int64_t naug);  // sweep_group() for a model of naug rows
double update_gemm_tiles_group(int64_t naug, int64_t ka0, int npan, int kx0, int kx1);
// The lower 128-tiles with I or J in block k+1, for k = 0 .. steps-2,
// concatenated (each step's list dealt to the XCDs like the bulk order);
// off[k] .. off[k+1] is step k's range.  ACE_XUPD=0 selects k_update_x.
bool cross_update_on_tiles();
std::vector<Tile> cross_update_tiles(int64_t naug, int steps, std::vector<int64_t> &off);
// k_update tile order: the tiles of `tl` grouped into S x S super-blocks of
// 128-tiles that are dealt whole to the 8 XCDs; list index b runs on XCD
// b % 8 (dispatch is round-robin).  Entries with I < 0 are padding.
std::vector<Tile> xcd_update_order(const std::vector<Tile> &tl, int S,
                                   const std::function<double(const Tile &)> &cost = nullptr);
// The tiles along a Hilbert curve cut into 8 equal-work pieces, one per XCD
// (ACE_BULK_CURVE=1: the bulk orders of pair_bulk_orders)
bool bulk_curve();
std::vector<Tile> curve_update_order(const std::vector<Tile> &tl,
                                     const std::function<double(const Tile &)> &cost = nullptr);
// per group of two steps, the bulk order with each XCD's cheap tiles last
// (ACE_TAIL_SORT=1): ngroups lists of *len entries
bool tail_sort();
// (sharded: rank r's own tiles of G)
// (Z: steps per group, sweep_group())
std::vector<Tile> pair_bulk_orders(int64_t naug, int steps, int64_t *len, int G = 1, int r = 0,
                                   int Z = 2);
// own lower tiles of size T over [0, ntile*T) in row-major order (ace_shard.cpp)
std::vector<Tile> own_tiles(int64_t ntile, int T, int G, int r);
// super-block size S of that order (0: row-major grid); ACE_UPD_ORDER=S
// overrides (diagnostic A/B switch)
int update_order_block();
// Lookahead: the panel sweep of step k+1 runs on `side` while the main
// stream updates the rest of step k.  `ev` needs 2*steps + 1 events.
struct SweepSync {
  hipStream_t side;
  hipStream_t side2 = nullptr;  // pair steps: the second block's cross (needs 4 steps + 4 events)
  hipEvent_t *ev;
  int nev;
  bool ready_recorded = false;  // caller already recorded ev[2 * steps] ("inputs ready")
  // recorded on the main stream after the whole assembly: the first group's
  // tail path waits for it when the assembly's second part leaves CUs to the
  // head path (ACE_ASM_PERSIST); null: it waits for ev[2 * steps]
  hipEvent_t tail_after = nullptr;
  // called on side2 after group 0's tail path, before its completion event
  // (ACE_ASM_FILL: the persistent assembly's filler launch)
  hipError_t (*fill)(void *, hipStream_t) = nullptr;
  bool tail_split = false;  // group 0's tail path after its whole head path
  void *fill_arg = nullptr;
};
// Optional timing of the dominant update launches (k_update<false>): event
// pairs in ev, executed GEMM flops per timed launch in flops[].
struct SweepTiming {
  hipEvent_t *ev;
  int nev;
  int *used;
  double *flops;
};
// Runs every step; A's K block ends holding -A^-1 (lower), the AUG rows hold
// (A^-1 R)^T and the corner -R^T A^-1 R.
hipError_t run_sweep(const SweepBufs &b, hipStream_t st, const SweepSync *sync,
                     const SweepTiming *timing);
double update_gemm_tiles(int64_t naug, int64_t k0, int kx, bool look);
// every GEMM flop of one sweep, whatever the schedule: each step's update of
// every lower tile outside its block (bulk + lookahead crosses) and its panel
// GEMM W_i = Pn_i W_kk
double sweep_flops(int64_t naug, int64_t npad);

// ---- sharded sweep (one rank's view; ace_shard.cpp drives the steps) --------
// Step k on rank r:  shard_pack -> [exchange: broadcast `low` from rank k%G,
// all-gather recv slot r -> recv] -> shard_unpack_chain (panel k on every rank,
// pivot chain run redundantly, W for the rows r consumes) -> updates.
struct ShardSweep {
  double *A;          // local column blocks, naug x (nloc * NB), ld = naug
  int64_t ld;         // naug
  int64_t npad;
  int G, r;
  double *P[8], *W[8];  // naug x NB: Pn = -panel (all rows), W (own rows); slot k % (2 Z)
  double *SW;
  double *S[2];
  double *piv;        // npad pivots (every rank records all of them)
  int *flag;
  double *low;        // (naug - k0) x NB broadcast block
  double *recv;       // G x shard_row_slots(k, G) x NB x NB; slot r holds the own
                      // row pieces (the in-place all-gather operand)
  const Tile *tiles;  // own 128-tiles (row-major lower), device
  int64_t ntiles;
};
int shard_row_slots(int k, int G);
hipError_t shard_pack(const ShardSweep &b, int k, hipStream_t st);
// own_done: the packing cross launch already wrote the rank's own panel rows
hipError_t shard_unpack_chain(const ShardSweep &b, int k, int buf, hipStream_t st,
                              bool own_done = false);
// cross tiles of block k+1 with panel k (buffer buf)
hipError_t shard_update_cross(const ShardSweep &b, int k, int buf, hipStream_t st);
// every own tile except the cross of block kx (kx < 0: none)
hipError_t shard_update_main(const ShardSweep &b, int k, int buf, int kx, hipStream_t st);
// npan steps from block kb in one launch (k_update_multi<true>; one panel:
// k_update), panels in slots (kb + j) % nslot, skipping blocks [kx0, kx1),
// on a tile list; kpack >= 0: the launch also writes the exchange buffers of
// step kpack (what shard_pack(kpack) would copy; G > 1) and the rank's own
// rows of panel kpack (slot kpack % nslot)
hipError_t shard_update_group(const ShardSweep &b, int kb, int npan, int nslot, int kx0, int kx1,
                              const Tile *tiles, int64_t nt, hipStream_t st, int kpack = -1,
                              double *lowp = nullptr, int64_t lr0 = 0, int64_t hh = -1);
// the head schedule's pieces (run_sweep_sharded_heads): a row range of the
// owner's column block (+ row pieces) into an exchange buffer; a row range of
// panel k from one; the pivot sub-steps alone; the head or tail panel GEMM
hipError_t shard_pack_part(const ShardSweep &b, int k, int64_t i_lo, int64_t i_hi, double *low,
                           int64_t lr0, int64_t hh, bool rows, hipStream_t st);
hipError_t shard_unpack_part(const ShardSweep &b, int k, int buf, int64_t i_lo, int64_t i_hi,
                             const double *low, int64_t lr0, int64_t hh, bool own_done,
                             hipStream_t st);
hipError_t shard_chain(const ShardSweep &b, int k, int buf, hipStream_t st);
hipError_t shard_pgemm(const ShardSweep &b, int k, int buf, int rt_lo, int rt_hi, bool head,
                       hipStream_t st);

// ---- small helpers -----------------------------------------------------------
// AUG rows of columns j < n: row 0 = y (zeros if y is null), row 1 = 1
// z0[0..n0) and z1[0..n1) (device ints, may be null) are zeroed by the same
// launch: the evaluation's flag and queue resets without fill launches
hipError_t launch_aug_init(double *A, int64_t ld, int64_t npad, int64_t n,
                           const double *y, hipStream_t st, int G = 1, int rank = 0,
                           int *z0 = nullptr, int n0 = 0, int *z1 = nullptr, int n1 = 0);
// out[0] = sum_j y_j (A^-1 1)_j (AUG row 1), out[1] = 1^T A^-1 1 (corner)
hipError_t launch_aug_dot(const double *A, int64_t ld, int64_t npad, int64_t n, const double *y,
                          double *out, hipStream_t st);
// sharded: vec = [u | v | yKy, yK1, 1K1] of the rank's own columns (zeros elsewhere)
hipError_t launch_aug_extract(const double *A, int64_t ld, int64_t npad, int G,
                              int rank, double *vec, hipStream_t st);
hipError_t launch_alpha_from_vec(const double *vec, int64_t npad, int64_t n,
                                 double theta1, int use_mu_solution, double *alpha,
                                 double *scal, hipStream_t st);
hipError_t launch_add(const double *x, double *y, int64_t count, hipStream_t st);
// alpha = u - mu_eff * v, u/v read from A's AUG rows; mu_eff = theta1 (or
// *theta1p, a device scalar, when given), or 0.5*yK1/1K1 when
// use_mu_solution; writes scal[0..2] = {yKy, yK1, 1K1}, scal[3] =
// mu_solution, scal[4] = mu_eff.
hipError_t launch_alpha_from_aug(const double *A, int64_t ld, int64_t npad,
                                 int64_t n, double theta1, int use_mu_solution,
                                 double *alpha, double *scal, hipStream_t st,
                                 const double *theta1p = nullptr);
hipError_t launch_colsum(const double *in, int64_t nrows, int ncols,
                         double *out, hipStream_t st);
// sums[0] = sum (ybar - s)^2, sums[1] = sum y*alpha, sums[2] = sum alpha,
// sums[3] = sum log(piv[0..npiv)), with ybar = y - *mu (device scalar).
// s == nullptr: ybar - s = sig * alpha (fused model, A = Kfull + sig I);
// sigp (device scalar) replaces sig when given; flag (device int) is copied
// to sums[4] when given, so that one read-back carries it.
hipError_t launch_final_sums(const double *y, const double *mu, const double *alpha,
                             const double *s, double sig, int64_t n, const double *piv,
                             int64_t npiv, double *sums, hipStream_t st,
                             const double *sigp = nullptr, const int *flag = nullptr);
// ---- device-fused training loop (ace_train.hip) -----------------------------
// theta tables of make_tab (ace_common.h) from a device theta, plus
// tab[2 B PM + B] = exp(theta[0]) (TabView::sig)
// the TabView::norms table: NS = B (+ 1 for the Matern gradient) rows of np
// points (ld np) from X (np x PM row-major), with mm_stage's arithmetic
hipError_t launch_slice_norms(const double *X, int PM, int64_t np, int B, int NS,
                              const double *wk, const double *wlast, double *norms,
                              hipStream_t st);
hipError_t launch_make_tab(const double *theta, int B, int p, int PM, double *tab,
                           hipStream_t st);
struct TrainCfg {
  int optimizer;  // ace_optimizer
  double lr, momentum, beta1, beta2;
  int clip;
  double clip_at, tol;
  int P, B, p, PM, kind;
  int64_t n;
  double std_y;
};
// One iteration's host-side tail of ace_model_train on the device (one
// workgroup): compose_grad + stats of para_update, norm clip, optimizer step,
// the mu overwrite and the convergence test.  st = [theta | m1 | m2 | g |
// prev] (5 P; prev = the theta the iteration's evaluation ran at), hist = the
// stats matrix (2 x (maxiter + 2)), ctl = {last iteration done, stop: 0
// running / 1 converged / 2 non-finite gradient}.  Once ctl[1] is set, later
// launches change nothing.
hipError_t launch_train_step(const TrainCfg &c, int it, const double *gsum, const double *sums,
                             const double *scal, const int *flag, double *st, double *hist,
                             int *ctl, hipStream_t stream);
// y = M x for M (m x k, col-major ld) ; y = M^T x
hipError_t launch_gemv(const double *M, int64_t ld, int64_t m, int64_t k,
                       const double *x, double *y, hipStream_t st);
hipError_t launch_gemv_t(const double *M, int64_t ld, int64_t m, int64_t k,
                         const double *x, double *y, hipStream_t st);
// C (m x n) = A (m x k) * B (k x n), col-major, fp64 MFMA.
hipError_t launch_gemm_nn(int64_t m, int64_t n, int64_t k, const double *A,
                          int64_t lda, const double *B, int64_t ldb, double *C,
                          int64_t ldc, hipStream_t st);
// Copies scale * A (lower) into a full symmetric n x n matrix (ld_out).
hipError_t launch_sym_from_lower(const double *A, int64_t ld, int64_t n,
                                 double scale, double *out, int64_t ld_out,
                                 hipStream_t st);
// Same from block-cyclic column storage: global column c of A lives in
// slot (c / NB) % G (slot_elems doubles each) at local column lcol(c, G).
hipError_t launch_sym_from_cyclic(const double *A, int64_t ld, int64_t n, int G,
                                  int64_t slot_elems, double scale, double *out,
                                  int64_t ld_out, hipStream_t st);
// dst[0:npad, 0:npad] (ld_dst) = src (n x n, ld n) + diag I, identity padding
hipError_t launch_prepare_A(const double *src, int64_t n, double diag,
                            double *dst, int64_t ld_dst, int64_t npad,
                            hipStream_t st);
hipError_t launch_fill(double *p, int64_t count, double v, hipStream_t st);
// Sum over b>=1 of cube slices (or slice 0 when B == 1): out m x n.
hipError_t launch_marginal_sum(const double *cube, int64_t m, int64_t n,
                               int B, double *out, hipStream_t st);
// Prediction rows: for r < nx: a = sum_c T[r,c] w[c]; q = sum_c T[r,c] K[r,c]
hipError_t launch_pred_rows(const double *T, const double *K, int64_t ld,
                            int64_t nx, int64_t nX, const double *w,
                            double *a, double *q, hipStream_t st);
// q[j] = w_j^T M w_j for three weight vectors packed in W (n x 3)
hipError_t launch_quad3(const double *M, int64_t ld, int64_t n,
                        const double *W, double *q, hipStream_t st);
hipError_t launch_log_abs(const double *Z, double *LZ, int64_t count,
                          hipStream_t st);

// ---- products with the resident inverse (ace_symm.hip) -----------------------
// out (n x k, ldo) = scale * S V, S = symmetric matrix with lower triangle in
// A (ld; block-cyclic columns for G > 1: only the rank's stored entries are
// used, so the ranks' outputs sum to S V).  vt: V[p][c] = V[c + p ldv].
hipError_t launch_symm(const double *A, int64_t ld, int64_t n, int G, int rank, const double *V,
                       int64_t ldv, bool vt, int64_t k, double scale, double *out, int64_t ldo,
                       hipStream_t st);
// a[c] = sum_q T[q + c ldt] w[q], d[c] = sum_q T[q + c ldt] K[c + q ldk], c < nx
hipError_t launch_pred_cols(const double *T, int64_t ldt, const double *K, int64_t ldk, int64_t n,
                            int64_t nx, const double *w, double *a, double *d, hipStream_t st);
// single GPU: out (n x k, ldo) = scale * L V^T, L the strictly lower part of
// the stored matrix, V given as k x n (V[p][c] = V[c + p ldv])
hipError_t launch_trmm_lower(const double *A, int64_t ld, int64_t n, const double *V, int64_t ldv,
                             int64_t k, double scale, double *out, int64_t ldo, hipStream_t st);
// a[c] = sum_q K[c][q] s[q], d[c] = sum_q K[c][q] (2 Y[q][c] + D[q] K[c][q])
hipError_t launch_pred_cols_tri(const double *Y, int64_t ldt, const double *K, int64_t ldk,
                                int64_t n, int64_t nx, const double *sv, const double *D, double *a,
                                double *d, hipStream_t st);
// D[q] = scale * A[q + q ld], q < n
hipError_t launch_diag_scaled(const double *A, int64_t ld, int64_t n, double scale, double *D,
                              hipStream_t st);
// w = y - mu
hipError_t launch_center(const double *y, int64_t n, double mu, double *w, hipStream_t st);

}  // namespace ace
