// ace_model.h -- the device-resident model shared by the C ABI (ace_api.cpp)
// and the resident-inverse products / prediction (ace_predict.cpp).
#pragma once
#include <functional>

#include "ace_common.h"
#include "ace_internal.h"

// Buffers of one Gauss-Jordan sweep and its lookahead events.
struct SweepWork {
  DBuf A, Ps[8], Ws[8], SW, S0, S1, piv, flag, order, xtiles, ptiles, gorder, htiles;
  int Z = 2;  // steps per bulk launch (sweep_group()), panel slots k % 2Z
  DBuf gtiles;                          // handle path: the gradient's tile list (build_grad_tiles)
  DBuf aq;                              // persistent assembly: tile counter, exits, CU claims
  DBuf bq;                              // small n: the bulk launches' work queues
  int breserve = 0;
  DBuf gpart, gwork, gsum;              // handle path: gradient partial-sum scratch
  DBuf norms;                           // handle path: slice norms (TabView::norms)
  int64_t ngtiles = 0, ngdiag = -2;     // -2: not built yet
  std::vector<int64_t> xoff, poff, hoff;
  int64_t glen = 0;
  std::vector<hipEvent_t> ev;
  int64_t n = 0, npad = 0, naug = 0, norder = 0;
  SweepWork() = default;
  SweepWork(const SweepWork &) = delete;
  ~SweepWork() {
    for (auto &e : ev) (void)hipEventDestroy(e);
  }
  void ensure(ace_ctx *ctx, int64_t n_) {
    n = n_;
    npad = round_up(n, NB);
    naug = npad + AUG;
    alloc(ctx, A, (size_t)(naug * naug) * sizeof(double), "alloc A");
    for (int j = 0; j < 2; ++j) {
      alloc(ctx, Ps[j], (size_t)(naug * NB) * sizeof(double), "alloc panel");
      alloc(ctx, Ws[j], (size_t)(naug * NB) * sizeof(double), "alloc panel");
    }
    alloc(ctx, SW, (size_t)SW_DOUBLES * sizeof(double), "alloc SW");
    alloc(ctx, S0, (size_t)(SUB * NB) * sizeof(double), "alloc S");
    alloc(ctx, S1, (size_t)(SUB * NB) * sizeof(double), "alloc S");
    alloc(ctx, piv, (size_t)npad * sizeof(double), "alloc piv");
    alloc(ctx, flag, 16, "alloc flag");
    alloc(ctx, aq, (2 + 64) * sizeof(int), "alloc assembly queue");
    norder = 0;
    if (const int S = update_order_block(); S > 0) {
      const std::vector<Tile> t = xcd_update_order(own_tiles(naug / UT, UT, 1, 0), S);
      alloc(ctx, order, t.size() * sizeof(Tile), "alloc tile order");
      upload_bytes(ctx, order.p, t.data(), t.size() * sizeof(Tile), "upload tile order");
      norder = (int64_t)t.size();
    }
    poff.clear();
    if (pair_steps() && cross_update_on_tiles() && npad / NB >= 2) {
      Z = sweep_group_n(naug);
      for (int j = 2; j < 2 * Z; ++j) {
        alloc(ctx, Ps[j], (size_t)(naug * NB) * sizeof(double), "alloc panel");
        alloc(ctx, Ws[j], (size_t)(naug * NB) * sizeof(double), "alloc panel");
      }
      const std::vector<Tile> t = pair_cross_tiles(naug, (int)(npad / NB), poff, Z);
      alloc(ctx, ptiles, std::max<size_t>(t.size(), 1) * sizeof(Tile), "alloc pair cross tiles");
      if (!t.empty())
        upload_bytes(ctx, ptiles.p, t.data(), t.size() * sizeof(Tile), "upload pair cross tiles");
      glen = 0;
      if (tail_sort()) {
        const std::vector<Tile> o = pair_bulk_orders(naug, (int)(npad / NB), &glen, 1, 0, Z);
        alloc(ctx, gorder, o.size() * sizeof(Tile), "alloc bulk orders");
        upload_bytes(ctx, gorder.p, o.data(), o.size() * sizeof(Tile), "upload bulk orders");
      }
      hoff.clear();
      if (heads_on()) {
        const std::vector<Tile> h = group_head_tiles(naug, (int)(npad / NB), Z, hoff);
        alloc(ctx, htiles, std::max<size_t>(h.size(), 1) * sizeof(Tile), "alloc head tiles");
        if (!h.empty())
          upload_bytes(ctx, htiles.p, h.data(), h.size() * sizeof(Tile), "upload head tiles");
      }
    }
    breserve = (Z > 2 && heads_on()) ? bulk_reserve(naug) : 0;
    if (breserve > 0) {
      // + per sweep step the barrier and exit counters of k_panel_split4 and
      // the D_0 counter of k_update_q4 (ACE_QSPLIT): zero
      // when allocated, reset by each launch's last workgroup (the per-sweep
      // memset covers the queues only: the first chain can start before it)
      void *const old = bq.p;
      alloc(ctx, bq, (size_t)((npad / NB + Z - 1) / Z * BQ_INTS + 3 * (npad / NB)) * sizeof(int),
            "alloc bulk queues");
      if (bq.p != old) ck(ctx, hipMemsetAsync(bq.p, 0, bq.bytes, ctx->stream), "memset queues");
    }
    xoff.clear();
    if (cross_update_on_tiles()) {
      const std::vector<Tile> t = cross_update_tiles(naug, (int)(npad / NB), xoff);
      alloc(ctx, xtiles, std::max<size_t>(t.size(), 1) * sizeof(Tile), "alloc cross tiles");
      if (!t.empty())
        upload_bytes(ctx, xtiles.p, t.data(), t.size() * sizeof(Tile), "upload cross tiles");
    }
    const size_t need = (size_t)(6 * (npad / NB) + 10);
    while (ev.size() < need) {
      hipEvent_t e;
      ck(ctx, hipEventCreateWithFlags(&e, ACE_SYNC_EVENT_FLAGS), "event");
      ev.push_back(e);
    }
  }
  SweepBufs bufs() const {
    SweepBufs b;
    b.A = A.d();
    b.ld = naug;
    b.npad = npad;
    for (int j = 0; j < 8; ++j) {
      b.P[j] = Ps[j].p ? Ps[j].d() : nullptr;
      b.W[j] = Ws[j].p ? Ws[j].d() : nullptr;
    }
    b.Z = Z;
    if (!poff.empty()) {
      b.ptiles = reinterpret_cast<const Tile *>(ptiles.p);
      b.poff = poff.data();
    }
    if (glen > 0) {
      b.gorder = reinterpret_cast<const Tile *>(gorder.p);
      b.glen = glen;
    }
    if (!hoff.empty()) {
      b.htiles = reinterpret_cast<const Tile *>(htiles.p);
      b.hoff = hoff.data();
    }
    if (breserve > 0 && bq.p) {
      b.bq = bq.i();
      b.breserve = breserve;
    }
    b.SW = SW.d();
    b.S[0] = S0.d();
    b.S[1] = S1.d();
    b.piv = piv.d();
    b.flag = flag.i();
    b.order = norder ? reinterpret_cast<const Tile *>(order.p) : nullptr;
    b.norder = norder;
    if (!xoff.empty()) {
      b.xtiles = reinterpret_cast<const Tile *>(xtiles.p);
      b.xoff = xoff.data();
    }
    return b;
  }
  SweepSync sync(ace_ctx *ctx) {
    SweepSync s;
    s.side = ctx->side;
    s.side2 = ctx->side2;
    s.ev = ev.data();
    s.nev = (int)ev.size();
    return s;
  }
};

// tv with TabView::norms computed into buf for the np points of X (np x PM,
// the padded side buffer): the assembly / gradient tiles then load their
// slice norms (bit-identical to computing them per tile)
inline TabView with_norms(ace_ctx *ctx, DBuf &buf, TabView tv, const Shape &s, const double *X,
                          int64_t np, hipStream_t st) {
  const bool m = s.kind == ACE_KERNEL_MATERN32;
  alloc(ctx, buf, (size_t)((s.B + 1) * np) * sizeof(double), "alloc norms");
  ck(ctx, launch_slice_norms(X, s.PM, np, s.B, m ? s.B + 1 : s.B, tv.wk,
                             m ? tv.wg + (s.B - 1) * s.PM : tv.wk, buf.d(), st),
     "slice norms");
  tv.norms = buf.d();
  tv.ldn = np;
  return tv;
}

// =====================================================================
// Device-resident model: one para_update per call, nothing materialised
// beyond A (the swept matrix) and O(n * tiles) partial sums.
// =====================================================================
struct ace_model {
  ace_ctx *ctx = nullptr;
  Shape s{};
  int64_t n = 0, npad = 0, naug = 0, ntiles = 0, ntr = 0;
  double std_y = 1.0;
  bool has_data = false;
  bool has_inverse = false;  // a para_update has left a resident inverse
  SideBufs side;
  DBuf y, tab, alpha, gpart, gwork;
  // the evaluation's results in one block, read back by one copy:
  // [gsum: grad_part_cols | sums: 8 (sums[4] = the sweep's flag) | scal: 16]
  DBuf res;
  DView gsum, sums, scal;
  DBuf norms;           // per-evaluation slice norms (TabView::norms), (B + 1) x npad
  DBuf gtiles;          // gradient tile list (grad_tile_order), or none
  int64_t ngdiag = -1;  // its leading diagonal tiles
  PinnedBuf hio;  // [theta tables | gsum | sums | scal | flag] host staging
  SweepWork sw;   // A = resident inverse of the last para_update
  SweepWork sw2;  // train_stats scratch (keeps sw's inverse, Q6)
  bool prof = false;
  // timing events in two sets: the set of evaluation t is read back while
  // evaluation t+1 runs (no host queries between evaluations)
  hipEvent_t ev_asm[4] = {}, ev_grad[4] = {};
  std::vector<hipEvent_t> ev_upd;  // 2 sets x 2 * steps
  std::vector<double> upd_flops;   // 2 sets x steps
  int upd_used[2] = {0, 0};
  int tset = 0, pend = -1;  // set the next timed evaluation records; set not yet read
  // [0] bulk update launches, [1] assembly, [2] gradient, [3] the sweep's
  // span (first bulk launch start -> last bulk launch end, every update /
  // cross / panel-GEMM flop of the sweep as its work)
  double t_ms[6] = {0, 0, 0, 0, 0, 0};
  int64_t t_launch[6] = {0, 0, 0, 0, 0, 0};
  double t_work[6] = {0, 0, 0, 0, 0, 0};
  ShardModel *shard = nullptr;  // block-column-sharded model (ace_shard.cpp)
};


// A = Kfull + sig I into w.A (AUG rows [y; 1], y may be null), then the
// sweep (ace_api.cpp; the fused model's and the handle path's common front)
void assemble_and_sweep(ace_ctx *ctx, SweepWork &w, const Shape &s, const PairSide &ps,
                        const TabView &tv, double sig, const double *y, int64_t n,
                        const SweepTiming *tmg, hipEvent_t *ev_asm);
// the gradient's XCD-dealt tile list for n (ace_api.cpp)
void build_grad_tiles(ace_ctx *ctx, int64_t n, DBuf &tiles, int64_t *ntiles, int64_t *ndiag);

// Operands of the device prediction pipeline (pred_pipeline, ace_predict.cpp).
struct PredOps {
  ace_ctx *ctx = nullptr;
  int64_t n = 0;            // training points
  const double *w = nullptr;  // y - mu on the device (n)
  // out (n x k, ld n) = A^-1 V^T for V = K_xX rows (k x n, ld ldv): this
  // rank's share when sharded (summed by allreduce)
  std::function<void(const double *V, int64_t ldv, int64_t k, double *out, DBuf &tmp)> symm;
  // optional (single GPU, ACE_PRED_TRI): the triangular form of the variance.
  // trmm: out (n x k) = L V^T, L the strictly lower part of A^-1; symv: out
  // (n x k) = A^-1 V for V n x k (ld ldv); sdiag: diag(A^-1) (n)
  std::function<void(const double *V, int64_t ldv, int64_t k, double *out)> trmm;
  std::function<void(const double *V, int64_t ldv, int64_t k, double *out, DBuf &tmp)> symv;
  const double *sdiag = nullptr;
  // optional: dst (n) = A^-1 w without a product (the model's swept AUG rows)
  std::function<void(double *dst)> ainv_w;
  std::function<void(double *buf, int64_t count)> allreduce;  // empty: single process
  // K_xX rows c0 .. c0 + nc (marginal slice sum for predict_marginal): a
  // device pointer with leading dimension *ld, possibly built in scratch
  std::function<const double *(int64_t c0, int64_t nc, int64_t *ld, DBuf &scratch)> cross;
  std::function<void(double *dst)> kdiag;  // diag(K_xx) (nx)
  // K_xx (nx x nx) for the ATE / ATT / ATU forms; scratch holds nx * nx
  std::function<const double *(int64_t *ld, DBuf &scratch)> kxx;
};
void pred_pipeline(const PredOps &op, int64_t nx, bool marginal, const double *Z_x, int ate,
                   double sigma, double mu, double mean_y, double std_y, double std_Z,
                   double *map, double *ci, double *var, double *avg);
