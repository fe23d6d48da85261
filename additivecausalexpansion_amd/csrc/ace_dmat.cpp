// ace_dmat.cpp -- device-matrix handles for the unchanged R6 call sequence.
//
// The reference's R6 kernel classes keep Kmat, Karray and invKmatn as R
// objects and pass them between .Call routines on every para_update
// (R/kernel_SE_R6.R:26-50: kernmat_*_symmetric_cpp -> invkernel_cpp ->
// mu_solution_cpp -> grad_*_cpp, then predict's pred_cpp at :75-97).  With
// host matrices that is 2-34 GB of PCIe traffic per iteration and, for
// Karray, an n x n x B cube (21.5 GB at C2).  The *_dev entry points below
// take and return ace_dmat handles instead, so the same sequence stays in
// HBM; the R shim wraps a handle in an ALTREP double vector that is only
// materialised if R code actually reads its values.
//
// Handle kinds:
//   DENSE  a column-major rows x cols (x slices) device array (ld = rows)
//   SWEPT  the Gauss-Jordan sweep's A: -A^-1 in the lower triangle of a
//          naug x naug array (the engine's inverse, never symmetrised unless read)
//   CUBE   the virtual `elements` cube of kernmat_*_cpp: X, Z, theta (as
//          device tables) are recorded; slices, or the marginal slice sums
//          of pred_marginal_cpp, are assembled on demand
//   KSYM   the virtual `full` matrix of kernmat_*_symmetric_cpp (same
//          record): invkernel_dev assembles A = Kfull + e^sigma I straight
//          into its sweep buffer (lower triangle, the fused model's kernels);
//          the n x n values are built only if read or consumed as a matrix
//
// Provenance: an inverse made from a KSYM handle remembers it, so that
// grad_dev / stats_dev given that same Kfull form the RMSE residual
// ybar - Kfull alpha as e^sigma alpha (A alpha = ybar, A = Kfull + e^sigma I:
// exact up to rounding) with no pass over Kfull.  Every SWEPT
// inverse carries A^-1 1 and 1^T A^-1 1 in its AUG rows (mu_solution_dev:
// no pass over the inverse either).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "../../include/ace_hip.h"

#include "ace_common.h"
#include "ace_internal.h"
#include "ace_model.h"

using namespace ace;

// What a virtual kernel handle records (shared by a kernmat call's `full`
// and `elements` handles): shape, the row / column sides (s2 unused if
// symmetric; s1 has n1 rounded up to NB rows for the sweep's assembly) and
// the theta tables.
struct KernSrc {
  Shape shape{};
  bool symmetric = false;
  std::shared_ptr<SideBufs> s1, s2;
  DBuf tab;
};

struct ace_dmat {
  enum Kind { DENSE, SWEPT, CUBE, KSYM };
  ace_ctx *ctx = nullptr;
  Kind kind = DENSE;
  int64_t rows = 0, cols = 0, slices = 1;
  DBuf buf;                             // DENSE data; SWEPT / CUBE / KSYM: materialised copy
  bool have_copy = false;               // SWEPT / CUBE / KSYM: buf holds the materialised values
  bool host_read = false;               // values were copied to the host (diagnostic)
  std::shared_ptr<SweepWork> sweep;     // SWEPT
  bool nonpd = false;                   // SWEPT: the sweep met a non-positive pivot
  double sig = 0.0;                     // SWEPT: e^sigma added on the diagonal
  std::shared_ptr<KernSrc> src;         // CUBE / KSYM; SWEPT: the KSYM it inverted (or null)
  std::shared_ptr<const std::vector<double>> yaug;  // SWEPT: the y swept along in AUG row 0
  DBuf msum;                            // dense CUBE: pred_marginal's slice sum (cached)
  bool have_msum = false;
  DBuf slice;                           // virtual CUBE: the last slice ace_dmat_read assembled
  int64_t slice_b = -1;                 // ... and its index (-1: none)
};

namespace {

ace_dmat *new_handle(ace_ctx *ctx, ace_dmat::Kind k, int64_t r, int64_t c, int64_t sl) {
  ace_dmat *h = new ace_dmat();
  h->ctx = ctx;
  h->kind = k;
  h->rows = r;
  h->cols = c;
  h->slices = sl;
  return h;
}

// Full values of a handle on the device (materialised on first use).
const double *values(ace_dmat *h) {
  ace_ctx *ctx = h->ctx;
  hipStream_t st = ctx->stream;
  if (h->kind == ace_dmat::DENSE || h->have_copy) return h->buf.d();
  const int64_t n1 = h->rows, n2 = h->cols;
  if (h->kind == ace_dmat::SWEPT) {
    alloc(ctx, h->buf, (size_t)(n1 * n2) * sizeof(double), "alloc inverse");
    if (h->nonpd)  // the reference's inverse of a non-PD matrix is non-finite
      ck(ctx, launch_fill(h->buf.d(), n1 * n2, kNaN, st), "fill");
    else
      ck(ctx, launch_sym_from_lower(h->sweep->A.d(), h->sweep->naug, n1, -1.0, h->buf.d(), n1, st),
         "symmetrize");
  } else if (h->kind == ace_dmat::KSYM) {
    const KernSrc &k = *h->src;
    const Shape &s = k.shape;
    alloc(ctx, h->buf, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
    ck(ctx, launch_assembly(1, s.kind, s.PM, k.s1->view(n1), k.s1->view(n1), n1, s.B, s.ZS,
                            tab_view(k.tab, s), 0.0, h->buf.d(), n1, nullptr, st),
       "assembly");
    sync(ctx);
  } else {
    const KernSrc &k = *h->src;
    const Shape &s = k.shape;
    DBuf full;
    alloc(ctx, full, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
    alloc(ctx, h->buf, (size_t)(n1 * n2 * s.B) * sizeof(double), "alloc cube");
    const PairSide a = k.s1->view(n1), b = k.symmetric ? k.s1->view(n1) : k.s2->view(n2);
    ck(ctx, launch_assembly(k.symmetric ? 1 : 2, s.kind, s.PM, a, b, 0, s.B, s.ZS,
                            tab_view(k.tab, s), 0.0, full.d(), n1, h->buf.d(), st),
       "cube assembly");
    sync(ctx);
  }
  h->have_copy = true;
  return h->buf.d();
}

// Marginal slice sum of a cube handle (src/pred_cpp.cpp:55-67): slices
// 1..B-1, or slice 0 when B == 1, assembled straight from X, Z, theta for a
// virtual cube (no cube is built), summed for a dense one.  Rows r0 .. r0+nr.
const double *marginal_rows(ace_dmat *h, int64_t r0, int64_t nr, int64_t *ld, DBuf &scratch) {
  ace_ctx *ctx = h->ctx;
  hipStream_t st = ctx->stream;
  const bool symmetric = h->src && h->src->symmetric;
  const int64_t n2 = symmetric ? h->rows : h->cols;
  const int B = (int)h->slices;
  alloc(ctx, scratch, (size_t)(nr * n2) * sizeof(double), "alloc marginal kernel");
  if (h->kind == ace_dmat::CUBE && !h->have_copy) {
    const KernSrc &k = *h->src;
    const Shape &s = k.shape;
    const int b0 = B > 1 ? 1 : 0, b1 = B > 1 ? B : 1;
    PairSide a = k.s1->view(nr);
    a.X += r0 * s.PM;
    a.Z += r0 * s.ZS;
    a.LZ += r0 * s.ZS;
    const PairSide b = symmetric ? k.s1->view(n2) : k.s2->view(n2);
    // the symmetric form's r < c ordering (mode 1) is only kept when the
    // block is the whole square matrix; row blocks use the cross form,
    // whose slice values agree with it to the last bit but the zero tests
    ck(ctx, launch_assembly(symmetric && r0 == 0 && nr == h->rows ? 1 : 2, s.kind, s.PM, a, b, 0,
                            B, s.ZS, tab_view(k.tab, s), 0.0, scratch.d(), nr, nullptr, st,
                            nullptr, 0, 1, 0, b0, b1),
       "marginal assembly");
  } else {
    // dense (or materialised) cube: the marginal slice sum is formed once and
    // kept with the handle (handles are immutable), then rows are copied out
    if (!h->have_msum) {
      const double *v = values(h);
      alloc(ctx, h->msum, (size_t)(h->rows * n2) * sizeof(double), "alloc marginal");
      ck(ctx, launch_marginal_sum(v, h->rows, n2, B, h->msum.d(), st), "marginal sum");
      h->have_msum = true;
    }
    ck(ctx, hipMemcpy2DAsync(scratch.d(), nr * sizeof(double), h->msum.d() + r0,
                             h->rows * sizeof(double), nr * sizeof(double), n2,
                             hipMemcpyDeviceToDevice, st),
       "copy rows");
    sync(ctx);
  }
  *ld = nr;
  return scratch.d();
}

// out (n x k, ld n) = inv * M^T for M (k x n, ld ldm): from the sweep's lower
// storage (scale -1) or a dense symmetric matrix (its lower triangle).
void inv_times(ace_dmat *inv, const double *M, int64_t ldm, bool vt, int64_t k, double *out) {
  ace_ctx *ctx = inv->ctx;
  const int64_t n = inv->rows;
  if (inv->kind == ace_dmat::SWEPT) {
    if (inv->nonpd) {
      ck(ctx, launch_fill(out, n * k, kNaN, ctx->stream), "fill");
      return;
    }
    ck(ctx, launch_symm(inv->sweep->A.d(), inv->sweep->naug, n, 1, 0, M, ldm, vt, k, -1.0, out, n,
                        ctx->stream),
       "symm");
  } else {
    ck(ctx, launch_symm(values(inv), n, n, 1, 0, M, ldm, vt, k, 1.0, out, n, ctx->stream), "symm");
  }
}

ace_dmat *as(const ace_dmat *h) { return const_cast<ace_dmat *>(h); }

// ACE_DMAT_DIRECT=0: invkernel_dev of a virtual Kfull materialises it and
// copies it into the sweep buffer (the round-2 path; A/B switch)
bool dmat_direct() {
  static const bool v = [] {
    const char *e = getenv("ACE_DMAT_DIRECT");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// Per-context state of the handle path (ace_ctx::dmat_state): the training
// inputs the R6 loop passes on every call, kept on the device.
//   side: X, Z (and log|Z|) packed for the pair kernels, n rounded up to NB
//         rows, reused while the caller's X and Z are bitwise the same;
//   y:    the response last passed to mu_solution_dev / grad_dev / stats_dev;
//         invkernel_dev sweeps it along in AUG row 0 (speculatively: grad_dev
//         checks it is still the same y, else it multiplies by the inverse).
struct DmatState {
  Shape shape{};
  int64_t n = -1;
  std::vector<double> X, Z;
  std::shared_ptr<SideBufs> side;
  std::shared_ptr<const std::vector<double>> y;
  DBuf ydev;
};

DmatState &dstate(ace_ctx *ctx) {
  if (!ctx->dmat_state) ctx->dmat_state = std::make_shared<DmatState>();
  return *static_cast<DmatState *>(ctx->dmat_state.get());
}

bool same_vals(const std::vector<double> &a, const double *b, size_t count) {
  return a.size() == count && (count == 0 || std::memcmp(a.data(), b, count * sizeof(double)) == 0);
}

// The packed training side for (X, Z): the cached one if X and Z are bitwise
// what it was built from, else a new upload (which becomes the cache).
std::shared_ptr<SideBufs> cached_side(ace_ctx *ctx, const Shape &s, int64_t n, const double *X,
                                      const double *Z) {
  DmatState &st = dstate(ctx);
  const size_t nx = (size_t)(n * s.p), nz = s.B > 1 ? (size_t)(n * (s.B - 1)) : 0;
  if (st.side && st.n == n && st.shape.kind == s.kind && st.shape.p == s.p && st.shape.B == s.B &&
      same_vals(st.X, X, nx) && same_vals(st.Z, Z, nz))
    return st.side;
  auto side = std::make_shared<SideBufs>();
  upload_side(ctx, *side, s, X, Z, n, round_up(n, NB));
  st.shape = s;
  st.n = n;
  st.X.assign(X, X + nx);
  st.Z.assign(Z ? Z : X, Z ? Z + nz : X);
  st.side = side;
  return side;
}

// Record y as the response the next invkernel_dev sweeps along.
void note_y(ace_ctx *ctx, const double *y, int64_t n) {
  DmatState &st = dstate(ctx);
  if (st.y && same_vals(*st.y, y, (size_t)n)) return;
  st.y = std::make_shared<const std::vector<double>>(y, y + n);
  upload(ctx, st.ydev, y, (size_t)n, "upload y");
}

// Sweep buffers for an inverse of size n: a pooled one from a freed handle
// (ace_dmat_free) when the size matches, else a new allocation.
std::shared_ptr<SweepWork> pooled_sweep(ace_ctx *ctx, int64_t n) {
  auto &pool = ctx->sweep_pool;
  for (size_t j = 0; j < pool.size(); ++j)
    if (pool[j]->n == n) {
      std::shared_ptr<SweepWork> w = pool[j];
      pool.erase(pool.begin() + (long)j);
      return w;
    }
  auto w = std::make_shared<SweepWork>();
  try {
    w->ensure(ctx, n);
  } catch (const Fail &f) {
    // out of device memory with pooled buffers of other sizes: drop them and
    // try once more (any other failure, e.g. ACE_ERR_TIMEOUT, propagates)
    if (f.code != ACE_ERR_OOM || pool.empty()) throw;
    pool.clear();
    w = std::make_shared<SweepWork>();
    w->ensure(ctx, n);
  }
  return w;
}

void check_square(ace_ctx *ctx, const ace_dmat *h, int64_t n, const char *what) {
  arg(ctx, h && h->rows == n && h->cols == n && h->kind != ace_dmat::CUBE, what);
}

}  // namespace

extern "C" {

int ace_dmat_upload(ace_ctx *ctx, int64_t rows, int64_t cols, int64_t slices, const double *host,
                    ace_dmat **out) {
  if (!ctx || !out) return ACE_ERR_ARG;
  *out = nullptr;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, rows >= 1 && cols >= 1 && slices >= 1 && host, "bad shape / null argument");
  std::unique_ptr<ace_dmat> h(new_handle(ctx, ace_dmat::DENSE, rows, cols, slices));
  upload(ctx, h->buf, host, (size_t)(rows * cols * slices), "upload matrix");
  *out = h.release();
  return ACE_OK;
  ACE_CATCH
}

int ace_dmat_dims(const ace_dmat *h, int64_t *rows, int64_t *cols, int64_t *slices) {
  if (!h) return ACE_ERR_ARG;
  if (rows) *rows = h->rows;
  if (cols) *cols = h->cols;
  if (slices) *slices = h->slices;
  return ACE_OK;
}

int ace_dmat_read(const ace_dmat *hc, int64_t offset, int64_t count, double *out) {
  if (!hc || !out) return ACE_ERR_ARG;
  ace_dmat *h = as(hc);
  ace_ctx *ctx = h->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  const int64_t total = h->rows * h->cols * h->slices;
  arg(ctx, offset >= 0 && count >= 0 && offset + count <= total, "read outside the matrix");
  if (h->kind == ace_dmat::CUBE && !h->have_copy) {
    // a virtual cube is read slice by slice (one n1 x n2 slice on the device
    // at a time, never the whole n1 x n2 x B cube: 21.5 GB at C2); a
    // one-slice sum [b, b+1) is that slice's values exactly
    const KernSrc &k = *h->src;
    const Shape &s = k.shape;
    const int64_t sl = h->rows * h->cols;
    // the last assembled slice stays on the handle: the R shim reads an
    // ALTREP vector element by element or 512 values at a time
    // (rcpp/ace_hip_shim.cpp Elt / Get_region), and each later read inside
    // that slice is then a plain download
    for (int64_t b = offset / sl; b < h->slices && b * sl < offset + count; ++b) {
      const int64_t lo = std::max(offset, b * sl), hi = std::min(offset + count, (b + 1) * sl);
      if (h->slice_b != b) {
        alloc(ctx, h->slice, (size_t)sl * sizeof(double), "alloc slice");
        h->slice_b = -1;
        const PairSide a = k.s1->view(h->rows), c = k.symmetric ? k.s1->view(h->rows) : k.s2->view(h->cols);
        ck(ctx, launch_assembly(k.symmetric ? 1 : 2, s.kind, s.PM, a, c, 0, s.B, s.ZS,
                                tab_view(k.tab, s), 0.0, h->slice.d(), h->rows, nullptr, ctx->stream,
                                nullptr, 0, 1, 0, (int)b, (int)b + 1),
           "slice assembly");
      }
      download(ctx, out + (lo - offset), h->slice.d() + (lo - b * sl), (size_t)(hi - lo),
               "download slice");
      sync(ctx);
      h->slice_b = b;
    }
    h->host_read = true;
    return ACE_OK;
  }
  const double *v = values(h);
  download(ctx, out, v + offset, (size_t)count, "download matrix");
  sync(ctx);
  h->host_read = true;
  return ACE_OK;
  ACE_CATCH
}

int ace_dmat_materialized(const ace_dmat *h) {
  return h ? ((h->kind == ace_dmat::DENSE || h->have_copy) ? 1 : 0) | (h->host_read ? 2 : 0) : 0;
}

void ace_dmat_free(ace_dmat *h) {
  if (!h) return;
  (void)hipSetDevice(h->ctx->device);
  // keep up to two sets of sweep buffers for the next invkernel_dev (the R6
  // loop frees one inverse per iteration); their contents are dead
  // (only sets of this n: a set of another size is dropped, not kept)
  if (h->kind == ace_dmat::SWEPT && h->sweep && h->sweep.use_count() == 1) {
    auto &pool = h->ctx->sweep_pool;
    const int64_t n = h->sweep->n;
    pool.erase(std::remove_if(pool.begin(), pool.end(),
                              [n](const std::shared_ptr<SweepWork> &w) { return w->n != n; }),
               pool.end());
    if (pool.size() >= 2) pool.erase(pool.begin());
    pool.push_back(std::move(h->sweep));
  }
  delete h;
}

int ace_kernmat_sym_dev(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *X,
                        const double *Z, const double *theta, ace_dmat **full,
                        ace_dmat **elements) {
  if (!ctx || !full) return ACE_ERR_ARG;
  *full = nullptr;
  if (elements) *elements = nullptr;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, n >= 1 && theta && (p == 0 || X) && (B == 1 || Z), "null argument");
  // nothing is assembled here: both outputs are virtual (X, Z, theta
  // recorded); the rows are padded to the sweep's NB multiple so that
  // invkernel_dev can assemble A straight into its sweep buffer
  auto src = std::make_shared<KernSrc>();
  src->shape = s;
  src->symmetric = true;
  src->s1 = cached_side(ctx, s, n, X, Z);
  std::vector<double> tab = make_tab(theta, s, false);
  upload(ctx, src->tab, tab.data(), tab.size(), "upload tables");
  std::unique_ptr<ace_dmat> K(new_handle(ctx, ace_dmat::KSYM, n, n, 1));
  K->src = src;
  std::unique_ptr<ace_dmat> E(new_handle(ctx, ace_dmat::CUBE, n, n, B));
  E->src = src;
  sync(ctx);
  *full = K.release();
  if (elements) *elements = E.release();
  return ACE_OK;
  ACE_CATCH
}

int ace_kernmat_cross_dev(ace_ctx *ctx, int kind, int64_t n1, int64_t n2, int p, int B,
                          const double *X1, const double *X2, const double *Z1, const double *Z2,
                          const double *theta, ace_dmat **full, ace_dmat **elements) {
  if (!ctx || !full) return ACE_ERR_ARG;
  *full = nullptr;
  if (elements) *elements = nullptr;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, n1 >= 1 && n2 >= 1 && theta, "bad shape / null argument");
  arg(ctx, (p == 0 || (X1 && X2)) && (B == 1 || (Z1 && Z2)), "null argument");
  auto src = std::make_shared<KernSrc>();
  src->shape = s;
  src->s1 = std::make_shared<SideBufs>();
  src->s2 = std::make_shared<SideBufs>();
  upload_side(ctx, *src->s1, s, X1, Z1, n1, n1);
  upload_side(ctx, *src->s2, s, X2, Z2, n2, n2);
  std::vector<double> tab = make_tab(theta, s, false);
  upload(ctx, src->tab, tab.data(), tab.size(), "upload tables");
  std::unique_ptr<ace_dmat> K(new_handle(ctx, ace_dmat::DENSE, n1, n2, 1));
  std::unique_ptr<ace_dmat> E(new_handle(ctx, ace_dmat::CUBE, n1, n2, B));
  E->src = src;
  alloc(ctx, K->buf, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
  ck(ctx, launch_assembly(2, kind, s.PM, src->s1->view(n1), src->s2->view(n2), 0, B, s.ZS,
                          tab_view(src->tab, s), 0.0, K->buf.d(), n1, nullptr, ctx->stream),
     "assembly");
  sync(ctx);
  *full = K.release();
  if (elements) *elements = E.release();
  return ACE_OK;
  ACE_CATCH
}

int ace_invkernel_dev(ace_ctx *ctx, const ace_dmat *K, double sigma, double *eigenval,
                      ace_dmat **inv) {
  if (!ctx || !inv) return ACE_ERR_ARG;
  *inv = nullptr;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, K && K->rows == K->cols && K->slices == 1 && K->kind != ace_dmat::CUBE,
      "pdmat must be a square matrix handle");
  const int64_t n = K->rows;
  std::unique_ptr<ace_dmat> h(new_handle(ctx, ace_dmat::SWEPT, n, n, 1));
  h->sweep = pooled_sweep(ctx, n);
  h->sig = std::exp(sigma);
  SweepWork &w = *h->sweep;
  // the response of the last mu_solution / grad call rides along in AUG row 0
  DmatState &ds = dstate(ctx);
  const bool with_y = ds.y && (int64_t)ds.y->size() == n;
  const double *ydev = with_y ? ds.ydev.d() : nullptr;
  if (with_y) h->yaug = ds.y;
  if (K->kind == ace_dmat::KSYM && dmat_direct()) {
    // the fused model's front: A = Kfull + e^sigma I assembled into the
    // sweep buffer (lower tiles) and swept, no n x n Kfull in between
    const KernSrc &k = *K->src;
    const TabView tv = with_norms(ctx, w.norms, tab_view(k.tab, k.shape), k.shape, k.s1->X.d(),
                                  w.npad, ctx->stream);
    assemble_and_sweep(ctx, w, k.shape, k.s1->view(n), tv, h->sig, ydev, n, nullptr, nullptr);
    h->src = K->src;
  } else {
    ck(ctx, launch_prepare_A(values(as(K)), n, h->sig, w.A.d(), w.naug, w.npad, ctx->stream),
       "prepare A");
    ck(ctx, launch_aug_init(w.A.d(), w.naug, w.npad, n, ydev, ctx->stream), "aug init");
    ck(ctx, hipMemsetAsync(w.flag.p, 0, sizeof(int), ctx->stream), "memset flag");
    const SweepSync sy = w.sync(ctx);
    ck(ctx, run_sweep(w.bufs(), ctx->stream, &sy, nullptr), "sweep");
  }
  int flag = 0;
  ck(ctx, hipMemcpyAsync(&flag, w.flag.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream),
     "download flag");
  if (eigenval) download(ctx, eigenval, w.piv.d(), (size_t)n, "download pivots");
  sync(ctx);
  h->nonpd = flag != 0;
  *inv = h.release();
  return ACE_OK;
  ACE_CATCH
}

int ace_mu_solution_dev(ace_ctx *ctx, int64_t n, const double *y, const ace_dmat *inv,
                        double *out) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, y && out, "null argument");
  check_square(ctx, inv, n, "invKmat must be an n x n matrix handle");
  double st = 0.0, sa = 0.0;
  DBuf dO;
  note_y(ctx, y, n);
  if (inv->kind == ace_dmat::SWEPT) {
    // sum(inv y) = y . (A^-1 1) and accu(inv) = 1^T A^-1 1: the swept AUG
    // row 1 and corner, no pass over the inverse
    alloc(ctx, dO, 2 * sizeof(double), "alloc");
    const SweepWork &w = *inv->sweep;
    ck(ctx, launch_aug_dot(w.A.d(), w.naug, w.npad, n, dstate(ctx).ydev.d(), dO.d(), ctx->stream),
       "aug dot");
    double o[2];
    download(ctx, o, dO.d(), 2, "download");
    sync(ctx);
    st = o[0];
    sa = o[1];
    if (inv->nonpd) st = sa = kNaN;
  } else {
    // [inv y | inv 1] in one product; sums on the host (n doubles each)
    std::vector<double> V((size_t)(2 * n), 1.0);
    std::copy(y, y + n, V.begin());
    DBuf dV;
    upload(ctx, dV, V.data(), V.size(), "upload y");
    alloc(ctx, dO, (size_t)(2 * n) * sizeof(double), "alloc");
    inv_times(as(inv), dV.d(), n, false, 2, dO.d());
    std::vector<double> o((size_t)(2 * n));
    download(ctx, o.data(), dO.d(), o.size(), "download");
    sync(ctx);
    for (int64_t j = 0; j < n; ++j) {
      st += o[(size_t)j];
      sa += o[(size_t)(n + j)];
    }
  }
  *out = 0.5 * st / sa;  // Q4 (src/utilities_cpp.cpp:9)
  return ACE_OK;
  ACE_CATCH
}

// alpha = inv (y - mu) on the device and the sums of k_final_sums with the
// residual ybar - Kfull alpha (src/kernel_SE_cpp.cpp:211-240).  alpha from
// the swept AUG rows (A^-1 y - mu A^-1 1) when this y was swept along, else a
// product with the inverse; the residual is e^sigma alpha when inv was swept
// from this same virtual Kfull (provenance), else the explicit Kfull alpha.
static void alpha_and_sums(ace_ctx *ctx, int64_t n, const double *y, double mu,
                           const ace_dmat *Kfull, const ace_dmat *inv, DBuf &dalpha,
                           DBuf &dsums) {
  note_y(ctx, y, n);
  const double *dy = dstate(ctx).ydev.d();
  DBuf ds, dmu, dscal;
  upload(ctx, dmu, &mu, 1, "upload mu");
  alloc(ctx, dalpha, (size_t)n * sizeof(double), "alloc alpha");
  alloc(ctx, dsums, 8 * sizeof(double), "alloc sums");
  const bool swept = inv->kind == ace_dmat::SWEPT;
  if (swept && !inv->nonpd && inv->yaug && same_vals(*inv->yaug, y, (size_t)n)) {
    const SweepWork &w = *inv->sweep;
    alloc(ctx, dscal, 8 * sizeof(double), "alloc scal");
    ck(ctx, launch_alpha_from_aug(w.A.d(), w.naug, w.npad, n, mu, 0, dalpha.d(), dscal.d(),
                                  ctx->stream),
       "alpha");
  } else {
    std::vector<double> ybar((size_t)n);
    for (int64_t r = 0; r < n; ++r) ybar[(size_t)r] = y[r] - mu;
    DBuf dyb;
    upload(ctx, dyb, ybar.data(), (size_t)n, "upload ybar");
    inv_times(as(inv), dyb.d(), n, false, 1, dalpha.d());
    sync(ctx);  // dyb is freed on return
  }
  const bool same = swept && inv->src && Kfull->kind == ace_dmat::KSYM && Kfull->src == inv->src;
  if (same) {
    ck(ctx, launch_final_sums(dy, dmu.d(), dalpha.d(), nullptr, inv->sig, n, nullptr, 0, dsums.d(),
                              ctx->stream),
       "final sums");
  } else {
    alloc(ctx, ds, (size_t)n * sizeof(double), "alloc s");
    ck(ctx, launch_gemv(values(as(Kfull)), n, n, n, dalpha.d(), ds.d(), ctx->stream),
       "gemv K alpha");
    ck(ctx, launch_final_sums(dy, dmu.d(), dalpha.d(), ds.d(), 0.0, n, nullptr, 0, dsums.d(),
                              ctx->stream),
       "final sums");
  }
  sync(ctx);  // ds, dmu and dscal are freed on return
}

int ace_stats_dev(ace_ctx *ctx, int64_t n, const double *y, const ace_dmat *Kmat,
                  const ace_dmat *inv, const double *eigenval, double mu, double std_y,
                  double *out) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, y && eigenval && out, "null argument");
  check_square(ctx, Kmat, n, "Kmat must be an n x n matrix handle");
  check_square(ctx, inv, n, "invKmatn must be an n x n matrix handle");
  DBuf dalpha, dsums;
  alpha_and_sums(ctx, n, y, mu, Kmat, inv, dalpha, dsums);
  double sums[4];
  download(ctx, sums, dsums.d(), 4, "download");
  sync(ctx);
  out[0] = std_y * std::sqrt(sums[0]) / std::sqrt((double)n);
  out[1] = -0.5 * (n * std::log(2.0 * M_PI) + host_logsum(eigenval, n) + sums[1]);
  if (inv->kind == ace_dmat::SWEPT && inv->nonpd) out[0] = out[1] = kNaN;
  return ACE_OK;
  ACE_CATCH
}

int ace_grad_dev(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *y,
                 const double *X, const double *Z, const ace_dmat *Kfull, const ace_dmat *Kel,
                 const ace_dmat *inv, const double *eigenval, const double *theta, double *stats,
                 double std_y, double *grad) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, y && eigenval && theta && stats && grad && (p == 0 || X) && (B == 1 || Z),
      "null argument");
  check_square(ctx, Kfull, n, "Kfull must be an n x n matrix handle");
  check_square(ctx, inv, n, "invKmatn must be an n x n matrix handle");
  arg(ctx, !Kel || (Kel->rows == n && Kel->cols == n && Kel->slices == B), "K must be n x n x B");
  const std::shared_ptr<SideBufs> sb = cached_side(ctx, s, n, X, Z);
  std::vector<double> tab = make_tab(theta, s);
  DBuf dtab, dalpha, dsums, dg0, dwork0, dgs0;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  alpha_and_sums(ctx, n, y, theta[1], Kfull, inv, dalpha, dsums);
  // the gradient recomputes K_b from X, Z, theta (a virtual cube is exactly
  // that); a dense cube handle is read like ace_grad's host cube
  const double *cube = (Kel && Kel->kind == ace_dmat::DENSE) ? Kel->buf.d() : nullptr;
  const bool swept = inv->kind == ace_dmat::SWEPT;
  const double *Ainv = swept ? inv->sweep->A.d() : values(as(inv));
  const int64_t ld = swept ? inv->sweep->naug : n;
  // the fused model's XCD-dealt tile order and partial-sum scratch, kept
  // with the sweep buffers
  const Tile *tl = nullptr;
  int64_t nt = grad_ntiles(n), ndiag = -1;
  DBuf *dg = &dg0, *dwork = &dwork0, *dgs = &dgs0;
  if (swept) {
    SweepWork &w = *inv->sweep;
    if (!cube) {
      if (w.ngdiag == -2) build_grad_tiles(ctx, n, w.gtiles, &w.ngtiles, &w.ngdiag);
      if (w.ngdiag >= 0) {
        tl = reinterpret_cast<const Tile *>(w.gtiles.p);
        nt = w.ngtiles;
        ndiag = w.ngdiag;
      }
    }
    dg = &w.gpart;
    dwork = &w.gwork;
    dgs = &w.gsum;
  }
  const int ldg = grad_part_cols(s.PM, B);
  alloc(ctx, *dg, (size_t)(nt * ldg) * sizeof(double), "alloc gpart");
  alloc(ctx, *dwork, (size_t)tile_sums_work(ldg) * sizeof(double), "alloc tile sums");
  alloc(ctx, *dgs, (size_t)ldg * sizeof(double), "alloc gsum");
  // swept (the resident inverse): the sweep buffers' norms table for the
  // cached side's npad rows; else the tiles compute their own
  const TabView tvg = swept && !cube ? with_norms(ctx, inv->sweep->norms, tab_view(dtab, s), s,
                                                  sb->X.d(), inv->sweep->npad, ctx->stream)
                                     : tab_view(dtab, s);
  ck(ctx, launch_grad(kind, s.PM, sb->view(n), B, s.ZS, tvg, Ainv, ld,
                      swept ? -1.0 : 1.0, dalpha.d(), cube, dg->d(), ctx->stream, tl, tl ? nt : 0, 1,
                      ndiag),
     "grad");
  ck(ctx, launch_tile_sums(dg->d(), nt, ldg, dwork->d(), dgs->d(), ctx->stream), "tile sums");
  std::vector<double> gs((size_t)ldg), sums(4);
  download(ctx, gs.data(), dgs->d(), gs.size(), "download gsum");
  download(ctx, sums.data(), dsums.d(), 4, "download sums");
  sync(ctx);
  compose_grad(s, theta, gs.data(), sums[2], grad);
  stats[0] = std_y * std::sqrt(sums[0]) / std::sqrt((double)n);
  stats[1] = -0.5 * (n * std::log(2.0 * M_PI) + host_logsum(eigenval, n) + sums[1]);
  if (swept && inv->nonpd) {
    const int P = 2 + B * (p + 1);
    for (int j = 0; j < P; ++j) grad[j] = kNaN;
    stats[0] = stats[1] = kNaN;
  }
  return ACE_OK;
  ACE_CATCH
}

int ace_pred_dev(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X, double sigma, double mu,
                 const ace_dmat *invK_XX, const ace_dmat *K_xX, const ace_dmat *K_xx,
                 double mean_y, double std_y, double *map, double *ci, double *var) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, y_X && map && ci && var, "null argument");
  check_square(ctx, invK_XX, nX, "invK_XX must be an nX x nX matrix handle");
  arg(ctx, K_xX && K_xX->rows == nx && K_xX->cols == nX && K_xX->kind != ace_dmat::CUBE,
      "K_xX must be an nx x nX matrix handle");
  check_square(ctx, K_xx, nx, "K_xx must be an nx x nx matrix handle");
  std::vector<double> w((size_t)nX);
  for (int64_t c = 0; c < nX; ++c) w[(size_t)c] = y_X[c] - mu;
  DBuf dw;
  upload(ctx, dw, w.data(), w.size(), "upload w");
  PredOps op;
  op.ctx = ctx;
  op.n = nX;
  op.w = dw.d();
  op.symm = [&](const double *V, int64_t ldv, int64_t k, double *out, DBuf &) {
    inv_times(as(invK_XX), V, ldv, true, k, out);
  };
  op.cross = [&](int64_t c0, int64_t, int64_t *ld, DBuf &) -> const double * {
    *ld = nx;
    return values(as(K_xX)) + c0;
  };
  op.kdiag = [&](double *dst) {
    const ace_dmat *h = K_xx;
    if (h->kind == ace_dmat::KSYM && !h->have_copy) {  // only the diagonal is used
      const KernSrc &k = *h->src;
      const Shape &s = k.shape;
      ck(ctx, launch_kdiag(s.kind, k.s1->view(nx), s.ZS, tab_view(k.tab, s), 0, s.B, dst,
                           ctx->stream),
         "kernel diagonal");
      return;
    }
    ck(ctx, hipMemcpy2DAsync(dst, sizeof(double), values(as(K_xx)), (size_t)(nx + 1) * sizeof(double),
                             sizeof(double), (size_t)nx, hipMemcpyDeviceToDevice, ctx->stream),
       "diag");
  };
  pred_pipeline(op, nx, false, nullptr, 0, sigma, mu, mean_y, std_y, 1.0, map, ci, var, nullptr);
  return ACE_OK;
  ACE_CATCH
}

int ace_pred_marginal_dev(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X,
                          const double *Z_x, double sigma, double mu, const ace_dmat *invK_XX,
                          const ace_dmat *K_xX, const ace_dmat *K_xx, double mean_y, double std_y,
                          double std_Z, int calculate_ate, double *map, double *ci, double *var,
                          double *avg) {
  (void)mean_y;
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, y_X && map && ci && var, "null argument");
  arg(ctx, !calculate_ate || (Z_x && avg), "calculate_ate needs Z_x and avg");
  check_square(ctx, invK_XX, nX, "invK_XX must be an nX x nX matrix handle");
  arg(ctx, K_xX && K_xX->rows == nx && K_xX->cols == nX, "K_xX must be nx x nX x B");
  arg(ctx, K_xx && K_xx->rows == nx && K_xx->cols == nx && K_xx->slices == K_xX->slices,
      "K_xx must be nx x nx x B");
  std::vector<double> w((size_t)nX);
  for (int64_t c = 0; c < nX; ++c) w[(size_t)c] = y_X[c] - mu;
  DBuf dw;
  upload(ctx, dw, w.data(), w.size(), "upload w");
  const int B = (int)K_xX->slices;
  PredOps op;
  op.ctx = ctx;
  op.n = nX;
  op.w = dw.d();
  op.symm = [&](const double *V, int64_t ldv, int64_t k, double *out, DBuf &) {
    inv_times(as(invK_XX), V, ldv, true, k, out);
  };
  op.cross = [&](int64_t c0, int64_t nc, int64_t *ld, DBuf &scratch) -> const double * {
    return marginal_rows(as(K_xX), c0, nc, ld, scratch);
  };
  op.kdiag = [&](double *dst) {
    ace_dmat *h = as(K_xx);
    // the r = c shortcut needs the symmetric kernel's record (a cross cube's
    // diagonal pairs rows of two different sides)
    if (h->kind == ace_dmat::CUBE && !h->have_copy && h->src->symmetric) {
      const KernSrc &k = *h->src;
      const Shape &s = k.shape;
      ck(ctx, launch_kdiag(s.kind, k.s1->view(nx), s.ZS, tab_view(k.tab, s), B > 1 ? 1 : 0,
                           B > 1 ? B : 1, dst, ctx->stream),
         "kernel diagonal");
    } else {
      DBuf m;
      int64_t ld = 0;
      const double *v = marginal_rows(h, 0, nx, &ld, m);
      ck(ctx, hipMemcpy2DAsync(dst, sizeof(double), v, (size_t)(ld + 1) * sizeof(double),
                               sizeof(double), (size_t)nx, hipMemcpyDeviceToDevice, ctx->stream),
         "diag");
      sync(ctx);
    }
  };
  op.kxx = [&](int64_t *ld, DBuf &scratch) -> const double * {
    return marginal_rows(as(K_xx), 0, nx, ld, scratch);
  };
  pred_pipeline(op, nx, true, Z_x, calculate_ate, sigma, mu, 0.0, std_y, std_Z, map, ci, var, avg);
  return ACE_OK;
  ACE_CATCH
}

}  // extern "C"
