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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <memory>
#include <vector>

#include "../../include/ace_hip.h"

#include "ace_common.h"
#include "ace_internal.h"
#include "ace_model.h"

using namespace ace;

struct ace_dmat {
  enum Kind { DENSE, SWEPT, CUBE };
  ace_ctx *ctx = nullptr;
  Kind kind = DENSE;
  int64_t rows = 0, cols = 0, slices = 1;
  DBuf buf;                             // DENSE data; SWEPT / CUBE: materialised copy
  bool have_copy = false;               // SWEPT / CUBE: buf holds the materialised values
  bool host_read = false;               // values were copied to the host (diagnostic)
  std::shared_ptr<SweepWork> sweep;     // SWEPT
  bool nonpd = false;                   // SWEPT: the sweep met a non-positive pivot
  Shape shape{};                        // CUBE
  bool symmetric = false;               // CUBE: kernmat_*_symmetric_cpp (else cross)
  SideBufs s1, s2;                      // CUBE: row / column sides (s2 unused if symmetric)
  DBuf tab;
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
  } else {
    const Shape &s = h->shape;
    DBuf full;
    alloc(ctx, full, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
    alloc(ctx, h->buf, (size_t)(n1 * n2 * s.B) * sizeof(double), "alloc cube");
    const PairSide a = h->s1.view(n1), b = h->symmetric ? h->s1.view(n1) : h->s2.view(n2);
    ck(ctx, launch_assembly(h->symmetric ? 1 : 2, s.kind, s.PM, a, b, 0, s.B, s.ZS,
                            tab_view(h->tab, s), 0.0, full.d(), n1, h->buf.d(), st),
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
  const int64_t n2 = h->symmetric ? h->rows : h->cols;
  const int B = (int)h->slices;
  alloc(ctx, scratch, (size_t)(nr * n2) * sizeof(double), "alloc marginal kernel");
  if (h->kind == ace_dmat::CUBE && !h->have_copy) {
    const Shape &s = h->shape;
    const int b0 = B > 1 ? 1 : 0, b1 = B > 1 ? B : 1;
    PairSide a = h->s1.view(nr);
    a.X += r0 * s.PM;
    a.Z += r0 * s.ZS;
    a.LZ += r0 * s.ZS;
    const PairSide b = h->symmetric ? h->s1.view(n2) : h->s2.view(n2);
    // the symmetric form's r < c ordering (mode 1) is only kept when the
    // block is the whole square matrix; row blocks use the cross form,
    // whose slice values agree with it to the last bit but the zero tests
    ck(ctx, launch_assembly(h->symmetric && r0 == 0 && nr == h->rows ? 1 : 2, s.kind, s.PM, a, b, 0,
                            B, s.ZS, tab_view(h->tab, s), 0.0, scratch.d(), nr, nullptr, st,
                            nullptr, 0, 1, 0, b0, b1),
       "marginal assembly");
  } else {
    const double *v = values(h);
    const int64_t mn = h->rows * n2;
    DBuf sum;
    alloc(ctx, sum, (size_t)mn * sizeof(double), "alloc marginal");
    ck(ctx, launch_marginal_sum(v, h->rows, n2, B, sum.d(), st), "marginal sum");
    ck(ctx, hipMemcpy2DAsync(scratch.d(), nr * sizeof(double), sum.d() + r0, h->rows * sizeof(double),
                             nr * sizeof(double), n2, hipMemcpyDeviceToDevice, st),
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
  std::unique_ptr<ace_dmat> K(new_handle(ctx, ace_dmat::DENSE, n, n, 1));
  std::unique_ptr<ace_dmat> E(new_handle(ctx, ace_dmat::CUBE, n, n, B));
  E->shape = s;
  E->symmetric = true;
  upload_side(ctx, E->s1, s, X, Z, n, n);
  std::vector<double> tab = make_tab(theta, s, false);
  upload(ctx, E->tab, tab.data(), tab.size(), "upload tables");
  alloc(ctx, K->buf, (size_t)(n * n) * sizeof(double), "alloc Kfull");
  ck(ctx, launch_assembly(1, kind, s.PM, E->s1.view(n), E->s1.view(n), n, B, s.ZS,
                          tab_view(E->tab, s), 0.0, K->buf.d(), n, nullptr, ctx->stream),
     "assembly");
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
  std::unique_ptr<ace_dmat> K(new_handle(ctx, ace_dmat::DENSE, n1, n2, 1));
  std::unique_ptr<ace_dmat> E(new_handle(ctx, ace_dmat::CUBE, n1, n2, B));
  E->shape = s;
  upload_side(ctx, E->s1, s, X1, Z1, n1, n1);
  upload_side(ctx, E->s2, s, X2, Z2, n2, n2);
  std::vector<double> tab = make_tab(theta, s, false);
  upload(ctx, E->tab, tab.data(), tab.size(), "upload tables");
  alloc(ctx, K->buf, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
  ck(ctx, launch_assembly(2, kind, s.PM, E->s1.view(n1), E->s2.view(n2), 0, B, s.ZS,
                          tab_view(E->tab, s), 0.0, K->buf.d(), n1, nullptr, ctx->stream),
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
  h->sweep = std::make_shared<SweepWork>();
  SweepWork &w = *h->sweep;
  w.ensure(ctx, n);
  ck(ctx, launch_prepare_A(values(as(K)), n, std::exp(sigma), w.A.d(), w.naug, w.npad, ctx->stream),
     "prepare A");
  ck(ctx, launch_aug_init(w.A.d(), w.naug, w.npad, 0, nullptr, ctx->stream), "aug init");
  ck(ctx, hipMemsetAsync(w.flag.p, 0, sizeof(int), ctx->stream), "memset flag");
  const SweepSync sy = w.sync(ctx);
  ck(ctx, run_sweep(w.bufs(), ctx->stream, &sy, nullptr), "sweep");
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
  // [inv y | inv 1] in one product; sums on the host (n doubles each)
  std::vector<double> V((size_t)(2 * n), 1.0);
  std::copy(y, y + n, V.begin());
  DBuf dV, dO;
  upload(ctx, dV, V.data(), V.size(), "upload y");
  alloc(ctx, dO, (size_t)(2 * n) * sizeof(double), "alloc");
  inv_times(as(inv), dV.d(), n, false, 2, dO.d());
  std::vector<double> o((size_t)(2 * n));
  download(ctx, o.data(), dO.d(), o.size(), "download");
  sync(ctx);
  double st = 0.0, sa = 0.0;
  for (int64_t j = 0; j < n; ++j) {
    st += o[(size_t)j];
    sa += o[(size_t)(n + j)];
  }
  *out = 0.5 * st / sa;  // Q4 (src/utilities_cpp.cpp:9)
  return ACE_OK;
  ACE_CATCH
}

// alpha = inv (y - mu) on the device; returns the explicit residual sums of
// k_final_sums with s = Kfull alpha (src/kernel_SE_cpp.cpp:211-240).
static void alpha_and_sums(ace_ctx *ctx, int64_t n, const double *y, double mu,
                           const ace_dmat *Kfull, const ace_dmat *inv, DBuf &dy, DBuf &dalpha,
                           DBuf &dsums) {
  std::vector<double> ybar((size_t)n);
  for (int64_t r = 0; r < n; ++r) ybar[(size_t)r] = y[r] - mu;
  DBuf dyb, ds, dmu;
  upload(ctx, dy, y, (size_t)n, "upload y");
  upload(ctx, dyb, ybar.data(), (size_t)n, "upload ybar");
  upload(ctx, dmu, &mu, 1, "upload mu");
  alloc(ctx, dalpha, (size_t)n * sizeof(double), "alloc alpha");
  alloc(ctx, ds, (size_t)n * sizeof(double), "alloc s");
  alloc(ctx, dsums, 8 * sizeof(double), "alloc sums");
  inv_times(as(inv), dyb.d(), n, false, 1, dalpha.d());
  ck(ctx, launch_gemv(values(as(Kfull)), n, n, n, dalpha.d(), ds.d(), ctx->stream), "gemv K alpha");
  ck(ctx, launch_final_sums(dy.d(), dmu.d(), dalpha.d(), ds.d(), 0.0, n, nullptr, 0, dsums.d(),
                            ctx->stream),
     "final sums");
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
  DBuf dy, dalpha, dsums;
  alpha_and_sums(ctx, n, y, mu, Kmat, inv, dy, dalpha, dsums);
  double sums[4];
  download(ctx, sums, dsums.d(), 4, "download");
  sync(ctx);
  out[0] = std_y * std::sqrt(sums[0]) / std::sqrt((double)n);
  out[1] = -0.5 * (n * std::log(2.0 * M_PI) + host_logsum(eigenval, n) + sums[1]);
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
  SideBufs sb;
  upload_side(ctx, sb, s, X, Z, n, (n + 63) / 64 * 64);
  std::vector<double> tab = make_tab(theta, s);
  DBuf dtab, dy, dalpha, dsums, dg, dwork, dgs;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  alpha_and_sums(ctx, n, y, theta[1], Kfull, inv, dy, dalpha, dsums);
  // the gradient recomputes K_b from X, Z, theta (a virtual cube is exactly
  // that); a dense cube handle is read like ace_grad's host cube
  const double *cube = (Kel && Kel->kind == ace_dmat::DENSE) ? Kel->buf.d() : nullptr;
  const bool swept = inv->kind == ace_dmat::SWEPT;
  const double *Ainv = swept ? inv->sweep->A.d() : values(as(inv));
  const int64_t ld = swept ? inv->sweep->naug : n;
  const int64_t nt = grad_ntiles(n);
  const int ldg = grad_part_cols(s.PM, B);
  alloc(ctx, dg, (size_t)(nt * ldg) * sizeof(double), "alloc gpart");
  alloc(ctx, dwork, (size_t)tile_sums_work(ldg) * sizeof(double), "alloc tile sums");
  alloc(ctx, dgs, (size_t)ldg * sizeof(double), "alloc gsum");
  ck(ctx, launch_grad(kind, s.PM, sb.view(n), B, s.ZS, tab_view(dtab, s), Ainv, ld,
                      swept ? -1.0 : 1.0, dalpha.d(), cube, dg.d(), ctx->stream),
     "grad");
  ck(ctx, launch_tile_sums(dg.d(), nt, ldg, dwork.d(), dgs.d(), ctx->stream), "tile sums");
  std::vector<double> gs((size_t)ldg), sums(4);
  download(ctx, gs.data(), dgs.d(), gs.size(), "download gsum");
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
    if (h->kind == ace_dmat::CUBE && !h->have_copy) {
      const Shape &s = h->shape;
      ck(ctx, launch_kdiag(s.kind, h->s1.view(nx), s.ZS, tab_view(h->tab, s), B > 1 ? 1 : 0,
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
