// ace_predict.cpp -- products with the resident inverse of a model: A^-1 V
// (ace_model_apply_inverse) and device-resident posterior prediction
// (ace_model_predict / ace_model_predict_marginal).
//
// The reference's predict path (R/kernel_SE_R6.R:75-97) builds K_xX and
// K_xx (or their n x n2 x B "elements" cubes) on the host, ships the stored
// invKmatn, and pred_cpp / pred_marginal_cpp (src/pred_cpp.cpp:8-126) form
// tmp = K_xX invK_XX with a full GEMM and the full n2 x n2 matrix
// K_xx - tmp K_xX^T, of which only the diagonal (and, for ATE/ATT/ATU,
// three quadratic forms) is used.  Here:
//   * the inverse is the one the last para_update left in HBM (Q6: the
//     theta_{T-1} inverse with kernels at the caller's theta_T), read from
//     the swept matrix's lower triangle (-A^-1) by k_symm -- never copied,
//     never sent to the host;
//   * K_xX (the marginal slice sum for predict_marginal) is assembled on the
//     device, test points in chunks, and T' = A^-1 K_xX^T (n x chunk) is one
//     MFMA product per chunk;
//   * only diag(K_xx) is formed (r2 = 0: launch_kdiag), and the ATE/ATT/ATU
//     quadratic forms use Km_xx (n2 x n2) and three n-vectors;
//   * sharded models: each rank multiplies by the inverse entries it stores
//     and the per-test-point sums are all-reduced (2 n2 + 3 doubles), never
//     the n x n2 products.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <vector>

#include "../../include/ace_hip.h"

#include "ace_common.h"
#include "ace_internal.h"
#include "ace_model.h"

using namespace ace;

namespace {

// test points per chunk: K_xX and T' are n x 8192 each (4.3 GB at n = 65536)
constexpr int64_t NXC = 8192;

struct PredScratch {
  DBuf K, T, Kxx;
};

// out (n x k, ld n) = A^-1 V, summed over the simulated ranks; on an RCCL
// rank the caller all-reduces (the partial holds this rank's entries only).
void symm_resident(ace_model *m, const double *V, int64_t ldv, bool vt, int64_t k, double *out,
                   DBuf &tmp) {
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  const int64_t n = m->n;
  if (!m->shard) {  // -A^-1 is stored: scale -1
    ck(ctx, launch_symm(m->sw.A.d(), m->naug, n, 1, 0, V, ldv, vt, k, -1.0, out, n, st), "symm");
    return;
  }
  const int G = shard_world(m->shard);
  for (int j = 0; j < shard_nlocal(m->shard); ++j) {
    double *dst = out;
    if (j > 0) {
      alloc(ctx, tmp, (size_t)(n * k) * sizeof(double), "alloc symm partial");
      dst = tmp.d();
    }
    ck(ctx, launch_symm(shard_A0(m->shard, j), m->naug, n, G, shard_rank_of(m->shard, j), V, ldv,
                        vt, k, -1.0, dst, n, st),
       "symm");
    if (j > 0) ck(ctx, launch_add(tmp.d(), out, n * k, st), "sim all-reduce");
  }
}

// ACE_PRED_TRI (default 1): single-GPU prediction takes the variance's
// quadratic form through the strictly lower triangle of A^-1 (half the
// MFMA work of the full symmetric product; 0 = the full product, A/B)
bool pred_tri() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_PRED_TRI");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

void require_inverse(ace_model *m) {
  arg(m->ctx, m->has_data, "ace_model_set_data() not called");
  arg(m->ctx, m->has_inverse, "no resident inverse: call ace_model_para_update() first");
}

}  // namespace

namespace {
void pred_pipeline_once(const PredOps &op, int64_t nx, bool marginal, const double *Z_x, int ate,
                        double sigma, double mu, double mean_y, double std_y, double std_Z,
                        double *map, double *ci, double *var, double *avg) {
  ace_ctx *ctx = op.ctx;
  hipStream_t st = ctx->stream;
  const int64_t n = op.n;
  // the large buffers live in the context between calls (ctx->pred_state);
  // this reference keeps them valid if an allocation failure drops it there
  std::shared_ptr<PredScratch> ps = std::static_pointer_cast<PredScratch>(ctx->pred_state);
  if (!ps) {
    ps = std::make_shared<PredScratch>();
    ctx->pred_state = ps;
  }
  DBuf &dKc = ps->K, &dT = ps->T, &dKmxx = ps->Kxx;
  DBuf dad, dkd, dtmp, dW3, dS3, dU3, dq3, dvt, ddot;
  const int64_t chunk = std::min<int64_t>(NXC, nx);
  alloc(ctx, dT, (size_t)(chunk * n) * sizeof(double), "alloc T");
  alloc(ctx, dad, (size_t)(2 * nx) * sizeof(double), "alloc sums");  // [a | d]
  alloc(ctx, dkd, (size_t)nx * sizeof(double), "alloc diag");
  std::vector<double> zx;
  if (ate) {  // weights 1, Z_x, (Z_x == 0) (src/pred_cpp.cpp:89-106)
    zx.assign(Z_x, Z_x + nx);
    std::vector<double> W3((size_t)(3 * nx));
    for (int64_t r = 0; r < nx; ++r) {
      W3[(size_t)r] = 1.0;
      W3[(size_t)(nx + r)] = zx[(size_t)r];
      W3[(size_t)(2 * nx + r)] = (zx[(size_t)r] == 0) ? 1.0 : 0.0;
    }
    upload(ctx, dW3, W3.data(), W3.size(), "upload weights");
    alloc(ctx, dS3, (size_t)(3 * n) * sizeof(double), "alloc s");
    alloc(ctx, dU3, (size_t)(3 * n) * sizeof(double), "alloc u");
    alloc(ctx, dvt, (size_t)n * sizeof(double), "alloc gemv");
    ck(ctx, launch_fill(dS3.d(), 3 * n, 0.0, st), "zero");
    ck(ctx, launch_fill(dU3.d(), 3 * n, 0.0, st), "zero");
  }
  // triangular form (op.trmm): the variance from Y = L K_xX^T, L the
  // strictly lower part of A^-1 (half of the full product's flops), the map
  // from s = A^-1 w, and u_j = A^-1 s_j once after the loop
  const bool tri = (bool)op.trmm;
  DBuf dsv;
  if (tri) {
    alloc(ctx, dsv, (size_t)n * sizeof(double), "alloc s");
    if (op.ainv_w)
      op.ainv_w(dsv.d());
    else
      op.symv(op.w, n, 1, dsv.d(), dtmp);
  }
  for (int64_t c0 = 0; c0 < nx; c0 += chunk) {
    const int64_t nc = std::min<int64_t>(chunk, nx - c0);
    int64_t ldk = 0;
    const double *Kc = op.cross(c0, nc, &ldk, dKc);  // K_xX rows c0 .. c0 + nc
    if (tri) {
      op.trmm(Kc, ldk, nc, dT.d());
      ck(ctx, launch_pred_cols_tri(dT.d(), n, Kc, ldk, n, nc, dsv.d(), op.sdiag, dad.d() + c0,
                                   dad.d() + nx + c0, st),
         "pred sums");
    } else {
      // T' = A^-1 K_xX^T (n x nc): the transpose of tmp = K_xX invK_XX
      op.symm(Kc, ldk, nc, dT.d(), dtmp);
      ck(ctx, launch_pred_cols(dT.d(), n, Kc, ldk, n, nc, op.w, dad.d() + c0, dad.d() + nx + c0, st),
         "pred sums");
    }
    if (ate)
      for (int j = 0; j < 3; ++j) {
        const double *wj = dW3.d() + j * nx + c0;
        // s_j += K_xX^T w_j, u_j += T' w_j = A^-1 K_xX^T w_j
        ck(ctx, launch_gemv_t(Kc, ldk, nc, n, wj, dvt.d(), st), "gemv_t");
        ck(ctx, launch_add(dvt.d(), dS3.d() + j * n, n, st), "add");
        if (tri) continue;
        ck(ctx, launch_gemv(dT.d(), n, n, nc, wj, dvt.d(), st), "gemv");
        ck(ctx, launch_add(dvt.d(), dU3.d() + j * n, n, st), "add");
      }
  }
  if (tri && ate) op.symv(dS3.d(), n, 3, dU3.d(), dtmp);  // u_j = A^-1 s_j
  op.kdiag(dkd.d());
  std::vector<double> q3(3, 0.0), dots(3, 0.0);
  if (ate) {
    // w_j^T Km_xx w_j with the full marginal test kernel
    int64_t ldx = 0;
    const double *Kxx = op.kxx(&ldx, dKmxx);
    alloc(ctx, dq3, (size_t)(3 * nx + 3) * sizeof(double), "alloc quad");
    ck(ctx, launch_quad3(Kxx, ldx, nx, dW3.d(), dq3.d(), st), "quad3");
    // s_j . u_j  (the rank's share of s_j^T A^-1 s_j)
    alloc(ctx, ddot, 3 * sizeof(double), "alloc dots");
    for (int j = 0; j < 3; ++j)
      ck(ctx, launch_gemv_t(dS3.d() + j * n, n, n, 1, dU3.d() + j * n, ddot.d() + j, st), "dot");
    if (op.allreduce) op.allreduce(ddot.d(), 3);
    download(ctx, q3.data(), dq3.d(), 3, "download quad");
    download(ctx, dots.data(), ddot.d(), 3, "download dots");
  }
  if (op.allreduce) op.allreduce(dad.d(), 2 * nx);
  std::vector<double> ad((size_t)(2 * nx)), kd((size_t)nx);
  download(ctx, ad.data(), dad.d(), ad.size(), "download sums");
  download(ctx, kd.data(), dkd.d(), kd.size(), "download diag");
  sync(ctx);
  if (!marginal) {
    finish_pred(nx, ad.data(), kd.data(), ad.data() + nx, sigma, mu, mean_y, std_y, map, ci, var);
    return;
  }
  std::vector<double> post(3);
  for (int j = 0; j < 3; ++j) post[(size_t)j] = q3[(size_t)j] - dots[(size_t)j];
  finish_marginal(nx, ad.data(), kd.data(), ad.data() + nx, std_y, std_Z,
                  ate ? zx.data() : nullptr, ate ? post.data() : nullptr, map, ci, var, avg);
}

// retained scratch above this size is released after the call (n = 16384,
// nx = 4096 keeps its 1.1 GB; n = 65536 with 8192-point chunks frees 8.6 GB)
constexpr size_t PRED_KEEP_BYTES = size_t(4) << 30;

void release_pred_state(ace_ctx *ctx) {
  if (auto ps = std::static_pointer_cast<PredScratch>(ctx->pred_state)) {
    ps->K.release();
    ps->T.release();
    ps->Kxx.release();
  }
  ctx->pred_state.reset();
}
}  // namespace

// The device prediction pipeline (pred_cpp / pred_marginal_cpp semantics)
// over abstract operands -- the device model's resident inverse here, and the
// device-matrix handles of the R6-faithful path in ace_dmat.cpp.  The large
// scratch (K_xX, T', K_xx chunks) stays in the context between calls; an
// allocation failure inside the call frees it -- all three buffers, including
// the ones the failed call still referenced -- and runs the call once more
// (outputs are written only at its end), and scratch above PRED_KEEP_BYTES
// is not kept past the call.
void pred_pipeline(const PredOps &op, int64_t nx, bool marginal, const double *Z_x, int ate,
                   double sigma, double mu, double mean_y, double std_y, double std_Z,
                   double *map, double *ci, double *var, double *avg) {
  ace_ctx *ctx = op.ctx;
  try {
    pred_pipeline_once(op, nx, marginal, Z_x, ate, sigma, mu, mean_y, std_y, std_Z, map, ci, var, avg);
  } catch (const Fail &f) {
    if (f.code != ACE_ERR_OOM) throw;
    (void)hipGetLastError();
    sync(ctx);  // the failed call's launches may still read the scratch
    release_pred_state(ctx);
    ctx->sweep_pool.clear();
    pred_pipeline_once(op, nx, marginal, Z_x, ate, sigma, mu, mean_y, std_y, std_Z, map, ci, var, avg);
  }
  if (auto ps = std::static_pointer_cast<PredScratch>(ctx->pred_state))
    if (ps->K.bytes + ps->T.bytes + ps->Kxx.bytes > PRED_KEEP_BYTES) release_pred_state(ctx);
}

namespace {

// ace_model_predict (marginal = false) / ace_model_predict_marginal: the
// model's resident inverse, K_xX assembled from the resident training side.
void predict_impl(ace_model *m, const double *theta, int64_t nx, const double *X2,
                  const double *Zt, bool marginal, const double *Z_x, int ate, double mean_y,
                  double std_y, double std_Z, double *map, double *ci, double *var, double *avg) {
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  const Shape &s = m->s;
  const int64_t n = m->n;
  const int B = s.B;
  const int b0 = marginal && B > 1 ? 1 : 0;  // src/pred_cpp.cpp:55-67
  const int b1 = marginal ? (B > 1 ? B : 1) : B;
  const double mu = theta[1];
  // kernels at the caller's theta (Q6)
  std::vector<double> tab = make_tab(theta, s, false);
  DBuf dtab, dw;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  const TabView tv = tab_view(dtab, s);
  SideBufs test;
  upload_side(ctx, test, s, X2, Zt, nx, nx);
  const PairSide train = m->shard ? shard_train_side(m->shard) : m->side.view(n);
  // w = y - mu: a = tmp (y - mu) with tmp^T = T' (src/pred_cpp.cpp:20, 70)
  alloc(ctx, dw, (size_t)n * sizeof(double), "alloc w");
  ck(ctx, launch_center(m->shard ? shard_train_y(m->shard) : m->y.d(), n, mu, dw.d(), st),
     "center y");
  PredOps op;
  op.ctx = ctx;
  op.n = n;
  op.w = dw.d();
  op.symm = [&](const double *V, int64_t ldv, int64_t k, double *out, DBuf &tmp) {
    symm_resident(m, V, ldv, true, k, out, tmp);
  };
  DBuf ddiag, dscal;
  if (!m->shard && pred_tri()) {  // -A^-1 is stored: scale -1
    alloc(ctx, ddiag, (size_t)n * sizeof(double), "alloc diag");
    ck(ctx, launch_diag_scaled(m->sw.A.d(), m->naug, n, -1.0, ddiag.d(), st), "diag");
    op.sdiag = ddiag.d();
    op.trmm = [&](const double *V, int64_t ldv, int64_t k, double *out) {
      ck(ctx, launch_trmm_lower(m->sw.A.d(), m->naug, n, V, ldv, k, -1.0, out, n, st), "trmm");
    };
    op.symv = [&](const double *V, int64_t ldv, int64_t k, double *out, DBuf &tmp) {
      symm_resident(m, V, ldv, false, k, out, tmp);
    };
    // A^-1 (y - mu) = A^-1 y - mu A^-1 1: the AUG rows the sweep left in A
    // (k_alpha_from_aug with the caller's mu), no n^2 pass
    alloc(ctx, dscal, 8 * sizeof(double), "alloc scalars");
    op.ainv_w = [&](double *dst) {
      ck(ctx, launch_alpha_from_aug(m->sw.A.d(), m->naug, m->npad, n, mu, 0, dst, dscal.d(), st,
                                    nullptr),
         "A^-1 w");
    };
  }
  if (m->shard) op.allreduce = [&](double *b, int64_t c) { shard_allreduce_sum(m->shard, b, c); };
  op.cross = [&](int64_t c0, int64_t nc, int64_t *ld, DBuf &scratch) -> const double * {
    alloc(ctx, scratch, (size_t)(nc * n) * sizeof(double), "alloc K_xX");
    PairSide tc = test.view(nc);
    tc.X += c0 * s.PM;
    tc.Z += c0 * s.ZS;
    tc.LZ += c0 * s.ZS;
    // kernmat_*_cpp(X2, X, Z2, Z): test side first
    ck(ctx, launch_assembly(2, s.kind, s.PM, tc, train, 0, B, s.ZS, tv, 0.0, scratch.d(), nc,
                            nullptr, st, nullptr, 0, 1, 0, b0, b1),
       "cross assembly");
    *ld = nc;
    return scratch.d();
  };
  op.kdiag = [&](double *dst) {
    ck(ctx, launch_kdiag(s.kind, test.view(nx), s.ZS, tv, b0, b1, dst, st), "kernel diagonal");
  };
  op.kxx = [&](int64_t *ld, DBuf &scratch) -> const double * {
    alloc(ctx, scratch, (size_t)(nx * nx) * sizeof(double), "alloc K_xx");
    ck(ctx, launch_assembly(1, s.kind, s.PM, test.view(nx), test.view(nx), 0, B, s.ZS, tv, 0.0,
                            scratch.d(), nx, nullptr, st, nullptr, 0, 1, 0, b0, b1),
       "symmetric assembly");
    *ld = nx;
    return scratch.d();
  };
  pred_pipeline(op, nx, marginal, Z_x, ate, theta[0], mu, mean_y, std_y, std_Z, map, ci, var, avg);
}

}  // namespace

extern "C" {

int ace_model_apply_inverse(ace_model *m, int64_t k, const double *V, double *out) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, k >= 1 && V && out, "bad shape / null argument");
  require_inverse(m);
  const int64_t n = m->n;
  DBuf dV, dout, dtmp;
  upload(ctx, dV, V, (size_t)(n * k), "upload V");
  alloc(ctx, dout, (size_t)(n * k) * sizeof(double), "alloc out");
  symm_resident(m, dV.d(), n, false, k, dout.d(), dtmp);
  if (m->shard) shard_allreduce_sum(m->shard, dout.d(), n * k);
  download(ctx, out, dout.d(), (size_t)(n * k), "download out");
  sync(ctx);
  return ACE_OK;
  ACE_CATCH
}

int ace_model_predict(ace_model *m, const double *theta, int64_t nx, const double *X2,
                      const double *Z2, double mean_y, double std_y, double *map, double *ci,
                      double *var) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, nx >= 1 && theta && map && ci && var && (m->s.p == 0 || X2) && (m->s.B == 1 || Z2),
      "bad shape / null argument");
  require_inverse(m);
  predict_impl(m, theta, nx, X2, Z2, false, nullptr, 0, mean_y, std_y, 1.0, map, ci, var, nullptr);
  return ACE_OK;
  ACE_CATCH
}

int ace_model_predict_marginal(ace_model *m, const double *theta, int64_t nx, const double *X2,
                               const double *dZ2, const double *Z_x, double std_y, double std_Z,
                               int calculate_ate, double *map, double *ci, double *var,
                               double *avg) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, nx >= 1 && theta && map && ci && var && (m->s.p == 0 || X2) && (m->s.B == 1 || dZ2),
      "bad shape / null argument");
  arg(ctx, !calculate_ate || (Z_x && avg), "calculate_ate needs Z_x and avg");
  require_inverse(m);
  predict_impl(m, theta, nx, X2, dZ2, true, Z_x, calculate_ate, 0.0, std_y, std_Z, map, ci, var,
               avg);
  return ACE_OK;
  ACE_CATCH
}

}  // extern "C"
