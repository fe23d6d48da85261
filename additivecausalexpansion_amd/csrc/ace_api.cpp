// ace_api.cpp -- C ABI (include/ace_hip.h) over the HIP kernels: context,
// argument checking, layout packing, the drop-in Rcpp-export equivalents
// and the device-resident para_update pipeline.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ace_hip.h"

#include "ace_common.h"
#include "ace_internal.h"
#include "ace_model.h"

using namespace ace;

std::string g_create_err;

namespace {
double sync_timeout_s() {
  static double v = -1.0;
  if (v < 0.0) {
    const char *e = getenv("ACE_SYNC_TIMEOUT");
    v = e ? std::max(0.0, atof(e)) : 600.0;
  }
  return v;
}
}  // namespace

// Bounded drain of one stream (ace_common.h).  Polls hipStreamQuery: yields
// for the first 100 ms (an evaluation is ~75 ms, so the common wait costs no
// extra latency), then sleeps 100 us between polls.  On the deadline the
// error names which of the context's streams still hold work, which is what
// a stalled hardware queue or a hung collective looks like from the host.
void ace_host::sync_stream(ace_ctx *ctx, hipStream_t s, const char *what) {
  const double lim = sync_timeout_s();
  if (lim <= 0.0) {
    ck(ctx, hipStreamSynchronize(s), what);
    return;
  }
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) ck(ctx, e, what);
    const double dt = std::chrono::duration<double>(clk::now() - t0).count();
    if (dt > lim) {
      std::string busy;
      const hipStream_t all[3] = {ctx->stream, ctx->side, ctx->side2};
      const char *names[3] = {"main", "side", "side2"};
      for (int i = 0; i < 3; ++i) {
        bool dup = false;
        for (int j = 0; j < i; ++j) dup = dup || all[j] == all[i];
        if (!all[i] || dup) continue;
        if (hipStreamQuery(all[i]) == hipErrorNotReady) busy += std::string(" ") + names[i];
      }
      char buf[160];
      snprintf(buf, sizeof buf, "%s: device work did not complete within %.0f s (streams still busy:%s)",
               what, lim, busy.empty() ? " none" : busy.c_str());
      ctx->err = buf;
      ctx->failed = true;  // later calls refuse to run (check_usable)
      fprintf(stderr, "ace: %s\n", buf);
      throw Fail{ACE_ERR_TIMEOUT};
    }
    if (dt < 0.1) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
}


extern "C" {

int ace_abi_version(void) { return ACE_ABI_VERSION; }

int ace_create(int device, ace_ctx **out) {
  if (!out) return ACE_ERR_ARG;
  *out = nullptr;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    g_create_err = std::string("no HIP device available: ") +
                   (e == hipSuccess ? "count == 0" : hipGetErrorString(e));
    return ACE_ERR_HIP;
  }
  if (device < 0 || device >= count) {
    g_create_err = "device index out of range";
    return ACE_ERR_ARG;
  }
  e = hipSetDevice(device);
  if (e != hipSuccess) {
    g_create_err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return ACE_ERR_HIP;
  }
  ace_ctx *c = new ace_ctx();
  c->device = device;
  // ACE_STREAMS: how many streams the context creates: 3 = main +
  // panel chain + tail path (default), 2 = the tail path on the panel
  // stream, 1 = everything on the main stream (no lookahead overlap).  The
  // results are bit-identical for every value.
  const char *vs = getenv("ACE_STREAMS");
  const int nstr = vs ? std::min(3, std::max(1, atoi(vs))) : 3;
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) c->nstreams = 1;
  if (e == hipSuccess && nstr >= 2) {
    // the lookahead streams are latency-bound: the highest priority, so their
    // workgroups take the first free CU slots next to the update kernel
    // (the range on the box: least 1, greatest -1, default 0)
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    e = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, hi);
    if (e == hipSuccess) c->nstreams = 2;
    if (e == hipSuccess && nstr >= 3) {
      // (at the main stream's priority instead: neutral)
      e = hipStreamCreateWithPriority(&c->side2, hipStreamNonBlocking, hi);
      if (e == hipSuccess) c->nstreams = 3;
    }
  }
  if (e != hipSuccess) {
    g_create_err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
    ace_destroy(c);
    return ACE_ERR_HIP;
  }
  // aliases for a smaller budget: a wait on an event of the same stream is
  // free, so the schedules run unchanged in host order
  if (!c->side) c->side = c->stream;
  if (!c->side2) c->side2 = c->side;
  *out = c;
  return ACE_OK;
}

void ace_destroy(ace_ctx *ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->side2 && ctx->side2 != ctx->side) (void)hipStreamDestroy(ctx->side2);
  if (ctx->side && ctx->side != ctx->stream) (void)hipStreamDestroy(ctx->side);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int ace_set_interrupt_poll(ace_ctx *ctx, int (*poll)(void *user), void *user) {
  if (!ctx) return ACE_ERR_ARG;
  ctx->poll = poll;
  ctx->poll_user = user;
  return ACE_OK;
}

const char *ace_last_error(const ace_ctx *ctx) {
  if (!ctx) return g_create_err.c_str();
  return ctx->err.c_str();
}

// ------------------------------------------------------------ assembly
int ace_kernmat_sym(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *X,
                    const double *Z, const double *theta, double *Kfull, double *Kel) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, n >= 1 && theta && Kfull && (p == 0 || X) && (B == 1 || Z), "null argument");
  SideBufs sb;
  upload_side(ctx, sb, s, X, Z, n, n);
  std::vector<double> tab = make_tab(theta, s, false);
  DBuf dtab, dK, dC;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  alloc(ctx, dK, (size_t)(n * n) * sizeof(double), "alloc Kfull");
  if (Kel) alloc(ctx, dC, (size_t)(n * n * B) * sizeof(double), "alloc cube");
  ck(ctx, launch_assembly(1, kind, s.PM, sb.view(n), sb.view(n), n, B, s.ZS, tab_view(dtab, s),
                          0.0, dK.d(), n, Kel ? dC.d() : nullptr, ctx->stream),
     "assembly");
  download(ctx, Kfull, dK.d(), (size_t)(n * n), "download Kfull");
  if (Kel) download(ctx, Kel, dC.d(), (size_t)(n * n * B), "download cube");
  sync(ctx);
  return ACE_OK;
  ACE_CATCH
}

int ace_kernmat_cross(ace_ctx *ctx, int kind, int64_t n1, int64_t n2, int p, int B,
                      const double *X1, const double *X2, const double *Z1, const double *Z2,
                      const double *theta, double *Kfull, double *Kel) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, n1 >= 1 && n2 >= 1 && theta && Kfull, "bad shape / null argument");
  arg(ctx, (p == 0 || (X1 && X2)) && (B == 1 || (Z1 && Z2)), "null argument");
  SideBufs s1, s2;
  upload_side(ctx, s1, s, X1, Z1, n1, n1);
  upload_side(ctx, s2, s, X2, Z2, n2, n2);
  std::vector<double> tab = make_tab(theta, s, false);
  DBuf dtab, dK, dC;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  alloc(ctx, dK, (size_t)(n1 * n2) * sizeof(double), "alloc Kfull");
  if (Kel) alloc(ctx, dC, (size_t)(n1 * n2 * B) * sizeof(double), "alloc cube");
  ck(ctx, launch_assembly(2, kind, s.PM, s1.view(n1), s2.view(n2), 0, B, s.ZS,
                          tab_view(dtab, s), 0.0, dK.d(), n1, Kel ? dC.d() : nullptr,
                          ctx->stream),
     "assembly");
  download(ctx, Kfull, dK.d(), (size_t)(n1 * n2), "download Kfull");
  if (Kel) download(ctx, Kel, dC.d(), (size_t)(n1 * n2 * B), "download cube");
  sync(ctx);
  return ACE_OK;
  ACE_CATCH
}

// ------------------------------------------------------------ inverse

int ace_invkernel(ace_ctx *ctx, int64_t n, const double *K, double sigma, double *eigenval,
                  double *inv) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, n >= 1 && K, "bad shape / null argument");
  SweepWork w;
  w.ensure(ctx, n);
  DBuf dK;
  upload(ctx, dK, K, (size_t)(n * n), "upload K");
  ck(ctx, launch_prepare_A(dK.d(), n, std::exp(sigma), w.A.d(), w.naug, w.npad, ctx->stream),
     "prepare A");
  ck(ctx, launch_aug_init(w.A.d(), w.naug, w.npad, 0, nullptr, ctx->stream), "aug init");
  ck(ctx, hipMemsetAsync(w.flag.p, 0, sizeof(int), ctx->stream), "memset flag");
  const SweepSync sy = w.sync(ctx);
  ck(ctx, run_sweep(w.bufs(), ctx->stream, &sy, nullptr), "sweep");
  int flag = 0;
  ck(ctx, hipMemcpyAsync(&flag, w.flag.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream),
     "download flag");
  if (inv) {
    ck(ctx, launch_sym_from_lower(w.A.d(), w.naug, n, -1.0, dK.d(), n, ctx->stream),
       "symmetrize");
    download(ctx, inv, dK.d(), (size_t)(n * n), "download inv");
  }
  if (eigenval) download(ctx, eigenval, w.piv.d(), (size_t)n, "download pivots");
  sync(ctx);
  if (flag && inv)  // not positive definite: the reference's inverse is NaN
    for (int64_t j = 0; j < n * n; ++j) inv[j] = kNaN;
  return ACE_OK;
  ACE_CATCH
}

// ------------------------------------------------------------ gradient
int ace_grad(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *y, const double *X,
             const double *Z, const double *Kfull, const double *Kel, const double *inv,
             const double *eigenval, const double *theta, double *stats, double std_y,
             double *grad) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  Shape s = check_shape(ctx, kind, p, B);
  arg(ctx, n >= 1 && y && Kfull && inv && eigenval && theta && stats && grad, "null argument");
  arg(ctx, (p == 0 || X) && (B == 1 || Z), "null argument");
  SideBufs sb;
  upload_side(ctx, sb, s, X, Z, n, (n + 63) / 64 * 64);  // k_grad reads whole 64-row tiles
  std::vector<double> tab = make_tab(theta, s);
  std::vector<double> ybar((size_t)n);
  for (int64_t r = 0; r < n; ++r) ybar[(size_t)r] = y[r] - theta[1];
  DBuf dtab, dy, dyb, dinv, dKf, dC, dalpha, ds, dg, dwork, dgs, dsums, dmu;
  upload(ctx, dtab, tab.data(), tab.size(), "upload tables");
  upload(ctx, dy, y, (size_t)n, "upload y");
  upload(ctx, dyb, ybar.data(), (size_t)n, "upload ybar");
  upload(ctx, dinv, inv, (size_t)(n * n), "upload inv");
  upload(ctx, dKf, Kfull, (size_t)(n * n), "upload Kfull");
  if (Kel) upload(ctx, dC, Kel, (size_t)(n * n * B), "upload cube");
  upload(ctx, dmu, &theta[1], 1, "upload mu");
  alloc(ctx, dalpha, (size_t)n * sizeof(double), "alloc alpha");
  alloc(ctx, ds, (size_t)n * sizeof(double), "alloc s");
  const int64_t nt = grad_ntiles(n);
  const int ncol = B * (s.PM + 1);
  const int ldg = grad_part_cols(s.PM, B);  // ncol + trace
  alloc(ctx, dg, (size_t)(nt * ldg) * sizeof(double), "alloc gpart");
  alloc(ctx, dwork, (size_t)tile_sums_work(ldg) * sizeof(double), "alloc tile sums");
  alloc(ctx, dgs, (size_t)ldg * sizeof(double), "alloc gsum");
  alloc(ctx, dsums, 8 * sizeof(double), "alloc sums");
  // alpha = invKmatn * ybar (src/kernel_SE_cpp.cpp:215)
  ck(ctx, launch_gemv(dinv.d(), n, n, n, dyb.d(), dalpha.d(), ctx->stream), "gemv alpha");
  ck(ctx, launch_grad(kind, s.PM, sb.view(n), B, s.ZS, tab_view(dtab, s), dinv.d(), n, 1.0,
                      dalpha.d(), Kel ? dC.d() : nullptr, dg.d(), ctx->stream),
     "grad");
  ck(ctx, launch_tile_sums(dg.d(), nt, ldg, dwork.d(), dgs.d(), ctx->stream), "tile sums");
  // Kfull * alpha for the RMSE (src/kernel_SE_cpp.cpp:238)
  ck(ctx, launch_gemv(dKf.d(), n, n, n, dalpha.d(), ds.d(), ctx->stream), "gemv K alpha");
  ck(ctx, launch_final_sums(dy.d(), dmu.d(), dalpha.d(), ds.d(), 0.0, n, nullptr, 0, dsums.d(),
                            ctx->stream),
     "final sums");
  std::vector<double> gs((size_t)(ncol + 1)), sums(8);
  download(ctx, gs.data(), dgs.d(), gs.size(), "download gsum");
  download(ctx, sums.data(), dsums.d(), 4, "download sums");
  sync(ctx);
  compose_grad(s, theta, gs.data(), sums[2], grad);
  const double logdet = host_logsum(eigenval, n);
  stats[0] = std_y * std::sqrt(sums[0]) / std::sqrt((double)n);
  stats[1] = -0.5 * (n * std::log(2.0 * M_PI) + logdet + sums[1]);
  return ACE_OK;
  ACE_CATCH
}

int ace_stats(ace_ctx *ctx, int64_t n, const double *y, const double *Kmat, const double *inv,
              const double *eigenval, double mu, double std_y, double *out) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, n >= 1 && y && Kmat && inv && eigenval && out, "null argument");
  std::vector<double> ybar((size_t)n);
  for (int64_t r = 0; r < n; ++r) ybar[(size_t)r] = y[r] - mu;
  DBuf dy, dyb, dinv, dK, dalpha, ds, dsums, dmu;
  upload(ctx, dy, y, (size_t)n, "upload y");
  upload(ctx, dyb, ybar.data(), (size_t)n, "upload ybar");
  upload(ctx, dinv, inv, (size_t)(n * n), "upload inv");
  upload(ctx, dK, Kmat, (size_t)(n * n), "upload K");
  upload(ctx, dmu, &mu, 1, "upload mu");
  alloc(ctx, dalpha, (size_t)n * sizeof(double), "alloc");
  alloc(ctx, ds, (size_t)n * sizeof(double), "alloc");
  alloc(ctx, dsums, 8 * sizeof(double), "alloc");
  ck(ctx, launch_gemv(dinv.d(), n, n, n, dyb.d(), dalpha.d(), ctx->stream), "gemv");
  ck(ctx, launch_gemv(dK.d(), n, n, n, dalpha.d(), ds.d(), ctx->stream), "gemv");
  ck(ctx, launch_final_sums(dy.d(), dmu.d(), dalpha.d(), ds.d(), 0.0, n, nullptr, 0, dsums.d(),
                            ctx->stream),
     "sums");
  double sums[4];
  download(ctx, sums, dsums.d(), 4, "download");
  sync(ctx);
  out[0] = std_y * std::sqrt(sums[0]) / std::sqrt((double)n);
  out[1] = -0.5 * (n * std::log(2.0 * M_PI) + host_logsum(eigenval, n) + sums[1]);
  return ACE_OK;
  ACE_CATCH
}

int ace_mu_solution(ace_ctx *ctx, int64_t n, const double *y, const double *inv, double *out) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, n >= 1 && y && inv && out, "null argument");
  DBuf dy, dinv, dt, dcs;
  upload(ctx, dy, y, (size_t)n, "upload y");
  upload(ctx, dinv, inv, (size_t)(n * n), "upload inv");
  alloc(ctx, dt, (size_t)n * sizeof(double), "alloc");
  alloc(ctx, dcs, (size_t)n * sizeof(double), "alloc");
  ck(ctx, launch_gemv(dinv.d(), n, n, n, dy.d(), dt.d(), ctx->stream), "gemv");
  ck(ctx, launch_colsum(dinv.d(), n, (int)n, dcs.d(), ctx->stream), "colsum");
  std::vector<double> t((size_t)n), cs((size_t)n);
  download(ctx, t.data(), dt.d(), (size_t)n, "download");
  download(ctx, cs.data(), dcs.d(), (size_t)n, "download");
  sync(ctx);
  double st = 0.0, sa = 0.0;
  for (int64_t j = 0; j < n; ++j) {
    st += t[(size_t)j];
    sa += cs[(size_t)j];
  }
  *out = 0.5 * st / sa;  // Q4
  return ACE_OK;
  ACE_CATCH
}

// ------------------------------------------------------------ prediction
int ace_pred(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X, double sigma, double mu,
             const double *invK_XX, const double *K_xX, const double *K_xx, double mean_y,
             double std_y, double *map, double *ci, double *var) {
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, nX >= 1 && nx >= 1 && y_X && invK_XX && K_xX && K_xx && map && ci && var,
      "null argument");
  std::vector<double> w((size_t)nX);
  for (int64_t c = 0; c < nX; ++c) w[(size_t)c] = y_X[c] - mu;
  DBuf dinv, dK, dT, dw, da, dq;
  upload(ctx, dinv, invK_XX, (size_t)(nX * nX), "upload inv");
  upload(ctx, dK, K_xX, (size_t)(nx * nX), "upload K_xX");
  upload(ctx, dw, w.data(), (size_t)nX, "upload w");
  alloc(ctx, dT, (size_t)(nx * nX) * sizeof(double), "alloc tmp");
  alloc(ctx, da, (size_t)nx * sizeof(double), "alloc");
  alloc(ctx, dq, (size_t)nx * sizeof(double), "alloc");
  // tmp = K_xX * invK_XX (src/pred_cpp.cpp:19)
  ck(ctx, launch_gemm_nn(nx, nX, nX, dK.d(), nx, dinv.d(), nX, dT.d(), nx, ctx->stream), "gemm");
  ck(ctx, launch_pred_rows(dT.d(), dK.d(), nx, nx, nX, dw.d(), da.d(), dq.d(), ctx->stream),
     "pred rows");
  std::vector<double> a((size_t)nx), q((size_t)nx);
  download(ctx, a.data(), da.d(), (size_t)nx, "download");
  download(ctx, q.data(), dq.d(), (size_t)nx, "download");
  sync(ctx);
  std::vector<double> kd((size_t)nx);
  for (int64_t r = 0; r < nx; ++r) kd[(size_t)r] = K_xx[r + r * nx];
  finish_pred(nx, a.data(), kd.data(), q.data(), sigma, mu, mean_y, std_y, map, ci, var);
  return ACE_OK;
  ACE_CATCH
}

int ace_pred_marginal(ace_ctx *ctx, int64_t nX, int64_t nx, int B, const double *y_X,
                      const double *Z_x, double sigma, double mu, const double *invK_XX,
                      const double *K_xX, const double *K_xx, double mean_y, double std_y,
                      double std_Z, int calculate_ate, double *map, double *ci, double *var,
                      double *avg) {
  (void)sigma;
  (void)mean_y;
  if (!ctx) return ACE_ERR_ARG;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, nX >= 1 && nx >= 1 && B >= 1 && y_X && invK_XX && K_xX && K_xx && map && ci && var,
      "null argument");
  arg(ctx, !calculate_ate || (Z_x && avg), "calculate_ate needs Z_x and avg");
  std::vector<double> w((size_t)nX);
  for (int64_t c = 0; c < nX; ++c) w[(size_t)c] = y_X[c] - mu;
  DBuf dinv, dcX, dcx, dmX, dmx, dT, dw, da, dq;
  upload(ctx, dinv, invK_XX, (size_t)(nX * nX), "upload inv");
  upload(ctx, dcX, K_xX, (size_t)(nx * nX * B), "upload K_xX");
  upload(ctx, dcx, K_xx, (size_t)(nx * nx * B), "upload K_xx");
  upload(ctx, dw, w.data(), (size_t)nX, "upload w");
  alloc(ctx, dmX, (size_t)(nx * nX) * sizeof(double), "alloc");
  alloc(ctx, dmx, (size_t)(nx * nx) * sizeof(double), "alloc");
  alloc(ctx, dT, (size_t)(nx * nX) * sizeof(double), "alloc");
  alloc(ctx, da, (size_t)nx * sizeof(double), "alloc");
  alloc(ctx, dq, (size_t)nx * sizeof(double), "alloc");
  ck(ctx, launch_marginal_sum(dcX.d(), nx, nX, B, dmX.d(), ctx->stream), "marginal sum");
  ck(ctx, launch_marginal_sum(dcx.d(), nx, nx, B, dmx.d(), ctx->stream), "marginal sum");
  ck(ctx, launch_gemm_nn(nx, nX, nX, dmX.d(), nx, dinv.d(), nX, dT.d(), nx, ctx->stream),
     "gemm");
  ck(ctx, launch_pred_rows(dT.d(), dmX.d(), nx, nx, nX, dw.d(), da.d(), dq.d(), ctx->stream),
     "pred rows");
  std::vector<double> a((size_t)nx), q((size_t)nx), dg((size_t)nx);
  download(ctx, a.data(), da.d(), (size_t)nx, "download");
  download(ctx, q.data(), dq.d(), (size_t)nx, "download");
  ck(ctx, hipMemcpy2DAsync(dg.data(), sizeof(double), dmx.d(), (size_t)(nx + 1) * sizeof(double),
                           sizeof(double), (size_t)nx, hipMemcpyDeviceToHost, ctx->stream),
     "download diag");
  std::vector<double> q3(3), tw((size_t)(3 * nX)), kw((size_t)(3 * nX));
  DBuf dW3, dq3, dtw, dkw;
  std::vector<double> zx;
  if (calculate_ate) {
    zx.assign(Z_x, Z_x + nx);
    std::vector<double> W3((size_t)(3 * nx));
    for (int64_t r = 0; r < nx; ++r) {
      W3[(size_t)r] = 1.0;
      W3[(size_t)(nx + r)] = zx[(size_t)r];
      W3[(size_t)(2 * nx + r)] = (zx[(size_t)r] == 0) ? 1.0 : 0.0;
    }
    upload(ctx, dW3, W3.data(), W3.size(), "upload weights");
    alloc(ctx, dq3, (size_t)(3 * nx + 3) * sizeof(double), "alloc");
    alloc(ctx, dtw, (size_t)(3 * nX) * sizeof(double), "alloc");
    alloc(ctx, dkw, (size_t)(3 * nX) * sizeof(double), "alloc");
    ck(ctx, launch_quad3(dmx.d(), nx, nx, dW3.d(), dq3.d(), ctx->stream), "quad3");
    for (int j = 0; j < 3; ++j) {
      ck(ctx, launch_gemv_t(dT.d(), nx, nx, nX, dW3.d() + j * nx, dtw.d() + j * nX, ctx->stream),
         "gemv_t");
      ck(ctx, launch_gemv_t(dmX.d(), nx, nx, nX, dW3.d() + j * nx, dkw.d() + j * nX,
                            ctx->stream),
         "gemv_t");
    }
    download(ctx, q3.data(), dq3.d(), 3, "download");
    download(ctx, tw.data(), dtw.d(), tw.size(), "download");
    download(ctx, kw.data(), dkw.d(), kw.size(), "download");
  }
  sync(ctx);
  std::vector<double> post;
  if (calculate_ate) {
    // posterior quadratic forms w^T (Km_xx - tmp Km_xX^T) w (src/pred_cpp.cpp:89-106)
    post.assign(3, 0.0);
    for (int j = 0; j < 3; ++j) {
      double cross = 0.0;
      for (int64_t c = 0; c < nX; ++c) cross += tw[(size_t)(j * nX + c)] * kw[(size_t)(j * nX + c)];
      post[(size_t)j] = q3[(size_t)j] - cross;
    }
  }
  finish_marginal(nx, a.data(), dg.data(), q.data(), std_y, std_Z, calculate_ate ? zx.data() : nullptr,
                  calculate_ate ? post.data() : nullptr, map, ci, var, avg);
  return ACE_OK;
  ACE_CATCH
}

}  // extern "C"

// CUs per shader engine the assembly's second part leaves to the first sweep group's
// head path (ACE_ASM_PERSIST, default 1; 0: the plain grid)
static int asm_persist_reserve() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_ASM_PERSIST");
    v = e ? std::max(0, std::min(2, atoi(e))) : 1;
  }
  return v;
}

// with the reservation: ACE_ASM_TAIL=1 (default) lets group 0's tail path run
// on the reserved CUs beside its head path, =2 after it (0: it waits for the
// whole assembly); ACE_ASM_FILL=1 (default) hands
// the reserved CUs back to the assembly's queue once group 0's lookahead is
// done (a filler launch on side2)
static int env_flag(const char *name, int dflt) {
  const char *e = getenv(name);
  return e ? atoi(e) : dflt;
}
static int asm_tail_mode() {
  static const int v = env_flag("ACE_ASM_TAIL", 1);
  return v;
}
static bool asm_fill_on() {
  static const bool v = env_flag("ACE_ASM_FILL", 1) != 0;
  return v;
}

struct AsmFill {
  int kind, PM, B, ZS, slots;
  PairSide ps;
  int64_t npad, naug;
  TabView tv;
  double sig;
  double *A;
  int *queue;
};

static hipError_t asm_fill(void *arg, hipStream_t st) {
  const AsmFill *f = (const AsmFill *)arg;
  return launch_assembly_persist(f->kind, f->PM, f->ps, f->npad, f->B, f->ZS, f->tv, f->sig, f->A,
                                 f->naug, st, f->queue, 0, f->slots);
}

// A = Kfull + sig I (lower 64-tiles, assembly mode 0) into w.A with the AUG
// rows [y; 1] (y null: the 1 row only), then the sweep.  The first sweep
// group's panels' columns are assembled first: that group's pivot chains and
// lookahead crosses (side stream) then run under the rest of the assembly.
// ev_asm (optional): two timing events around the assembly.
void assemble_and_sweep(ace_ctx *ctx, SweepWork &w, const Shape &s, const PairSide &ps,
                        const TabView &tv, double sig, const double *y, int64_t n,
                        const SweepTiming *tmg, hipEvent_t *ev_asm) {
  hipStream_t st = ctx->stream;
  const int steps = (int)(w.npad / NB);
  SweepSync sy = w.sync(ctx);
  // ACE_ASM_PERSIST=R: the second part as a persistent work queue that
  // leaves R CUs of every shader engine to the first group's head path
  // (DESIGN §5); the queue is reset before anything can join it
  const int R = asm_persist_reserve();
  const bool persist = R > 0 && sy.side && sy.nev >= 5 * steps + 6 && pairs_use_mm(s.PM, false) &&
                       mm_lds_ok(s.PM, s.B, s.kind, false);
  // (the flag and the persistent assembly's queue are zeroed by the same launch)
  ck(ctx, launch_aug_init(w.A.d(), w.naug, w.npad, n, y, st, 1, 0, w.flag.i(), 1,
                          persist ? w.aq.i() : nullptr, persist ? 2 + 64 : 0),
     "aug init");
  if (ev_asm) ck(ctx, hipEventRecord(ev_asm[0], st), "event");
  ck(ctx, launch_assembly(0, s.kind, s.PM, ps, ps, w.npad, s.B, s.ZS, tv, sig, w.A.d(), w.naug,
                          nullptr, st, nullptr, 0, 1, 1),
     "assembly (first panel)");
  if (sy.side && sy.nev >= 2 * steps + 1) {  // run_sweep's "inputs ready" event
    ck(ctx, hipEventRecord(sy.ev[2 * steps], st), "event");
    sy.ready_recorded = true;
  }
  AsmFill fill;
  if (persist && sy.ready_recorded) {
    ck(ctx, launch_assembly_persist(s.kind, s.PM, ps, w.npad, s.B, s.ZS, tv, sig, w.A.d(), w.naug,
                                    st, w.aq.i(), R),
       "assembly (persistent)");
    const int tail = asm_tail_mode();
    if (tail == 0) {  // group 0's tail path after the whole assembly
      sy.tail_after = sy.ev[5 * steps + 5];
      ck(ctx, hipEventRecord(sy.tail_after, st), "event");
    }
    sy.tail_split = tail == 2;  // ... after group 0's head path
    const int per = asm_fill_on() ? assembly_persist_per_cu(s.kind, s.PM, s.B) : 0;
    if (per > 0) {  // the reserved CUs: R per engine, 4 engines per XCD, 8 XCDs
      fill = AsmFill{s.kind, s.PM, s.B, s.ZS, 32 * R * per, ps, w.npad, w.naug, tv, sig, w.A.d(), w.aq.i()};
      sy.fill = asm_fill;
      sy.fill_arg = &fill;
    }
  } else {
    ck(ctx, launch_assembly(0, s.kind, s.PM, ps, ps, w.npad, s.B, s.ZS, tv, sig, w.A.d(), w.naug,
                            nullptr, st, nullptr, 0, 1, 2),
       "assembly");
  }
  // with the persistent queue this marks the MAIN launch's end: the tiles
  // the filler launch (side2, after group 0's lookahead) takes are counted in
  // the assembly's work but not in this interval (DESIGN §8 note)
  if (ev_asm) ck(ctx, hipEventRecord(ev_asm[1], st), "event");
  ck(ctx, run_sweep(w.bufs(), st, &sy, tmg), "sweep");
}

// The gradient's tile list for n: diagonal 64-tiles first, then the strictly
// lower ones dealt to the XCDs in S x S super-blocks (a launch's block b runs
// on XCD b % 8).  *ndiag = -1 (and no list) for the row-major grid.
void build_grad_tiles(ace_ctx *ctx, int64_t n, DBuf &tiles, int64_t *ntiles, int64_t *ndiag) {
  *ntiles = grad_ntiles(n);
  *ndiag = -1;
  const int S = grad_order_block();
  if (S <= 0) return;
  const int64_t ntr = (n + AT - 1) / AT;
  std::vector<Tile> lst, low;
  for (int64_t I = 0; I < ntr; ++I) lst.push_back(Tile{(int)I, (int)I});
  for (int64_t I = 1; I < ntr; ++I)
    for (int64_t J = 0; J < I; ++J) low.push_back(Tile{(int)I, (int)J});
  const std::vector<Tile> o = xcd_update_order(low, S);
  lst.insert(lst.end(), o.begin(), o.end());
  alloc(ctx, tiles, lst.size() * sizeof(Tile), "alloc grad tiles");
  upload_bytes(ctx, tiles.p, lst.data(), lst.size() * sizeof(Tile), "upload grad tiles");
  *ntiles = (int64_t)lst.size();
  *ndiag = ntr;
}

// ACE_NORMS=0: every pair tile computes its own slice norms (A/B switch;
// the table is bit-identical)
static bool slice_norms_on() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_NORMS");
    v = e ? (atoi(e) != 0) : 1;
  }
  return v != 0;
}

namespace {

// One evaluation on the stream.  theta_dev != nullptr: theta is a device
// vector (the device-fused training loop) -- tables, exp(theta[0]) and
// theta[1] are then read on the device and `theta` is not used.
void model_pipeline(ace_model *m, SweepWork &w, const double *theta, int use_mu, bool timed,
                    const double *theta_dev = nullptr) {
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  const Shape &s = m->s;
  TabView tv = tab_view(m->tab, s);
  double sig = 0.0;
  if (theta_dev) {
    ck(ctx, launch_make_tab(theta_dev, s.B, s.p, s.PM, m->tab.d(), st), "tables");
    tv.sig = m->tab.d() + 2 * s.B * s.PM + s.B;
  } else {
    std::vector<double> tab = make_tab(theta, s);
    // pinned staging, async on the stream: the previous evaluation's results
    // were synchronised before this one started, so the region is free
    double *h = m->hio.ensure(ctx, tab.size() + m->res.bytes / sizeof(double));
    std::copy(tab.begin(), tab.end(), h);
    ck(ctx, hipMemcpyAsync(m->tab.p, h, tab.size() * sizeof(double), hipMemcpyHostToDevice, st),
       "upload tables");
    sig = std::exp(theta[0]);
  }
  const PairSide ps = m->side.view(m->n);
  if (m->norms.p) {  // the slice norms once per point, for the assembly and the gradient
    const int NS = s.kind == ACE_KERNEL_MATERN32 ? s.B + 1 : s.B;
    ck(ctx, launch_slice_norms(ps.X, s.PM, m->npad, s.B, NS, tv.wk,
                               s.kind == ACE_KERNEL_MATERN32 ? tv.wg + (s.B - 1) * s.PM : tv.wk,
                               m->norms.d(), st),
       "slice norms");
    tv.norms = m->norms.d();
    tv.ldn = m->npad;
  }
  const int ts = m->tset;
  SweepTiming tmg;
  const size_t nset = m->ev_upd.size() / 2;
  tmg.ev = m->ev_upd.data() + ts * nset;
  tmg.nev = (int)nset;
  tmg.used = &m->upd_used[ts];
  tmg.flops = m->upd_flops.data() + ts * (nset / 2);
  assemble_and_sweep(ctx, w, s, ps, tv, sig, m->y.d(), m->n, timed ? &tmg : nullptr,
                     timed ? m->ev_asm + 2 * ts : nullptr);
  ck(ctx, launch_alpha_from_aug(w.A.d(), w.naug, w.npad, m->n, theta_dev ? 0.0 : theta[1], use_mu,
                                m->alpha.d(), m->scal.d(), st, theta_dev ? theta_dev + 1 : nullptr),
     "alpha");
  // RMSE residual ybar - Kfull alpha = sig alpha (A = Kfull + sig I is what
  // the sweep inverted): no Kfull copy and no pass over it (k_final_sums)
  if (timed) ck(ctx, hipEventRecord(m->ev_grad[2 * ts], st), "event");
  ck(ctx, launch_grad(s.kind, s.PM, ps, s.B, s.ZS, tv, w.A.d(), w.naug, -1.0, m->alpha.d(),
                      nullptr, m->gpart.d(), st, reinterpret_cast<const Tile *>(m->gtiles.p),
                      m->ngdiag >= 0 ? m->ntiles : 0, 1, m->ngdiag),
     "grad");
  if (timed) ck(ctx, hipEventRecord(m->ev_grad[2 * ts + 1], st), "event");
  const int ldg = grad_part_cols(s.PM, s.B);
  ck(ctx, launch_tile_sums(m->gpart.d(), m->ntiles, ldg, m->gwork.d(), m->gsum.d(), st),
     "tile sums");
  ck(ctx, launch_final_sums(m->y.d(), m->scal.d() + 4, m->alpha.d(), nullptr, sig, m->n,
                            w.piv.d(), w.npad, m->sums.d(), st, tv.sig, w.flag.i()),
     "final sums");
}

// Reads the event set `ts` of an evaluation whose work has completed.
void model_collect_timing(ace_model *m, int ts) {
  const int nupd = m->upd_used[ts];
  const size_t nset = m->ev_upd.size() / 2;
  const hipEvent_t *ev = m->ev_upd.data() + ts * nset;
  const double *fl = m->upd_flops.data() + ts * (nset / 2);
  float ms = 0.f;
  ck(m->ctx, hipEventElapsedTime(&ms, m->ev_asm[2 * ts], m->ev_asm[2 * ts + 1]), "elapsed");
  m->t_ms[1] += ms;
  m->t_launch[1] += 1;
  ck(m->ctx, hipEventElapsedTime(&ms, m->ev_grad[2 * ts], m->ev_grad[2 * ts + 1]), "elapsed");
  m->t_ms[2] += ms;
  m->t_launch[2] += 1;
  for (int j = 0; j + 1 < nupd; j += 2) {
    ck(m->ctx, hipEventElapsedTime(&ms, ev[j], ev[j + 1]), "elapsed");
    m->t_ms[0] += ms;
    m->t_launch[0] += 1;
    m->t_work[0] += fl[j / 2];
  }
  if (nupd >= 2) {  // the sweep's span and all of its flops (schedule-independent)
    ck(m->ctx, hipEventElapsedTime(&ms, ev[0], ev[nupd - 1]), "elapsed");
    m->t_ms[3] += ms;
    m->t_launch[3] += 1;
    m->t_work[3] += sweep_flops(m->sw.naug, m->sw.npad);
    // the lead-in: the assembly's (main) launch end to the first bulk start
    ck(m->ctx, hipEventElapsedTime(&ms, m->ev_asm[2 * ts + 1], ev[0]), "elapsed");
    m->t_ms[4] += ms;
    m->t_launch[4] += 1;
  }
  // the evaluation's device span: assembly start to gradient end
  ck(m->ctx, hipEventElapsedTime(&ms, m->ev_asm[2 * ts], m->ev_grad[2 * ts + 1]), "elapsed");
  m->t_ms[5] += ms;
  m->t_launch[5] += 1;
  const double n = (double)m->n, pairs = n * (n + 1) / 2, B = m->s.B, p = m->s.p;
  // work: the update launches' GEMM flops (counted per launch
  // from its tiles), pair kernels by their algorithmic flop formulas
  m->t_work[1] += pairs * B * (3 * p + 3);
  m->t_work[2] += pairs * (4 * B * p + 2 * p) + (m->s.kind == ACE_KERNEL_MATERN32 ? pairs * B * p : 0);
}

// Host syncs of the device-fused training loop: every ACE_TRAIN_SYNC
// iterations (default 4).  Iterations enqueued after the one that converged
// still run but change nothing in theta or the stats (k_train_step checks the
// stop flag); their evaluations do overwrite the resident inverse, so the
// stopping iteration's evaluation is re-run once at its saved theta.  A fit
// spends at most ACE_TRAIN_SYNC extra evaluations.
int train_sync_every() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("ACE_TRAIN_SYNC");
    v = e ? std::max(1, atoi(e)) : 4;
  }
  return v;
}

// ace_model_train of an unsharded model: theta, the optimizer moments and
// the stats matrix live in HBM; each iteration is the evaluation pipeline
// (tables from the device theta) + k_train_step, enqueued without a host
// round trip.
int train_device(ace_model *m, int optimizer, double learn_rate, double momentum, double beta1,
                 double beta2, int norm_clip, double clip_at, int maxiter, double tol,
                 double *theta, double *stats, int *iters, int *converged) {
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, m->has_data, "ace_model_set_data() not called");
  const Shape &s = m->s;
  const int P = 2 + s.B * (s.p + 1);
  hipStream_t st = ctx->stream;
  DBuf dst, dhist, dctl;
  std::vector<double> init((size_t)(5 * P), 0.0);
  std::copy(theta, theta + P, init.begin());
  upload(ctx, dst, init.data(), init.size(), "upload train state");
  std::vector<double> hz((size_t)(2 * (maxiter + 2)), 0.0);
  upload(ctx, dhist, hz.data(), hz.size(), "upload stats");
  alloc(ctx, dctl, 4 * sizeof(int), "alloc train control");
  ck(ctx, hipMemsetAsync(dctl.p, 0, 4 * sizeof(int), st), "memset control");
  TrainCfg c;
  c.optimizer = optimizer;
  c.lr = learn_rate;
  c.momentum = momentum;
  c.beta1 = beta1;
  c.beta2 = beta2;
  c.clip = norm_clip;
  c.clip_at = clip_at;
  c.tol = tol;
  c.P = P;
  c.B = s.B;
  c.p = s.p;
  c.PM = s.PM;
  c.kind = s.kind;
  c.n = m->n;
  c.std_y = m->std_y;
  const int K = train_sync_every();
  int ctl[4] = {0, 0, 0, 0};
  bool interrupted = false;
  int queued = 0;  // last iteration enqueued
  for (int it = 1; it <= maxiter; ++it) {
    if (ctx->poll && ctx->poll(ctx->poll_user)) {  // before iteration it, like para_update
      interrupted = true;
      break;
    }
    model_pipeline(m, m->sw, nullptr, it == 1 ? 1 : 0, false, dst.d());
    ck(ctx, launch_train_step(c, it, m->gsum.d(), m->sums.d(), m->scal.d(), m->sw.flag.i(), dst.d(),
                              dhist.d(), dctl.i(), st),
       "train step");
    queued = it;
    if (it % K == 0 || it == maxiter) {
      ck(ctx, hipMemcpyAsync(ctl, dctl.p, sizeof(ctl), hipMemcpyDeviceToHost, st), "download control");
      sync(ctx);
      if (ctl[1] != 0) break;
    }
  }
  ck(ctx, hipMemcpyAsync(ctl, dctl.p, sizeof(ctl), hipMemcpyDeviceToHost, st), "download control");
  sync(ctx);
  if (ctl[0] >= 1 && queued > ctl[0]) {
    // iterations queued after the stopping one ran their evaluation at the
    // final theta into m->sw; the reference's invKmatn is the one of the last
    // para_update (Q6, R/main_ace.R:215-227, R/kernel_SE_R6.R:37): re-run
    // iteration ctl[0]'s evaluation at the theta it saw (deterministic, so
    // bit-identical to what that iteration left)
    model_pipeline(m, m->sw, nullptr, ctl[0] == 1 ? 1 : 0, false, dst.d() + 4 * P);
  }
  download(ctx, theta, dst.d(), (size_t)P, "download theta");
  download(ctx, stats, dhist.d(), (size_t)(2 * (maxiter + 2)), "download stats");
  sync(ctx);
  m->has_inverse = ctl[0] > 0;
  const int it = ctl[0];
  if (iters) *iters = it;
  if (converged) *converged = 0;
  if (interrupted) {
    ctx->err = "interrupted";
    return ACE_ERR_INTERRUPTED;
  }
  if (ctl[1] == 2) {
    ctx->err = "Some gradients are not finite, NaN, or NA. Often this is due to too large "
               "learning rates.";
    return ACE_ERR_NONFINITE;
  }
  double fin[2];
  const int rc = ace_model_train_stats(m, theta, fin);
  if (rc != ACE_OK) return rc;
  stats[2 * (it + 1)] = fin[0];
  stats[2 * (it + 1) + 1] = fin[1];
  if (converged) *converged = it < maxiter ? 1 : 0;
  return ACE_OK;
  ACE_CATCH
}

}  // namespace

extern "C" {

int ace_model_create(ace_ctx *ctx, int kind, int64_t n, int p, int B, ace_model **out) {
  if (!ctx || !out) return ACE_ERR_ARG;
  *out = nullptr;
  ace_model *m = new ace_model();
  m->ctx = ctx;
  try {
    ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    m->s = check_shape(ctx, kind, p, B);
    arg(ctx, n >= 2, "n must be >= 2");
    m->n = n;
    m->sw.ensure(ctx, n);
    m->npad = m->sw.npad;
    m->naug = m->sw.naug;
    m->ntiles = grad_ntiles(n);
    m->ntr = (n + AT - 1) / AT;
    build_grad_tiles(ctx, n, m->gtiles, &m->ntiles, &m->ngdiag);
    const Shape &s = m->s;
    alloc(ctx, m->y, (size_t)m->npad * sizeof(double), "alloc y");
    alloc(ctx, m->tab, (size_t)(2 * s.B * s.PM + s.B + 1) * sizeof(double), "alloc tab");
    if (slice_norms_on())
      alloc(ctx, m->norms, (size_t)((s.B + 1) * m->npad) * sizeof(double), "alloc norms");
    alloc(ctx, m->alpha, (size_t)m->npad * sizeof(double), "alloc alpha");
    const int ldg = grad_part_cols(s.PM, s.B);
    alloc(ctx, m->gpart, (size_t)(m->ntiles * ldg) * sizeof(double), "alloc gpart");
    alloc(ctx, m->gwork, (size_t)tile_sums_work(ldg) * sizeof(double), "alloc tile sums");
    alloc(ctx, m->res, (size_t)(ldg + 8 + 16) * sizeof(double), "alloc results");
    m->gsum.p = m->res.d();
    m->sums.p = m->res.d() + ldg;
    m->scal.p = m->res.d() + ldg + 8;
    ck(ctx, hipMemsetAsync(m->sw.A.p, 0, m->sw.A.bytes, ctx->stream), "memset A");
    const int steps = (int)(m->npad / NB);
    m->ev_upd.assign((size_t)(4 * steps), nullptr);
    m->upd_flops.assign((size_t)(2 * steps), 0.0);
    for (auto &e : m->ev_upd) ck(ctx, hipEventCreateWithFlags(&e, ACE_TIMING_EVENT_FLAGS), "event");
    for (int j = 0; j < 4; ++j) {
      ck(ctx, hipEventCreateWithFlags(&m->ev_asm[j], ACE_TIMING_EVENT_FLAGS), "event");
      ck(ctx, hipEventCreateWithFlags(&m->ev_grad[j], ACE_TIMING_EVENT_FLAGS), "event");
    }
    sync(ctx);
  } catch (const Fail &f) {
    ace_model_destroy(m);
    return f.code;
  }
  *out = m;
  return ACE_OK;
}

void ace_model_destroy(ace_model *m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  if (m->shard) shard_destroy(m->shard);
  for (auto &e : m->ev_upd)
    if (e) (void)hipEventDestroy(e);
  for (int j = 0; j < 4; ++j) {
    if (m->ev_asm[j]) (void)hipEventDestroy(m->ev_asm[j]);
    if (m->ev_grad[j]) (void)hipEventDestroy(m->ev_grad[j]);
  }
  delete m;
}

int ace_model_set_data(ace_model *m, const double *y, const double *X, const double *Z,
                       double std_y) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, y && (m->s.p == 0 || X) && (m->s.B == 1 || Z), "null argument");
  if (m->shard) {
    shard_set_data(m->shard, y, X, Z);
    m->std_y = std_y;
    m->has_data = true;
    return ACE_OK;
  }
  upload_side(ctx, m->side, m->s, X, Z, m->n, m->npad);
  std::vector<double> yp((size_t)m->npad, 0.0);
  std::copy(y, y + m->n, yp.begin());
  upload_bytes(ctx, m->y.p, yp.data(), yp.size() * sizeof(double), "upload y");
  m->std_y = std_y;
  sync(ctx);
  m->has_data = true;
  return ACE_OK;
  ACE_CATCH
}

#ifdef ACE_HOST_TRACE
// diagnostic builds only (tools/build_variant.sh TAG -DACE_HOST_TRACE): host
// timestamps of one para_update on stderr -- entry, enqueue done, results
// synchronised, exit -- and the time since the previous call's exit
static double host_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
static double g_ht_exit = 0.0;
#define ACE_HT(name) const double name = host_us()
#else
#define ACE_HT(name)
#endif

int ace_model_para_update(ace_model *m, int iter, double *theta, double *grad, double *stats,
                          double *mu_post) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_HT(t_in);
  ACE_TRY
  int stop = (ctx->poll && ctx->poll(ctx->poll_user)) ? 1 : 0;
  // sharded over RCCL: every rank votes (also ranks without a poll), so that
  // all of them stop before the same evaluation
  if (m->shard) stop = shard_any(m->shard, stop);
  if (stop) {
    ctx->err = "interrupted";
    return ACE_ERR_INTERRUPTED;
  }
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, m->has_data, "ace_model_set_data() not called");
  arg(ctx, theta && grad && stats, "null argument");
  const Shape &s = m->s;
  const bool timed = m->prof;
  const int ncol = s.B * (s.PM + 1);
  std::vector<double> gs((size_t)(ncol + 1));
  double sums[4], scal[5];
  int flag = 0;
  if (m->shard) {
    shard_eval(m->shard, theta, iter == 1 ? 1 : 0, 0, timed, gs.data(), sums, scal, &flag);
    if (timed) shard_collect_timing(m->shard, m->t_ms, m->t_launch, m->t_work);
  } else {
    model_pipeline(m, m->sw, theta, iter == 1 ? 1 : 0, timed);
    ACE_HT(t_enq);
    // the previous timed evaluation's events completed before its results
    // were read: read them back while this evaluation runs
    if (m->pend >= 0) {
      model_collect_timing(m, m->pend);
      m->pend = -1;
    }
    // the result block into the pinned region behind the tables: one copy
    // and one (bounded) synchronisation -- pinned, so the copy is queued
    // without draining the stream first as download() does for pageable
    // memory; four drained small copies cost ~20 us each at C1
    double *h = m->hio.p + (2 * s.B * s.PM + s.B);
    ck(ctx, hipMemcpyAsync(h, m->res.p, m->res.bytes, hipMemcpyDeviceToHost, ctx->stream),
       "download results");
    sync(ctx);
    const double *hs = h + (m->sums.d() - m->res.d()), *hc = h + (m->scal.d() - m->res.d());
    std::copy(h, h + gs.size(), gs.begin());
    std::copy(hs, hs + 4, sums);
    std::copy(hc, hc + 5, scal);
    flag = hs[4] != 0.0;
    if (timed) {
      m->pend = m->tset;
      m->tset ^= 1;
    }
#ifdef ACE_HOST_TRACE
    const double t_sync = host_us();
    fprintf(stderr, "ace_host_trace it %d: since last exit %.1f us, enqueue %.1f us, wait %.1f us\n",
            iter, g_ht_exit > 0 ? t_in - g_ht_exit : -1.0, t_enq - t_in, t_sync - t_enq);
#endif
  }
  m->has_inverse = true;
  if (iter == 1) theta[1] = scal[3];  // mean_solution before the gradient (R/kernel_SE_R6.R:45)
  compose_grad(s, theta, gs.data(), sums[2], grad);
  stats[0] = m->std_y * std::sqrt(sums[0]) / std::sqrt((double)m->n);
  stats[1] = -0.5 * (m->n * std::log(2.0 * M_PI) + sums[3] + sums[1]);
  if (mu_post) *mu_post = scal[3];
  if (flag) {  // not positive definite: the reference's outputs are non-finite
    const int P = 2 + s.B * (s.p + 1);
    for (int j = 0; j < P; ++j) grad[j] = kNaN;
    stats[0] = stats[1] = kNaN;
    if (mu_post) *mu_post = kNaN;
  }
#ifdef ACE_HOST_TRACE
  g_ht_exit = host_us();
#endif
  return ACE_OK;
  ACE_CATCH
}

int ace_model_train_stats(ace_model *m, const double *theta, double *stats) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, m->has_data && theta && stats, "null argument / no data");
  double sums[4];
  int flag = 0;
  if (m->shard) {
    std::vector<double> gs((size_t)(m->s.B * (m->s.PM + 1) + 1));
    double scal[5];
    shard_eval(m->shard, theta, 0, 1, false, gs.data(), sums, scal, &flag);
  } else {
    m->sw2.ensure(ctx, m->n);
    model_pipeline(m, m->sw2, theta, 0, false);
    double hs[5];
    download(ctx, hs, m->sums.d(), 5, "download sums");
    sync(ctx);
    std::copy(hs, hs + 4, sums);
    flag = hs[4] != 0.0;
  }
  stats[0] = m->std_y * std::sqrt(sums[0]) / std::sqrt((double)m->n);
  stats[1] = -0.5 * (m->n * std::log(2.0 * M_PI) + sums[3] + sums[1]);
  if (flag) stats[0] = stats[1] = kNaN;
  return ACE_OK;
  ACE_CATCH
}

int ace_model_get_inverse(ace_model *m, double *inv) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  ACE_TRY
  ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
  arg(ctx, inv != nullptr, "null argument");
  if (m->shard) {
    shard_get_inverse(m->shard, inv);
    return ACE_OK;
  }
  DBuf out;
  alloc(ctx, out, (size_t)(m->n * m->n) * sizeof(double), "alloc inverse");
  ck(ctx, launch_sym_from_lower(m->sw.A.d(), m->naug, m->n, -1.0, out.d(), m->n, ctx->stream),
     "symmetrize");
  download(ctx, inv, out.d(), (size_t)(m->n * m->n), "download inverse");
  sync(ctx);
  return ACE_OK;
  ACE_CATCH
}

int ace_model_profile(ace_model *m, int enable) {
  if (!m) return ACE_ERR_ARG;
  m->prof = enable != 0;
  m->pend = -1;  // counters restart: drop an unread set
  for (int j = 0; j < 6; ++j) {
    m->t_ms[j] = 0;
    m->t_launch[j] = 0;
    m->t_work[j] = 0;
  }
  return ACE_OK;
}

int ace_model_kernel_time(ace_model *m, int which, double *ms, int64_t *launches, double *work) {
  if (!m || which < 0 || which > 5) return ACE_ERR_ARG;
  if (m->pend >= 0) {  // the last timed evaluation's set (its work is complete)
    try {
      model_collect_timing(m, m->pend);
    } catch (const Fail &f) {
      return f.code;
    }
    m->pend = -1;
  }
  if (ms) *ms = m->t_ms[which];
  if (launches) *launches = m->t_launch[which];
  if (work) *work = m->t_work[which];
  return ACE_OK;
}

int ace_comm_unique_id(unsigned char *id) {
  if (!id) return ACE_ERR_ARG;
  try {
    shard_unique_id(id);
  } catch (const std::exception &e) {
    g_create_err = e.what();
    return ACE_ERR_HIP;
  }
  return ACE_OK;
}

int ace_model_create_sharded(ace_ctx *ctx, int kind, int64_t n, int p, int B, int world,
                             int rank, const unsigned char *id, ace_model **out) {
  if (!ctx || !out) return ACE_ERR_ARG;
  *out = nullptr;
  ace_model *m = new ace_model();
  m->ctx = ctx;
  try {
    ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    m->s = check_shape(ctx, kind, p, B);
    arg(ctx, n >= 2, "n must be >= 2");
    arg(ctx, world >= 1 && world <= 64 && rank >= 0 && rank < world, "bad world / rank");
    arg(ctx, id != nullptr || rank == 0, "simulated group (id == NULL) is created as rank 0");
    m->n = n;
    m->npad = round_up(n, NB);
    m->naug = m->npad + AUG;
    m->shard = shard_create(ctx, m->s, n, world, rank, id);
  } catch (const Fail &f) {
    ace_model_destroy(m);
    return f.code;
  }
  *out = m;
  return ACE_OK;
}

int ace_model_create_sharded_host(ace_ctx *ctx, int kind, int64_t n, int p, int B, int world,
                                  int rank, const ace_comm_ops *ops, ace_model **out) {
  if (!ctx || !out) return ACE_ERR_ARG;
  *out = nullptr;
  if (!ops || !ops->broadcast || !ops->allgather || !ops->allreduce) {
    ctx->err = "ace_model_create_sharded_host: incomplete ace_comm_ops";
    return ACE_ERR_ARG;
  }
  ace_model *m = new ace_model();
  m->ctx = ctx;
  try {
    ck(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    m->s = check_shape(ctx, kind, p, B);
    arg(ctx, n >= 2, "n must be >= 2");
    arg(ctx, world >= 1 && world <= 64 && rank >= 0 && rank < world, "bad world / rank");
    m->n = n;
    m->npad = round_up(n, NB);
    m->naug = m->npad + AUG;
    m->shard = shard_create_host(ctx, m->s, n, world, rank, *ops);
  } catch (const Fail &f) {
    ace_model_destroy(m);
    return f.code;
  }
  *out = m;
  return ACE_OK;
}

int ace_model_shard_info(const ace_model *m, int *world, int *rank) {
  if (!m) return ACE_ERR_ARG;
  if (world) *world = m->shard ? shard_world(m->shard) : 1;
  if (rank) *rank = m->shard ? shard_rank(m->shard) : 0;
  return ACE_OK;
}

int ace_model_comm_calls(const ace_model *m, int64_t *counts) {
  if (!m || !counts) return ACE_ERR_ARG;
  for (int j = 0; j < ACE_COMM_KINDS; ++j) counts[j] = 0;
  if (m->shard) shard_comm_calls(m->shard, counts);
  return ACE_OK;
}

int ace_model_train(ace_model *m, int optimizer, double learn_rate, double momentum, double beta1,
                    double beta2, int norm_clip, double clip_at, int maxiter, double tol,
                    double *theta, double *stats, int *iters, int *converged) {
  if (!m) return ACE_ERR_ARG;
  ace_ctx *ctx = m->ctx;
  if (!theta || !stats || maxiter < 1 ||
      (optimizer != ACE_OPT_NESTEROV && optimizer != ACE_OPT_ADAM && optimizer != ACE_OPT_NADAM)) {
    ctx->err = "ace_model_train: bad argument";
    return ACE_ERR_ARG;
  }
  const int P = 2 + m->s.B * (m->s.p + 1);
  for (int64_t j = 0; j < 2 * (int64_t)(maxiter + 2); ++j) stats[j] = 0.0;
  if (!m->shard)
    return train_device(m, optimizer, learn_rate, momentum, beta1, beta2, norm_clip, clip_at,
                        maxiter, tol, theta, stats, iters, converged);
  // sharded: the host loop (every rank runs the same iterations)
  std::vector<double> g((size_t)P), mom1((size_t)P, 0.0), mom2((size_t)P, 0.0);
  int it = 0;
  for (it = 1; it <= maxiter; ++it) {
    double st[2], mu = 0.0;
    const int rc = ace_model_para_update(m, it, theta, g.data(), st, &mu);
    if (rc != ACE_OK) {  // interrupted (or failed) before iteration `it`
      if (iters) *iters = it - 1;
      if (converged) *converged = 0;
      return rc;
    }
    stats[2 * it] = st[0];
    stats[2 * it + 1] = st[1];
    ace_norm_clip(norm_clip, P, g.data(), clip_at);  // Optim$update (R/optimizer_classes.R)
    int ok = 0;
    if (optimizer == ACE_OPT_NADAM)
      ok = ace_nadam(P, it, learn_rate, beta1, beta2, 1e-8, mom1.data(), mom2.data(), g.data(), theta);
    else if (optimizer == ACE_OPT_ADAM)
      ok = ace_adam(P, it, learn_rate, beta1, beta2, 1e-8, mom1.data(), mom2.data(), g.data(), theta);
    else
      ok = ace_nesterov(P, learn_rate, momentum, mom1.data(), g.data(), theta);
    if (!ok) {
      ctx->err = "Some gradients are not finite, NaN, or NA. Often this is due to too large "
                 "learning rates.";
      if (iters) *iters = it;
      if (converged) *converged = 0;
      return ACE_ERR_NONFINITE;
    }
    theta[1] = mu;  // private$mean_solution(y) with this iteration's inverse
    const double change = std::fabs(stats[2 * it + 1] - stats[2 * (it - 1) + 1]);
    if (change < tol && it > 3) break;
  }
  if (it > maxiter) it = maxiter;
  double fin[2];
  const int rc = ace_model_train_stats(m, theta, fin);
  if (rc != ACE_OK) return rc;
  stats[2 * (it + 1)] = fin[0];
  stats[2 * (it + 1) + 1] = fin[1];
  if (iters) *iters = it;
  if (converged) *converged = it < maxiter ? 1 : 0;
  return ACE_OK;
}

}  // extern "C"

