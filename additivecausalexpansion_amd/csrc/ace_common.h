// ace_common.h -- host-side helpers shared by the C ABI (ace_api.cpp) and the
// sharded model (ace_shard.cpp): the context, device buffers, argument and
// error handling, theta tables, pair-side uploads and gradient composition.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "../../include/ace_hip.h"
#include "ace_internal.h"

struct SweepWork;  // ace_model.h

// Streams (DESIGN §5 "Streams and hardware queues"): all non-blocking, so
// nothing the runtime or another library puts on the legacy null stream is
// ordered against them, and the library itself never uses the null stream.
// ACE_STREAMS = 3 (default) / 2 / 1 creates that many; with fewer, side2
// aliases side and side aliases stream.  Every cross-stream wait is enqueued
// after the record it waits for, so any serialisation of the three in host
// order -- one stream, or two sharing a hardware queue -- is a valid
// execution of the same graph with bit-identical results.
struct ace_ctx {
  int device = 0;
  int nstreams = 0;              // distinct streams created (1..3)
  hipStream_t stream = nullptr;  // main stream (every ABI call syncs it)
  hipStream_t side = nullptr;    // sweep lookahead: panel factorisation
  hipStream_t side2 = nullptr;   // sweep lookahead: the second block's cross update
  int (*poll)(void *) = nullptr; // optional interrupt poll (ace_set_interrupt_poll)
  void *poll_user = nullptr;
  std::string err;
  // set when a bounded sync timed out (ACE_ERR_TIMEOUT): copies enqueued
  // before the deadline may still land, so every later call on this context
  // refuses to run (ACE_ERR_TIMEOUT) instead of reusing its buffers
  bool failed = false;
  // sweep buffers of freed inverse handles (ace_dmat.cpp), reused by the
  // next invkernel_dev of the same n instead of a new 2 n^2-byte allocation
  std::vector<std::shared_ptr<SweepWork>> sweep_pool;
  std::shared_ptr<void> dmat_state;  // the handle path's cached inputs (ace_dmat.cpp)
  // prediction's n x nx scratch (K_xX, the product, K_xx; ace_predict.cpp),
  // kept between calls -- a fresh 0.5 GB hipMalloc / hipFree pair per call
  // costs more than the kernels it feeds; dropped when an allocation fails
  std::shared_ptr<void> pred_state;
};

extern std::string g_create_err;

// Events that only order work on this device (the sweep's cross-stream
// hand-offs) or time it: no system-scope fence on record / wait -- the
// default release writes back L2 for host visibility, ~20 us per sweep step.
#define ACE_SYNC_EVENT_FLAGS (hipEventDisableTiming | (unsigned)hipEventDisableSystemFence)
#define ACE_TIMING_EVENT_FLAGS ((unsigned)hipEventDisableSystemFence)

namespace ace_host {
using namespace ace;

inline const double kNaN = std::numeric_limits<double>::quiet_NaN();

struct Fail {
  int code;
};

// RAII device buffer
struct DBuf {
  void *p = nullptr;
  size_t bytes = 0;
  DBuf() = default;
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  ~DBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  double *d() const { return static_cast<double *>(p); }
  int *i() const { return static_cast<int *>(p); }
};

// A non-owning sub-range of a DBuf.
struct DView {
  double *p = nullptr;
  double *d() const { return p; }
};

inline void ck(ace_ctx *ctx, hipError_t e, const char *what) {
  if (e == hipSuccess) return;
  ctx->err = std::string(what) + ": " + hipGetErrorString(e);
  throw Fail{e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? ACE_ERR_OOM
                                                                          : ACE_ERR_HIP};
}

inline void arg(ace_ctx *ctx, bool ok, const char *msg) {
  if (ok) return;
  ctx->err = msg;
  throw Fail{ACE_ERR_ARG};
}

// A failed allocation first drops the pooled sweep buffers of freed inverse
// handles (dead contents, ace_dmat_free) and retries once.
inline void alloc(ace_ctx *ctx, DBuf &b, size_t bytes, const char *what) {
  if (b.bytes >= bytes && b.p) return;
  b.release();
  if (bytes == 0) bytes = 16;
  hipError_t e = hipMalloc(&b.p, bytes);
  if ((e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) &&
      (!ctx->sweep_pool.empty() || ctx->pred_state)) {
    (void)hipGetLastError();
    ctx->sweep_pool.clear();
    ctx->pred_state.reset();  // (a caller allocating into it holds its own reference)
    e = hipMalloc(&b.p, bytes);
  }
  if (e != hipSuccess) b.p = nullptr;
  ck(ctx, e, what);
  b.bytes = bytes;
}

// Waits until everything enqueued on `s` has run, bounded: after
// ACE_SYNC_TIMEOUT seconds (default 600; 0 = an unbounded
// hipStreamSynchronize) the call fails with ACE_ERR_TIMEOUT and ctx->err
// names the context's streams that still hold work, instead of blocking the
// host forever on a stalled queue or collective (ace_api.cpp).
void sync_stream(ace_ctx *ctx, hipStream_t s, const char *what);
inline void sync(ace_ctx *ctx) { sync_stream(ctx, ctx->stream, "hipStreamSynchronize"); }

// Host <-> device copies: stream-ordered on the main stream (never the null
// stream).  The stream is drained (bounded) BEFORE a copy is queued: a
// pageable copy blocks inside the runtime until earlier stream work is done,
// which would bypass ACE_SYNC_TIMEOUT, and a timeout then leaves no copy
// into caller memory queued.  Uploads are complete on return (pageable host
// buffers may be temporaries); downloads complete at the caller's next sync.
inline void upload(ace_ctx *ctx, DBuf &b, const double *h, size_t count, const char *what) {
  alloc(ctx, b, count * sizeof(double), what);
  if (!count) return;
  sync_stream(ctx, ctx->stream, what);
  ck(ctx, hipMemcpyAsync(b.p, h, count * sizeof(double), hipMemcpyHostToDevice, ctx->stream), what);
  sync_stream(ctx, ctx->stream, what);
}
// the same for any trivially copyable host array (tile lists)
inline void upload_bytes(ace_ctx *ctx, void *d, const void *h, size_t bytes, const char *what) {
  if (!bytes) return;
  sync_stream(ctx, ctx->stream, what);
  ck(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream), what);
  sync_stream(ctx, ctx->stream, what);
}

inline void download(ace_ctx *ctx, double *h, const double *d, size_t count, const char *what) {
  if (!count) return;
  sync_stream(ctx, ctx->stream, what);
  ck(ctx, hipMemcpyAsync(h, d, count * sizeof(double), hipMemcpyDeviceToHost, ctx->stream), what);
}

// Pinned host staging for the per-evaluation traffic (theta tables up, the
// gradient sums and statistics down): pageable copies each take a host
// round trip through the runtime's staging buffer (~100 us apiece).
struct PinnedBuf {
  double *p = nullptr;
  size_t n = 0;
  PinnedBuf() = default;
  PinnedBuf(const PinnedBuf &) = delete;
  PinnedBuf &operator=(const PinnedBuf &) = delete;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  double *ensure(ace_ctx *ctx, size_t count) {
    if (count > n) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      n = 0;
      ck(ctx, hipHostMalloc((void **)&p, count * sizeof(double), hipHostMallocDefault),
         "pinned host alloc");
      n = count;
    }
    return p;
  }
};

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

struct Shape {
  int kind, p, B, PM, ZS;
};

inline Shape check_shape(ace_ctx *ctx, int kind, int p, int B) {
  arg(ctx, kind == ACE_KERNEL_SE || kind == ACE_KERNEL_MATERN32, "unknown kernel kind");
  arg(ctx, p >= 0 && B >= 1, "p must be >= 0 and B >= 1");
  if (p > PMAX || B > BMAX) {
    ctx->err = "unsupported shape: p <= 64 and B <= 32 are compiled";
    throw Fail{ACE_ERR_UNSUPPORTED};
  }
  Shape s;
  s.kind = kind;
  s.p = p;
  s.B = B;
  s.PM = pm_bucket(p < 1 ? 1 : p);
  s.ZS = B > 1 ? B - 1 : 1;
  return s;
}

// column-major X (n x p) -> row-major n x PM, zero padded
inline std::vector<double> pack_rows(const double *M, int64_t n, int cols, int width) {
  std::vector<double> out((size_t)(n * width), 0.0);
  for (int i = 0; i < cols; ++i)
    for (int64_t r = 0; r < n; ++r) out[(size_t)(r * width + i)] = M[r + i * n];
  return out;
}

// theta tables (b-major), see TabView in ace_internal.h.  The kernel reads
// theta up to index 1 + B (p + 1) - 1 = P - 2 only, so the kernel-matrix
// entry points (with_grad = false) accept a theta one entry short, as the
// reference's kernmat_* do; the gradient-indexed weights need all P.
inline std::vector<double> make_tab(const double *theta, const Shape &s, bool with_grad = true) {
  const int B = s.B, PM = s.PM;
  std::vector<double> t((size_t)(2 * B * PM + B), 0.0);
  for (int b = 0; b < B; ++b) {
    for (int i = 0; i < s.p; ++i) {
      t[(size_t)(b * PM + i)] = std::exp(-theta[1 + b + B * (i + 1)]);  // Q1 kernel index
      if (with_grad)
        t[(size_t)(B * PM + b * PM + i)] = std::exp(-theta[2 + B + b + B * i]);  // gradient index
    }
    t[(size_t)(2 * B * PM + b)] = theta[2 + b];
  }
  return t;
}

inline TabView tab_view(const DBuf &b, const Shape &s) {
  TabView v;
  v.wk = b.d();
  v.wg = b.d() + s.B * s.PM;
  v.lam = b.d() + 2 * s.B * s.PM;
  return v;
}

// Device copy of one pair side (X, Z, log|Z|).
struct SideBufs {
  DBuf X, Z, LZ;
  PairSide view(int64_t n) const {
    PairSide ps;
    ps.X = X.d();
    ps.Z = Z.d();
    ps.LZ = LZ.d();
    ps.n = n;
    return ps;
  }
};

inline void upload_side(ace_ctx *ctx, SideBufs &sb, const Shape &s, const double *X, const double *Z,
                 int64_t n, int64_t nalloc) {
  std::vector<double> xr = pack_rows(X, n, s.p, s.PM);
  xr.resize((size_t)(nalloc * s.PM), 0.0);
  upload(ctx, sb.X, xr.data(), xr.size(), "upload X");
  std::vector<double> zr((size_t)(nalloc * s.ZS), 0.0);
  if (s.B > 1 && Z) {
    std::vector<double> t = pack_rows(Z, n, s.B - 1, s.ZS);
    std::copy(t.begin(), t.end(), zr.begin());
  }
  upload(ctx, sb.Z, zr.data(), zr.size(), "upload Z");
  alloc(ctx, sb.LZ, zr.size() * sizeof(double), "alloc LZ");
  if (s.kind == ACE_KERNEL_SE)
    ck(ctx, launch_log_abs(sb.Z.d(), sb.LZ.d(), (int64_t)zr.size(), ctx->stream), "log_abs");
}

inline double host_logsum(const double *w, int64_t n) {
  double s = 0.0;
  for (int64_t j = 0; j < n; ++j) s += std::log(w[j]);
  return s;
}

// Final composition of the P-gradient from the device sums.
//   gsum[b*(PM+1)+i] : sum T K_b d_i^2 (SE) / sum T K_b/(1+sqrt(3 r~2)) d_i^2 (Matern)
//   gsum[b*(PM+1)+PM]: sum T K_b ; gsum[B*(PM+1)] : trace T
inline void compose_grad(const Shape &s, const double *theta, const double *gsum, double sum_alpha,
                  double *grad) {
  const int B = s.B, PM = s.PM, P = 2 + B * (s.p + 1);
  for (int j = 0; j < P; ++j) grad[j] = 0.0;
  grad[0] = -0.5 * gsum[B * (PM + 1)] * std::exp(theta[0]);  // sigma_gradient
  for (int b = 0; b < B; ++b) grad[2 + b] = -0.5 * gsum[b * (PM + 1) + PM];
  for (int i = 0; i < s.p; ++i)
    for (int b = 0; b < B; ++b) {
      const int j = 2 + B + b + B * i;
      const double sum = gsum[b * (PM + 1) + i];
      if (s.kind == ACE_KERNEL_SE) grad[j] = -0.5 * (sum * std::exp(-theta[j]));
      else grad[j] = -0.25 * 9 * sum * std::exp(-theta[j]);
    }
  grad[1] = (s.kind == ACE_KERNEL_SE) ? sum_alpha : 0.0;
}

// Host tail of pred_cpp (src/pred_cpp.cpp:20-33): from a = tmp (y - mu),
// kd = diag(K_xx), qd = diag(tmp K_xX^T).
inline void finish_pred(int64_t nx, const double *a, const double *kd, const double *qd,
                        double sigma, double mu, double mean_y, double std_y, double *map,
                        double *ci, double *var) {
  const double es = std::exp(sigma);
  for (int64_t r = 0; r < nx; ++r) {
    const double yx = mean_y + std_y * (a[r] + mu);
    const double d = (kd[r] - qd[r]) + es;
    const double sd = std_y * std::sqrt(std::fabs(d));
    map[r] = yx;
    ci[r] = yx - 1.96 * sd;
    ci[r + nx] = yx + 1.96 * sd;
    var[r] = std::pow(sd, 2);
  }
}

// Host tail of pred_marginal_cpp (src/pred_cpp.cpp:69-126): a, kd, qd of the
// marginal kernels; with zx != NULL also ATE / ATT / ATU from the posterior
// quadratic forms post[j] = w_j^T (Km_xx - tmp Km_xX^T) w_j for w = 1, Z_x,
// (Z_x == 0).  avg (12) as ace_pred_marginal.
inline void finish_marginal(int64_t nx, const double *a, const double *kd, const double *qd,
                            double std_y, double std_Z, const double *zx, const double *post,
                            double *map, double *ci, double *var, double *avg) {
  std::vector<double> yx((size_t)nx);
  for (int64_t r = 0; r < nx; ++r) {
    yx[(size_t)r] = std_y * a[r] / std_Z;
    const double d = kd[r] - qd[r];
    const double sd = std_y * std::sqrt(std::fabs(d)) / std_Z;
    map[r] = yx[(size_t)r];
    ci[r] = yx[(size_t)r] - 1.96 * sd;
    ci[r + nx] = yx[(size_t)r] + 1.96 * sd;
    var[r] = std::pow(sd, 2);
  }
  if (!zx || !post) return;
  double sy = 0.0, syz = 0.0, sz = 0.0;
  for (int64_t r = 0; r < nx; ++r) {
    sy += yx[(size_t)r];
    syz += yx[(size_t)r] * zx[r];
    sz += zx[r];
  }
  const double ate = sy / (double)nx;
  const double ate_sd = std_y * std::sqrt(post[0]) / (double)nx;
  const unsigned int ntx = (unsigned int)sz;  // unsigned int in the reference
  const double att = syz / ntx;
  const double att_sd = std_y * std::sqrt(post[1]) / ntx;
  const unsigned int nux = (unsigned int)nx - ntx;
  const double atu = (ate * nx - att * ntx) / nux;
  const double atu_sd = std_y * std::sqrt(post[2]) / nux;
  const double m3[3] = {ate, att, atu}, s3[3] = {ate_sd, att_sd, atu_sd};
  for (int j = 0; j < 3; ++j) {
    avg[4 * j + 0] = m3[j];
    avg[4 * j + 1] = m3[j] - 1.96 * s3[j];
    avg[4 * j + 2] = m3[j] + 1.96 * s3[j];
    avg[4 * j + 3] = std::pow(s3[j], 2);
  }
}

}  // namespace ace_host
using namespace ace_host;

// Every ABI entry point: a context whose bounded sync timed out refuses work
inline void check_usable(ace_ctx *ctx) {
  if (!ctx->failed) return;
  ctx->err = "context unusable: an earlier call timed out (ACE_ERR_TIMEOUT); destroy it";
  throw Fail{ACE_ERR_TIMEOUT};
}

#define ACE_TRY \
  try {         \
    check_usable(ctx);
#define ACE_CATCH \
  }               \
  catch (const Fail &f) { return f.code; }

// ---- sharded model (ace_shard.cpp); errors throw Fail with ctx->err set ----
struct ShardModel;
void shard_unique_id(unsigned char *id);  // throws std::runtime_error
ShardModel *shard_create(ace_ctx *ctx, const Shape &s, int64_t n, int world, int rank,
                         const unsigned char *id);
// host-callback collectives (ace_model_create_sharded_host)
ShardModel *shard_create_host(ace_ctx *ctx, const Shape &s, int64_t n, int world, int rank,
                              const ace_comm_ops &ops);
void shard_destroy(ShardModel *m);
void shard_set_data(ShardModel *m, const double *y, const double *X, const double *Z);
void shard_eval(ShardModel *m, const double *theta, int use_mu, int which, bool timed,
                double *gsum, double *sums, double *scal, int *flag);
void shard_get_inverse(ShardModel *m, double *inv);
void shard_collect_timing(ShardModel *m, double *t_ms, int64_t *t_launch, double *t_work);
int shard_world(const ShardModel *m);
void shard_comm_calls(const ShardModel *m, int64_t *counts);  // ACE_COMM_KINDS entries
int shard_any(ShardModel *m, int local);  // collective OR (RCCL), local value (simulated)
int shard_nlocal(const ShardModel *m);                // ranks simulated in this process (1 with RCCL)
PairSide shard_train_side(const ShardModel *m);       // the replicated training X, Z, log|Z|
const double *shard_train_y(const ShardModel *m);     // the replicated y (npad, device)
const double *shard_A0(const ShardModel *m, int j);   // local rank j's resident A (column blocks)
int shard_rank_of(const ShardModel *m, int j);
void shard_allreduce_sum(ShardModel *m, double *buf, int64_t count);
int shard_rank(const ShardModel *m);
