// ace_shard.cpp -- block-column-sharded para_update across GPUs.
//
// Layout: A (naug x naug, lower triangle, the AUG rows [y; 1] appended) is
// split into NB-wide column blocks, block j on rank j % G, stored as local
// block j / G of a naug x (nloc NB) column-major array with the global row
// index (ace_internal.h lcol).  X, Z, y are replicated (<= 26 MB at C4).
//
// One evaluation on rank r:
//   assembly      own lower 64-tiles (+ identity padding, sigma diagonal)
//   sweep step k  pack -> exchange -> unpack + pivot chain -> update
//                 exchange = RCCL group { broadcast of panel rows >= k0 from
//                 rank k % G, all-gather of the row pieces A[k, j<k] }; the
//                 NB x NB pivot sweep runs redundantly on every rank (it is
//                 one workgroup of latency) so no second collective carries
//                 D^-1 or the pivots.  Lookahead as on one GPU: the cross of
//                 block k+1 is updated first, then pack/exchange/chain of
//                 panel k+1 run on the side stream under the bulk update.
//   alpha         AUG rows of own columns -> all-reduce (u, v, corner)
//   gradient      own 64-tiles of T = -A^-1 - alpha alpha^T
//   reduce        one all-reduce of the gradient sums (the RMSE residual is
//                 sig alpha, k_final_sums: no pass over Kfull)
// Every rank then holds identical sums and composes the same P-gradient.
//
// The communicator is RCCL (one process per GPU, loaded with dlopen so the
// library has no link-time RCCL dependency and shares the RCCL a host
// process such as PyTorch has already loaded) or, with id == NULL, an
// in-process group that simulates all G ranks on one device with device
// copies -- the validation mode: same kernels, same packing, same
// collective semantics.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <stdexcept>

#include "ace_common.h"
#include "ace_internal.h"

using namespace ace;

namespace {

// ------------------------------------------------------------------ RCCL
struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*Broadcast)(const void *, void *, size_t, ncclDataType_t, int, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t,
                            ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char *(*GetErrorString)(ncclResult_t) = nullptr;
  // optional: the head schedule's second communicator (null: that schedule
  // is not used over RCCL)
  ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t *, ncclConfig_t *) = nullptr;

  Rccl() {
    // an RCCL already in the process (e.g. PyTorch's) is reused by soname
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      err = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
#define ACE_SYM(f, name)                                              \
  f = reinterpret_cast<decltype(f)>(dlsym(h, name));                  \
  if (!f) {                                                           \
    err = std::string("librccl.so.1 lacks ") + name;                  \
    return;                                                           \
  }
    ACE_SYM(GetUniqueId, "ncclGetUniqueId");
    ACE_SYM(CommInitRank, "ncclCommInitRank");
    ACE_SYM(CommDestroy, "ncclCommDestroy");
    ACE_SYM(Broadcast, "ncclBroadcast");
    ACE_SYM(AllGather, "ncclAllGather");
    ACE_SYM(AllReduce, "ncclAllReduce");
    ACE_SYM(GroupStart, "ncclGroupStart");
    ACE_SYM(GroupEnd, "ncclGroupEnd");
    ACE_SYM(GetErrorString, "ncclGetErrorString");
#undef ACE_SYM
    CommSplit = reinterpret_cast<decltype(CommSplit)>(dlsym(h, "ncclCommSplit"));
    ok = true;
  }
};

Rccl &rccl() {
  static Rccl r;
  return r;
}

void nck(ace_ctx *ctx, ncclResult_t e, const char *what) {
  if (e == ncclSuccess) return;
  ctx->err = std::string(what) + ": " + rccl().GetErrorString(e);
  throw Fail{ACE_ERR_HIP};
}

// Host-callback collectives: stage through pinned host buffers owned by the
// model (a timed-out copy can never land in freed memory), every copy
// stream-ordered on `st` with the stream drained (bounded) before it is
// queued and after it, before the host touches the buffer.
struct HostStage {
  PinnedBuf a, b;
};
void d2h(ace_ctx *ctx, void *h, const void *d, size_t bytes, hipStream_t st) {
  sync_stream(ctx, st, "stage");
  ck(ctx, hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st), "stage");
  sync_stream(ctx, st, "stage");
}
void h2d(ace_ctx *ctx, void *d, const void *h, size_t bytes, hipStream_t st) {
  sync_stream(ctx, st, "unstage");
  ck(ctx, hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st), "unstage");
  sync_stream(ctx, st, "unstage");
}
void hck(ace_ctx *ctx, int rc, const char *what) {
  if (rc == 0) return;
  ctx->err = std::string(what) + ": host collective returned " + std::to_string(rc);
  throw Fail{ACE_ERR_HIP};
}

void host_bcast(ace_ctx *ctx, const ace_comm_ops &o, HostStage &hs, double *dbuf, size_t count,
                int root, hipStream_t st) {
  double *h = hs.a.ensure(ctx, count);
  d2h(ctx, h, dbuf, count * sizeof(double), st);
  hck(ctx, o.broadcast(o.user, h, (int64_t)count, root), "broadcast");
  h2d(ctx, dbuf, h, count * sizeof(double), st);
}

void host_allgather(ace_ctx *ctx, const ace_comm_ops &o, HostStage &hs, const double *dsend,
                    double *drecv, size_t count, int world, hipStream_t st) {
  double *s = hs.a.ensure(ctx, count);
  double *r = hs.b.ensure(ctx, count * (size_t)world);
  d2h(ctx, s, dsend, count * sizeof(double), st);
  hck(ctx, o.allgather(o.user, s, r, (int64_t)count), "allgather");
  h2d(ctx, drecv, r, count * (size_t)world * sizeof(double), st);
}

void host_allreduce(ace_ctx *ctx, const ace_comm_ops &o, HostStage &hs, double *dbuf,
                    size_t count, int op, hipStream_t st) {
  double *h = hs.a.ensure(ctx, count);
  d2h(ctx, h, dbuf, count * sizeof(double), st);
  hck(ctx, o.allreduce(o.user, h, (int64_t)count, op), "allreduce");
  h2d(ctx, dbuf, h, count * sizeof(double), st);
}

// ------------------------------------------------------------------ rank
struct RankState {
  int r = 0;
  DBuf A[2];  // A[1]: train_stats scratch (keeps A[0]'s inverse, Q6)
  DBuf P[8], W[8], SW, S[2], piv, flag, low, recv;  // panel slots k % (2 Z)
  DBuf tupd, tasm, tgrad;  // device tile lists
  int64_t nupd = 0, nasm = 0, nasm1 = 0, ngrad = 0, ndiag = 0;  // nasm1: first-part tiles
  std::vector<Tile> hupd;  // host copy (flop accounting)
  // pair schedule: own lookahead cross tiles (XCD-dealt), one device list
  // with host offsets -- xoff[k] .. xoff[k + 1]: tiles with I or J in block
  // k + 1 (the single-step cross with panel k); poff[2 g], poff[2 g + 1]:
  // group g's pair cross, block 2 g first, then block 2 g + 1 minus block 2 g
  DBuf tx, tp;
  std::vector<int64_t> xoff, poff;
  // head schedule: the own tiles of group_head_tiles' lists (device, host
  // offsets hoff[G 2Z + m]) and the head part's exchange buffer (Z NB x NB)
  DBuf th, lowh;
  std::vector<int64_t> hoff;
  DBuf y, tab, alpha, scal, gpart, gwork, red, sums, augvec;
  SideBufs side;
};

}  // namespace

struct ShardModel {
  ace_ctx *ctx = nullptr;
  Shape s{};
  int64_t n = 0, npad = 0, naug = 0, ntr = 0;
  int G = 1, rank = 0;
  int Z = 2;          // sweep steps per bulk launch of the group schedule (sweep_group())
  bool sim = true;    // every rank simulated in this process (device copies)
  // timing-only proxy (-DACE_DIAG_SHARD_PROXY builds, unique_id NULL): rank
  // `rank` of `world` alone, scheduled as an RCCL rank (lookahead on the
  // side streams), every collective replaced by device copies of the bytes
  // that rank would receive; results wrong, per-rank time right
  bool proxy = false;
  DBuf proxy_buf;  // the broadcast's landing buffer
  bool host = false;  // host-callback collectives (ace_comm_ops)
  ace_comm_ops ops{};
  HostStage stage;  // pinned staging of the host-callback collectives
  ncclComm_t comm = nullptr;
  // head schedule (run_sweep_sharded_heads): its tail exchanges run on a
  // second communicator, so they are never ordered behind the head path's
  // (one communicator's collectives execute in issue order on any stream)
  bool heads = false;
  ncclComm_t comm2 = nullptr;
  std::vector<std::unique_ptr<RankState>> ranks;  // 1 (RCCL) or G (simulated)
  // collectives this rank issued (ace_model_comm_calls): RCCL calls or host
  // callbacks, by ace_comm_kind; simulated and proxy groups issue none
  int64_t calls[ACE_COMM_KINDS] = {};
  // a real RCCL communicator: its collectives run at every world size,
  // world 1 included (the simulated, proxy and host-callback groups treat a
  // one-rank collective as the identity)
  bool live() const { return comm != nullptr; }
  DBuf vote;                                       // shard_any: one double
  std::vector<hipEvent_t> ev;                      // lookahead events
  // timing of local rank 0 (update launches, assembly, gradient)
  std::vector<hipEvent_t> ev_upd;
  std::vector<double> upd_flops;
  hipEvent_t ev_asm[2] = {nullptr, nullptr}, ev_grad[2] = {nullptr, nullptr};
  int upd_used = 0;
  PinnedBuf hio;  // [tables | gsum | sums | scal | one flag per local rank] host staging
  ~ShardModel() {
    for (auto e : ev) (void)hipEventDestroy(e);
    for (auto e : ev_upd) (void)hipEventDestroy(e);
    for (int j = 0; j < 2; ++j) {
      if (ev_asm[j]) (void)hipEventDestroy(ev_asm[j]);
      if (ev_grad[j]) (void)hipEventDestroy(ev_grad[j]);
    }
    if (comm2) (void)rccl().CommDestroy(comm2);
    if (comm) (void)rccl().CommDestroy(comm);
  }
};

namespace {

int64_t ncols_local(int64_t naug, int G, int r) {
  const int64_t nblk = (naug + NB - 1) / NB;  // column blocks incl. the AUG block
  int64_t cnt = 0;
  for (int64_t j = r; j < nblk; j += G) ++cnt;
  return cnt * NB;
}


void upload_tiles(ace_ctx *ctx, DBuf &b, const std::vector<Tile> &t) {
  alloc(ctx, b, std::max<size_t>(t.size(), 1) * sizeof(Tile), "alloc tiles");
  upload_bytes(ctx, b.p, t.data(), t.size() * sizeof(Tile), "upload tiles");
}

ShardSweep sweep_view(const ShardModel &m, RankState &R, int which) {
  ShardSweep b;
  b.A = R.A[which].d();
  b.ld = m.naug;
  b.npad = m.npad;
  b.G = m.G;
  b.r = R.r;
  for (int j = 0; j < 8; ++j) {
    b.P[j] = R.P[j].p ? R.P[j].d() : nullptr;
    b.W[j] = R.W[j].p ? R.W[j].d() : nullptr;
  }
  for (int j = 0; j < 2; ++j) b.S[j] = R.S[j].d();
  b.SW = R.SW.d();
  b.piv = R.piv.d();
  b.flag = R.flag.i();
  b.low = R.low.d();
  b.recv = R.recv.d();
  b.tiles = reinterpret_cast<const Tile *>(R.tupd.p);
  b.ntiles = R.nupd;
  return b;
}

// GEMM flops of one k_update launch on a tile list (tiles outside block k
// and outside the cross of kx; a tile of the AUG row block computes 16 rows)
double update_flops(const std::vector<Tile> &tl, int64_t naug, int64_t k0, int kx) {
  const int KT = NB / UT, kt0 = (int)(k0 / UT), kt1 = kt0 + KT;
  const int taug = (int)(naug / UT) - 1;
  double cnt = 0.0;
  for (const Tile &t : tl) {
    if (t.I < 0) continue;  // padding of the XCD order
    if (kx >= 0 && ((t.I >= kx * KT && t.I < (kx + 1) * KT) || (t.J >= kx * KT && t.J < (kx + 1) * KT)))
      continue;
    const bool Ik = t.I >= kt0 && t.I < kt1, Jk = t.J >= kt0 && t.J < kt1;
    if (!(Ik || Jk)) cnt += (t.I == taug) ? 16.0 / UT : 1.0;
  }
  return cnt * 2.0 * UT * UT * NB;
}

// GEMM flops of one k_update_multi launch (npan steps from block ka) on a tile
// list, skipping the cross of blocks [kx0, kx1): a tile in group block jm
// starts from W_jm and takes the later panels, any other tile every panel
// (the kernel's rule; update_gemm_tiles_group over the whole triangle)
double update_flops_group(const std::vector<Tile> &tl, int64_t naug, int64_t ka0, int npan, int kx0,
                          int kx1) {
  constexpr int KT = NB / UT;
  const int ta0 = (int)(ka0 / UT);
  const int taug = (int)(naug / UT) - 1;
  double cnt = 0.0;
  for (const Tile &t : tl) {
    if (t.I < 0) continue;
    if (kx0 >= 0 && ((t.I >= kx0 * KT && t.I < kx1 * KT) || (t.J >= kx0 * KT && t.J < kx1 * KT)))
      continue;
    const int di = t.I - ta0, dj = t.J - ta0;
    const int bi = (di >= 0 && di < npan * KT) ? di / KT : -1;
    const int bj = (dj >= 0 && dj < npan * KT) ? dj / KT : -1;
    const int jm = std::max(bi, bj);
    if (jm == npan - 1) continue;
    cnt += ((t.I == taug) ? 16.0 / UT : 1.0) * (jm >= 0 ? npan - 1 - jm : npan);
  }
  return cnt * 2.0 * UT * UT * NB;
}

// The rank's own lookahead cross lists of the group schedule (RankState):
// per step k the tiles with I or J in block k + 1 (xoff), per group g >= 1
// (blocks kb = Z g .. kb + z - 1) the cross of block kb (poff[2 g]) and the
// rest of the group's cross (poff[2 g + 1]).
void build_cross_lists(ace_ctx *ctx, RankState &R, int64_t naug, int steps, int G, int Z) {
  constexpr int KT = NB / UT;
  const std::vector<Tile> own = own_tiles(naug / UT, UT, G, R.r);
  auto in_blk = [&](int t, int blk) { return t >= blk * KT && t < (blk + 1) * KT; };
  const int S = update_order_block();
  auto deal = [&](const std::vector<Tile> &t) { return S > 0 ? xcd_update_order(t, S) : t; };
  std::vector<Tile> x, pr;
  R.xoff.assign(1, 0);
  for (int k = 0; k + 1 < steps; ++k) {
    std::vector<Tile> t;
    for (const Tile &q : own)
      if (in_blk(q.I, k + 1) || in_blk(q.J, k + 1)) t.push_back(q);
    const std::vector<Tile> o = deal(t);
    x.insert(x.end(), o.begin(), o.end());
    R.xoff.push_back((int64_t)x.size());
  }
  const int ng = (steps + Z - 1) / Z;
  R.poff.assign(2 * ng + 1, 0);
  for (int g = 1; g < ng; ++g) {
    const int b0 = Z * g, b1 = std::min(steps, Z * (g + 1));  // blocks [b0, b1)
    std::vector<Tile> ta, tb;
    for (const Tile &q : own) {
      if (in_blk(q.I, b0) || in_blk(q.J, b0)) {
        ta.push_back(q);
        continue;
      }
      for (int bb = b0 + 1; bb < b1; ++bb)
        if (in_blk(q.I, bb) || in_blk(q.J, bb)) {
          tb.push_back(q);
          break;
        }
    }
    R.poff[2 * g] = (int64_t)pr.size();
    const std::vector<Tile> oa = deal(ta), ob = deal(tb);
    pr.insert(pr.end(), oa.begin(), oa.end());
    R.poff[2 * g + 1] = (int64_t)pr.size();
    pr.insert(pr.end(), ob.begin(), ob.end());
    R.poff[2 * g + 2] = (int64_t)pr.size();
  }
  upload_tiles(ctx, R.tx, x);
  upload_tiles(ctx, R.tp, pr);
}

// The head schedule's tile lists on rank R: group_head_tiles' lists (the
// single-GPU head / tail split, ace_sweep.hip) restricted to the rank's own
// tiles (column block owned), offsets hoff[G 2Z + m].
void build_head_lists(ace_ctx *ctx, RankState &R, int64_t naug, int steps, int G, int Z) {
  constexpr int KT = NB / UT;
  std::vector<int64_t> off;
  const std::vector<Tile> all = group_head_tiles(naug, steps, Z, off);
  std::vector<Tile> mine;
  R.hoff.assign(off.size(), 0);
  for (size_t m = 0; m + 1 < off.size(); ++m) {
    for (int64_t i = off[m]; i < off[m + 1]; ++i) {
      const Tile &t = all[(size_t)i];
      if (t.I >= 0 && (t.J / KT) % G == R.r) mine.push_back(t);
    }
    R.hoff[m + 1] = (int64_t)mine.size();
  }
  upload_tiles(ctx, R.th, mine);
}

// ACE_SHARD_HEADS=0: the sharded sweep keeps the group schedule without the
// head / tail split (run_sweep_sharded); default on
bool shard_heads_on() {
  static const bool v = [] {
    const char *e = getenv("ACE_SHARD_HEADS");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// ---- collectives over the local ranks -------------------------------------
// Panel exchange of step k on stream st.
void exchange(ShardModel &m, int k, hipStream_t st) {
  ace_ctx *ctx = m.ctx;
  if (m.G == 1 && !m.live()) return;  // one simulated rank: the identity
  const int64_t k0 = (int64_t)k * NB;
  const size_t nlow = (size_t)((m.naug - k0) * NB);
  const int slots = shard_row_slots(k, m.G);
  const size_t nrow = (size_t)slots * NB * NB;
  const int root = k % m.G;
  // the all-gather operand of rank r is slot r of recv (in place)
  auto own = [&](RankState &R) { return R.recv.d() + (size_t)R.r * nrow; };
  if (m.host) {
    RankState &R = *m.ranks[0];
    host_bcast(ctx, m.ops, m.stage, R.low.d(), nlow, root, st);
    ++m.calls[ACE_COMM_BROADCAST];
    if (nrow > 0) {
      host_allgather(ctx, m.ops, m.stage, own(R), R.recv.d(), nrow, m.G, st);
      ++m.calls[ACE_COMM_ALLGATHER];
    }
    return;
  }
  if (m.proxy) {  // the bytes this rank receives, as device copies
    RankState &R = *m.ranks[0];
    if (R.r != root) {
      alloc(ctx, m.proxy_buf, nlow * sizeof(double), "alloc proxy");
      ck(ctx, hipMemcpyAsync(m.proxy_buf.p, R.low.p, nlow * sizeof(double), hipMemcpyDeviceToDevice, st),
         "proxy broadcast");
    }
    if (nrow > 0)
      for (int q = 0; q < m.G; ++q)
        if (q != R.r)
          ck(ctx, hipMemcpyAsync(R.recv.d() + (size_t)q * nrow, own(R), nrow * sizeof(double),
                                 hipMemcpyDeviceToDevice, st),
             "proxy all-gather");
    return;
  }
  if (!m.sim) {
    RankState &R = *m.ranks[0];
    nck(ctx, rccl().GroupStart(), "ncclGroupStart");
    nck(ctx, rccl().Broadcast(R.low.p, R.low.p, nlow, ncclDouble, root, m.comm, st),
        "ncclBroadcast");
    ++m.calls[ACE_COMM_BROADCAST];
    if (nrow > 0) {
      nck(ctx, rccl().AllGather(own(R), R.recv.p, nrow, ncclDouble, m.comm, st), "ncclAllGather");
      ++m.calls[ACE_COMM_ALLGATHER];
    }
    nck(ctx, rccl().GroupEnd(), "ncclGroupEnd");
    ++m.calls[ACE_COMM_GROUPS];
    return;
  }
  RankState &src = *m.ranks[(size_t)root];
  for (auto &Rp : m.ranks) {
    RankState &R = *Rp;
    if (R.r != root)
      ck(ctx, hipMemcpyAsync(R.low.p, src.low.p, nlow * sizeof(double), hipMemcpyDeviceToDevice, st),
         "sim broadcast");
    if (nrow > 0)
      for (auto &Sp : m.ranks)
        if (Sp->r != R.r)
          ck(ctx, hipMemcpyAsync(R.recv.d() + (size_t)Sp->r * nrow, own(*Sp), nrow * sizeof(double),
                                 hipMemcpyDeviceToDevice, st),
             "sim all-gather");
  }
}

// The head schedule's two exchanges of panel k: head = the owner's column
// rows [k0, hend) (rows x NB doubles in lowh, broadcast, on the head path's
// stream); tail = the rows [hend, naug) (in low, broadcast) and the row
// pieces (all-gather), on the tail path's stream and the second communicator
// (host-callback groups: both through the callbacks, each blocking the host
// between its stream's drain before and after, so the host issues the head
// and tail exchanges one at a time, in the same order on every rank).
void exchange_part(ShardModel &m, int k, bool head, int64_t rows, hipStream_t st) {
  ace_ctx *ctx = m.ctx;
  if (m.G == 1 && !m.live()) return;  // one simulated rank: the identity
  const size_t nlow = (size_t)(rows * NB);
  const size_t nrow = head ? 0 : (size_t)shard_row_slots(k, m.G) * NB * NB;
  const int root = k % m.G;
  auto lowp = [&](RankState &R) { return head ? R.lowh.d() : R.low.d(); };
  auto own = [&](RankState &R) { return R.recv.d() + (size_t)R.r * nrow; };
  if (m.host) {
    RankState &R = *m.ranks[0];
    if (nlow > 0) {
      host_bcast(ctx, m.ops, m.stage, lowp(R), nlow, root, st);
      ++m.calls[ACE_COMM_BROADCAST];
    }
    if (nrow > 0) {
      host_allgather(ctx, m.ops, m.stage, own(R), R.recv.d(), nrow, m.G, st);
      ++m.calls[ACE_COMM_ALLGATHER];
    }
    return;
  }
  if (m.proxy) {  // the bytes this rank receives, as device copies (timing only)
    RankState &R = *m.ranks[0];
    if (R.r != root && nlow > 0) {
      alloc(ctx, m.proxy_buf, std::max(m.proxy_buf.bytes, nlow * sizeof(double)), "alloc proxy");
      ck(ctx, hipMemcpyAsync(m.proxy_buf.p, lowp(R), nlow * sizeof(double), hipMemcpyDeviceToDevice, st),
         "proxy broadcast");
    }
    if (nrow > 0)
      for (int q = 0; q < m.G; ++q)
        if (q != R.r)
          ck(ctx, hipMemcpyAsync(R.recv.d() + (size_t)q * nrow, own(R), nrow * sizeof(double),
                                 hipMemcpyDeviceToDevice, st),
             "proxy all-gather");
    return;
  }
  if (!m.sim) {
    RankState &R = *m.ranks[0];
    ncclComm_t c = head ? m.comm : m.comm2;
    nck(ctx, rccl().GroupStart(), "ncclGroupStart");
    if (nlow > 0) {
      nck(ctx, rccl().Broadcast(lowp(R), lowp(R), nlow, ncclDouble, root, c, st), "ncclBroadcast");
      ++m.calls[ACE_COMM_BROADCAST];
    }
    if (nrow > 0) {
      nck(ctx, rccl().AllGather(own(R), R.recv.p, nrow, ncclDouble, c, st), "ncclAllGather");
      ++m.calls[ACE_COMM_ALLGATHER];
    }
    nck(ctx, rccl().GroupEnd(), "ncclGroupEnd");
    ++m.calls[ACE_COMM_GROUPS];
    return;
  }
  RankState &src = *m.ranks[(size_t)root];
  for (auto &Rp : m.ranks) {
    RankState &R = *Rp;
    if (R.r != root && nlow > 0)
      ck(ctx, hipMemcpyAsync(lowp(R), lowp(src), nlow * sizeof(double), hipMemcpyDeviceToDevice, st),
         "sim broadcast");
    if (nrow > 0)
      for (auto &Sp : m.ranks)
        if (Sp->r != R.r)
          ck(ctx, hipMemcpyAsync(R.recv.d() + (size_t)Sp->r * nrow, own(*Sp), nrow * sizeof(double),
                                 hipMemcpyDeviceToDevice, st),
             "sim all-gather");
  }
}

// In-place sum over ranks of `count` doubles at offset `off` of buffer `which`
// (0: augvec, 1: red).
void allreduce(ShardModel &m, int which, int64_t count, hipStream_t st) {
  ace_ctx *ctx = m.ctx;
  if (m.G == 1 && !m.live()) return;  // one simulated rank: the identity
  auto buf = [&](RankState &R) { return which == 0 ? R.augvec.d() : R.red.d(); };
  if (m.host) {
    host_allreduce(ctx, m.ops, m.stage, buf(*m.ranks[0]), (size_t)count, 0, st);
    ++m.calls[ACE_COMM_ALLREDUCE];
    return;
  }
  if (m.proxy) {  // a same-size device copy in place of the ring all-reduce
    double *b = buf(*m.ranks[0]);
    alloc(ctx, m.proxy_buf, std::max(m.proxy_buf.bytes, (size_t)count * sizeof(double)), "alloc proxy");
    ck(ctx, hipMemcpyAsync(m.proxy_buf.p, b, (size_t)count * sizeof(double), hipMemcpyDeviceToDevice, st),
       "proxy all-reduce");
    return;
  }
  if (!m.sim) {
    double *b = buf(*m.ranks[0]);
    nck(ctx, rccl().AllReduce(b, b, (size_t)count, ncclDouble, ncclSum, m.comm, st),
        "ncclAllReduce");
    ++m.calls[ACE_COMM_ALLREDUCE];
    return;
  }
  double *acc = buf(*m.ranks[0]);
  for (size_t j = 1; j < m.ranks.size(); ++j)
    ck(ctx, launch_add(buf(*m.ranks[j]), acc, count, st), "sim all-reduce");
  for (size_t j = 1; j < m.ranks.size(); ++j)
    ck(ctx, hipMemcpyAsync(buf(*m.ranks[j]), acc, (size_t)count * sizeof(double),
                           hipMemcpyDeviceToDevice, st),
       "sim all-reduce");
}

// RCCL connects a communicator's peers at its first collective (host
// bootstrap exchanges, device buffers).  Each communicator runs here, with
// no kernel of this library in flight, the grouped broadcast + all-gather
// the sweep issues on it (and the all-reduce on the first), synchronised: the
// first evaluation's sweep then finds every connection made.
void rccl_warmup(ShardModel &m) {
  ace_ctx *ctx = m.ctx;
  hipStream_t st = ctx->stream;
  DBuf w;
  alloc(ctx, w, (size_t)(m.G + 1) * sizeof(double), "alloc warm-up");
  ck(ctx, hipMemsetAsync(w.p, 0, w.bytes, st), "memset warm-up");
  double *b = w.d();
  for (ncclComm_t c : {m.comm, m.comm2}) {
    if (!c) continue;
    nck(ctx, rccl().GroupStart(), "ncclGroupStart");
    nck(ctx, rccl().Broadcast(b, b, 1, ncclDouble, 0, c, st), "ncclBroadcast (warm-up)");
    nck(ctx, rccl().AllGather(b + m.rank, b, 1, ncclDouble, c, st), "ncclAllGather (warm-up)");
    nck(ctx, rccl().GroupEnd(), "ncclGroupEnd");
    m.calls[ACE_COMM_BROADCAST] += 1;
    m.calls[ACE_COMM_ALLGATHER] += 1;
    m.calls[ACE_COMM_GROUPS] += 1;
    sync_stream(ctx, st, "RCCL warm-up");
  }
  nck(ctx, rccl().AllReduce(b + m.G, b + m.G, 1, ncclDouble, ncclSum, m.comm, st),
      "ncclAllReduce (warm-up)");
  m.calls[ACE_COMM_ALLREDUCE] += 1;
  sync_stream(ctx, st, "RCCL warm-up");
}

// ---- the sharded sweep -------------------------------------------------------
bool fuse_pack() {
  static const bool v = [] {
    const char *e = getenv("ACE_FUSE_PACK");
    return !(e && atoi(e) == 0);
  }();
  return v;
}

// One step per update launch, lookahead only over RCCL (ACE_PAIR=0: the
// round-2 schedule, kept for A/B and for npad < 2 NB).
void run_sweep_sharded_steps(ShardModel &m, int which, bool timed) {
  ace_ctx *ctx = m.ctx;
  hipStream_t st = ctx->stream;
  // the simulated and the host-callback groups run everything in order on
  // one stream (their exchanges are synchronous)
  const bool lookahead = !m.sim && !m.host;
  hipStream_t side = lookahead ? ctx->side : st;
  const int steps = (int)(m.npad / NB);
  std::vector<ShardSweep> v;
  for (auto &R : m.ranks) v.push_back(sweep_view(m, *R, which));
  auto rec = [&](int idx, hipStream_t s) {
    if (lookahead) ck(ctx, hipEventRecord(m.ev[(size_t)idx], s), "event");
  };
  auto wait = [&](hipStream_t s, int idx) {
    if (lookahead) ck(ctx, hipStreamWaitEvent(s, m.ev[(size_t)idx], 0), "event wait");
  };
  auto prepare = [&](int k, int buf) {  // panel k into buffer buf, on `side`
    for (auto &b : v) ck(ctx, shard_pack(b, k, side), "shard pack");
    exchange(m, k, side);
    for (auto &b : v) ck(ctx, shard_unpack_chain(b, k, buf, side), "shard panel");
  };
  rec(2 * steps, st);  // inputs ready
  wait(side, 2 * steps);
  prepare(0, 0);
  rec(0, side);
  m.upd_used = 0;
  for (int k = 0; k < steps; ++k) {
    const int buf = k & 1;
    const bool more = k + 1 < steps;
    wait(st, 2 * k);  // panel k ready
    if (more) {
      // side stream, under the bulk update k: cross of block k+1 (after the
      // bulk update k-1), then pack / exchange / sweep of panel k+1
      rec(2 * k + 1, st);
      wait(side, 2 * k + 1);
      for (auto &b : v) ck(ctx, shard_update_cross(b, k, buf, side), "shard cross update");
      prepare(k + 1, buf ^ 1);
      rec(2 * (k + 1), side);
    }
    const bool tm = timed && m.upd_used + 2 <= (int)m.ev_upd.size();
    for (size_t j = 0; j < v.size(); ++j) {
      if (tm && j == 0) ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used], st), "event");
      ck(ctx, shard_update_main(v[j], k, buf, more ? k + 1 : -1, st), "shard update");
      if (tm && j == 0) {
        ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used + 1], st), "event");
        m.upd_flops[(size_t)m.upd_used / 2] =
            update_flops(m.ranks[0]->hupd, m.naug, (int64_t)k * NB, more ? k + 1 : -1);
        m.upd_used += 2;
      }
    }
  }
}

// Z sweep steps per bulk launch (Z = sweep_group(), 4 by default), the
// single-GPU group schedule (ace_sweep.hip run_sweep_groups) on each rank's own
// tiles.  Group g = steps Z g .. Z g + z - 1, panels in slots k % (2 Z):
//   main:  wait(ready g) -> k_update_multi over the own tiles outside group
//          g+1's cross (group g's z panels, K = z NB per tile) -> bulkdone(g)
//   side:  wait(bulkdone g-1) -> group g's panels on block kb's cross (the
//          launch that finalises block kb also packs step kb's exchange
//          buffers) -> prepare(kb) [exchange, unpack + pivot chain + W] ->
//          [wait side2] for j = 1 .. z-1: panels kb .. kb+j-1 on block
//          kb+j's cross (packing kb+j) -> prepare(kb+j) -> ready(g+1)
//   side2: group g's panels on the rest of group g+1's cross, concurrently
//          with block kb's chain
// Every mode runs the lookahead: RCCL exchanges on the side stream; the
// simulated group's device copies on the side stream (all simulated ranks
// share the three streams, so their bulk launches overlap the side path as
// one rank's do); the host-callback group synchronises the side stream and
// exchanges on the host while the already enqueued bulk launch runs.  The
// bulk launch of group g is enqueued before the side path of group g+1 so
// that a blocking (host) exchange overlaps it.  Every tile sees the
// single-step schedule's MFMA chains in the same order (k_update_multi's
// per-tile rule): bit-identical to run_sweep_sharded_steps
// (tests/test_shard_gpu.py).
// The single-GPU head / tail schedule (run_sweep_heads) on each
// rank's own tiles, with the exchange split the same way.  Group G = blocks
// [kb, kb + z), hend = (kb + z) NB:
//   side (head path): Q over the group's square (own tiles) packs panel kb's
//     column rows [kb NB, hend) -> head exchange (a broadcast of at most
//     Z NB x NB doubles from the block's owner) -> unpack -> the pivot
//     sub-steps -> the panel GEMM of the rows [k0 + NB, hend) -> Q_{j+1}
//     packs panel k + 1's head rows -> ...
//   side2 (tail path): the rest of the group's cross packs panel kb's rows
//     [hend, naug) and the row pieces -> tail exchange (broadcast +
//     all-gather, second communicator) -> unpack -> [after the sub-steps] the
//     panel GEMM of the other rows -> [after the head GEMM] T_{j+1} packs
//     panel k + 1's tail -> ...
//   main: [ready g, ready2 g] -> the bulk launch of group g.
// A panel's pivot chain then waits only for its head rows: the full column
// cross, the row-piece all-gather and the panel GEMM of every other row run
// beside it.  Every tile sees the same launches' MFMA chains as in
// run_sweep_heads (the same lists, restricted to the rank's tiles):
// bit-identical to the single-GPU model (tests/test_shard_gpu.py).
void run_sweep_sharded_heads(ShardModel &m, int which, bool timed) {
  ace_ctx *ctx = m.ctx;
  const int steps = (int)(m.npad / NB);
  const int Z = m.Z, NS = 2 * Z;
  const int ng = (steps + Z - 1) / Z;
  constexpr int KT = NB / UT;
  const int64_t naug = m.naug;
  hipStream_t st = ctx->stream, side = ctx->side, side2 = ctx->side2;
  auto zsize = [&](int g) { return std::min(Z, steps - Z * g); };
  std::vector<ShardSweep> v;
  for (auto &R : m.ranks) v.push_back(sweep_view(m, *R, which));
  auto EV = [&](int i) { return m.ev[(size_t)i]; };
  const int E_IN = 0;  // recorded by shard_eval: the first group's columns assembled
  auto E_READY = [&](int g) { return 1 + g; };          // group g's head path done
  auto E_READY2 = [&](int g) { return 1 + ng + g; };    // group g's tail path done
  auto E_SP = [&](int k) { return 2 + 3 * ng + 2 * k; };  // panel k's sub-steps done
  auto E_GH = [&](int k) { return 3 + 3 * ng + 2 * k; };  // panel k's head GEMM done
  // main, before bulk g: bulk g-1 done and group g's head and tail paths
  // done -- what group g+1's lists need (its tiles were last touched by bulk
  // g-1; the W rows of its blocks come from group g's tail panel GEMMs)
  auto E_PRE = [&](int g) { return 2 + 3 * ng + 2 * steps + g; };
  // bulk g done (g = -1: the main stream's work before the sweep): the head
  // path of group g+2 waits for it and group g+1's tail path directly -- one
  // cross-stream hop instead of two through E_PRE (single GPU: the same in
  // run_sweep_heads, profiles/r05_v14_qdirect.txt)
  auto E_BULK = [&](int g) { return 3 + 4 * ng + 2 * steps + g; };
  auto rec = [&](int i, hipStream_t s_) { ck(ctx, hipEventRecord(EV(i), s_), "event"); };
  auto wait = [&](hipStream_t s_, int i) { ck(ctx, hipStreamWaitEvent(s_, EV(i), 0), "event wait"); };
  auto hend_of = [&](int G) { return (int64_t)(Z * G + zsize(G)) * NB; };
  // own tiles of list m of group G (group_head_tiles' numbering)
  auto hlist = [&](size_t q, int G, int mm, int64_t &n) {
    RankState &R = *m.ranks[q];
    const size_t i = (size_t)G * 2 * Z + (size_t)mm;
    n = R.hoff[i + 1] - R.hoff[i];
    return (const Tile *)R.th.p + R.hoff[i];
  };
  // a launch on list mm of group G: npan panels from block kb0, packing
  // panel kp's head (head = true) or tail part
  auto launch = [&](int G, int mm, int npan, int kb0, int kp, bool head, hipStream_t s_) {
    const int64_t k0 = (int64_t)kp * NB, he = hend_of(G);
    for (size_t q = 0; q < v.size(); ++q) {
      int64_t n;
      const Tile *tl = hlist(q, G, mm, n);
      RankState &R = *m.ranks[q];
      ck(ctx, shard_update_group(v[q], kb0, npan, NS, -1, -1, tl, n, s_, kp,
                                 head ? R.lowh.d() : R.low.d(), head ? 0 : he - k0,
                                 head ? he - k0 : naug - he),
         head ? "shard head update" : "shard tail update");
    }
  };
  // panel k's head rows in: exchange (+ pack when no launch packed them) + unpack
  auto head_in = [&](int k, int G, bool packed) {
    const int64_t k0 = (int64_t)k * NB, he = hend_of(G);
    if (!packed)
      for (size_t q = 0; q < v.size(); ++q)
        ck(ctx, shard_pack_part(v[q], k, k0, he, m.ranks[q]->lowh.d(), 0, he - k0, false, side),
           "shard head pack");
    exchange_part(m, k, true, he - k0, side);
    for (size_t q = 0; q < v.size(); ++q)
      ck(ctx, shard_unpack_part(v[q], k, k % NS, k0, he, m.ranks[q]->lowh.d(), 0, he - k0, packed, side),
         "shard head unpack");
  };
  auto tail_in = [&](int k, int G, bool packed) {
    const int64_t k0 = (int64_t)k * NB, he = hend_of(G);
    if (!packed)
      for (size_t q = 0; q < v.size(); ++q)
        ck(ctx, shard_pack_part(v[q], k, he, naug, m.ranks[q]->low.d(), he - k0, naug - he, true, side2),
           "shard tail pack");
    exchange_part(m, k, false, naug - he, side2);
    for (size_t q = 0; q < v.size(); ++q) {
      ck(ctx, shard_unpack_part(v[q], k, k % NS, 0, k0, m.ranks[q]->low.d(), 0, 0, packed, side2),
         "shard tail unpack");
      ck(ctx, shard_unpack_part(v[q], k, k % NS, he, naug, m.ranks[q]->low.d(), he - k0, naug - he,
                                packed, side2),
         "shard tail unpack");
    }
  };
  // group G's head path (side) and tail path (side2)
  auto produce = [&](int G) {
    const int kb = Z * G, zb = zsize(G);
    const int hT = (int)(hend_of(G) / UT);
    if (G == 0) {
      head_in(0, 0, false);
      tail_in(0, 0, false);
    } else {
      launch(G, 0, zsize(G - 1), Z * (G - 1), kb, true, side);    // Q
      head_in(kb, G, true);
      launch(G, 1, zsize(G - 1), Z * (G - 1), kb, false, side2);  // the rest of the cross
      tail_in(kb, G, true);
    }
    for (int j = 0; j < zb; ++j) {
      const int k = kb + j;
      // head
      for (auto &b : v) ck(ctx, shard_chain(b, k, k % NS, side), "shard chain");
      rec(E_SP(k), side);
      for (auto &b : v) ck(ctx, shard_pgemm(b, k, k % NS, (k + 1) * KT, hT, true, side), "shard head GEMM");
      rec(E_GH(k), side);
      if (j + 1 < zb) {
        launch(G, 2 + j, 1, k, k + 1, true, side);  // panel k on Q_{j+1}
        head_in(k + 1, G, true);
      }
      // tail
      wait(side2, E_SP(k));
      for (auto &b : v) ck(ctx, shard_pgemm(b, k, k % NS, (k + 1) * KT, hT, false, side2), "shard tail GEMM");
      if (j + 1 < zb) {
        wait(side2, E_GH(k));
        launch(G, zb + j + 1, j + 1, kb, k + 1, false, side2);  // T_{j+1}
        tail_in(k + 1, G, true);
      }
    }
    rec(E_READY(G), side);
    rec(E_READY2(G), side2);
  };
  wait(side, E_IN);
  wait(side2, E_IN);
  produce(0);
  rec(E_BULK(-1), st);
  m.upd_used = 0;
  for (int g = 0; g < ng; ++g) {
    const int kg = Z * g;
    const bool more = g + 1 < ng;
    const int kb = Z * (g + 1), zb = more ? zsize(g + 1) : 0;
    wait(st, E_READY(g));
    wait(st, E_READY2(g));
    rec(E_PRE(g), st);
    const bool tm = timed && m.upd_used + 2 <= (int)m.ev_upd.size();
    const int kx0 = more ? kb : -1, kx1 = more ? kb + zb : -1;
    for (size_t j = 0; j < v.size(); ++j) {
      RankState &R = *m.ranks[j];
      if (tm && j == 0) ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used], st), "event");
      ck(ctx, shard_update_group(v[j], kg, zsize(g), NS, kx0, kx1, (const Tile *)R.tupd.p, R.nupd, st),
         "shard group update");
      if (tm && j == 0) {
        ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used + 1], st), "event");
        m.upd_flops[(size_t)m.upd_used / 2] =
            update_flops_group(R.hupd, m.naug, (int64_t)kg * NB, zsize(g), kx0, kx1);
        m.upd_used += 2;
      }
    }
    if (!more) break;
    rec(E_BULK(g), st);
    wait(side, E_READY2(g));
    wait(side, E_BULK(g - 1));
    wait(side2, E_PRE(g));
    produce(g + 1);
  }
}

void run_sweep_sharded(ShardModel &m, int which, bool timed) {
  ace_ctx *ctx = m.ctx;
  const int steps = (int)(m.npad / NB);
  const int Z = m.Z;
  if (m.heads && steps >= 2) {
    run_sweep_sharded_heads(m, which, timed);
    return;
  }
  if (!pair_steps() || steps < 2 || Z < 2 || !m.ranks[0]->P[2 * Z - 1].p) {
    run_sweep_sharded_steps(m, which, timed);
    return;
  }
  const int NS = 2 * Z;  // panel slots
  hipStream_t st = ctx->stream, side = ctx->side, side2 = ctx->side2;
  const int ng = (steps + Z - 1) / Z;
  auto zsize = [&](int g) { return std::min(Z, steps - Z * g); };
  std::vector<ShardSweep> v;
  for (auto &R : m.ranks) v.push_back(sweep_view(m, *R, which));
  // events: [0] inputs, ready(g) 1.., bulkdone(g) 1+ng.., side2 start / done,
  // [4 ng + 1] the assembly done
  auto EV = [&](int i) { return m.ev[(size_t)i]; };
  const int E_IN = 0;
  auto E_READY = [&](int g) { return 1 + g; };
  auto E_BULK = [&](int g) { return 1 + ng + g; };
  auto E_S2A = [&](int g) { return 1 + 2 * ng + g; };
  auto E_S2B = [&](int g) { return 1 + 3 * ng + g; };
  const int E_ASM = 1 + 4 * ng;  // the whole assembly (part 2 included) done
  auto rec = [&](int i, hipStream_t s_) { ck(ctx, hipEventRecord(EV(i), s_), "event"); };
  auto wait = [&](hipStream_t s_, int i) { ck(ctx, hipStreamWaitEvent(s_, EV(i), 0), "event wait"); };
  // the cross launch that finalises block k's tiles also writes the exchange
  // buffers of step k (ACE_FUSE_PACK=0: separate k_pack_* launches)
  const bool fuse = fuse_pack();
  auto prepare = [&](int k, bool packed) {  // panel k into slot k % NS, on `side`
    if (!packed)
      for (auto &b : v) ck(ctx, shard_pack(b, k, side), "shard pack");
    exchange(m, k, side);
    for (auto &b : v) ck(ctx, shard_unpack_chain(b, k, k % NS, side, packed), "shard panel");
  };
  // blocks kb + 1 .. kb + z - 1 of a group from its own panels, each followed
  // by its exchange and chain (on `side`)
  auto inner = [&](int kb, int z) {
    for (int j = 1; j < z; ++j) {
      const int k = kb + j - 1;  // xoff list k: the own tiles with I or J in block k + 1
      for (size_t q = 0; q < v.size(); ++q) {
        RankState &R = *m.ranks[q];
        const int64_t x0 = R.xoff[(size_t)k], nx = R.xoff[(size_t)k + 1] - x0;
        ck(ctx, shard_update_group(v[q], kb, j, NS, -1, -1, (const Tile *)R.tx.p + x0, nx, side,
                                   fuse ? kb + j : -1),
           "shard cross update");
      }
      prepare(kb + j, fuse);
    }
  };
  // E_IN: recorded by shard_eval after the first group's panels' columns,
  // the AUG rows and the flag (the rest of the assembly runs on under it)
  wait(side, E_IN);
  prepare(0, false);
  inner(0, zsize(0));
  rec(E_READY(0), side);
  m.upd_used = 0;
  rec(E_ASM, st);  // group 1's cross tiles include assembly part-2 tiles
  for (int g = 0; g < ng; ++g) {
    const int kg = Z * g;
    const bool more = g + 1 < ng;
    const int kb = Z * (g + 1), zb = more ? zsize(g + 1) : 0;
    wait(st, E_READY(g));
    const bool tm = timed && m.upd_used + 2 <= (int)m.ev_upd.size();
    const int kx0 = more ? kb : -1, kx1 = more ? kb + zb : -1;
    for (size_t j = 0; j < v.size(); ++j) {
      RankState &R = *m.ranks[j];
      if (tm && j == 0) ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used], st), "event");
      ck(ctx, shard_update_group(v[j], kg, zsize(g), NS, kx0, kx1, (const Tile *)R.tupd.p, R.nupd,
                                 st),
         "shard group update");
      if (tm && j == 0) {
        ck(ctx, hipEventRecord(m.ev_upd[(size_t)m.upd_used + 1], st), "event");
        m.upd_flops[(size_t)m.upd_used / 2] =
            update_flops_group(R.hupd, m.naug, (int64_t)kg * NB, zsize(g), kx0, kx1);
        m.upd_used += 2;
      }
    }
    rec(E_BULK(g), st);
    if (!more) break;
    // side path of group g + 1 (its cross tiles were last touched by bulk g-1)
    wait(side, g > 0 ? E_BULK(g - 1) : E_ASM);
    const bool rest = zb > 1;
    if (rest) {  // the rest of group g+1's cross on side2, concurrently
      rec(E_S2A(g + 1), side);
      wait(side2, E_S2A(g + 1));
      for (size_t j = 0; j < v.size(); ++j) {
        RankState &R = *m.ranks[j];
        const int64_t p0 = R.poff[(size_t)(2 * (g + 1) + 1)], np = R.poff[(size_t)(2 * (g + 1) + 2)] - p0;
        ck(ctx, shard_update_group(v[j], kg, zsize(g), NS, -1, -1, (const Tile *)R.tp.p + p0, np,
                                   side2),
           "shard group cross");
      }
      rec(E_S2B(g + 1), side2);
    }
    for (size_t j = 0; j < v.size(); ++j) {
      RankState &R = *m.ranks[j];
      const int64_t p0 = R.poff[(size_t)(2 * (g + 1))], np = R.poff[(size_t)(2 * (g + 1) + 1)] - p0;
      ck(ctx, shard_update_group(v[j], kg, zsize(g), NS, -1, -1, (const Tile *)R.tp.p + p0, np, side,
                                 fuse ? kb : -1),
         "shard group cross");
    }
    prepare(kb, fuse);
    if (rest) wait(side, E_S2B(g + 1));
    inner(kb, zb);
    rec(E_READY(g + 1), side);
  }
}

}  // namespace

// ---- entry points used by ace_api.cpp ------------------------------------------
void shard_unique_id(unsigned char *id) {
  Rccl &R = rccl();
  if (!R.ok) throw std::runtime_error(R.err);
  ncclUniqueId u;
  if (R.GetUniqueId(&u) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
  std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
}

namespace {
ShardModel *shard_create_any(ace_ctx *ctx, const Shape &s, int64_t n, int world, int rank,
                             const unsigned char *id, const ace_comm_ops *ops) {
  std::unique_ptr<ShardModel> m(new ShardModel());
  m->ctx = ctx;
  m->s = s;
  m->n = n;
  m->npad = round_up(n, NB);
  m->naug = m->npad + AUG;
  m->ntr = (n + AT - 1) / AT;
  m->G = world;
  m->rank = rank;
  m->Z = sweep_group_n(m->naug);
  m->host = ops != nullptr;
  if (ops) m->ops = *ops;
  m->sim = id == nullptr && !m->host;
#ifdef ACE_DIAG_SHARD_PROXY
  m->proxy = m->sim && world > 1;
  if (m->proxy) m->sim = false;
#endif
  const int64_t naug = m->naug, npad = m->npad;
  if (!m->sim && !m->host && !m->proxy) {
    if (!rccl().ok) {
      ctx->err = rccl().err;
      throw Fail{ACE_ERR_HIP};
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
    nck(ctx, rccl().CommInitRank(&m->comm, world, u, rank), "ncclCommInitRank");
  }
  const int nlocal = m->sim ? world : 1;
  const int steps = (int)(npad / NB);
  // the head schedule in every mode (the host-callback group's head and tail
  // exchanges block the host one at a time, in issue order)
  m->heads = shard_heads_on() && heads_on() && pair_steps() && steps >= 2 && m->Z >= 2 &&
             (m->sim || m->proxy || m->host || rccl().CommSplit);
  if (m->heads && m->comm)
    nck(ctx, rccl().CommSplit(m->comm, 0, rank, &m->comm2, nullptr), "ncclCommSplit");
  if (m->comm) rccl_warmup(*m);
  const int maxslots = shard_row_slots(steps, world);
  const int ncol = s.B * (s.PM + 1);
  for (int j = 0; j < nlocal; ++j) {
    std::unique_ptr<RankState> R(new RankState());
    R->r = m->sim ? j : rank;
    // every rank allocates the largest local width (rank 0's), so that the
    // local arrays are equal-sized all-gather operands (shard_get_inverse);
    // the extra block column of the smaller ranks is never touched otherwise
    const int64_t nloc = ncols_local(naug, world, 0);
    alloc(ctx, R->A[0], (size_t)(naug * nloc) * sizeof(double), "alloc local A");
    ck(ctx, hipMemsetAsync(R->A[0].p, 0, R->A[0].bytes, ctx->stream), "memset A");
    // group schedule: 2 Z panel slots (k % 2Z); the one-step schedule: 2
    const int nslot = pair_steps() && steps >= 2 ? 2 * m->Z : 2;
    for (int b = 0; b < nslot; ++b) {
      alloc(ctx, R->P[b], (size_t)(naug * NB) * sizeof(double), "alloc panel");
      alloc(ctx, R->W[b], (size_t)(naug * NB) * sizeof(double), "alloc panel");
    }
    for (int b = 0; b < 2; ++b) alloc(ctx, R->S[b], (size_t)(SUB * NB) * sizeof(double), "alloc S");
    if (nslot > 2) build_cross_lists(ctx, *R, naug, steps, world, m->Z);
    if (m->heads) {
      build_head_lists(ctx, *R, naug, steps, world, m->Z);
      alloc(ctx, R->lowh, (size_t)(m->Z * NB * NB) * sizeof(double), "alloc head exchange");
    }
    alloc(ctx, R->SW, (size_t)SW_DOUBLES * sizeof(double), "alloc SW");
    alloc(ctx, R->piv, (size_t)npad * sizeof(double), "alloc piv");
    alloc(ctx, R->flag, 16, "alloc flag");
    alloc(ctx, R->low, (size_t)(naug * NB) * sizeof(double), "alloc exchange");
    alloc(ctx, R->recv, (size_t)world * std::max(1, maxslots) * NB * NB * sizeof(double),
          "alloc exchange");
    if (m->proxy) {  // what the proxy never receives is zeros, not stale memory
      ck(ctx, hipMemsetAsync(R->low.p, 0, R->low.bytes, ctx->stream), "memset exchange");
      ck(ctx, hipMemsetAsync(R->recv.p, 0, R->recv.bytes, ctx->stream), "memset exchange");
    }
    R->hupd = own_tiles(naug / UT, UT, world, R->r);
    if (const int S = update_order_block(); S > 0) R->hupd = xcd_update_order(R->hupd, S);
    R->nupd = (int64_t)R->hupd.size();
    upload_tiles(ctx, R->tupd, R->hupd);
    std::vector<Tile> ta = own_tiles(npad / AT, AT, world, R->r);
    // the first group's panels' columns first (the group schedule's first
    // side path runs under the rest of the assembly, as model_pipeline's)
    const int jb = m->Z * NB / AT;
    R->nasm1 = std::stable_partition(ta.begin(), ta.end(), [&](const Tile &t) { return t.J < jb; }) -
               ta.begin();
    R->nasm = (int64_t)ta.size();
    upload_tiles(ctx, R->tasm, ta);
    std::vector<Tile> tg = own_tiles(m->ntr, AT, world, R->r);
    // diagonal tiles first: the gradient kernel runs them separately
    std::stable_partition(tg.begin(), tg.end(), [](const Tile &t) { return t.I == t.J; });
    R->ngrad = (int64_t)tg.size();
    for (const Tile &t : tg) R->ndiag += t.I == t.J;
    upload_tiles(ctx, R->tgrad, tg);
    alloc(ctx, R->y, (size_t)npad * sizeof(double), "alloc y");
    alloc(ctx, R->tab, (size_t)(2 * s.B * s.PM + s.B) * sizeof(double), "alloc tab");
    alloc(ctx, R->alpha, (size_t)npad * sizeof(double), "alloc alpha");
    alloc(ctx, R->scal, 16 * sizeof(double), "alloc scal");
    const int ldg = grad_part_cols(s.PM, s.B);
    alloc(ctx, R->gpart, (size_t)(std::max<int64_t>(R->ngrad, 1) * ldg) * sizeof(double),
          "alloc gpart");
    alloc(ctx, R->gwork, (size_t)tile_sums_work(ldg) * sizeof(double), "alloc tile sums");
    alloc(ctx, R->red, (size_t)(ncol + 1 + npad) * sizeof(double), "alloc reduction");
    alloc(ctx, R->sums, 8 * sizeof(double), "alloc sums");
    alloc(ctx, R->augvec, (size_t)(2 * npad + 8) * sizeof(double), "alloc aug vector");
    m->ranks.push_back(std::move(R));
  }
  // lookahead events: the step schedule's 2 steps + 1, the pair schedule's
  // 4 ngroups + 2
  const int ngr = (steps + m->Z - 1) / std::max(1, m->Z);
  m->ev.assign((size_t)std::max({2 * steps + 1, 4 * ((steps + 1) / 2) + 2, 4 + 5 * ngr + 2 * steps}),
               nullptr);
  for (auto &e : m->ev) ck(ctx, hipEventCreateWithFlags(&e, ACE_SYNC_EVENT_FLAGS), "event");
  m->ev_upd.assign((size_t)(2 * steps), nullptr);
  m->upd_flops.assign((size_t)steps, 0.0);
  for (auto &e : m->ev_upd) ck(ctx, hipEventCreateWithFlags(&e, ACE_TIMING_EVENT_FLAGS), "event");
  for (int j = 0; j < 2; ++j) {
    ck(ctx, hipEventCreateWithFlags(&m->ev_asm[j], ACE_TIMING_EVENT_FLAGS), "event");
    ck(ctx, hipEventCreateWithFlags(&m->ev_grad[j], ACE_TIMING_EVENT_FLAGS), "event");
  }
  sync(ctx);
  return m.release();
}
}  // namespace

ShardModel *shard_create(ace_ctx *ctx, const Shape &s, int64_t n, int world, int rank,
                         const unsigned char *id) {
  return shard_create_any(ctx, s, n, world, rank, id, nullptr);
}

ShardModel *shard_create_host(ace_ctx *ctx, const Shape &s, int64_t n, int world, int rank,
                              const ace_comm_ops &ops) {
  return shard_create_any(ctx, s, n, world, rank, nullptr, &ops);
}

void shard_destroy(ShardModel *m) { delete m; }

void shard_set_data(ShardModel *m, const double *y, const double *X, const double *Z) {
  ace_ctx *ctx = m->ctx;
  std::vector<double> yp((size_t)m->npad, 0.0);
  std::copy(y, y + m->n, yp.begin());
  for (auto &R : m->ranks) {
    upload_side(ctx, R->side, m->s, X, Z, m->n, m->npad);
    upload_bytes(ctx, R->y.p, yp.data(), yp.size() * sizeof(double), "upload y");
  }
  sync(ctx);
}

// One evaluation at theta into A[which]; the host receives (local rank 0's
// copy of the all-reduced) gradient sums, final sums, scalars and the flag.
void shard_eval(ShardModel *m, const double *theta, int use_mu, int which, bool timed,
                double *gsum, double *sums, double *scal, int *flag) {
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  const Shape &s = m->s;
  const int ncol = s.B * (s.PM + 1);
  const int64_t naug = m->naug, npad = m->npad, n = m->n;
  std::vector<double> tab = make_tab(theta, s);
  const double sig = std::exp(theta[0]);
  // pinned staging, async on the stream: the previous evaluation's results
  // were synchronised before this one started, so the region is free
  const size_t nl = m->ranks.size();
  double *h = m->hio.ensure(ctx, tab.size() + (size_t)(ncol + 1) + 4 + 5 + nl);
  std::copy(tab.begin(), tab.end(), h);
  for (auto &R : m->ranks) {
    if (which == 1) {
      alloc(ctx, R->A[1], R->A[0].bytes, "alloc local A (train stats)");
      ck(ctx, hipMemsetAsync(R->A[1].p, 0, R->A[1].bytes, st), "memset A");
    }
    ck(ctx, hipMemcpyAsync(R->tab.p, h, tab.size() * sizeof(double), hipMemcpyHostToDevice, st),
       "upload tables");
  }
  // assembly (own tiles) + AUG rows: the first group's panels' columns, the
  // AUG rows and the flag, then (the sweep's first side path may start) the rest
  if (timed) ck(ctx, hipEventRecord(m->ev_asm[0], st), "event");
  for (int part = 0; part < 2; ++part) {
    for (size_t j = 0; j < m->ranks.size(); ++j) {
      RankState &R = *m->ranks[j];
      const TabView tv = tab_view(R.tab, s);
      const PairSide ps = R.side.view(n);
      const int64_t t0 = part ? R.nasm1 : 0, nt = part ? R.nasm - R.nasm1 : R.nasm1;
      if (nt > 0)
        ck(ctx, launch_assembly(0, s.kind, s.PM, ps, ps, npad, s.B, s.ZS, tv, sig, R.A[which].d(),
                                naug, nullptr, st, (const Tile *)R.tasm.p + t0, nt, m->G),
           "assembly");
      if (part == 0) {
        ck(ctx, launch_aug_init(R.A[which].d(), naug, npad, n, R.y.d(), st, m->G, R.r), "aug init");
        ck(ctx, hipMemsetAsync(R.flag.p, 0, sizeof(int), st), "memset flag");
      }
    }
    if (part == 0) ck(ctx, hipEventRecord(m->ev[0], st), "event");  // the sweep's inputs ready
  }
  if (timed) ck(ctx, hipEventRecord(m->ev_asm[1], st), "event");
  run_sweep_sharded(*m, which, timed);
  // alpha, mu_solution
  for (auto &R : m->ranks)
    ck(ctx, launch_aug_extract(R->A[which].d(), naug, npad, m->G, R->r, R->augvec.d(), st),
       "aug extract");
  allreduce(*m, 0, 2 * npad + 3, st);
  for (auto &R : m->ranks)
    ck(ctx, launch_alpha_from_vec(R->augvec.d(), npad, n, theta[1], use_mu, R->alpha.d(),
                                  R->scal.d(), st),
       "alpha");
  // gradient partial sums of own tiles
  for (size_t j = 0; j < m->ranks.size(); ++j) {
    RankState &R = *m->ranks[j];
    const TabView tv = tab_view(R.tab, s);
    const PairSide ps = R.side.view(n);
    const Tile *tg = (const Tile *)R.tgrad.p;
    if (timed && j == 0) ck(ctx, hipEventRecord(m->ev_grad[0], st), "event");
    ck(ctx, launch_grad(s.kind, s.PM, ps, s.B, s.ZS, tv, R.A[which].d(), naug, -1.0, R.alpha.d(),
                        nullptr, R.gpart.d(), st, tg, R.ngrad, m->G, R.ndiag),
       "grad");
    if (timed && j == 0) ck(ctx, hipEventRecord(m->ev_grad[1], st), "event");
    // a rank without gradient tiles contributes zeros (tile sums over none)
    ck(ctx, launch_tile_sums(R.gpart.d(), R.ngrad, ncol + 1, R.gwork.d(), R.red.d(), st),
       "tile sums");
  }
  allreduce(*m, 1, ncol + 1, st);
  // RMSE residual ybar - Kfull alpha = sig alpha (k_final_sums): no Kfull pass
  for (auto &R : m->ranks)
    ck(ctx, launch_final_sums(R->y.d(), R->scal.d() + 4, R->alpha.d(), nullptr, sig, n,
                              R->piv.d(), npad, R->sums.d(), st),
       "final sums");
  // into the pinned region behind the tables, one synchronisation
  RankState &R0 = *m->ranks[0];
  double *hg = h + tab.size(), *hs = hg + ncol + 1, *hc = hs + 4, *hf = hc + 5;
  ck(ctx, hipMemcpyAsync(hg, R0.red.p, (size_t)(ncol + 1) * sizeof(double), hipMemcpyDeviceToHost, st),
     "download gsum");
  ck(ctx, hipMemcpyAsync(hs, R0.sums.p, 4 * sizeof(double), hipMemcpyDeviceToHost, st),
     "download sums");
  ck(ctx, hipMemcpyAsync(hc, R0.scal.p, 5 * sizeof(double), hipMemcpyDeviceToHost, st),
     "download scal");
  for (size_t j = 0; j < nl; ++j)
    ck(ctx, hipMemcpyAsync(hf + j, m->ranks[j]->flag.p, sizeof(int), hipMemcpyDeviceToHost, st),
       "download flag");
  sync(ctx);
  std::copy(hg, hg + ncol + 1, gsum);
  std::copy(hs, hs + 4, sums);
  std::copy(hc, hc + 5, scal);
  *flag = 0;
  for (size_t j = 0; j < nl; ++j) {
    int f;
    std::memcpy(&f, hf + j, sizeof(int));
    *flag |= f;
  }
}

// Full symmetric inverse (n x n) of the resident A[0] on every rank.  The
// ranks' local arrays (equal-sized, see shard_create) are gathered into one
// naug x (G * nloc) buffer, slot r = rank r's local columns -- an RCCL
// all-gather, or device copies in the simulated group -- and the mirror
// kernel reads global column c from slot (c / NB) % G at local column
// lcol(c).  One gathered copy per process, no sums.
void shard_get_inverse(ShardModel *m, double *inv) {
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  const int64_t n = m->n, naug = m->naug;
  const int64_t slot = naug * ncols_local(naug, m->G, 0);  // doubles per rank
  DBuf gath, out;
  alloc(ctx, gath, (size_t)(slot * m->G) * sizeof(double), "alloc gathered inverse");
  if (m->sim || m->proxy) {
    for (auto &R : m->ranks)
      ck(ctx, hipMemcpyAsync(gath.d() + (size_t)R->r * slot, R->A[0].p, (size_t)slot * sizeof(double),
                             hipMemcpyDeviceToDevice, st),
         "gather local columns");
  } else if (m->host) {
    host_allgather(ctx, m->ops, m->stage, m->ranks[0]->A[0].d(), gath.d(), (size_t)slot, m->G, st);
    ++m->calls[ACE_COMM_ALLGATHER];
  } else {
    nck(ctx, rccl().AllGather(m->ranks[0]->A[0].p, gath.p, (size_t)slot, ncclDouble, m->comm, st),
        "ncclAllGather (inverse)");
    ++m->calls[ACE_COMM_ALLGATHER];
  }
  alloc(ctx, out, (size_t)(n * n) * sizeof(double), "alloc inverse");
  ck(ctx, launch_sym_from_cyclic(gath.d(), naug, n, m->G, slot, -1.0, out.d(), n, st),
     "symmetrize");
  download(ctx, inv, out.d(), (size_t)(n * n), "download inverse");
  sync(ctx);
}

void shard_collect_timing(ShardModel *m, double *t_ms, int64_t *t_launch, double *t_work) {
  float ms = 0.f;
  ck(m->ctx, hipEventElapsedTime(&ms, m->ev_asm[0], m->ev_asm[1]), "elapsed");
  t_ms[1] += ms;
  t_launch[1] += 1;
  ck(m->ctx, hipEventElapsedTime(&ms, m->ev_grad[0], m->ev_grad[1]), "elapsed");
  t_ms[2] += ms;
  t_launch[2] += 1;
  for (int j = 0; j + 1 < m->upd_used; j += 2) {
    ck(m->ctx, hipEventElapsedTime(&ms, m->ev_upd[(size_t)j], m->ev_upd[(size_t)j + 1]),
       "elapsed");
    t_ms[0] += ms;
    t_launch[0] += 1;
    t_work[0] += m->upd_flops[(size_t)(j / 2)];
  }
  // pair kernels: local rank 0's share of the algorithmic flops
  const RankState &R = *m->ranks[0];
  const double pairs = (double)(R.ngrad - R.ndiag) * AT * AT + (double)R.ndiag * AT * (AT + 1) / 2;
  const double B = m->s.B, p = m->s.p;
  t_work[1] += pairs * B * (3 * p + 3);
  t_work[2] += pairs * (4 * B * p + 2 * p) + (m->s.kind == ACE_KERNEL_MATERN32 ? pairs * B * p : 0);
}

// Collective OR of a per-rank flag (the interrupt poll of ace_model_para_update):
// with RCCL every rank must take the same branch, or the ranks that stop
// leave the others blocked in the next sweep's collectives.  Simulated
// groups share the process's poll, so the local value is already common.
int shard_any(ShardModel *m, int local) {
  if (m->sim || m->proxy || (m->G == 1 && !m->live())) return local;
  ace_ctx *ctx = m->ctx;
  hipStream_t st = ctx->stream;
  ++m->calls[ACE_COMM_ALLREDUCE];
  if (m->host) {
    double v = local ? 1.0 : 0.0;
    hck(ctx, m->ops.allreduce(m->ops.user, &v, 1, 1), "allreduce (interrupt vote)");
    return v != 0.0;
  }
  alloc(ctx, m->vote, sizeof(double), "alloc vote");
  double v = local ? 1.0 : 0.0;
  ck(ctx, hipMemcpyAsync(m->vote.p, &v, sizeof(double), hipMemcpyHostToDevice, st), "vote up");
  nck(ctx, rccl().AllReduce(m->vote.p, m->vote.p, 1, ncclDouble, ncclMax, m->comm, st),
      "ncclAllReduce (interrupt vote)");
  ck(ctx, hipMemcpyAsync(&v, m->vote.p, sizeof(double), hipMemcpyDeviceToHost, st), "vote down");
  sync(ctx);
  return v != 0.0;
}

// ---- access for the resident-inverse products (ace_predict.cpp) --------------
int shard_nlocal(const ShardModel *m) { return (int)m->ranks.size(); }
PairSide shard_train_side(const ShardModel *m) { return m->ranks[0]->side.view(m->n); }
const double *shard_train_y(const ShardModel *m) { return m->ranks[0]->y.d(); }
const double *shard_A0(const ShardModel *m, int j) { return m->ranks[(size_t)j]->A[0].d(); }
int shard_rank_of(const ShardModel *m, int j) { return m->ranks[(size_t)j]->r; }

// Sum over ranks of `count` doubles (in place, device).  Simulated groups
// sum their local partials themselves, so only RCCL has work to do.
void shard_allreduce_sum(ShardModel *m, double *buf, int64_t count) {
  if (m->sim || m->proxy || (m->G == 1 && !m->live()) || count <= 0) return;
  ++m->calls[ACE_COMM_ALLREDUCE];
  if (m->host) {
    host_allreduce(m->ctx, m->ops, m->stage, buf, (size_t)count, 0, m->ctx->stream);
    return;
  }
  nck(m->ctx, rccl().AllReduce(buf, buf, (size_t)count, ncclDouble, ncclSum, m->comm,
                               m->ctx->stream),
      "ncclAllReduce");
}

int shard_world(const ShardModel *m) { return m->G; }
void shard_comm_calls(const ShardModel *m, int64_t *counts) {
  for (int j = 0; j < ACE_COMM_KINDS; ++j) counts[j] = m->calls[j];
}
int shard_rank(const ShardModel *m) { return m->rank; }
