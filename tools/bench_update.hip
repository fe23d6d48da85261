// bench_update.hip -- standalone timing of the sweep update kernel (the
// dominant kernel of one eval) and candidate variants, interleaved in one
// process (cdna_hip_programming.md §5.4 rule 24).  Random operands.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I additivecausalexpansion_amd/csrc \
//          -o tools/bench_update tools/bench_update.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../additivecausalexpansion_amd/csrc/ace_sweep.hip"

using namespace ace;

// Variant 1: 8 waves per block (wave grid 2 rows x 4 cols of 64x32), so that
// accumulators are 32 doubles per lane and 4 waves fit per SIMD.
__global__ __launch_bounds__(512, 2) void k_update_w8(double *__restrict__ A, int64_t ld,
                                                      const double *__restrict__ W,
                                                      const double *__restrict__ Pn,
                                                      int64_t ldp, int64_t k0, int kx) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  const int J = blockIdx.x, I = blockIdx.y;
  if (J > I) return;
  constexpr int KT = NB / UT;
  if (kx >= 0 && ((I >= kx * KT && I < (kx + 1) * KT) || (J >= kx * KT && J < (kx + 1) * KT)))
    return;
  const int kt0 = (int)(k0 / UT), kt1 = kt0 + KT;
  if ((I >= kt0 && I < kt1) || (J >= kt0 && J < kt1)) return;  // write-back tiles: not timed here
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 64*wr, cols 32*wc
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = A[r + (c + 4 * j) * ld];
    }
  // staging: 512 threads, each 4 doubles of W and 4 of P per chunk
  const int sk = tid >> 5, sm = (tid & 31) * 4;
  const double *gW = W + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = Pn + (C0 + sm) + (int64_t)sk * ldp;
  double2 rw[2], rp[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    rw[e] = *reinterpret_cast<const double2 *>(gW + 2 * e);
    rp[e] = *reinterpret_cast<const double2 *>(gP + 2 * e);
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    *reinterpret_cast<double2 *>(&sW[0][sk][sm + 2 * e]) = rw[e];
    *reinterpret_cast<double2 *>(&sP[0][sk][sm + 2 * e]) = rp[e];
  }
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCH) {
      const int64_t off = (int64_t)(ch + 1) * BK * ldp;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        rw[e] = *reinterpret_cast<const double2 *>(gW + off + 2 * e);
        rp[e] = *reinterpret_cast<const double2 *>(gP + off + 2 * e);
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
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + 2 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + 2 * e]) = rp[e];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) A[r + (c + 4 * j) * ld] = acc[ci][ri][j];
    }
}

// Variant: 1-D grid over a precomputed lower-tile table (order chosen on the host)
__global__ __launch_bounds__(512, 2) void k_update_tab(const int *__restrict__ tiles, double *__restrict__ A, int64_t ld,
                                                      const double *__restrict__ W,
                                                      const double *__restrict__ Pn,
                                                      int64_t ldp, int64_t k0, int kx) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  const int tv = tiles[blockIdx.x];
  const int I = tv >> 16, J = tv & 0xffff;
  constexpr int KT = NB / UT;
  if (kx >= 0 && ((I >= kx * KT && I < (kx + 1) * KT) || (J >= kx * KT && J < (kx + 1) * KT)))
    return;
  const int kt0 = (int)(k0 / UT), kt1 = kt0 + KT;
  if ((I >= kt0 && I < kt1) || (J >= kt0 && J < kt1)) return;  // write-back tiles: not timed here
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;  // rows 64*wr, cols 32*wc
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = A[r + (c + 4 * j) * ld];
    }
  // staging: 512 threads, each 4 doubles of W and 4 of P per chunk
  const int sk = tid >> 5, sm = (tid & 31) * 4;
  const double *gW = W + (R0 + sm) + (int64_t)sk * ldp;
  const double *gP = Pn + (C0 + sm) + (int64_t)sk * ldp;
  double2 rw[2], rp[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    rw[e] = *reinterpret_cast<const double2 *>(gW + 2 * e);
    rp[e] = *reinterpret_cast<const double2 *>(gP + 2 * e);
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    *reinterpret_cast<double2 *>(&sW[0][sk][sm + 2 * e]) = rw[e];
    *reinterpret_cast<double2 *>(&sP[0][sk][sm + 2 * e]) = rp[e];
  }
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const int cur = ch & 1;
    if (ch + 1 < NCH) {
      const int64_t off = (int64_t)(ch + 1) * BK * ldp;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        rw[e] = *reinterpret_cast<const double2 *>(gW + off + 2 * e);
        rp[e] = *reinterpret_cast<const double2 *>(gP + off + 2 * e);
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
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + 2 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + 2 * e]) = rp[e];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) A[r + (c + 4 * j) * ld] = acc[ci][ri][j];
    }
}

__global__ void k_rand(double *p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)(i * 2654435761u) ^ seed;
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    p[i] = (double)(x & 0xffffff) / 16777216.0 - 0.5;
  }
}

int main(int argc, char **argv) {
  const int64_t npad = argc > 1 ? atoll(argv[1]) : 16384;
  const int64_t naug = npad + AUG, ld = naug;
  double *A, *W, *P;
  if (hipMalloc(&A, sizeof(double) * naug * naug) != hipSuccess) return 1;
  if (hipMalloc(&W, sizeof(double) * naug * NB) != hipSuccess) return 1;
  if (hipMalloc(&P, sizeof(double) * naug * NB) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, A, (size_t)(naug * naug), 1u);
  hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, W, (size_t)(naug * NB), 2u);
  hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, P, (size_t)(naug * NB), 3u);
  (void)hipDeviceSynchronize();
  const unsigned nT = (unsigned)(naug / UT);
  const int64_t k0 = (npad / NB / 2) * NB;  // a middle step
  const double flops = (double)update_gemm_tiles(naug, k0, -1, false) * 2.0 * UT * UT * NB;
  // tile tables: (0) row-major lower order, (S) S x S supertiles, each XCD
  // (blockIdx % 8) given a contiguous range of the order
  auto make_table = [&](int S, bool xcd) {
    std::vector<int> order;
    const int nt = (int)nT;
    if (S <= 1) {
      for (int I = 0; I < nt; ++I)
        for (int J = 0; J <= I; ++J) order.push_back((I << 16) | J);
    } else {
      for (int SI = 0; SI * S < nt; ++SI)
        for (int SJ = 0; SJ <= SI; ++SJ)
          for (int i = 0; i < S; ++i)
            for (int j = 0; j < S; ++j) {
              const int I = SI * S + i, J = SJ * S + j;
              if (I < nt && J <= I) order.push_back((I << 16) | J);
            }
    }
    const int N = (int)order.size();
    std::vector<int> tab(N);
    if (!xcd) {
      tab = order;
    } else {
      // block L runs on XCD L % 8, as the (L / 8)-th block of that XCD
      const int per = (N + 7) / 8;
      int L = 0;
      std::vector<int> slot(N, -1);
      // blocks L = 8*q + x  ->  order index x*per + q (skipping past N)
      std::vector<int> out;
      for (int q = 0; q < per; ++q)
        for (int x = 0; x < 8; ++x) {
          const int o = x * per + q;
          if (o < N) out.push_back(order[o]);
        }
      tab = out;
      (void)L;
      (void)slot;
    }
    int *d;
    (void)hipMalloc(&d, sizeof(int) * N);
    (void)hipMemcpy(d, tab.data(), sizeof(int) * N, hipMemcpyHostToDevice);
    return std::make_pair(d, N);
  };
  struct V { const char *name; int *tab; int N; };
  std::vector<V> vars;
  vars.push_back({"k_update(library, 2-D grid)", nullptr, 0});
  {
    auto t = make_table(1, false); vars.push_back({"table row-major", t.first, t.second});
    t = make_table(4, true); vars.push_back({"table S4 xcd", t.first, t.second});
    t = make_table(8, true); vars.push_back({"table S8 xcd", t.first, t.second});
    t = make_table(16, true); vars.push_back({"table S16 xcd", t.first, t.second});
    t = make_table(8, false); vars.push_back({"table S8 no-xcd", t.first, t.second});
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 10;
  for (int round = 0; round < 3; ++round) {
    for (size_t v = 0; v < vars.size(); ++v) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) {
        if (v == 0)
          hipLaunchKernelGGL(k_update<false>, dim3(nT * (nT + 1) / 2), dim3(UTHREADS), 0, 0, A, ld, W, P, ld, k0, -1);
        else
          hipLaunchKernelGGL(k_update_tab, dim3(vars[v].N), dim3(512), 0, 0, vars[v].tab, A, ld, W,
                             P, ld, k0, -1);
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("{\"variant\": \"%s\", \"round\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.2f}\n",
             vars[v].name, round, ms / reps, flops / (ms / reps * 1e-3) / 1e12);
    }
  }
  return 0;
}
