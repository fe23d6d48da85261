// bench_update.hip -- standalone timing of the sweep update kernel's GEMM
// tiles (the dominant kernel of one eval) and diagnostic variants,
// interleaved in one process (cdna_hip_programming.md §5.4 rule 24).
// Random operands, one middle sweep step, no side-stream contention.
//   V0 library structure (C tile loaded into the accumulators first)
//   V1 no C load (acc = 0)            -- cost of the C-tile load
//   V2 no C load, no C store          -- the staged MFMA loop alone
//   V3 acc = 0, C loaded + added at the end
//   V4 V0 with s_setprio raised around the MFMA block
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bench_update tools/bench_update.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef KDEPTH
#define KDEPTH 256
#endif
constexpr int NB = KDEPTH, UT = 128, AUG = 128, BK = 16, LDL = 144, NCH = NB / BK;
typedef double d4 __attribute__((ext_vector_type(4)));

template <int V>
__global__ __launch_bounds__(512, 2) void k_upd(double *__restrict__ A, int64_t ld,
                                                const double *__restrict__ W,
                                                const double *__restrict__ Pn, int64_t ldp) {
  __shared__ __attribute__((aligned(16))) double sW[2][BK][LDL];
  __shared__ __attribute__((aligned(16))) double sP[2][BK][LDL];
  const int t = blockIdx.x;
  int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  const int I = i, J = t - i * (i + 1) / 2;
  const int64_t R0 = (int64_t)I * UT, C0 = (int64_t)J * UT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wr = wv & 1, wc = wv >> 1;
  const int lr = lane & 15, lk = lane >> 4;
  d4 acc[2][4];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[ci][ri][j] = (V == 0 || V == 4) ? A[r + (c + 4 * j) * ld] : 0.0;
    }
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
    if (V == 4) __builtin_amdgcn_s_setprio(2);
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
    if (V == 4) __builtin_amdgcn_s_setprio(0);
    if (ch + 1 < NCH) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        *reinterpret_cast<double2 *>(&sW[cur ^ 1][sk][sm + 2 * e]) = rw[e];
        *reinterpret_cast<double2 *>(&sP[cur ^ 1][sk][sm + 2 * e]) = rp[e];
      }
    }
    __syncthreads();
  }
  if (V == 2) {
    // keep the result live without a full store
    double s = 0;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int ri = 0; ri < 4; ++ri) s += acc[ci][ri][0] + acc[ci][ri][1] + acc[ci][ri][2] + acc[ci][ri][3];
    if (s == 12345.678) A[0] = s;
    return;
  }
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int ri = 0; ri < 4; ++ri) {
      const int64_t r = R0 + 64 * wr + 16 * ri + lr;
      const int64_t c = C0 + 32 * wc + 16 * ci + lk;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double v = acc[ci][ri][j];
        if (V == 3) v += A[r + (c + 4 * j) * ld];
        A[r + (c + 4 * j) * ld] = v;
      }
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
  const unsigned ntiles = nT * (nT + 1) / 2;
  const double flops = (double)ntiles * 2.0 * UT * UT * NB;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 10;
  const char *names[] = {"V0 library", "V1 no C load", "V2 no C load/store", "V3 C added at end",
                         "V4 setprio"};
  for (int round = 0; round < 3; ++round) {
    for (int v = 0; v < 5; ++v) {
      (void)hipEventRecord(e0);
      for (int r = 0; r < reps; ++r) {
        switch (v) {
          case 0: hipLaunchKernelGGL(k_upd<0>, dim3(ntiles), dim3(512), 0, 0, A, ld, W, P, ld); break;
          case 1: hipLaunchKernelGGL(k_upd<1>, dim3(ntiles), dim3(512), 0, 0, A, ld, W, P, ld); break;
          case 2: hipLaunchKernelGGL(k_upd<2>, dim3(ntiles), dim3(512), 0, 0, A, ld, W, P, ld); break;
          case 3: hipLaunchKernelGGL(k_upd<3>, dim3(ntiles), dim3(512), 0, 0, A, ld, W, P, ld); break;
          case 4: hipLaunchKernelGGL(k_upd<4>, dim3(ntiles), dim3(512), 0, 0, A, ld, W, P, ld); break;
        }
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("{\"variant\": \"%s\", \"round\": %d, \"ms_per_launch\": %.4f, \"tflops\": %.2f}\n",
             names[v], round, ms / reps, flops / (ms / reps * 1e-3) / 1e12);
    }
  }
  return 0;
}
