// bench_panel.hip -- uncontended timing of one step's panel chain
// (k_gather, 4 x (k_pivot, k_panel)) at the C2 size.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bench_panel tools/bench_panel.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../additivecausalexpansion_amd/csrc/ace_sweep.hip"

using namespace ace;

__global__ void k_spd(double *A, int64_t ld, int64_t n) {
  // A = 0.01 * hash + n * I (lower triangle used)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i % n, c = i / n;
    unsigned x = (unsigned)((r < c ? r * 131071 + c : c * 131071 + r) * 2654435761u);
    x ^= x >> 15;
    A[r + c * ld] = 0.01 * ((double)(x & 0xffff) / 65536.0 - 0.5) + (r == c ? 4.0 : 0.0);
  }
}

int main() {
  const int64_t npad = 16384, naug = npad + AUG, ld = naug;
  double *A, *P[2], *W[2], *SW, *S[2], *piv;
  int *flag;
  (void)hipMalloc(&A, sizeof(double) * naug * naug);
  for (int i = 0; i < 2; ++i) {
    (void)hipMalloc(&P[i], sizeof(double) * naug * NB);
    (void)hipMalloc(&W[i], sizeof(double) * naug * NB);
    (void)hipMalloc(&S[i], sizeof(double) * SUB * NB);
  }
  (void)hipMalloc(&SW, sizeof(double) * SUB * SUB);
  (void)hipMalloc(&piv, sizeof(double) * npad);
  (void)hipMalloc(&flag, 16);
  hipLaunchKernelGGL(k_spd, dim3(8192), dim3(256), 0, 0, A, ld, naug);
  (void)hipDeviceSynchronize();
  hipEvent_t ev[12];
  for (auto &e : ev) (void)hipEventCreate(&e);
  const int64_t k0 = 8192;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(ev[0]);
    hipLaunchKernelGGL(k_gather, dim3((unsigned)(naug / 64), NB / 64), dim3(256), 0, 0, A, ld, k0,
                       P[0], W[0], ld, S[0]);
    (void)hipEventRecord(ev[1]);
    for (int s = 0; s < NB / SUB; ++s) {
      hipLaunchKernelGGL(k_pivot, dim3(1), dim3(256), 0, 0, S[s & 1], s, SW, piv,
                         k0 + (int64_t)s * SUB, flag);
      (void)hipEventRecord(ev[2 + 2 * s]);
      hipLaunchKernelGGL(k_panel, dim3(NB / SUB), dim3(256), 0, 0, W[0], ld, k0, s,
                         SW, S[s & 1], S[(s + 1) & 1], k0);
      (void)hipEventRecord(ev[3 + 2 * s]);
    }
    hipLaunchKernelGGL(k_panel_gemm, dim3((unsigned)(naug / SUB)), dim3(512), 0, 0, W[0], P[0], ld, k0);
    (void)hipEventRecord(ev[10]);
    (void)hipEventSynchronize(ev[10]);
    float g, t;
    (void)hipEventElapsedTime(&g, ev[0], ev[1]);
    (void)hipEventElapsedTime(&t, ev[0], ev[9]);
    printf("{\"rep\": %d, \"gather_us\": %.1f", rep, g * 1e3);
    for (int s = 0; s < 4; ++s) {
      float a, b;
      (void)hipEventElapsedTime(&a, ev[s == 0 ? 1 : 1 + 2 * s], ev[2 + 2 * s]);
      (void)hipEventElapsedTime(&b, ev[2 + 2 * s], ev[3 + 2 * s]);
      printf(", \"pivot%d_us\": %.1f, \"panel%d_us\": %.1f", s, a * 1e3, s, b * 1e3);
    }
    float gm;
    (void)hipEventElapsedTime(&gm, ev[9], ev[10]);
    (void)hipEventElapsedTime(&t, ev[0], ev[10]);
    printf(", \"panel_gemm_us\": %.1f, \"chain_us\": %.1f}\n", gm * 1e3, t * 1e3);
  }
  return 0;
}
