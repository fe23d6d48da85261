// Probe of the fp64 MFMA shapes on gfx950 (run on the box):
//  1. the lane layout of v_mfma_f64_4x4x4_4b_f64 (A, B, C/D), from 64
//     one-hot experiments (wave e: A = 1 at lane e only, B[l] = l + 1,
//     so D is B's entries routed through A's one slot);
//  2. issue cost in cycles of v_mfma_f64_4x4x4_4b_f64 against
//     v_mfma_f64_16x16x4f64 (8 independent accumulators per wave, one wave
//     per SIMD on every CU, s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(double *out) {
  const int e = blockIdx.x, l = threadIdx.x;
  const double a = (l == e) ? 1.0 : 0.0;
  const double b = (double)(l + 1);
  double acc = 0.0;
  acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc, 0, 0, 0);
  out[e * 64 + l] = acc;
  // the same with the roles swapped: B one-hot, A encoded
  double acc2 = 0.0;
  acc2 = __builtin_amdgcn_mfma_f64_4x4x4f64((double)(l + 1), a, acc2, 0, 0, 0);
  out[64 * 64 + e * 64 + l] = acc2;
}

template <int SHAPE>
__global__ void k_rate(double *out, long long *cyc, int iters) {
  const int l = threadIdx.x;
  double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
  long long t0 = clock64();
  if (SHAPE == 4) {
    double acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = 0.0;
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[j], 0, 0, 0);
    double s = 0.0;
    for (int j = 0; j < 8; ++j) s += acc[j];
    out[blockIdx.x * 64 + l] = s;
  } else {
    d4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    double s = 0.0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * 64 + l] = s;
  }
  long long t1 = clock64();
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double *d;
  long long *c;
  hipMalloc(&d, 2 * 64 * 64 * sizeof(double) + 4096 * 64 * 8);
  hipMalloc(&c, 4096 * sizeof(long long));
  hipLaunchKernelGGL(k_layout, dim3(64), dim3(64), 0, 0, d);
  std::vector<double> h(2 * 64 * 64);
  hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
  printf("layout_A_onehot\n");
  for (int e = 0; e < 64; ++e) {
    printf("A%d:", e);
    for (int l = 0; l < 64; ++l)
      if (h[e * 64 + l] != 0.0) printf(" %d=%g", l, h[e * 64 + l]);
    printf("\n");
  }
  printf("layout_B_onehot\n");
  for (int e = 0; e < 64; ++e) {
    printf("B%d:", e);
    for (int l = 0; l < 64; ++l)
      if (h[4096 + e * 64 + l] != 0.0) printf(" %d=%g", l, h[4096 + e * 64 + l]);
    printf("\n");
  }
  const int nb = 1024, iters = 4096;  // 4 waves per CU = 1 per SIMD on 256 CUs
  std::vector<long long> hc(nb);
  for (int shape : {4, 16}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (shape == 4) hipLaunchKernelGGL(k_rate<4>, dim3(nb), dim3(64), 0, 0, d, c, iters);
      else hipLaunchKernelGGL(k_rate<16>, dim3(nb), dim3(64), 0, 0, d, c, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(hc.data(), c, nb * 8, hipMemcpyDeviceToHost);
      double avg = 0;
      for (auto v : hc) avg += v;
      avg /= nb;
      const double flops = (shape == 4 ? 512.0 : 2048.0) * 8 * iters * nb;
      printf("shape %d: %.1f cycles per MFMA per wave (clock64), %.3f ms, %.1f TFLOP/s\n", shape,
             avg / (8.0 * iters), ms, flops / (ms * 1e-3) / 1e12);
    }
  }
  return 0;
}
