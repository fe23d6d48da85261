// microbench_f64_mix.hip -- can v_mfma_f64 and v_fma_f64 overlap on gfx950?
// Times fixed amounts of MFMA and VALU fp64 work issued (a) alone, (b) by the
// same wave interleaved, (c) by different waves of one workgroup.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench_f64_mix tools/microbench_f64_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>  // 0 mfma only, 1 valu only, 2 same-wave mix, 3 split waves (even mfma)
__global__ __launch_bounds__(512) void k_mix(double *out, int iters, double seed) {
  d4 acc[8];
  double c[16];
  for (int j = 0; j < 8; ++j) acc[j] = d4{seed * j, 0.0, 1.0, seed};
  for (int j = 0; j < 16; ++j) c[j] = seed * j;
  const double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  const double fa = 1.0 - 1e-9 * threadIdx.x, fb = 1e-7 * seed;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool do_m = MODE == 0 || MODE == 2 || (MODE == 3 && (wv & 1) == 0);
  const bool do_v = MODE == 1 || MODE == 2 || (MODE == 3 && (wv & 1) == 1);
  const int it_m = (MODE == 3) ? 2 * iters : iters;  // same total work per workgroup
  if (do_m && do_v) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
        c[2 * j] = fma(c[2 * j], fa, fb);
        c[2 * j + 1] = fma(c[2 * j + 1], fa, fb);
      }
    }
  } else if (do_m) {
    for (int it = 0; it < it_m; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
  } else if (do_v) {
    for (int it = 0; it < it_m; ++it) {
#pragma unroll
      for (int j = 0; j < 16; ++j) c[j] = fma(c[j], fa, fb);
    }
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
  for (int j = 0; j < 16; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE>
float run(double *out, int blocks, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_mix<MODE>, dim3(blocks), dim3(512), 0, 0, out, 50, 1.0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_mix<MODE>, dim3(blocks), dim3(512), 0, 0, out, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  const int blocks = 256 * 4, iters = 2000;
  double *out;
  if (hipMalloc(&out, sizeof(double) * blocks * 512) != hipSuccess) return 1;
  const float m = run<0>(out, blocks, iters), v = run<1>(out, blocks, iters);
  const float mix = run<2>(out, blocks, iters), split = run<3>(out, blocks, iters);
  // per workgroup: 8 waves x iters x (8 MFMA = 16384 flop) and 8 waves x 64 lanes x iters x 16 FMA
  const double fm = (double)blocks * 8 * iters * 8 * 2048.0;
  const double fv = (double)blocks * 8 * 64 * iters * 16 * 2.0;
  printf("{\"mfma_only_ms\": %.3f, \"mfma_tflops\": %.2f, \"valu_only_ms\": %.3f, "
         "\"valu_tflops\": %.2f, \"same_wave_mix_ms\": %.3f, \"mix_tflops\": %.2f, "
         "\"split_waves_ms\": %.3f, \"split_tflops\": %.2f}\n",
         m, fm / (m * 1e-3) / 1e12, v, fv / (v * 1e-3) / 1e12, mix,
         (fm + fv) / (mix * 1e-3) / 1e12, split, (fm + fv) / (split * 1e-3) / 1e12);
  return 0;
}
