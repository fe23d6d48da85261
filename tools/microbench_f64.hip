// microbench_f64.hip -- measured fp64 peaks on gfx950 for the roofline:
//   * v_mfma_f64_16x16x4_f64 issue rate (8 independent accumulators per wave)
//   * v_fma_f64 VALU rate (8 independent chains per lane)
//   * HBM stream copy (fp64, 16 B per lane)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench_f64 tools/microbench_f64.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ __launch_bounds__(256) void k_mfma(double *out, int iters, double seed) {
  d4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = d4{seed * j, 0.0, 1.0, seed};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_valu(double *out, int iters, double seed) {
  double c[8];
  for (int j = 0; j < 8; ++j) c[j] = seed * j;
  const double a = 1.0 - 1e-9 * threadIdx.x, b = 1e-7 * seed;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(c[j], a, b);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_copy(const double2 *__restrict__ in,
                                              double2 *__restrict__ out, size_t n2) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 4000;
  double *out;
  CK(hipMalloc(&out, sizeof(double) * blocks * threads));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  // warm
  hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(threads), 0, 0, out, 100, 1.0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(threads), 0, 0, out, iters, 1.0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double mfma_flops = (double)blocks * (threads / 64) * iters * 8 * 2048.0;
  const double mfma_tf = mfma_flops / (ms * 1e-3) / 1e12;
  hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(threads), 0, 0, out, 100, 1.0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(threads), 0, 0, out, iters * 4, 1.0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms2;
  CK(hipEventElapsedTime(&ms2, e0, e1));
  const double valu_flops = (double)blocks * threads * (iters * 4.0) * 8 * 2.0;
  const double valu_tf = valu_flops / (ms2 * 1e-3) / 1e12;
  // HBM copy, 4 GiB each way
  const size_t bytes = (size_t)4 << 30;
  double2 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  hipLaunchKernelGGL(k_copy, dim3(256 * 16), dim3(256), 0, 0, a, b, bytes / 16);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(k_copy, dim3(256 * 16), dim3(256), 0, 0, a, b, bytes / 16);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms3;
  CK(hipEventElapsedTime(&ms3, e0, e1));
  const double gbs = 5.0 * 2.0 * bytes / (ms3 * 1e-3) / 1e9;
  printf("{\"mfma_f64_16x16x4_tflops\": %.2f, \"valu_fma_f64_tflops\": %.2f, "
         "\"hbm_copy_gbs\": %.1f, \"mfma_ms\": %.3f, \"valu_ms\": %.3f}\n",
         mfma_tf, valu_tf, gbs, ms, ms2);
  return 0;
}
