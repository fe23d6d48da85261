// Issue cost of the VALU instructions on the pair kernels' per-pair chains
// (gfx950): each kernel runs 8 independent chains of one instruction per
// lane, four waves per SIMD on every CU (nb = 4096 blocks of 64 threads), and
// reports cycles per instruction per wave from the kernel time (HIP events)
// at the measured clock, plus the rate.  Instructions: fp64 fma / mul / add,
// v_rsq_f64, v_rcp_f64, v_ldexp_f64, v_rndne_f64, v_cvt_i32_f64,
// 32-bit v_add_u32 / v_and_b32, v_cndmask (via a select), v_mov_b32_dpp.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAINS 8
template <int OP>
__global__ void k_op(double *out, int iters) {
  double x[CHAINS];
  int ix[CHAINS];
  for (int j = 0; j < CHAINS; ++j) {
    x[j] = 1.0 + 1e-3 * (threadIdx.x + j);
    ix[j] = threadIdx.x + 7 * j;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < CHAINS; ++j) {
      if (OP == 0) x[j] = fma(x[j], 0.999999, 1e-7);
      if (OP == 1) x[j] = x[j] * 1.0000001;
      if (OP == 2) x[j] = __builtin_amdgcn_rsq(x[j]);
      if (OP == 3) x[j] = __builtin_amdgcn_rcp(x[j]);
      if (OP == 4) x[j] = __builtin_amdgcn_ldexp(x[j], (it & 1) ? 1 : -1);
      if (OP == 5) x[j] = __builtin_rint(x[j]) + 0.25;
      if (OP == 6) ix[j] = (int)x[j] + ix[j];
      if (OP == 7) ix[j] = (ix[j] + 0x1234567) & 0x7ffffff;
      if (OP == 8) ix[j] = __builtin_amdgcn_mov_dpp(ix[j], 0xB1, 0xf, 0xf, false) + 1;
      if (OP == 9) x[j] = (ix[j] & 1) ? x[j] : -x[j];
    }
  }
  double s = 0.0;
  for (int j = 0; j < CHAINS; ++j) s += x[j] + ix[j];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int OP>
void run(const char *name, double *d, int ops_per_iter) {
  const int nb = 4096, iters = 20000;  // 4 waves per SIMD
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k_op<OP>, dim3(nb), dim3(64), 0, 0, d, 100);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k_op<OP>, dim3(nb), dim3(64), 0, 0, d, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  int clk = 0;
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);  // kHz
  // four waves per SIMD: SIMD cycles per wave-instruction = time * clock / (4 * instructions)
  const double inst = 4.0 * iters * CHAINS * ops_per_iter;
  printf("%-14s %.2f cycles per wave-instruction at %.0f MHz (%.3f ms)\n", name,
         ms * 1e-3 * clk * 1e3 / inst, clk / 1e3, ms);
}

int main() {
  double *d;
  (void)hipMalloc(&d, 4096 * 64 * sizeof(double));
  run<0>("v_fma_f64", d, 1);
  run<1>("v_mul_f64", d, 1);
  run<2>("v_rsq_f64", d, 1);
  run<3>("v_rcp_f64", d, 1);
  run<4>("v_ldexp_f64", d, 1);
  run<5>("rndne+add_f64", d, 2);
  run<6>("cvt_i32_f64+add", d, 2);
  run<7>("add_u32+and", d, 2);
  run<8>("mov_dpp+add", d, 2);
  run<9>("and+cndmask x2", d, 4);
  return 0;
}
