// probe_cumask.hip -- how hipExtStreamCreateWithCUMask bits map to CUs on this
// box: for a stream mask it reports which (XCC, SE, CU) slots workgroups ran on
// and the throughput of an fp64 FMA kernel, so a chain stream can be given a
// few CUs the bulk stream never uses.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_cumask tools/probe_cumask.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <cstdio>
#include <set>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

// hwreg(HW_REG_HW_ID) = 4 and hwreg(HW_REG_XCC_ID) = 20, all 32 bits
__global__ void k_where(unsigned *out, int iters, double *sink) {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  double a = 1.0 + threadIdx.x * 1e-9, c[4] = {0.1, 0.2, 0.3, 0.4};
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = fma(c[j], a, 1e-7);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
  }
  if (c[0] + c[1] + c[2] + c[3] == 12345.0) sink[0] = 1.0;
}

static int run(hipStream_t s, const char *name, int nblk, int iters, unsigned *d, double *sink) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_where, dim3(nblk), dim3(256), 0, s, d, iters, sink);  // warm
  CK(hipEventRecord(e0, s));
  hipLaunchKernelGGL(k_where, dim3(nblk), dim3(256), 0, s, d, iters, sink);
  CK(hipEventRecord(e1, s));
  // bounded wait: a mask that selects no usable CU would never drain
  for (int t = 0; hipEventQuery(e1) == hipErrorNotReady; ++t) {
    if (t > 3000) {
      printf("%-28s TIMEOUT (no CU of this mask picks up work)\n", name);
      fflush(stdout);
      return 2;
    }
    usleep(1000);
  }
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned> h(2 * nblk);
  CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
  std::set<unsigned> cus;
  std::set<unsigned> xccs;
  for (int b = 0; b < nblk; ++b) {
    const unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
    const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
    cus.insert((xcc << 8) | (se << 5) | (sh << 4) | cu);
    xccs.insert(xcc);
  }
  printf("%-28s %8.3f ms  distinct CU slots %3zu  XCCs %zu :", name, ms, cus.size(), xccs.size());
  int shown = 0;
  for (unsigned v : cus) {
    if (shown++ < 12) printf(" x%u.se%u.sh%u.cu%u", v >> 8, (v >> 5) & 7, (v >> 4) & 1, v & 15);
  }
  printf("\n");
  return 0;
}

int main() {
  setvbuf(stdout, nullptr, _IONBF, 0);
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  printf("multiProcessorCount %d\n", p.multiProcessorCount);
  const int words = (p.multiProcessorCount + 31) / 32;
  hipStream_t s0;
  CK(hipStreamCreate(&s0));
  std::vector<uint32_t> m(words + 2, 0);
  CK(hipExtStreamGetCUMask(s0, (uint32_t)m.size(), m.data()));
  printf("default mask:");
  for (uint32_t w : m) printf(" %08x", w);
  printf("\n");
  unsigned *d;
  double *sink;
  CK(hipMalloc(&d, 2 * 4 * 8192));
  CK(hipMalloc(&sink, 8));
  const int nblk = 4096, iters = 20000;
  if (run(s0, "default stream", nblk, iters, d, sink)) return 1;
  for (int R : {4, 8, 16}) {
    // only bits 0..R-1
    std::vector<uint32_t> only(words, 0), rest(words, 0);
    for (int i = 0; i < p.multiProcessorCount; ++i) {
      if (i < R) only[i / 32] |= 1u << (i % 32);
      else rest[i / 32] |= 1u << (i % 32);
    }
    hipStream_t a, b;
    CK(hipExtStreamCreateWithCUMask(&a, p.multiProcessorCount, only.data()));
    CK(hipExtStreamCreateWithCUMask(&b, p.multiProcessorCount, rest.data()));
    char nm[64];
    snprintf(nm, sizeof nm, "bits [0,%d)", R);
    if (run(a, nm, 64, iters / 10, d, sink)) return 1;
    snprintf(nm, sizeof nm, "bits [%d,%d)", R, p.multiProcessorCount);
    if (run(b, nm, nblk, iters, d, sink)) return 1;
    // strided: bit i*32 for i < R (one per 32-bit word)
    std::vector<uint32_t> sonly(words, 0), srest(words, 0);
    std::set<int> pick;
    for (int i = 0; i < R; ++i) pick.insert((i * 32 + (i / words)) % p.multiProcessorCount);
    for (int i = 0; i < p.multiProcessorCount; ++i) {
      if (pick.count(i)) sonly[i / 32] |= 1u << (i % 32);
      else srest[i / 32] |= 1u << (i % 32);
    }
    hipStream_t c, e;
    CK(hipExtStreamCreateWithCUMask(&c, p.multiProcessorCount, sonly.data()));
    CK(hipExtStreamCreateWithCUMask(&e, p.multiProcessorCount, srest.data()));
    snprintf(nm, sizeof nm, "strided %d bits", R);
    if (run(c, nm, 64, iters / 10, d, sink)) return 1;
    snprintf(nm, sizeof nm, "all but strided %d", R);
    if (run(e, nm, nblk, iters, d, sink)) return 1;
    CK(hipStreamDestroy(a));
    CK(hipStreamDestroy(b));
    CK(hipStreamDestroy(c));
    CK(hipStreamDestroy(e));
  }
  return 0;
}
