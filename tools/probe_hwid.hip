// Which hardware IDs identify a CU on gfx950: one 64-thread block per
// launch slot (4 per CU), each records HW_REG_XCC_ID and HW_REG_HW_ID; the
// host decodes the gfx9 HW_ID fields (CU_ID [11:8], SH_ID [12], SE_ID
// [15:13]) and counts distinct (XCC, SE, SH, CU) tuples (expect one per CU).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_ids(unsigned *out) {
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc;
    __builtin_amdgcn_s_sleep(100);
  }
}

int main() {
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int nb = 4 * p.multiProcessorCount;
  unsigned *d;
  (void)hipMalloc(&d, 2 * nb * sizeof(unsigned));
  // 40 KB of LDS each: at most 4 blocks per CU, so the 4 x CUs blocks cover every CU
  hipLaunchKernelGGL(k_ids, dim3(nb), dim3(64), 40 * 1024, 0, d);
  std::vector<unsigned> h(2 * nb);
  (void)hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
  std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cus;
  std::set<unsigned> se, sh, cu, xc;
  for (int b = 0; b < nb; ++b) {
    const unsigned hw = h[2 * b], x = h[2 * b + 1] & 0xf;
    const unsigned c = (hw >> 8) & 0xf, s = (hw >> 12) & 1, e = (hw >> 13) & 7;
    cus.insert({x, e, s, c});
    se.insert(e); sh.insert(s); cu.insert(c); xc.insert(x);
    if (b < 16) printf("block %d: HW_ID 0x%08x XCC_ID 0x%x -> xcc %u se %u sh %u cu %u\n", b, hw, h[2 * b + 1], x, e, s, c);
  }
  printf("CUs reported %d; distinct (xcc, se, sh, cu) %zu; xcc values %zu, se %zu, sh %zu, cu_id %zu\n",
         p.multiProcessorCount, cus.size(), xc.size(), se.size(), sh.size(), cu.size());
  int n0 = 0;
  for (auto &t : cus) if (std::get<1>(t) == 0 && std::get<2>(t) == 0 && std::get<3>(t) == 0) ++n0;
  printf("CUs with se = sh = cu_id = 0: %d\n", n0);
  return 0;
}
