// ace_wgtime.h -- ACE_DIAG_WGTIME (diagnostic builds only, tools/wg_timeline.py):
// per workgroup of the instrumented kernels, the wall clock (100 MHz) at
// entry, at up to four marks of wave 0, and per wave at exit, the CU
// (HW_REG_HW_ID / XCC_ID) and the launch's grid, into a device record array
// of the including translation unit, read back by its extern "C"
// ace_diag_wgtime* entry.  Instrumented workgroups start with one extra
// barrier.  Compiles to nothing without -DACE_DIAG_WGTIME.
#pragma once
#include <algorithm>
#include <hip/hip_runtime.h>

namespace ace {
#ifdef ACE_DIAG_WGTIME
constexpr int WGT_REC = 16, WGT_CAP = 1 << 18;
static __device__ unsigned long long d_wgt_rec[(size_t)WGT_CAP * WGT_REC];
static __device__ unsigned d_wgt_cnt;
struct WgTime {
  unsigned slot = ~0u;
  __device__ WgTime(int kid, unsigned *sh, bool on) {
    if (!on) return;
    const unsigned long long t0 = wall_clock64();
    if (threadIdx.x == 0) {
      const unsigned sl = atomicAdd(&d_wgt_cnt, 1u);
      *sh = sl;
      if (sl < WGT_CAP) {
        unsigned long long *r = d_wgt_rec + (size_t)sl * WGT_REC;
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 15;
        r[0] = (unsigned long long)kid | ((unsigned long long)blockIdx.x << 8) |
               ((unsigned long long)gridDim.x << 36);
        r[1] = (unsigned long long)hw | ((unsigned long long)xcc << 32) |
               ((unsigned long long)(blockDim.x >> 6) << 40);
        r[2] = t0;
        r[3] = (unsigned long long)blockIdx.y | ((unsigned long long)gridDim.y << 32);
        for (int k = 4; k < WGT_REC; ++k) r[k] = 0;  // no stale exits / marks
      }
    }
    __syncthreads();
    slot = *sh;
  }
  __device__ void mark(int i) const {  // intermediate clock of wave 0 (records 12..15)
    if (slot < WGT_CAP && threadIdx.x == 0) d_wgt_rec[(size_t)slot * WGT_REC + 12 + i] = wall_clock64();
  }
  __device__ ~WgTime() {
    if (slot < WGT_CAP && (threadIdx.x & 63) == 0)
      d_wgt_rec[(size_t)slot * WGT_REC + 4 + (threadIdx.x >> 6)] = wall_clock64();
  }
};
#define ACE_WGT(kid, on)                 \
  __shared__ unsigned wgt_slot_sh_;      \
  WgTime wgt_(kid, &wgt_slot_sh_, (on))
#define ACE_WGT_MARK(i) wgt_.mark(i)

// copies up to cap records (16 x u64 each) to dst; returns how many the
// device wrote since the last reset (reset != 0 zeroes the counter after the
// copy).  Device-synchronous.
static inline long long wgt_read(void *dst, long long cap, int reset) {
  unsigned cnt = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(d_wgt_cnt), sizeof(cnt)) != hipSuccess) return -1;
  const long long n = std::min<long long>(std::min<long long>(cnt, WGT_CAP), cap);
  if (dst && n > 0 &&
      hipMemcpyFromSymbol(dst, HIP_SYMBOL(d_wgt_rec), (size_t)n * WGT_REC * 8) != hipSuccess)
    return -1;
  if (reset) {
    const unsigned z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(d_wgt_cnt), &z, sizeof(z)) != hipSuccess) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  return (long long)cnt;
}
#else
#define ACE_WGT(kid, on)
#define ACE_WGT_MARK(i)
#endif
}  // namespace ace
