// probe_trans.hip -- accuracy of the fp64 hardware reciprocal / rsqrt
// (v_rcp_f64, v_rsq_f64) and of one / two Newton steps after them, in ulps
// against the correctly rounded host results, over [1, 4) x 2^k.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_trans tools/probe_trans.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_trans(const double *x, double *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  double q = __builtin_amdgcn_rcp(v);
  out[6 * i + 0] = q;
  double e = fma(-v, q, 1.0);
  const double q1 = fma(q, e, q);
  out[6 * i + 1] = q1;
  e = fma(-v, q1, 1.0);
  out[6 * i + 2] = fma(q1, e, q1);
  const double y = __builtin_amdgcn_rsq(v);
  out[6 * i + 3] = y;
  // sqrt from rsq: s = v y, one Goldschmidt step, one / two corrections
  double s = v * y, h = 0.5 * y;
  const double g = fma(-h, s, 0.5);
  s = fma(s, g, s);
  h = fma(h, g, h);
  double d = fma(-s, s, v);
  const double s1 = fma(d, h, s);
  out[6 * i + 4] = s1;
  d = fma(-s1, s1, v);
  out[6 * i + 5] = fma(d, h, s1);
}

static double ulps(double a, double b) {
  if (a == b) return 0.0;
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  return std::fabs((double)(ia - ib));
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n);
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;  // [0,1)
    x[i] = std::ldexp(1.0 + 3.0 * u, (int)(s % 41) - 20);
  }
  double *dx, *dout;
  (void)hipMalloc(&dx, n * 8);
  (void)hipMalloc(&dout, 6 * (size_t)n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_trans, dim3(n / 256), dim3(256), 0, 0, dx, dout, n);
  std::vector<double> o(6 * (size_t)n);
  (void)hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
  double m[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < n; ++i) {
    const double r = 1.0 / x[i], q = std::sqrt(x[i]), rs = 1.0 / std::sqrt(x[i]);
    m[0] = std::fmax(m[0], ulps(o[6 * i + 0], r));
    m[1] = std::fmax(m[1], ulps(o[6 * i + 1], r));
    m[2] = std::fmax(m[2], ulps(o[6 * i + 2], r));
    m[3] = std::fmax(m[3], ulps(o[6 * i + 3], rs));
    m[4] = std::fmax(m[4], ulps(o[6 * i + 4], q));
    m[5] = std::fmax(m[5], ulps(o[6 * i + 5], q));
  }
  printf("max ulp over %d inputs: rcp %.0f, rcp+1NR %.0f, rcp+2NR %.0f | rsq %.0f, "
         "sqrt(rsq+GS+1) %.0f, sqrt(rsq+GS+2) %.0f\n",
         n, m[0], m[1], m[2], m[3], m[4], m[5]);
  return 0;
}
