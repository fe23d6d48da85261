// ace_train.hip -- the per-iteration host tail of ace.train on the device, so
// that the training loop (R/main_ace.R:213-235) enqueues iteration after
// iteration without a host round trip.
//
//   k_make_tab   : the theta tables of make_tab (ace_common.h) from the
//                  device theta, plus exp(theta[0]) for the diagonal;
//   k_train_step : para_update's compose_grad + stats (ace_api.cpp), the
//                  norm clip (src/utilities_cpp.cpp:121-129, Q5), the
//                  optimizer (src/optimizer_cpp.cpp:8-63, Q8), the mu
//                  overwrite (R/kernel_SE_R6.R:45,58) and the convergence test
//                  (R/main_ace.R:221-226), one workgroup.
#include "../../include/ace_hip.h"
#include "ace_internal.h"

namespace ace {

__global__ void k_make_tab(const double *__restrict__ th, int B, int p, int PM,
                           double *__restrict__ tab) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int nk = B * PM;
  if (e < 2 * nk) {
    const int gi = e >= nk;  // 0: kernel weights (Q1 index), 1: gradient weights
    const int q = e - gi * nk;
    const int b = q / PM, i = q - b * PM;
    double v = 0.0;
    if (i < p) v = exp(-th[gi ? 2 + B + b + B * i : 1 + b + B * (i + 1)]);
    tab[e] = v;
  } else if (e < 2 * nk + B) {
    tab[e] = th[2 + (e - 2 * nk)];
  } else if (e == 2 * nk + B) {
    tab[e] = exp(th[0]);
  }
}

hipError_t launch_make_tab(const double *theta, int B, int p, int PM, double *tab,
                           hipStream_t st) {
  const int total = 2 * B * PM + B + 1;
  hipLaunchKernelGGL(k_make_tab, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, theta,
                     B, p, PM, tab);
  return hipGetLastError();
}

namespace {

__device__ __forceinline__ double wsum64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// block sum of 1024 threads, every thread gets the result
__device__ __forceinline__ double bsum(double v, double *sh) {
  v = wsum64(v);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) sh[wv] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int q = 0; q < 16; ++q) r += sh[q];
  __syncthreads();
  return r;
}

}  // namespace

__global__ __launch_bounds__(1024) void k_train_step(TrainCfg c, int it,
                                                     const double *__restrict__ gsum,
                                                     const double *__restrict__ sums,
                                                     const double *__restrict__ scal,
                                                     const int *__restrict__ flag,
                                                     double *__restrict__ st,
                                                     double *__restrict__ hist,
                                                     int *__restrict__ ctl) {
  __shared__ double sh[16];
  if (ctl[1] != 0) return;  // stopped at an earlier iteration: this one is discarded
  const int P = c.P, B = c.B, PM = c.PM, tid = threadIdx.x;
  double *th = st, *m1 = st + P, *m2 = st + 2 * P, *g = st + 3 * P, *prev = st + 4 * P;
  // the theta this iteration's evaluation ran at: the host re-runs it into
  // the resident inverse when later, discarded iterations overwrote it
  // (Q6: predict uses invKmatn of the last para_update, R/kernel_SE_R6.R:37)
  for (int j = tid; j < P; j += 1024) prev[j] = th[j];
  __syncthreads();
  const double kNaN = __builtin_nan("");
  const double mu = scal[3];
  const bool bad = *flag != 0;  // not positive definite: non-finite outputs
  const bool se = c.kind == ACE_KERNEL_SE;
  // compose_grad (ace_common.h); theta[1] <- mu_solution at iter 1 happens
  // before it in para_update but compose_grad does not read theta[1]
  for (int j = tid; j < P; j += 1024) {
    double v;
    if (j == 0) {
      v = -0.5 * gsum[B * (PM + 1)] * exp(th[0]);
    } else if (j == 1) {
      v = se ? sums[2] : 0.0;
    } else if (j < 2 + B) {
      v = -0.5 * gsum[(j - 2) * (PM + 1) + PM];
    } else {
      const int q = j - 2 - B, b = q % B, i = q / B;
      const double sm = gsum[b * (PM + 1) + i];
      v = se ? -0.5 * (sm * exp(-th[j])) : -0.25 * 9 * sm * exp(-th[j]);
    }
    g[j] = bad ? kNaN : v;
  }
  double s0 = c.std_y * sqrt(sums[0]) / sqrt((double)c.n);
  double s1 = -0.5 * ((double)c.n * log(2.0 * M_PI) + sums[3] + sums[1]);
  if (bad) s0 = s1 = kNaN;
  if (tid == 0) {
    hist[2 * it] = s0;
    hist[2 * it + 1] = s1;
    if (it == 1) th[1] = mu;  // mean_solution before the gradient (R/kernel_SE_R6.R:45)
  }
  __syncthreads();
  // Optim$update: norm clip, then the finite test and the step
  double ss = 0.0, nf = 0.0;
  for (int j = tid; j < P; j += 1024) {
    ss += g[j] * g[j];
    nf += isfinite(g[j]) ? 0.0 : 1.0;
  }
  ss = bsum(ss, sh);
  nf = bsum(nf, sh);
  const double L2 = sqrt(ss);
  const bool clip = c.clip && (L2 > c.clip_at) && isfinite(L2) && (L2 != 0);
  if (nf > 0.0) {  // the optimizer classes' stop(): theta stays as it was
    if (tid == 0) {
      ctl[0] = it;
      ctl[1] = 2;
    }
    return;
  }
  const double b1 = c.beta1, b2 = c.beta2, eps = 1e-8;
  const double c1 = 1 - pow(b1, (double)it), c2 = 1 - pow(b2, (double)it);
  for (int j = tid; j < P; j += 1024) {
    const double gj = clip ? g[j] / L2 : g[j];
    if (c.optimizer == ACE_OPT_NESTEROV) {
      m1[j] = c.momentum * m1[j] + c.lr * gj;
      th[j] = th[j] + m1[j];
    } else if (c.optimizer == ACE_OPT_NADAM) {
      m1[j] = b1 * m1[j] + (1 - b1) * gj;
      m2[j] = b2 * m2[j] + (1 - b2) * (gj * gj);
      th[j] = th[j] + c.lr * ((b1 * m1[j] + (1 - b1) * gj) / c1) / (sqrt(m2[j] / c2) + eps);
    } else {
      m1[j] = (b1 * m1[j]) + (1 - b1) * gj;
      m2[j] = b2 * m2[j] + (1 - b2) * (gj * gj);
      th[j] = th[j] + c.lr * (m1[j] / c1) / (sqrt(m2[j] / c2) + eps);
    }
  }
  __syncthreads();
  if (tid == 0) {
    th[1] = mu;  // private$mean_solution(y) with this iteration's inverse
    const double change = fabs(s1 - hist[2 * (it - 1) + 1]);
    ctl[0] = it;
    if (change < c.tol && it > 3) ctl[1] = 1;
  }
}

hipError_t launch_train_step(const TrainCfg &c, int it, const double *gsum, const double *sums,
                             const double *scal, const int *flag, double *st, double *hist,
                             int *ctl, hipStream_t stream) {
  hipLaunchKernelGGL(k_train_step, dim3(1), dim3(1024), 0, stream, c, it, gsum, sums, scal, flag,
                     st, hist, ctl);
  return hipGetLastError();
}

}  // namespace ace
