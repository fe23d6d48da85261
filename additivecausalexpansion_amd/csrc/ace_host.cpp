// ace_host.cpp -- host-only entry points of the C ABI (no GPU, no context):
// the optimizer steps, norm clipping, the natural-cubic-spline basis and the
// data normalisation.  They run once per iteration on P <= 818 doubles or
// once per fit, so they stay on the host.
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/ace_hip.h"

namespace {

bool all_finite(int64_t P, const double *g) {
  for (int64_t j = 0; j < P; ++j)
    if (!std::isfinite(g[j])) return false;
  return true;
}

}  // namespace

extern "C" {

// Nesterov_cpp (src/optimizer_cpp.cpp:8-20)
int ace_nesterov(int64_t P, double learn_rate, double momentum, double *nu, const double *grad,
                 double *para) {
  const bool ok = all_finite(P, grad);
  for (int64_t j = 0; j < P; ++j) {
    nu[j] = momentum * nu[j] + learn_rate * grad[j];
    para[j] = para[j] + nu[j];
  }
  return ok ? 1 : 0;
}

// Nadam_cpp (src/optimizer_cpp.cpp:23-42): the Nesterov term uses the
// already-updated m (Q8).
int ace_nadam(int64_t P, double iter, double learn_rate, double beta1, double beta2, double eps,
              double *m, double *v, const double *grad, double *para) {
  const bool ok = all_finite(P, grad);
  const double c1 = 1 - std::pow(beta1, iter), c2 = 1 - std::pow(beta2, iter);
  for (int64_t j = 0; j < P; ++j) {
    m[j] = beta1 * m[j] + (1 - beta1) * grad[j];
    v[j] = beta2 * v[j] + (1 - beta2) * std::pow(grad[j], 2);
    para[j] = para[j] + learn_rate * ((beta1 * m[j] + (1 - beta1) * grad[j]) / c1) /
                            (std::sqrt(v[j] / c2) + eps);
  }
  return ok ? 1 : 0;
}

// Adam_cpp (src/optimizer_cpp.cpp:45-63)
int ace_adam(int64_t P, double iter, double learn_rate, double beta1, double beta2, double eps,
             double *m, double *v, const double *grad, double *para) {
  const bool ok = all_finite(P, grad);
  const double c1 = 1 - std::pow(beta1, iter), c2 = 1 - std::pow(beta2, iter);
  for (int64_t j = 0; j < P; ++j) {
    m[j] = (beta1 * m[j]) + (1 - beta1) * grad[j];
    v[j] = beta2 * v[j] + (1 - beta2) * std::pow(grad[j], 2);
    para[j] = para[j] + learn_rate * (m[j] / c1) / (std::sqrt(v[j] / c2) + eps);
  }
  return ok ? 1 : 0;
}

// norm_clip_cpp (src/utilities_cpp.cpp:121-129), Q5
void ace_norm_clip(int flag, int64_t P, double *grads, double max_length) {
  if (!flag) return;
  double ss = 0.0;
  for (int64_t j = 0; j < P; ++j) ss += grads[j] * grads[j];
  const double L2 = std::sqrt(ss);
  if ((L2 > max_length) && std::isfinite(L2) && (L2 != 0)) {
    for (int64_t j = 0; j < P; ++j) grads[j] = grads[j] / L2;
  }
}

// generate_ncs_matrix / generate_ncs_derivative_matrix (src/ncs_basis_cpp.cpp:5-58)
static void ncs_columns(int64_t n, const double *x, const std::vector<double> &kn, bool deriv,
                        double *out /* n x (K-1), ld n */) {
  const int64_t K = (int64_t)kn.size();
  std::vector<double> d((size_t)(n * K), 0.0);
  auto f = [&](double xv, double k) {
    const double gt = (xv > k) ? 1.0 : 0.0;
    return deriv ? 3 * gt * std::pow(xv - k, 2) : gt * std::pow(xv - k, 3);
  };
  for (int64_t r = 0; r < n; ++r) d[r + (K - 1) * n] = f(x[r], kn[K - 1]);
  for (int64_t i = 0; i < K - 1; ++i)
    for (int64_t r = 0; r < n; ++r)
      d[r + i * n] = (f(x[r], kn[i]) - d[r + (K - 1) * n]) / (kn[K - 1] - kn[i]);
  for (int64_t r = 0; r < n; ++r) d[r + (K - 1) * n] = 0.0;
  for (int64_t i = 0; i < K - 2; ++i)
    for (int64_t r = 0; r < n; ++r) out[r + i * n] = d[r + i * n] - d[r + (K - 2) * n];
  for (int64_t r = 0; r < n; ++r) out[r + (K - 2) * n] = -d[r + (K - 2) * n];
}

static int ncs_common(int64_t n, const double *x, int64_t nknots, const double *knots,
                      double *design, int64_t *ncols, bool deriv) {
  if (n < 0 || nknots < 2 || !x || !knots || !design) return ACE_ERR_ARG;
  std::vector<double> kn(knots, knots + nknots);
  std::sort(kn.begin(), kn.end());
  kn.erase(std::unique(kn.begin(), kn.end()), kn.end());
  const int64_t K = (int64_t)kn.size();
  if (K < 2) return ACE_ERR_ARG;
  for (int64_t r = 0; r < n; ++r) design[r] = deriv ? 1.0 : x[r];
  ncs_columns(n, x, kn, deriv, design + n);
  if (ncols) *ncols = K;
  return ACE_OK;
}

// ncs_basis (src/ncs_basis_cpp.cpp:61-79)
int ace_ncs_basis(int64_t n, const double *x, int64_t nknots, const double *knots,
                  double *design, int64_t *ncols) {
  return ncs_common(n, x, nknots, knots, design, ncols, false);
}

// ncs_basis_deriv (src/ncs_basis_cpp.cpp:82-99)
int ace_ncs_basis_deriv(int64_t n, const double *x, int64_t nknots, const double *knots,
                        double *design, int64_t *ncols) {
  return ncs_common(n, x, nknots, knots, design, ncols, true);
}

static double median_of(const double *p, int64_t n) {
  std::vector<double> v(p, p + n);
  std::sort(v.begin(), v.end());
  if (n % 2) return v[(size_t)(n / 2)];
  return (v[(size_t)(n / 2 - 1)] + v[(size_t)(n / 2)]) / 2.0;
}

static void unique_minmax(const double *p, int64_t n, int64_t *count, double *mn, double *mx) {
  std::vector<double> v(p, p + n);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  *count = (int64_t)v.size();
  *mn = v.empty() ? 0.0 : v.front();
  *mx = v.empty() ? 0.0 : v.back();
}

// normalize_train (src/utilities_cpp.cpp:13-104).  Quirks kept: binary
// columns store their location/scale in row i (not i+1) of the moments, a
// constant Z column zeroes Z.col(i) with the X-offset index, and the Z
// rescale tests isbinary(i - px - 1) (X's flags).
int ace_normalize_train(int64_t n, int px, int pz, double *y, double *X, double *Z,
                        double *mom) {
  if (n < 2 || px < 0 || pz < 0) return ACE_ERR_ARG;
  const int64_t mr = 1 + px + pz;
  auto M = [&](int64_t r, int c) -> double & { return mom[r + c * mr]; };
  for (int64_t r = 0; r < mr; ++r) {
    M(r, 0) = 0.0;
    M(r, 1) = 1.0;
    M(r, 2) = 0.0;
  }
  std::vector<int> isb((size_t)(px + pz), 0);
  for (int i = 0; i < px; ++i) {
    double *col = X + (int64_t)i * n;
    int64_t cnt;
    double mn, mx;
    unique_minmax(col, n, &cnt, &mn, &mx);
    if (cnt == 2) {
      isb[i] = 1;
      M(i + 1, 2) = 1;
      if (mn != 0) M(i, 0) = mn;
      if (mx != 1) M(i, 1) = (mx - mn);
      for (int64_t r = 0; r < n; ++r) col[r] -= M(i, 0);
      for (int64_t r = 0; r < n; ++r) col[r] /= M(i, 1);
    } else if (cnt == 1) {
      for (int64_t r = 0; r < n; ++r) col[r] = 0.0;
    }
  }
  for (int i = px; i < px + pz; ++i) {
    double *col = Z + (int64_t)(i - px) * n;
    int64_t cnt;
    double mn, mx;
    unique_minmax(col, n, &cnt, &mn, &mx);
    if (cnt == 2) {
      isb[i] = 1;
      M(i + 1, 2) = 1;
      if (mn != 0) M(i, 0) = mn;
      if (mx != 1) M(i, 1) = (mx - mn);
      for (int64_t r = 0; r < n; ++r) col[r] -= M(i, 0);
      for (int64_t r = 0; r < n; ++r) col[r] /= M(i, 1);
    } else if (cnt == 1) {
      if (i >= pz) return ACE_ERR_ARG;  // Z.col(i) out of bounds in the reference
      double *zc = Z + (int64_t)i * n;
      for (int64_t r = 0; r < n; ++r) zc[r] = 0.0;
    }
  }
  double s = 0.0;
  for (int64_t r = 0; r < n; ++r) s += y[r];
  M(0, 0) = s / (double)n;
  for (int64_t r = 0; r < n; ++r) y[r] = y[r] - M(0, 0);
  for (int i = 1; i < px + 1; ++i)
    if (isb[i - 1] == 0) {
      double *col = X + (int64_t)(i - 1) * n;
      M(i, 0) = median_of(col, n);
      for (int64_t r = 0; r < n; ++r) col[r] -= M(i, 0);
    }
  for (int i = px + 1; i < px + pz + 1; ++i)
    if (isb[i - 1] == 0) {
      double *col = Z + (int64_t)(i - px - 1) * n;
      M(i, 0) = median_of(col, n);
      for (int64_t r = 0; r < n; ++r) col[r] -= M(i, 0);
    }
  double mean = 0.0;
  for (int64_t r = 0; r < n; ++r) mean += y[r];
  mean /= (double)n;
  double ss = 0.0;
  for (int64_t r = 0; r < n; ++r) ss += (y[r] - mean) * (y[r] - mean);
  M(0, 1) = std::sqrt(ss / (double)(n - 1));
  for (int64_t r = 0; r < n; ++r) y[r] = y[r] / M(0, 1);
  for (int i = 1; i < px + 1; ++i)
    if (isb[i - 1] == 0) {
      double *col = X + (int64_t)(i - 1) * n;
      double mx = 0.0;
      for (int64_t r = 0; r < n; ++r) mx = std::max(mx, std::fabs(col[r]));
      M(i, 1) = mx;
      for (int64_t r = 0; r < n; ++r) col[r] /= M(i, 1);
    }
  for (int i = px + 1; i < px + pz + 1; ++i)
    if (i - px - 1 < (int)isb.size() && isb[i - px - 1] == 0) {
      double *col = Z + (int64_t)(i - px - 1) * n;
      double mx = 0.0;
      for (int64_t r = 0; r < n; ++r) mx = std::max(mx, std::fabs(col[r]));
      M(i, 1) = mx;
      for (int64_t r = 0; r < n; ++r) col[r] = col[r] / M(i, 1);
    }
  return ACE_OK;
}

// normalize_test (src/utilities_cpp.cpp:108-118)
int ace_normalize_test(int64_t n, int px, int pz, double *X, double *Z, const double *mom,
                       int64_t mr) {
  if (mr < 1 + px + pz) return ACE_ERR_ARG;
  for (int i = 0; i < px; ++i)
    for (int64_t r = 0; r < n; ++r)
      X[r + i * n] = (X[r + i * n] - mom[(i + 1)]) / mom[(i + 1) + mr];
  for (int i = 0; i < pz; ++i)
    for (int64_t r = 0; r < n; ++r)
      Z[r + i * n] = (Z[r + i * n] - mom[(i + 1 + px)]) / mom[(i + 1 + px) + mr];
  return ACE_OK;
}

}  // extern "C"
