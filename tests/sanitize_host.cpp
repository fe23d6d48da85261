// sanitize_host.cpp -- AddressSanitizer / UBSan driver for the host-side code
// of the C ABI (additivecausalexpansion_amd/csrc/ace_host.cpp: optimizers,
// norm clip, ncs basis, normalisation) and the oracle's C restatement
// (oracle/ace_ref.c), SURVEY.md §5 "Race detection / sanitizers".  Built and
// run by tests/test_sanitize_cpu.py with -fsanitize=address,undefined; any
// report aborts the process (halt_on_error).  Test infrastructure only.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/ace_hip.h"

extern "C" {
// oracle/ace_ref.c
int ref_kernmat_sym(int kind, int64_t n, int p, int B, const double *X, const double *Z,
                    const double *theta, double *Kfull, double *Kel);
int ref_grad(int kind, int64_t n, int p, int B, const double *y, const double *X,
             const double *Kfull, const double *Kel, const double *inv, double logdet,
             const double *theta, double *stats, double std_y, double *grad);
double ref_mu_solution(int64_t n, const double *y, const double *inv);
}

static int failures = 0;
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                                 \
    }                                                                             \
  } while (0)

int main() {
  std::mt19937_64 rng(7);
  std::normal_distribution<double> N(0.0, 1.0);
  std::uniform_real_distribution<double> U(-1.0, 1.0);

  // optimizers + norm clip, including P = 1 and a non-finite gradient
  for (int64_t P : {1, 17, 818}) {
    std::vector<double> g(P), m(P, 0.0), v(P, 0.0), nu(P, 0.0), th(P);
    for (auto &x : g) x = N(rng);
    for (auto &x : th) x = N(rng);
    ace_norm_clip(1, P, g.data(), 1.0);
    for (int it = 1; it <= 5; ++it) {
      CHECK(ace_nadam(P, it, 0.01, 0.9, 0.999, 1e-8, m.data(), v.data(), g.data(), th.data()) == 1);
      CHECK(ace_adam(P, it, 0.01, 0.9, 0.999, 1e-8, m.data(), v.data(), g.data(), th.data()) == 1);
      CHECK(ace_nesterov(P, 0.01, 0.5, nu.data(), g.data(), th.data()) == 1);
    }
    g[P - 1] = NAN;
    CHECK(ace_nadam(P, 6, 0.01, 0.9, 0.999, 1e-8, m.data(), v.data(), g.data(), th.data()) == 0);
    ace_norm_clip(1, P, g.data(), 1.0);  // non-finite norm: untouched
  }

  // ncs basis (+ derivative), duplicated / unsorted knots, n = 0 and 1
  for (int64_t n : {0, 1, 200}) {
    std::vector<double> x(n + 1), knots = {0.5, -1.0, 0.1, 1.0, 0.1};  // n = 0: non-null x
    for (auto &e : x) e = U(rng);
    std::vector<double> design((size_t)(n * 4) + 1);
    int64_t nc = 0;
    CHECK(ace_ncs_basis(n, x.data(), (int64_t)knots.size(), knots.data(), design.data(), &nc) ==
          ACE_OK);
    CHECK(nc == 4);
    CHECK(ace_ncs_basis_deriv(n, x.data(), (int64_t)knots.size(), knots.data(), design.data(),
                              &nc) == ACE_OK);
  }
  {
    double k1[1] = {0.0}, x1[1] = {0.0}, d1[4];
    int64_t nc;
    CHECK(ace_ncs_basis(1, x1, 1, k1, d1, &nc) == ACE_ERR_ARG);
  }

  // normalisation: continuous, binary and constant columns
  {
    const int64_t n = 101;
    const int px = 3, pz = 2;
    std::vector<double> y(n), X((size_t)(n * px)), Z((size_t)(n * pz)),
        mom((size_t)(3 * (1 + px + pz)));
    for (auto &e : y) e = N(rng);
    for (int64_t r = 0; r < n; ++r) {
      X[r] = U(rng);
      X[r + n] = (r % 2) ? 3.0 : 5.0;  // binary
      X[r + 2 * n] = 2.0 * U(rng);
      Z[r] = N(rng);
      Z[r + n] = (r % 3) ? 1.0 : 0.0;  // binary
    }
    CHECK(ace_normalize_train(n, px, pz, y.data(), X.data(), Z.data(), mom.data()) == ACE_OK);
    std::vector<double> X2 = X, Z2 = Z;
    CHECK(ace_normalize_test(n, px, pz, X2.data(), Z2.data(), mom.data(), 1 + px + pz) == ACE_OK);
    // constant Z column with px >= pz: Z.col(i) is out of range in the reference
    std::vector<double> Zc((size_t)n, 4.0), y2 = y, X3((size_t)(n * px));
    std::vector<double> mom2((size_t)(3 * (1 + px + 1)));
    for (auto &e : X3) e = U(rng);
    CHECK(ace_normalize_train(n, px, 1, y2.data(), X3.data(), Zc.data(), mom2.data()) ==
          ACE_ERR_ARG);
  }

  // oracle restatement: assembly + gradient + mu at a small size
  {
    const int64_t n = 37;
    const int p = 3, B = 4, P = 2 + B * (p + 1);
    std::vector<double> X((size_t)(n * p)), Z((size_t)(n * (B - 1))), th(P), y(n);
    for (auto &e : X) e = U(rng);
    for (auto &e : Z) e = (U(rng) > 0.3) ? N(rng) : 0.0;
    for (auto &e : y) e = N(rng);
    th[0] = -2.0;
    th[1] = 0.1;
    for (int j = 2; j < P; ++j) th[j] = 0.3 * N(rng);
    std::vector<double> full((size_t)(n * n)), el((size_t)(n * n * B));
    for (int kind = 0; kind < 2; ++kind) {
      CHECK(ref_kernmat_sym(kind, n, p, B, X.data(), Z.data(), th.data(), full.data(),
                            el.data()) == 0);
      // a diagonal SPD stand-in for the inverse (the restatement only reads it)
      std::vector<double> inv((size_t)(n * n), 0.0);
      for (int64_t r = 0; r < n; ++r) inv[r + r * n] = 1.0 / (1.0 + full[r + r * n]);
      double stats[2] = {0.0, 0.0};
      std::vector<double> g(P);
      ref_grad(kind, n, p, B, y.data(), X.data(), full.data(), el.data(), inv.data(), 0.0,
               th.data(), stats, 1.3, g.data());
      for (double e : g) CHECK(std::isfinite(e));
      CHECK(std::isfinite(ref_mu_solution(n, y.data(), inv.data())));
    }
  }

  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::puts("sanitize_host: OK");
  return 0;
}
