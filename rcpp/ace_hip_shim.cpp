// ace_hip_shim.cpp -- Rcpp shim that keeps the reference package's `.Call`
// surface (R/RcppExports.R:4-78) and forwards every routine to the C ABI in
// include/ace_hip.h.  Drop-in for ace 0.4.1: replace src/kernel_SE_cpp.cpp,
// src/kernel_Matern_cpp.cpp, src/pred_cpp.cpp, src/stats_cpp.cpp,
// src/optimizer_cpp.cpp, src/utilities_cpp.cpp and src/ncs_basis_cpp.cpp by
// this file, re-run Rcpp::compileAttributes(), and link libace_hip.so
// (INTEGRATION.md).  UNTESTED HERE: R and Rcpp are not installed in the
// build image; the same entry points are exercised through the Python
// ctypes binding (additivecausalexpansion_amd/_lib.py) by tests/.
//
// Semantics kept from the reference:
//  * arguments the reference takes by non-const arma reference are mutated
//    in place (stats, m/v/nu/para, grads, y/X/Z): an Rcpp NumericVector /
//    NumericMatrix argument shares the R object's memory, exactly like the
//    RcppArmadillo `arma::vec&` view;
//  * list names `full`/`elements`, `eigenval`/`inv`, `map`/`ci`/`var`
//    [/`ate`/`att`/`atu`];
//  * a non-zero ace status becomes Rcpp::stop(ace_last_error()).
#include <Rcpp.h>

#include "ace_hip.h"

using namespace Rcpp;

namespace {

// Rcpp::checkUserInterrupt() equivalent: R_CheckUserInterrupt longjmps, so
// it runs under R_ToplevelExec and a FALSE return means "interrupt pending".
void check_interrupt(void *) { R_CheckUserInterrupt(); }
int r_poll(void *) { return R_ToplevelExec(check_interrupt, nullptr) == FALSE; }

ace_ctx *ctx() {
  static ace_ctx *c = nullptr;
  if (!c) {
    if (ace_create(0, &c) != ACE_OK) Rcpp::stop(std::string("ace: ") + ace_last_error(nullptr));
    ace_set_interrupt_poll(c, r_poll, nullptr);
  }
  return c;
}

void ok(int status) {
  if (status == ACE_ERR_INTERRUPTED) throw Rcpp::internal::InterruptedException();
  if (status != ACE_OK) Rcpp::stop(std::string("ace: ") + ace_last_error(ctx()));
}

NumericVector cube(int64_t n1, int64_t n2, int B) {
  NumericVector c((R_xlen_t)(n1 * n2 * B));
  c.attr("dim") = IntegerVector::create((int)n1, (int)n2, B);
  return c;
}

List kernmat_cross(int kind, NumericMatrix X1, NumericMatrix X2, NumericMatrix Z1,
                   NumericMatrix Z2, NumericVector parameters) {
  const int64_t n1 = X1.nrow(), n2 = X2.nrow();
  const int p = X2.ncol(), B = Z1.ncol() + 1;
  NumericMatrix full(n1, n2);
  NumericVector el = cube(n1, n2, B);
  ok(ace_kernmat_cross(ctx(), kind, n1, n2, p, B, X1.begin(), X2.begin(), Z1.begin(),
                       Z2.begin(), parameters.begin(), full.begin(), el.begin()));
  return List::create(_["full"] = full, _["elements"] = el);
}

List kernmat_sym(int kind, NumericMatrix X, NumericMatrix Z, NumericVector parameters) {
  const int64_t n = X.nrow();
  const int p = X.ncol(), B = Z.ncol() + 1;
  NumericMatrix full(n, n);
  NumericVector el = cube(n, n, B);
  ok(ace_kernmat_sym(ctx(), kind, n, p, B, X.begin(), Z.begin(), parameters.begin(),
                     full.begin(), el.begin()));
  return List::create(_["full"] = full, _["elements"] = el);
}

NumericVector grad(int kind, NumericVector y, NumericMatrix X, NumericMatrix Z,
                   NumericMatrix Kfull, NumericVector K, NumericMatrix invKmatn,
                   NumericVector eigenval, NumericVector parameters, NumericVector stats,
                   unsigned int B, double std_y) {
  NumericVector g(parameters.size());
  ok(ace_grad(ctx(), kind, X.nrow(), X.ncol(), (int)B, y.begin(), X.begin(), Z.begin(),
              Kfull.begin(), K.size() ? K.begin() : nullptr, invKmatn.begin(),
              eigenval.begin(), parameters.begin(), stats.begin(), std_y, g.begin()));
  return g;  // stats was written in place (src/kernel_SE_cpp.cpp:238-240)
}

}  // namespace

// [[Rcpp::export]]
List kernmat_SE_cpp(NumericMatrix X1, NumericMatrix X2, NumericMatrix Z1, NumericMatrix Z2,
                    NumericVector parameters) {
  return kernmat_cross(ACE_KERNEL_SE, X1, X2, Z1, Z2, parameters);
}

// [[Rcpp::export]]
List kernmat_SE_symmetric_cpp(NumericMatrix X, NumericMatrix Z, NumericVector parameters) {
  return kernmat_sym(ACE_KERNEL_SE, X, Z, parameters);
}

// [[Rcpp::export]]
List kernmat_Matern32_cpp(NumericMatrix X1, NumericMatrix X2, NumericMatrix Z1,
                          NumericMatrix Z2, NumericVector parameters) {
  return kernmat_cross(ACE_KERNEL_MATERN32, X1, X2, Z1, Z2, parameters);
}

// [[Rcpp::export]]
List kernmat_Matern32_symmetric_cpp(NumericMatrix X, NumericMatrix Z, NumericVector parameters) {
  return kernmat_sym(ACE_KERNEL_MATERN32, X, Z, parameters);
}

// [[Rcpp::export]]
List invkernel_cpp(NumericMatrix pdmat, double sigma) {
  const int64_t n = pdmat.nrow();
  NumericVector ev(n);
  NumericMatrix inv(n, n);
  ok(ace_invkernel(ctx(), n, pdmat.begin(), sigma, ev.begin(), inv.begin()));
  return List::create(_["eigenval"] = ev, _["inv"] = inv);
}

// [[Rcpp::export]]
NumericVector grad_SE_cpp(NumericVector y, NumericMatrix X, NumericMatrix Z,
                          NumericMatrix Kfull, NumericVector K, NumericMatrix invKmatn,
                          NumericVector eigenval, NumericVector parameters,
                          NumericVector stats, unsigned int B, double std_y) {
  return grad(ACE_KERNEL_SE, y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y);
}

// [[Rcpp::export]]
NumericVector grad_Matern_cpp(NumericVector y, NumericMatrix X, NumericMatrix Z,
                              NumericMatrix Kfull, NumericVector K, NumericMatrix invKmatn,
                              NumericVector eigenval, NumericVector parameters,
                              NumericVector stats, unsigned int B, double std_y) {
  return grad(ACE_KERNEL_MATERN32, y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B,
              std_y);
}

// [[Rcpp::export]]
NumericVector stats_cpp(NumericVector y, NumericMatrix Kmat, NumericMatrix invKmatn,
                        NumericVector eigenval, double mu, double std_y = 1) {
  NumericVector out(2);
  ok(ace_stats(ctx(), y.size(), y.begin(), Kmat.begin(), invKmatn.begin(), eigenval.begin(), mu,
               std_y, out.begin()));
  return out;
}

// [[Rcpp::export]]
double mu_solution_cpp(NumericVector y, NumericMatrix invKmat) {
  double mu = 0;
  ok(ace_mu_solution(ctx(), y.size(), y.begin(), invKmat.begin(), &mu));
  return mu;
}

// [[Rcpp::export]]
List pred_cpp(NumericVector y_X, double sigma, double mu, NumericMatrix invK_XX,
              NumericMatrix K_xX, NumericMatrix K_xx, double mean_y, double std_y) {
  const int64_t nx = K_xX.nrow(), nX = K_xX.ncol();
  NumericVector map(nx), var(nx);
  NumericMatrix ci(nx, 2);
  ok(ace_pred(ctx(), nX, nx, y_X.begin(), sigma, mu, invK_XX.begin(), K_xX.begin(),
              K_xx.begin(), mean_y, std_y, map.begin(), ci.begin(), var.begin()));
  return List::create(_["map"] = map, _["ci"] = ci, _["var"] = var);
}

// [[Rcpp::export]]
List pred_marginal_cpp(NumericVector y_X, NumericVector Z_x, double sigma, double mu,
                       NumericMatrix invK_XX, NumericVector K_xX, NumericVector K_xx,
                       double mean_y, double std_y, double std_Z, bool calculate_ate) {
  IntegerVector d = K_xX.attr("dim");
  const int64_t nx = d[0], nX = d[1];
  const int B = d[2];
  NumericVector map(nx), var(nx), avg(12);
  NumericMatrix ci(nx, 2);
  ok(ace_pred_marginal(ctx(), nX, nx, B, y_X.begin(), Z_x.begin(), sigma, mu, invK_XX.begin(),
                       K_xX.begin(), K_xx.begin(), mean_y, std_y, std_Z, calculate_ate ? 1 : 0,
                       map.begin(), ci.begin(), var.begin(), avg.begin()));
  if (!calculate_ate) return List::create(_["map"] = map, _["ci"] = ci, _["var"] = var);
  auto one = [&](int j) {
    return List::create(_["map"] = avg[4 * j],
                        _["ci"] = NumericVector::create(avg[4 * j + 1], avg[4 * j + 2]),
                        _["var"] = avg[4 * j + 3]);
  };
  return List::create(_["map"] = map, _["ci"] = ci, _["var"] = var, _["ate"] = one(0),
                      _["att"] = one(1), _["atu"] = one(2));
}

// [[Rcpp::export]]
bool Nesterov_cpp(double learn_rate, double momentum, NumericVector nu, NumericVector grad,
                  NumericVector para) {
  return ace_nesterov(para.size(), learn_rate, momentum, nu.begin(), grad.begin(),
                      para.begin()) != 0;
}

// [[Rcpp::export]]
bool Nadam_cpp(double iter, double learn_rate, double beta1, double beta2, double eps,
               NumericVector m, NumericVector v, NumericVector grad, NumericVector para) {
  return ace_nadam(para.size(), iter, learn_rate, beta1, beta2, eps, m.begin(), v.begin(),
                   grad.begin(), para.begin()) != 0;
}

// [[Rcpp::export]]
bool Adam_cpp(double iter, double learn_rate, double beta1, double beta2, double eps,
              NumericVector m, NumericVector v, NumericVector grad, NumericVector para) {
  return ace_adam(para.size(), iter, learn_rate, beta1, beta2, eps, m.begin(), v.begin(),
                  grad.begin(), para.begin()) != 0;
}

// [[Rcpp::export]]
void norm_clip_cpp(bool flag, NumericVector grads, double max_length) {
  ace_norm_clip(flag ? 1 : 0, grads.size(), grads.begin(), max_length);
}

// [[Rcpp::export]]
NumericMatrix ncs_basis(NumericVector x, NumericVector knots) {
  NumericMatrix d(x.size(), knots.size());
  int64_t k = 0;
  ok(ace_ncs_basis(x.size(), x.begin(), knots.size(), knots.begin(), d.begin(), &k));
  return d(Range(0, x.size() - 1), Range(0, k - 1));
}

// [[Rcpp::export]]
NumericMatrix ncs_basis_deriv(NumericVector x, NumericVector knots) {
  NumericMatrix d(x.size(), knots.size());
  int64_t k = 0;
  ok(ace_ncs_basis_deriv(x.size(), x.begin(), knots.size(), knots.begin(), d.begin(), &k));
  return d(Range(0, x.size() - 1), Range(0, k - 1));
}

// [[Rcpp::export]]
NumericMatrix normalize_train(NumericVector y, NumericMatrix X, NumericMatrix Z) {
  NumericMatrix mom(1 + X.ncol() + Z.ncol(), 3);
  ok(ace_normalize_train(y.size(), X.ncol(), Z.ncol(), y.begin(), X.begin(), Z.begin(),
                         mom.begin()));
  return mom;  // y, X, Z normalised in place (src/utilities_cpp.cpp:13)
}

// [[Rcpp::export]]
void normalize_test(NumericMatrix X, NumericMatrix Z, NumericMatrix moments) {
  ok(ace_normalize_test(X.nrow(), X.ncol(), Z.ncol(), X.begin(), Z.begin(), moments.begin(),
                        moments.nrow()));
}

// ---- optional device-resident fast path -------------
// An R6 para_update can call these instead of the kernmat/invkernel/grad
// trio to keep X, Z, y and the inverse in HBM (no n x n x B cube in R).

// [[Rcpp::export]]
SEXP ace_model_new(int kind, NumericVector y, NumericMatrix X, NumericMatrix Z, double std_y) {
  ace_model *m = nullptr;
  ok(ace_model_create(ctx(), kind, X.nrow(), X.ncol(), Z.ncol() + 1, &m));
  ok(ace_model_set_data(m, y.begin(), X.begin(), Z.begin(), std_y));
  XPtr<ace_model, PreserveStorage, ace_model_destroy, true> p(m, true);
  return p;
}

// [[Rcpp::export]]
List ace_model_step(SEXP model, int iter, NumericVector parameters) {
  XPtr<ace_model, PreserveStorage, ace_model_destroy, true> m(model);
  NumericVector g(parameters.size()), st(2);
  double mu = 0;
  ok(ace_model_para_update(m.get(), iter, parameters.begin(), g.begin(), st.begin(), &mu));
  return List::create(_["gradients"] = g, _["stats"] = st, _["mu"] = mu);
}

// The whole ace.train loop (R/main_ace.R:213-235) natively; optimizer
// 0 = Nesterov, 1 = Adam, 2 = Nadam.  parameters is updated in place.
// [[Rcpp::export]]
List ace_model_fit(SEXP model, int optimizer, double learn_rate, double momentum, double beta1,
                   double beta2, bool norm_clip, double clip_at, int maxiter, double tol,
                   NumericVector parameters) {
  XPtr<ace_model, PreserveStorage, ace_model_destroy, true> m(model);
  if (maxiter < 1) Rcpp::stop("ace: maxiter must be >= 1");
  // the R loop's matrix(0, 2, maxiter + 2) (R/main_ace.R:213): the library
  // writes all 2 x (maxiter + 2) entries
  NumericMatrix st(2, maxiter + 2);
  int iters = 0, converged = 0;
  ok(ace_model_train(m.get(), optimizer, learn_rate, momentum, beta1, beta2, norm_clip ? 1 : 0,
                     clip_at, maxiter, tol, parameters.begin(), st.begin(), &iters, &converged));
  // stats[, 3:(iter + 2)] as ace.train returns it (R/main_ace.R:235)
  NumericMatrix out = st(_, Range(2, iters + 1));
  return List::create(_["stats"] = out, _["iterations"] = iters, _["converged"] = converged != 0);
}
