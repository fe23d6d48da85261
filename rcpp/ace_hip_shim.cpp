// ace_hip_shim.cpp -- Rcpp shim that keeps the reference package's `.Call`
// surface (R/RcppExports.R:4-78) and forwards every routine to the C ABI in
// include/ace_hip.h.  Drop-in for ace 0.4.1: replace src/kernel_SE_cpp.cpp,
// src/kernel_Matern_cpp.cpp, src/pred_cpp.cpp, src/stats_cpp.cpp,
// src/optimizer_cpp.cpp, src/utilities_cpp.cpp and src/ncs_basis_cpp.cpp by
// this file, re-run Rcpp::compileAttributes(), and link libace_hip.so
// (INTEGRATION.md).  The R6 classes and every other R file stay unchanged.
// UNTESTED HERE: R and Rcpp are not installed in the build image; the same
// entry points and the same call sequence are exercised through the Python
// ctypes binding by tests/ (tests/test_r6_handles_gpu.py drives the R6
// sequence over the device handles this shim wraps).
//
// Device handles.  The R6 kernel classes keep Kmat, Karray and invKmatn as R
// objects and pass them from routine to routine (R/kernel_SE_R6.R:26-50).
// Here the matrix results of kernmat_* and invkernel_cpp are ace_dmat
// handles wrapped in an ALTREP double vector (class "ace_dmat", with the R
// dim attribute of the reference's result):
//   * passing one back into a routine of this shim uses the device data --
//     Kmat, the inverse and the `elements` cube never cross PCIe, and the
//     cube (21.5 GB at n = 16384, B = 10) is never assembled at all: the
//     gradient recomputes its slices, prediction assembles only the marginal
//     slice sums it needs;
//   * reading one from R (x[i], dim arithmetic, sum(), print(), ...)
//     materialises it transparently (Elt / Get_region read ranges; Dataptr
//     copies the whole object once into a host vector);
//   * an object R has written to (Dataptr with writeable = TRUE) is from then
//     on a plain host vector: later calls upload it like any R matrix.
// options(ace.device_handles = FALSE) returns plain R matrices instead.
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
#include <R_ext/Altrep.h>

#include <memory>
#include <vector>

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

// Device memory held by handles R no longer references is released by R's
// garbage collector, which does not see it: a device allocation that fails
// runs the collector once and retries (each R6 iteration drops the previous
// iteration's Kmat / inverse handles).
template <class F>
void ok_gc(F call) {
  int st = call();
  if (st == ACE_ERR_OOM) {
    R_gc();
    st = call();
  }
  ok(st);
}

// Status check for code R calls from its C internals (the ALTREP methods):
// no BEGIN_RCPP/END_RCPP guard surrounds those frames, so a C++ exception
// must not unwind through them.  Rf_error longjmps to R's handler instead;
// nothing on these frames needs a destructor (R objects are PROTECTed and
// unwound by R).
void ok_altrep(int status) {
  if (status != ACE_OK) Rf_error("ace: %s", ace_last_error(ctx()));
}

bool use_handles() {
  SEXP o = Rf_GetOption1(Rf_install("ace.device_handles"));
  return o == R_NilValue || Rf_asLogical(o) != FALSE;
}

// ---------------------------------------------------------------- ALTREP class
R_altrep_class_t dmat_class;

ace_dmat *handle_of(SEXP x) {
  return static_cast<ace_dmat *>(R_ExternalPtrAddr(R_altrep_data1(x)));
}

R_xlen_t dmat_length(SEXP x) {
  int64_t r = 0, c = 0, s = 0;
  ace_dmat_dims(handle_of(x), &r, &c, &s);
  return (R_xlen_t)(r * c * s);
}

// data2: the host copy (R_NilValue until R asks for the data pointer)
SEXP materialise(SEXP x) {
  SEXP d2 = R_altrep_data2(x);
  if (d2 == R_NilValue) {
    const R_xlen_t n = dmat_length(x);
    d2 = PROTECT(Rf_allocVector(REALSXP, n));
    ok_altrep(ace_dmat_read(handle_of(x), 0, (int64_t)n, REAL(d2)));
    R_set_altrep_data2(x, d2);
    UNPROTECT(1);
  }
  return d2;
}

void *dmat_dataptr(SEXP x, Rboolean writeable) {
  SEXP d2 = materialise(x);
  // once written through this pointer the host copy is the truth:
  // as_dmat() below then uploads it instead of using the stale handle
  if (writeable) Rf_setAttrib(x, Rf_install("ace.host_owned"), Rf_ScalarLogical(TRUE));
  return REAL(d2);
}

const void *dmat_dataptr_or_null(SEXP x) {
  SEXP d2 = R_altrep_data2(x);
  return d2 == R_NilValue ? nullptr : REAL(d2);
}

double dmat_elt(SEXP x, R_xlen_t i) {
  SEXP d2 = R_altrep_data2(x);
  if (d2 != R_NilValue) return REAL(d2)[i];
  double v = NA_REAL;
  ok_altrep(ace_dmat_read(handle_of(x), (int64_t)i, 1, &v));
  return v;
}

R_xlen_t dmat_get_region(SEXP x, R_xlen_t i, R_xlen_t n, double *buf) {
  const R_xlen_t len = dmat_length(x);
  const R_xlen_t m = (i + n > len) ? len - i : n;
  if (m <= 0) return 0;
  SEXP d2 = R_altrep_data2(x);
  if (d2 != R_NilValue) {
    std::copy(REAL(d2) + i, REAL(d2) + i + m, buf);
  } else {
    ok_altrep(ace_dmat_read(handle_of(x), (int64_t)i, (int64_t)m, buf));
  }
  return m;
}

Rboolean dmat_inspect(SEXP x, int, int, int, void (*)(SEXP, int, int, int)) {
  Rprintf(" ace_dmat device handle (%s)\n",
          R_altrep_data2(x) == R_NilValue ? "device only" : "host copy present");
  return TRUE;
}

// the handle is immutable: a duplicate shares it (R's GC owns the pointer)
SEXP dmat_duplicate(SEXP x, Rboolean) {
  SEXP d2 = R_altrep_data2(x);
  SEXP y = PROTECT(R_new_altrep(dmat_class, R_altrep_data1(x),
                                d2 == R_NilValue ? R_NilValue : Rf_duplicate(d2)));
  UNPROTECT(1);
  return y;
}

void dmat_finalize(SEXP p) {
  ace_dmat *h = static_cast<ace_dmat *>(R_ExternalPtrAddr(p));
  if (h) ace_dmat_free(h);
  R_ClearExternalPtr(p);
}

// a handle as an R double vector with the reference result's dim attribute
SEXP wrap_dmat(ace_dmat *h) {
  SEXP ptr = PROTECT(R_MakeExternalPtr(h, R_NilValue, R_NilValue));
  R_RegisterCFinalizerEx(ptr, dmat_finalize, TRUE);
  SEXP x = PROTECT(R_new_altrep(dmat_class, ptr, R_NilValue));
  int64_t r = 0, c = 0, s = 0;
  ace_dmat_dims(h, &r, &c, &s);
  if (s > 1) Rf_setAttrib(x, R_DimSymbol, IntegerVector::create((int)r, (int)c, (int)s));
  else Rf_setAttrib(x, R_DimSymbol, IntegerVector::create((int)r, (int)c));
  UNPROTECT(2);
  return x;
}

bool is_device(SEXP x) {
  return ALTREP(x) && R_altrep_inherits(x, dmat_class) &&
         Rf_getAttrib(x, Rf_install("ace.host_owned")) == R_NilValue;
}

// Handle for a matrix argument: the object's own handle, or (a plain R
// matrix, or one R has written to) a temporary upload kept alive in `tmp`.
struct Temps {
  std::vector<ace_dmat *> h;
  ~Temps() {
    for (ace_dmat *p : h) ace_dmat_free(p);
  }
};
const ace_dmat *as_dmat(SEXP x, Temps &tmp) {
  if (is_device(x)) return handle_of(x);
  SEXP dim = Rf_getAttrib(x, R_DimSymbol);
  int64_t r = Rf_xlength(x), c = 1, s = 1;
  if (dim != R_NilValue) {
    r = INTEGER(dim)[0];
    c = Rf_length(dim) > 1 ? INTEGER(dim)[1] : 1;
    s = Rf_length(dim) > 2 ? INTEGER(dim)[2] : 1;
  }
  ace_dmat *h = nullptr;
  ok(ace_dmat_upload(ctx(), r, c, s, REAL(x), &h));
  tmp.h.push_back(h);
  return h;
}

bool any_device(std::initializer_list<SEXP> xs) {
  for (SEXP x : xs)
    if (is_device(x)) return true;
  return false;
}

NumericVector cube(int64_t n1, int64_t n2, int B) {
  NumericVector c((R_xlen_t)(n1 * n2 * B));
  c.attr("dim") = IntegerVector::create((int)n1, (int)n2, B);
  return c;
}

int ncols_of(SEXP M) {
  SEXP dim = Rf_getAttrib(M, R_DimSymbol);
  return dim == R_NilValue ? 1 : INTEGER(dim)[1];
}
int64_t nrows_of(SEXP M) {
  SEXP dim = Rf_getAttrib(M, R_DimSymbol);
  return dim == R_NilValue ? Rf_xlength(M) : INTEGER(dim)[0];
}

// ---------------------------------------------------------------- kernels
List kernmat_cross(int kind, NumericMatrix X1, NumericMatrix X2, SEXP Z1, SEXP Z2,
                   NumericVector parameters) {
  const int64_t n1 = X1.nrow(), n2 = X2.nrow();
  const int p = X2.ncol(), B = ncols_of(Z1) + 1;
  if (use_handles()) {
    ace_dmat *full = nullptr, *el = nullptr;
    ok_gc([&] {
      return ace_kernmat_cross_dev(ctx(), kind, n1, n2, p, B, X1.begin(), X2.begin(), REAL(Z1),
                                   REAL(Z2), parameters.begin(), &full, &el);
    });
    return List::create(_["full"] = wrap_dmat(full), _["elements"] = wrap_dmat(el));
  }
  NumericMatrix full(n1, n2);
  NumericVector el = cube(n1, n2, B);
  ok(ace_kernmat_cross(ctx(), kind, n1, n2, p, B, X1.begin(), X2.begin(), REAL(Z1), REAL(Z2),
                       parameters.begin(), full.begin(), el.begin()));
  return List::create(_["full"] = full, _["elements"] = el);
}

List kernmat_sym(int kind, NumericMatrix X, SEXP Z, NumericVector parameters) {
  const int64_t n = X.nrow();
  const int p = X.ncol(), B = ncols_of(Z) + 1;
  if (use_handles()) {
    ace_dmat *full = nullptr, *el = nullptr;
    ok_gc([&] {
      return ace_kernmat_sym_dev(ctx(), kind, n, p, B, X.begin(), REAL(Z), parameters.begin(),
                                 &full, &el);
    });
    return List::create(_["full"] = wrap_dmat(full), _["elements"] = wrap_dmat(el));
  }
  NumericMatrix full(n, n);
  NumericVector el = cube(n, n, B);
  ok(ace_kernmat_sym(ctx(), kind, n, p, B, X.begin(), REAL(Z), parameters.begin(), full.begin(),
                     el.begin()));
  return List::create(_["full"] = full, _["elements"] = el);
}

NumericVector grad(int kind, NumericVector y, NumericMatrix X, SEXP Z, SEXP Kfull, SEXP K,
                   SEXP invKmatn, NumericVector eigenval, NumericVector parameters,
                   NumericVector stats, unsigned int B, double std_y) {
  NumericVector g(parameters.size());
  if (any_device({Kfull, K, invKmatn})) {
    Temps t;
    // the gradient recomputes K_b from X, Z, theta: a virtual cube is never read
    ok(ace_grad_dev(ctx(), kind, X.nrow(), X.ncol(), (int)B, y.begin(), X.begin(), REAL(Z),
                    as_dmat(Kfull, t), is_device(K) ? handle_of(K) : nullptr, as_dmat(invKmatn, t),
                    eigenval.begin(), parameters.begin(), stats.begin(), std_y, g.begin()));
    return g;  // stats was written in place (src/kernel_SE_cpp.cpp:238-240)
  }
  ok(ace_grad(ctx(), kind, X.nrow(), X.ncol(), (int)B, y.begin(), X.begin(), REAL(Z),
              REAL(Kfull), Rf_xlength(K) ? REAL(K) : nullptr, REAL(invKmatn), eigenval.begin(),
              parameters.begin(), stats.begin(), std_y, g.begin()));
  return g;  // stats was written in place (src/kernel_SE_cpp.cpp:238-240)
}

}  // namespace

// Registers the ALTREP class when the package's DLL loads (R_init_ace).
// [[Rcpp::init]]
void ace_altrep_init(DllInfo *dll) {
  dmat_class = R_make_altreal_class("ace_dmat", "ace", dll);
  R_set_altrep_Length_method(dmat_class, dmat_length);
  R_set_altrep_Inspect_method(dmat_class, dmat_inspect);
  R_set_altrep_Duplicate_method(dmat_class, dmat_duplicate);
  R_set_altvec_Dataptr_method(dmat_class, dmat_dataptr);
  R_set_altvec_Dataptr_or_null_method(dmat_class, dmat_dataptr_or_null);
  R_set_altreal_Elt_method(dmat_class, dmat_elt);
  R_set_altreal_Get_region_method(dmat_class, dmat_get_region);
}

// [[Rcpp::export]]
List kernmat_SE_cpp(NumericMatrix X1, NumericMatrix X2, SEXP Z1, SEXP Z2,
                    NumericVector parameters) {
  return kernmat_cross(ACE_KERNEL_SE, X1, X2, Z1, Z2, parameters);
}

// [[Rcpp::export]]
List kernmat_SE_symmetric_cpp(NumericMatrix X, SEXP Z, NumericVector parameters) {
  return kernmat_sym(ACE_KERNEL_SE, X, Z, parameters);
}

// [[Rcpp::export]]
List kernmat_Matern32_cpp(NumericMatrix X1, NumericMatrix X2, SEXP Z1, SEXP Z2,
                          NumericVector parameters) {
  return kernmat_cross(ACE_KERNEL_MATERN32, X1, X2, Z1, Z2, parameters);
}

// [[Rcpp::export]]
List kernmat_Matern32_symmetric_cpp(NumericMatrix X, SEXP Z, NumericVector parameters) {
  return kernmat_sym(ACE_KERNEL_MATERN32, X, Z, parameters);
}

// `$eigenval` holds the sweep's pivots (the squared Cholesky diagonal), not
// the eigenvalues src/kernel_SE_cpp.cpp:144-156 returns.  Every in-package
// consumer uses only sum(log(eigenval)) (src/kernel_SE_cpp.cpp:240,
// src/kernel_Matern_cpp.cpp:463, src/stats_cpp.cpp:29), which is log det A
// for both, bit for bit as before.  A caller reading the values themselves
// is told by attr(x, "ace_kind") = "pivots" only -- no warning: the
// package's own R code is the caller, and a warning under options(warn = 2)
// would longjmp out of the export past C++ destructors.
static void mark_pivots(NumericVector &ev) { ev.attr("ace_kind") = "pivots"; }

// [[Rcpp::export]]
List invkernel_cpp(SEXP pdmat, double sigma) {
  const int64_t n = nrows_of(pdmat);
  NumericVector ev(n);
  mark_pivots(ev);
  if (use_handles() || is_device(pdmat)) {
    Temps t;
    ace_dmat *inv = nullptr;
    const ace_dmat *K = as_dmat(pdmat, t);
    ok_gc([&] { return ace_invkernel_dev(ctx(), K, sigma, ev.begin(), &inv); });
    return List::create(_["eigenval"] = ev, _["inv"] = wrap_dmat(inv));
  }
  NumericMatrix inv(n, n);
  ok(ace_invkernel(ctx(), n, REAL(pdmat), sigma, ev.begin(), inv.begin()));
  return List::create(_["eigenval"] = ev, _["inv"] = inv);
}

// [[Rcpp::export]]
NumericVector grad_SE_cpp(NumericVector y, NumericMatrix X, SEXP Z, SEXP Kfull, SEXP K,
                          SEXP invKmatn, NumericVector eigenval, NumericVector parameters,
                          NumericVector stats, unsigned int B, double std_y) {
  return grad(ACE_KERNEL_SE, y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B, std_y);
}

// [[Rcpp::export]]
NumericVector grad_Matern_cpp(NumericVector y, NumericMatrix X, SEXP Z, SEXP Kfull, SEXP K,
                              SEXP invKmatn, NumericVector eigenval, NumericVector parameters,
                              NumericVector stats, unsigned int B, double std_y) {
  return grad(ACE_KERNEL_MATERN32, y, X, Z, Kfull, K, invKmatn, eigenval, parameters, stats, B,
              std_y);
}

// [[Rcpp::export]]
NumericVector stats_cpp(NumericVector y, SEXP Kmat, SEXP invKmatn, NumericVector eigenval,
                        double mu, double std_y = 1) {
  NumericVector out(2);
  if (any_device({Kmat, invKmatn})) {
    Temps t;
    ok(ace_stats_dev(ctx(), y.size(), y.begin(), as_dmat(Kmat, t), as_dmat(invKmatn, t),
                     eigenval.begin(), mu, std_y, out.begin()));
    return out;
  }
  ok(ace_stats(ctx(), y.size(), y.begin(), REAL(Kmat), REAL(invKmatn), eigenval.begin(), mu,
               std_y, out.begin()));
  return out;
}

// [[Rcpp::export]]
double mu_solution_cpp(NumericVector y, SEXP invKmat) {
  double mu = 0;
  if (is_device(invKmat)) {
    ok(ace_mu_solution_dev(ctx(), y.size(), y.begin(), handle_of(invKmat), &mu));
    return mu;
  }
  ok(ace_mu_solution(ctx(), y.size(), y.begin(), REAL(invKmat), &mu));
  return mu;
}

// [[Rcpp::export]]
List pred_cpp(NumericVector y_X, double sigma, double mu, SEXP invK_XX, SEXP K_xX, SEXP K_xx,
              double mean_y, double std_y) {
  const int64_t nx = nrows_of(K_xX), nX = nrows_of(invK_XX);
  NumericVector map(nx), var(nx);
  NumericMatrix ci(nx, 2);
  if (any_device({invK_XX, K_xX, K_xx})) {
    Temps t;
    ok(ace_pred_dev(ctx(), nX, nx, y_X.begin(), sigma, mu, as_dmat(invK_XX, t), as_dmat(K_xX, t),
                    as_dmat(K_xx, t), mean_y, std_y, map.begin(), ci.begin(), var.begin()));
  } else {
    ok(ace_pred(ctx(), nX, nx, y_X.begin(), sigma, mu, REAL(invK_XX), REAL(K_xX), REAL(K_xx),
                mean_y, std_y, map.begin(), ci.begin(), var.begin()));
  }
  return List::create(_["map"] = map, _["ci"] = ci, _["var"] = var);
}

// [[Rcpp::export]]
List pred_marginal_cpp(NumericVector y_X, NumericVector Z_x, double sigma, double mu,
                       SEXP invK_XX, SEXP K_xX, SEXP K_xx, double mean_y, double std_y,
                       double std_Z, bool calculate_ate) {
  IntegerVector d = Rf_getAttrib(K_xX, R_DimSymbol);
  const int64_t nx = d[0], nX = d[1];
  const int B = d.size() > 2 ? d[2] : 1;
  NumericVector map(nx), var(nx), avg(12);
  NumericMatrix ci(nx, 2);
  if (any_device({invK_XX, K_xX, K_xx})) {
    Temps t;
    ok(ace_pred_marginal_dev(ctx(), nX, nx, y_X.begin(), Z_x.begin(), sigma, mu,
                             as_dmat(invK_XX, t), as_dmat(K_xX, t), as_dmat(K_xx, t), mean_y,
                             std_y, std_Z, calculate_ate ? 1 : 0, map.begin(), ci.begin(),
                             var.begin(), avg.begin()));
  } else {
    ok(ace_pred_marginal(ctx(), nX, nx, B, y_X.begin(), Z_x.begin(), sigma, mu, REAL(invK_XX),
                         REAL(K_xX), REAL(K_xx), mean_y, std_y, std_Z, calculate_ate ? 1 : 0,
                         map.begin(), ci.begin(), var.begin(), avg.begin()));
  }
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

// ---- optional fused device model (one call per para_update) ---------------
// The R6 classes above already stay on the device through the handles; these
// entry points additionally fuse kernel + inverse + gradient into one call
// (ace_model_para_update: no Kfull copy, no separate GEMV passes) for a
// caller that opts in.

// [[Rcpp::export]]
SEXP ace_model_new(int kind, NumericVector y, NumericMatrix X, SEXP Z, double std_y) {
  ace_model *m = nullptr;
  ok(ace_model_create(ctx(), kind, X.nrow(), X.ncol(), ncols_of(Z) + 1, &m));
  ok(ace_model_set_data(m, y.begin(), X.begin(), REAL(Z), std_y));
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

// Device-resident predict with the fused model's resident inverse (Q6).
// [[Rcpp::export]]
List ace_model_predict_r(SEXP model, NumericVector parameters, NumericMatrix X2, SEXP Z2,
                         double mean_y, double std_y) {
  XPtr<ace_model, PreserveStorage, ace_model_destroy, true> m(model);
  const int64_t nx = X2.nrow();
  NumericVector map(nx), var(nx);
  NumericMatrix ci(nx, 2);
  ok(ace_model_predict(m.get(), parameters.begin(), nx, X2.begin(), REAL(Z2), mean_y, std_y,
                       map.begin(), ci.begin(), var.begin()));
  return List::create(_["map"] = map, _["ci"] = ci, _["var"] = var);
}
