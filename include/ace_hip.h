/*
 * ace_hip.h -- C ABI of the MI355X-native engine for the `ace` hot path.
 *
 * Drop-in boundary: every entry point below replaces one Rcpp-exported
 * routine of the reference (R package `ace` 0.4.1).  The reference routine
 * is cited as file:line next to each declaration; the R-side `.Call`
 * wrapper names are in R/RcppExports.R:4-78 and are kept unchanged by the
 * Rcpp shim shown in INTEGRATION.md.
 *
 * Conventions
 *  - All matrices are column-major fp64 (R / Armadillo layout) with explicit
 *    64-bit dimensions; cubes are n1 x n2 x B, slice-major (arma::cube).
 *  - The library never allocates or frees caller memory.  Outputs go to
 *    caller buffers; buffers documented "in/out" are mutated in place
 *    exactly as the reference mutates the R vectors it receives by
 *    non-const reference (SURVEY.md §8b "Ownership").
 *  - Functions taking an `ace_ctx*` run on the GPU; they return ACE_OK (0)
 *    or a non-zero status, and ace_last_error() describes the failure.  The
 *    Rcpp shim turns a non-zero status into Rcpp::stop().
 *  - A matrix that is not positive definite does NOT raise an error: as in
 *    the reference (a failed eig_sym only prints, src/kernel_SE_cpp.cpp:144-146)
 *    the affected outputs come out non-finite, so R's optimizer classes
 *    stop() on the non-finite gradient (R/optimizer_classes.R:26-29).
 *  - Host-only functions (optimizers, norm clip, spline basis, normalisation)
 *    need no context and never touch the GPU.
 *  - Calls are blocking and not re-entrant per context (the reference runs
 *    everything synchronously on the R main thread).
 */
#ifndef ACE_HIP_H
#define ACE_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACE_ABI_VERSION 1

enum ace_kernel_kind { ACE_KERNEL_SE = 0, ACE_KERNEL_MATERN32 = 1 };

enum ace_status {
  ACE_OK = 0,
  ACE_ERR_ARG = 1,         /* invalid argument / shape                          */
  ACE_ERR_HIP = 2,         /* HIP runtime failure (no device, launch failure)   */
  ACE_ERR_OOM = 3,         /* device allocation failed                          */
  ACE_ERR_UNSUPPORTED = 4, /* shape outside the compiled range (p > 64, B > 32) */
  ACE_ERR_NONFINITE = 5,   /* non-finite gradient in ace_model_train (R's stop()) */
  ACE_ERR_INTERRUPTED = 6, /* the interrupt poll asked to stop                  */
  ACE_ERR_TIMEOUT = 7      /* device work did not drain within ACE_SYNC_TIMEOUT
                              seconds (default 600): a stalled queue or a hung
                              collective; ace_last_error names the busy streams.
                              The context is then failed: later calls on it
                              return ACE_ERR_TIMEOUT at once (destroy it), and
                              host buffers passed to the timed-out call must
                              not be freed or reused (a copy queued before the
                              deadline may still land in them)            */
};

typedef struct ace_ctx ace_ctx;
typedef struct ace_model ace_model;

/* ---------------------------------------------------------------- context */
int ace_abi_version(void);
/* Creates a context on HIP device `device` (one process per GPU).  It owns
 * up to three non-blocking HIP streams (ACE_STREAMS = 3, 2 or 1; results are
 * bit-identical for every value) and never uses the null stream. */
int ace_create(int device, ace_ctx **out);
void ace_destroy(ace_ctx *ctx);
/* Message of the last failure on this context ("" if none).  NULL ctx gives
 * the message of the last failed ace_create in this process. */
const char *ace_last_error(const ace_ctx *ctx);
/* Optional interrupt poll (the reference calls Rcpp::checkUserInterrupt() in
 * its row loops, src/kernel_SE_cpp.cpp): poll(user) is called between
 * iterations of ace_model_train and before every ace_model_para_update; a
 * non-zero return stops the call with ACE_ERR_INTERRUPTED (the R shim maps
 * it to R's interrupt).  poll == NULL removes it.  On a model sharded over
 * RCCL the ranks' poll results are OR-ed by a one-double all-reduce before
 * every para_update (ranks without a poll vote 0), so all ranks stop before
 * the same evaluation and none is left inside a collective. */
int ace_set_interrupt_poll(ace_ctx *ctx, int (*poll)(void *user), void *user);

/* ------------------------------------------------ Rcpp-export equivalents */

/* kernmat_SE_cpp / kernmat_Matern32_cpp (src/kernel_SE_cpp.cpp:9-64,
 * src/kernel_Matern_cpp.cpp:52-93).  X1 n1 x p, X2 n2 x p, Z1 n1 x (B-1),
 * Z2 n2 x (B-1), theta P = 2 + B(p+1).  Writes Kfull (n1 x n2, list item
 * `full`) and, if Kel != NULL, the n1 x n2 x B cube (`elements`). */
int ace_kernmat_cross(ace_ctx *ctx, int kind, int64_t n1, int64_t n2, int p,
                      int B, const double *X1, const double *X2,
                      const double *Z1, const double *Z2, const double *theta,
                      double *Kfull, double *Kel);

/* kernmat_SE_symmetric_cpp / kernmat_Matern32_symmetric_cpp
 * (src/kernel_SE_cpp.cpp:67-134, src/kernel_Matern_cpp.cpp:190-240).
 * Kfull n x n (`full`); Kel n x n x B (`elements`) or NULL. */
int ace_kernmat_sym(ace_ctx *ctx, int kind, int64_t n, int p, int B,
                    const double *X, const double *Z, const double *theta,
                    double *Kfull, double *Kel);

/* invkernel_cpp (src/kernel_SE_cpp.cpp:137-157).  A = K + exp(sigma) I.
 * inv (n x n) = A^-1.  `eigenval` (n) receives the pivots of A's
 * symmetric elimination (Cholesky diagonal squared) instead of A's
 * eigenvalues: every consumer in the reference only uses sum(log(eigenval))
 * (src/kernel_SE_cpp.cpp:240, src/kernel_Matern_cpp.cpp:463,
 * src/stats_cpp.cpp:29), and sum(log(pivots)) == log det A.
 * Either output pointer may be NULL. */
int ace_invkernel(ace_ctx *ctx, int64_t n, const double *K, double sigma,
                  double *eigenval, double *inv);

/* grad_SE_cpp / grad_Matern_cpp (src/kernel_SE_cpp.cpp:192-243,
 * src/kernel_Matern_cpp.cpp:420-467).  Kel (n x n x B) may be NULL: the
 * engine then recomputes the slices from X, Z, theta on the device (the R6
 * caller always passes the cube of the same theta).  stats (2) is in/out:
 * stats[0] = RMSE, stats[1] = log evidence.  grad receives P values. */
int ace_grad(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *y,
             const double *X, const double *Z, const double *Kfull,
             const double *Kel, const double *inv, const double *eigenval,
             const double *theta, double *stats, double std_y, double *grad);

/* stats_cpp (src/stats_cpp.cpp:9-32): out[0] = RMSE, out[1] = log evidence. */
int ace_stats(ace_ctx *ctx, int64_t n, const double *y, const double *Kmat,
              const double *inv, const double *eigenval, double mu,
              double std_y, double *out);

/* mu_solution_cpp (src/utilities_cpp.cpp:6-10). */
int ace_mu_solution(ace_ctx *ctx, int64_t n, const double *y,
                    const double *inv, double *out);

/* pred_cpp (src/pred_cpp.cpp:8-34).  nX training rows, nx test rows.
 * K_xX nx x nX, K_xx nx x nx.  map (nx), ci (nx x 2), var (nx). */
int ace_pred(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X,
             double sigma, double mu, const double *invK_XX,
             const double *K_xX, const double *K_xx, double mean_y,
             double std_y, double *map, double *ci, double *var);

/* pred_marginal_cpp (src/pred_cpp.cpp:37-126).  K_xX nx x nX x B,
 * K_xx nx x nx x B.  When calculate_ate != 0, `avg` (12) receives
 * [ate.map, ate.ci0, ate.ci1, ate.var, att.map, att.ci0, att.ci1, att.var,
 *  atu.map, atu.ci0, atu.ci1, atu.var]; otherwise avg may be NULL. */
int ace_pred_marginal(ace_ctx *ctx, int64_t nX, int64_t nx, int B,
                      const double *y_X, const double *Z_x, double sigma,
                      double mu, const double *invK_XX, const double *K_xX,
                      const double *K_xx, double mean_y, double std_y,
                      double std_Z, int calculate_ate, double *map, double *ci,
                      double *var, double *avg);

/* ------------------------------- device-matrix handles (unchanged R6 flow)
 *
 * The R6 kernel classes keep Kmat, Karray and invKmatn as R objects and
 * pass them between the routines above on every para_update
 * (R/kernel_SE_R6.R:26-50; predict: :75-97).  The *_dev variants keep
 * those objects in HBM as ace_dmat handles; the R shim wraps a handle in an
 * ALTREP double vector that is materialised only when R reads its values
 * (INTEGRATION.md), so the unchanged R6 code moves no n x n matrix and no
 * n x n x B cube.  Semantics, argument order and outputs are those of the
 * host-buffer routine of the same name.
 *   kernmat_*_dev: *full is a device n1 x n2 matrix; *elements (optional) is
 *     VIRTUAL: X, Z and theta are recorded and slices (or pred_marginal's
 *     slice sums) are assembled only when read or consumed.
 *   invkernel_dev: *inv is the sweep's device result (never symmetrised or
 *     copied unless read); eigenval (n, host) receives the pivots.
 *   grad_dev / stats_dev: RMSE from the explicit residual ybar - Kfull alpha
 *     (src/kernel_SE_cpp.cpp:238), like the host-buffer routines.
 * Handles belong to the context that made them; ace_dmat_free releases one. */
typedef struct ace_dmat ace_dmat;
int ace_dmat_upload(ace_ctx *ctx, int64_t rows, int64_t cols, int64_t slices,
                    const double *host, ace_dmat **out);
int ace_dmat_dims(const ace_dmat *h, int64_t *rows, int64_t *cols, int64_t *slices);
/* count doubles from column-major linear index offset (materialises a
 * virtual cube / the symmetric inverse on the device on first read) */
int ace_dmat_read(const ace_dmat *h, int64_t offset, int64_t count, double *out);
/* bit 0: full values exist on the device; bit 1: values were read to the host */
int ace_dmat_materialized(const ace_dmat *h);
void ace_dmat_free(ace_dmat *h);
int ace_kernmat_sym_dev(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *X,
                        const double *Z, const double *theta, ace_dmat **full,
                        ace_dmat **elements);
int ace_kernmat_cross_dev(ace_ctx *ctx, int kind, int64_t n1, int64_t n2, int p, int B,
                          const double *X1, const double *X2, const double *Z1, const double *Z2,
                          const double *theta, ace_dmat **full, ace_dmat **elements);
int ace_invkernel_dev(ace_ctx *ctx, const ace_dmat *K, double sigma, double *eigenval,
                      ace_dmat **inv);
int ace_mu_solution_dev(ace_ctx *ctx, int64_t n, const double *y, const ace_dmat *inv,
                        double *out);
int ace_stats_dev(ace_ctx *ctx, int64_t n, const double *y, const ace_dmat *Kmat,
                  const ace_dmat *inv, const double *eigenval, double mu, double std_y,
                  double *out);
int ace_grad_dev(ace_ctx *ctx, int kind, int64_t n, int p, int B, const double *y,
                 const double *X, const double *Z, const ace_dmat *Kfull, const ace_dmat *Kel,
                 const ace_dmat *inv, const double *eigenval, const double *theta, double *stats,
                 double std_y, double *grad);
int ace_pred_dev(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X, double sigma, double mu,
                 const ace_dmat *invK_XX, const ace_dmat *K_xX, const ace_dmat *K_xx,
                 double mean_y, double std_y, double *map, double *ci, double *var);
int ace_pred_marginal_dev(ace_ctx *ctx, int64_t nX, int64_t nx, const double *y_X,
                          const double *Z_x, double sigma, double mu, const ace_dmat *invK_XX,
                          const ace_dmat *K_xX, const ace_dmat *K_xx, double mean_y, double std_y,
                          double std_Z, int calculate_ate, double *map, double *ci, double *var,
                          double *avg);

/* ---------------------------------------------- host-only (no GPU, no ctx) */

/* Nesterov_cpp / Nadam_cpp / Adam_cpp (src/optimizer_cpp.cpp:8-63).  All
 * vectors are P long and mutated in place; the return value is the
 * reference's bool: 1 if every gradient is finite, else 0.  Ascent (Q8). */
int ace_nesterov(int64_t P, double learn_rate, double momentum, double *nu,
                 const double *grad, double *para);
int ace_nadam(int64_t P, double iter, double learn_rate, double beta1,
              double beta2, double eps, double *m, double *v,
              const double *grad, double *para);
int ace_adam(int64_t P, double iter, double learn_rate, double beta1,
             double beta2, double eps, double *m, double *v,
             const double *grad, double *para);

/* norm_clip_cpp (src/utilities_cpp.cpp:121-129), in place.  Q5: rescales
 * to unit norm (not to max_length) when ||grads|| > max_length. */
void ace_norm_clip(int flag, int64_t P, double *grads, double max_length);

/* ncs_basis / ncs_basis_deriv (src/ncs_basis_cpp.cpp:61-99).  knots are
 * de-duplicated and sorted; design must hold n x (#unique knots) doubles;
 * *ncols receives #unique knots. */
int ace_ncs_basis(int64_t n, const double *x, int64_t nknots,
                  const double *knots, double *design, int64_t *ncols);
int ace_ncs_basis_deriv(int64_t n, const double *x, int64_t nknots,
                        const double *knots, double *design, int64_t *ncols);

/* normalize_train (src/utilities_cpp.cpp:13-104): in place on y (n),
 * X (n x px), Z (n x pz); moments is (1+px+pz) x 3 column-major.
 * normalize_test (src/utilities_cpp.cpp:108-118): in place on X, Z. */
int ace_normalize_train(int64_t n, int px, int pz, double *y, double *X,
                        double *Z, double *moments);
int ace_normalize_test(int64_t n, int px, int pz, double *X, double *Z,
                       const double *moments, int64_t moment_rows);

/* ------------------------------- device-resident hot path (one model fit)
 *
 * The R6 kernel classes ship Kmat, the n x n x B cube and invKmatn through
 * R on every iteration (R/kernel_SE_R6.R:26-39, 47-50).  The model below
 * keeps X, Z, y, the swept matrix and the training inverse resident in HBM
 * and never materialises the cube: one ace_model_para_update() is the
 * native work of one para_update (R/kernel_SE_R6.R:40-62,
 * R/kernel_Matern32_R6.R:39-60) -- kernel assembly, factorisation +
 * inverse + log-determinant, and every gradient and statistic.
 */
int ace_model_create(ace_ctx *ctx, int kind, int64_t n, int p, int B,
                     ace_model **out);
void ace_model_destroy(ace_model *m);
/* Uploads y (n), X (n x p), Z (n x (B-1)) and the std_y moment. */
int ace_model_set_data(ace_model *m, const double *y, const double *X,
                       const double *Z, double std_y);
/* One para_update's native work at theta (P, in/out).  If iter == 1,
 * theta[1] is first overwritten with mu_solution (R/kernel_SE_R6.R:45).
 * grad (P) receives the gradient, stats (2) the RMSE and log evidence,
 * *mu_post the mu_solution of this iteration's inverse, which the caller
 * writes into theta[1] after its optimizer step (R/kernel_SE_R6.R:54).
 * The inverse stays resident for ace_model_predict. */
int ace_model_para_update(ace_model *m, int iter, double *theta, double *grad,
                          double *stats, double *mu_post);
/* get_train_stats (R/kernel_SE_R6.R:63-74): kernel + inverse at theta and
 * stats_cpp with mu = theta[1]; the resident inverse is NOT replaced. */
int ace_model_train_stats(ace_model *m, const double *theta, double *stats);
/* Copies the resident training inverse (n x n) to the host. */
int ace_model_get_inverse(ace_model *m, double *inv);
/* out (n x k) = A^-1 V with the resident inverse of the last para_update,
 * V and out column-major n x k on the host.  The inverse never leaves HBM
 * (sharded: each rank multiplies by the entries it stores, one all-reduce of
 * n x k).  ACE_ERR_ARG before the first para_update. */
int ace_model_apply_inverse(ace_model *m, int64_t k, const double *V, double *out);

/* Device-resident predict (R/kernel_SE_R6.R:75-83 -> pred_cpp,
 * src/pred_cpp.cpp:8-34): kernels at `theta` (P, the caller's current
 * parameters), inverse = the resident one of the last para_update (Q6: the
 * R6 invKmatn).  X2 nx x p, Z2 nx x (B-1) column-major (the test basis).
 * map (nx), ci (nx x 2), var (nx) as pred_cpp's list.  K_xX is assembled
 * on the device, only diag(K_xx) is formed; nothing n x n crosses PCIe.
 * Single GPU: diag(K_xX A^-1 K_xX^T) through the strictly lower triangle of
 * A^-1 (half the flops of the full product) and K_xX A^-1 (y - mu) from the
 * sweep's augmented rows; results equal the full-product form up to
 * rounding (ACE_PRED_TRI=0 selects it). */
int ace_model_predict(ace_model *m, const double *theta, int64_t nx, const double *X2,
                      const double *Z2, double mean_y, double std_y, double *map, double *ci,
                      double *var);
/* Device-resident predict_marginal (R/kernel_SE_R6.R:84-97 ->
 * pred_marginal_cpp, src/pred_cpp.cpp:37-126): the marginal kernels are the
 * slice sums b >= 1 (slice 0 if B == 1) of the cross / test kernels built
 * with dZ2 (nx x (B-1), the basis derivative at the test treatments).
 * Z_x (nx) is the treatment column the reference receives as Z2; it is read
 * only when calculate_ate != 0.  avg (12) as ace_pred_marginal. */
int ace_model_predict_marginal(ace_model *m, const double *theta, int64_t nx, const double *X2,
                               const double *dZ2, const double *Z_x, double std_y, double std_Z,
                               int calculate_ate, double *map, double *ci, double *var,
                               double *avg);
/* Per-kernel device timing for the roofline report: when enabled, HIP
 * events bracket every launch of the dense update kernel (`which` = 0),
 * the assembly kernel (1) and the gradient kernel (2) on the model's
 * stream.  *ms = summed duration, *launches = count, *work = algorithmic
 * flops issued by those launches.  `which` = 3: the
 * sweep's span per evaluation (first bulk update launch start to the last
 * one's end) with every update / cross / panel-GEMM flop of the sweep as
 * its work (unsharded models); 4: from the end of the assembly's main
 * launch to the first bulk update launch's start (unsharded); 5: the
 * evaluation's device span, assembly start to gradient end.  Enabling resets the
 * counters.  An evaluation's events are read back while the next one runs
 * (no host queries between evaluations); ace_model_kernel_time reads the
 * last timed evaluation's set first, so its totals cover every timed
 * evaluation. */
int ace_model_profile(ace_model *m, int enable);
int ace_model_kernel_time(ace_model *m, int which, double *ms,
                          int64_t *launches, double *work);

/* The whole ace.train optimisation loop (R/main_ace.R:213-235) in native
 * code, with no per-iteration round trip through the host language:
 *   for iter = 1..maxiter:
 *     para_update (R/kernel_SE_R6.R:40-62): kernel, inverse, gradient, stats,
 *       theta[1] <- mu_solution at iter 1;
 *     norm clip (Q5, src/utilities_cpp.cpp:121-129), optimizer step (Q8,
 *       src/optimizer_cpp.cpp:8-63), theta[1] <- mu_solution (Q4);
 *     stop when |Delta log evidence| < tol and iter > 3;
 *   then get_train_stats at the final theta (R/kernel_SE_R6.R:63-74).
 * optimizer: ACE_OPT_NESTEROV (also "GD" with momentum 0), ACE_OPT_ADAM,
 * ACE_OPT_NADAM; eps = 1e-8 as in R/optimizer_classes.R.  theta (P) in/out.
 * stats: 2 x (maxiter + 2) column-major, zero-filled like the R matrix;
 * column j (1..iter) holds [RMSE, log evidence] of iteration j and column
 * iter + 1 the final train stats.  *iters = iterations run, *converged =
 * (iter < maxiter).  A non-finite gradient returns ACE_ERR_NONFINITE (the
 * optimizer classes' stop(), R/optimizer_classes.R:26-29) with theta and
 * stats as of that iteration.  Works on sharded models (collective). */
enum ace_optimizer { ACE_OPT_NESTEROV = 0, ACE_OPT_ADAM = 1, ACE_OPT_NADAM = 2 };
int ace_model_train(ace_model *m, int optimizer, double learn_rate,
                    double momentum, double beta1, double beta2, int norm_clip,
                    double clip_at, int maxiter, double tol, double *theta,
                    double *stats, int *iters, int *converged);

/* ------------------------------- multi-GPU: block-column-sharded model
 *
 * For n beyond what one evaluation should spend on one GPU (SURVEY.md §8e,
 * configs C3/C4).  The reference has no multi-process path (one R process,
 * BLAS threads only); this is the scale-out of the same para_update.
 * A is distributed by NB = 256-wide column blocks, block-cyclic over the
 * `world` ranks (block j on rank j % world), one process per GPU.  Each
 * sweep step broadcasts the pivot block's column panel from its owner and
 * all-gathers the panel's row pieces (RCCL over xGMI); assembly, update and
 * gradient work only on the rank's own columns; one all-reduce per
 * evaluation combines the swept [y; 1] rows (alpha, mu) and a second one the
 * gradient partial sums (the RMSE residual is sig * alpha, so no Kfull*alpha
 * pass exists).  Every rank returns identical grad / stats.
 *
 * Bootstrap: rank 0 calls ace_comm_unique_id() and sends the 128 bytes to
 * every rank out of band (MPI, torch.distributed, a file); each rank then
 * calls ace_model_create_sharded() with the same id (blocks until all
 * `world` ranks have joined).  With id == NULL all `world` ranks are
 * simulated inside this process on ctx's device and the exchanges are
 * device copies: the validation mode the single-GPU tests use.
 * The returned model takes every ace_model_* call above; calls are
 * collective (every rank makes the same sequence of calls). */
#define ACE_UNIQUE_ID_BYTES 128
int ace_comm_unique_id(unsigned char *id);
int ace_model_create_sharded(ace_ctx *ctx, int kind, int64_t n, int p, int B,
                             int world, int rank, const unsigned char *id,
                             ace_model **out);
/* world / rank of a model (1 / 0 for ace_model_create models) */
int ace_model_shard_info(const ace_model *m, int *world, int *rank);

/* Collectives this rank has issued since the model was created, by kind
 * (counts[ACE_COMM_KINDS]): RCCL calls of an ace_model_create_sharded model
 * -- at every world size, 1 included -- or host callbacks of an
 * ace_model_create_sharded_host model.  ACE_COMM_GROUPS counts the RCCL
 * ncclGroupStart/End launches (a sweep step's broadcast + all-gather).
 * Simulated groups (id == NULL) and single-GPU models issue none.  Per
 * evaluation of the head / tail sweep over S = ceil(n / 256) steps: 2 S
 * broadcasts, the all-gathers of steps with row pieces, 2 all-reduces plus
 * the interrupt vote; creation adds RCCL's warm-up calls. */
enum ace_comm_kind {
  ACE_COMM_BROADCAST = 0,
  ACE_COMM_ALLGATHER = 1,
  ACE_COMM_ALLREDUCE = 2,
  ACE_COMM_GROUPS = 3,
  ACE_COMM_KINDS = 4
};
int ace_model_comm_calls(const ace_model *m, int64_t *counts);

/* Host-callback collectives: the same sharded model with every exchange
 * (panel broadcast + all-gather per sweep step, the two all-reduces per
 * evaluation, the interrupt vote, the inverse gather) routed through
 * caller-supplied functions on HOST buffers -- the library stages device ->
 * host, calls, and copies back.  One process per rank with its own ace_ctx
 * (any devices, also one shared GPU); for validating the per-process
 * packing / ownership logic over a CPU transport such as gloo (not a
 * performance path: every step synchronises).  Callbacks return 0 on
 * success; op of allreduce: 0 = sum, 1 = max.  allgather: recv holds
 * world x count doubles, rank r's block at r * count. */
typedef struct ace_comm_ops {
  void *user;
  int (*broadcast)(void *user, double *buf, int64_t count, int root);
  int (*allgather)(void *user, const double *send, double *recv, int64_t count);
  int (*allreduce)(void *user, double *buf, int64_t count, int op);
} ace_comm_ops;
int ace_model_create_sharded_host(ace_ctx *ctx, int kind, int64_t n, int p, int B,
                                  int world, int rank, const ace_comm_ops *ops,
                                  ace_model **out);

#ifdef __cplusplus
}
#endif

#endif /* ACE_HIP_H */
