/*
 * ace_ref.c -- literal single-threaded C restatement of the reference's
 * native loops (ace 0.4.1).  TEST INFRASTRUCTURE ONLY: used by tests/ as an
 * independent cross-check of oracle/ace_oracle.py and by bench.py's
 * cpu_baseline leg (timed, never shipped).  PARITY UNPINNED (see
 * oracle/ace_oracle.py header and DESIGN.md: the reference cannot be built
 * here and holds no golden vectors).
 *
 * Layout: Armadillo/R column-major.  X is n x p (X[r + i*n]); Z is
 * n x (B-1); matrices n x n; the cube is n x n x B (slice-major).
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, like R's default flags:
 * no FMA contraction, so the products and sums round as the reference's).
 *
 * The packed-triangle loop order, the in-loop exp and the per-(i,b) trace
 * passes are kept on purpose: this is also the CPU baseline timing.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define SQRT3 1.7320508075688772 /* sqrt(3) promoted to double */

static double sgn(double x) { return (double)((0 < x) - (x < 0)); }

/* uppertri2symmat (src/include/ace_kernel_utils.hpp:7-20) */
static void unpack_upper(const double *vec, int64_t n, double *out) {
  int64_t cnt = 0;
  for (int64_t r = 0; r < n; r++)
    for (int64_t c = r; c < n; c++) {
      out[r + c * n] = vec[cnt];
      out[c + r * n] = vec[cnt];
      cnt++;
    }
}

/* kernmat_{SE,Matern32}_symmetric_cpp: src/kernel_SE_cpp.cpp:67-134,
 * src/kernel_Matern_cpp.cpp:190-240.  kind 0 = SE, 1 = Matern32.
 * Kel may be NULL (then only Kfull is produced).  Returns 0 / -1 (OOM). */
int ref_kernmat_sym(int kind, int64_t n, int p, int B, const double *X,
                    const double *Z, const double *theta, double *Kfull,
                    double *Kel) {
  int64_t np = n * (n + 1) / 2;
  double *tmpX = (double *)calloc((size_t)(np * B), sizeof(double));
  if (!tmpX) return -1;
  for (int i = 0; i < p; i++) {
    int64_t cnt = 0;
    for (int64_t r = 0; r < n; r++)
      for (int64_t c = r; c < n; c++) {
        double d = X[r + i * n] - X[c + i * n];
        double tmp = d * d;
        for (int b = 0; b < B; b++)
          tmpX[cnt + b * np] += tmp * exp(-theta[1 + b + B * (i + 1)]);
        cnt++;
      }
  }
  if (kind == 1)
    for (int64_t j = 0; j < np * B; j++) tmpX[j] = sqrt(tmpX[j]);
  /* slice 0 */
  for (int64_t j = 0; j < np; j++) {
    double t = tmpX[j];
    tmpX[j] = (kind == 0) ? exp(theta[2] - t)
                          : (1 + SQRT3 * t) * exp(theta[2] - SQRT3 * t);
  }
  if (Kel) unpack_upper(tmpX, n, Kel);
  for (int b = 1; b < B; b++) {
    double *col = tmpX + b * np;
    const double *zb = Z + (int64_t)(b - 1) * n;
    int64_t cnt = 0;
    for (int64_t r = 0; r < n; r++) {
      if (zb[r] == 0) {
        for (int64_t c = r; c < n; c++) col[cnt++] = 0;
        continue;
      }
      for (int64_t c = r; c < n; c++) {
        double t = col[cnt];
        if (kind == 0) {
          if (zb[c] == 0)
            col[cnt] = 0;
          else
            col[cnt] = (sgn(zb[r]) * sgn(zb[c])) *
                       exp(theta[2 + b] - t + log(fabs(zb[r])) + log(fabs(zb[c])));
        } else {
          col[cnt] = (1 + SQRT3 * t) * exp(theta[2 + b] - SQRT3 * t) * zb[r] * zb[c];
        }
        cnt++;
      }
    }
    if (Kel) unpack_upper(col, n, Kel + (int64_t)b * n * n);
    for (int64_t j = 0; j < np; j++) tmpX[j] += col[j];
  }
  unpack_upper(tmpX, n, Kfull);
  free(tmpX);
  return 0;
}

/* kernmat_{SE,Matern32}_cpp (cross): src/kernel_SE_cpp.cpp:9-64,
 * src/kernel_Matern_cpp.cpp:52-93.  X1 n1 x p, X2 n2 x p, Z1 n1 x (B-1),
 * Z2 n2 x (B-1).  Kel (n1 x n2 x B) may be NULL. */
int ref_kernmat_cross(int kind, int64_t n1, int64_t n2, int p, int B,
                      const double *X1, const double *X2, const double *Z1,
                      const double *Z2, const double *theta, double *Kfull,
                      double *Kel) {
  int64_t nn = n1 * n2;
  double *cube = Kel ? Kel : (double *)malloc((size_t)(nn * B) * sizeof(double));
  if (!cube) return -1;
  memset(cube, 0, (size_t)(nn * B) * sizeof(double));
  for (int i = 0; i < p; i++)
    for (int64_t r = 0; r < n1; r++)
      for (int b = 0; b < B; b++) {
        double e = exp(-theta[1 + b + B * (i + 1)]);
        for (int64_t c = 0; c < n2; c++) {
          double d = X1[r + i * n1] - X2[c + i * n2];
          cube[r + c * n1 + b * nn] += (d * d) * e;
        }
      }
  if (kind == 1)
    for (int64_t j = 0; j < nn * B; j++) cube[j] = sqrt(cube[j]);
  for (int64_t j = 0; j < nn; j++) {
    double t = cube[j];
    cube[j] = (kind == 0) ? exp(theta[2] - t)
                          : (1 + SQRT3 * t) * exp(theta[2] - SQRT3 * t);
    Kfull[j] = cube[j];
  }
  for (int b = 1; b < B; b++) {
    double *sl = cube + b * nn;
    const double *z1 = Z1 + (int64_t)(b - 1) * n1;
    const double *z2 = Z2 + (int64_t)(b - 1) * n2;
    for (int64_t r = 0; r < n1; r++) {
      for (int64_t c = 0; c < n2; c++) {
        double t = sl[r + c * n1];
        double v;
        if (z1[r] == 0 || z2[c] == 0)
          v = 0;
        else if (kind == 0)
          v = (sgn(z1[r]) * sgn(z2[c])) *
              exp(theta[2 + b] - t + log(fabs(z1[r])) + log(fabs(z2[c])));
        else
          v = (1 + SQRT3 * t) * exp(theta[2 + b] - SQRT3 * t) * z1[r] * z2[c];
        sl[r + c * n1] = v;
      }
    }
    for (int64_t j = 0; j < nn; j++) Kfull[j] += sl[j];
  }
  if (!Kel) free(cube);
  return 0;
}

/* grad_SE_cpp / grad_Matern_cpp: src/kernel_SE_cpp.cpp:161-243 and
 * src/kernel_Matern_cpp.cpp:340-467.  `logdet` = sum(log(eigenval)).
 * Kel is the n x n x B cube.  stats[0..1] written in place. */
int ref_grad(int kind, int64_t n, int p, int B, const double *y,
             const double *X, const double *Kfull, const double *Kel,
             const double *inv, double logdet, const double *theta,
             double *stats, double std_y, double *grad) {
  int P = 2 + B * (p + 1);
  double *ybar = (double *)malloc(n * sizeof(double));
  double *alpha = (double *)malloc(n * sizeof(double));
  double *T = (double *)malloc((size_t)(n * n) * sizeof(double));
  double *D2 = (double *)malloc((size_t)(n * n) * sizeof(double));
  double *F = NULL;
  if (!ybar || !alpha || !T || !D2) return -1;
  for (int j = 0; j < P; j++) grad[j] = 0;
  for (int64_t r = 0; r < n; r++) ybar[r] = y[r] - theta[1];
  for (int64_t r = 0; r < n; r++) {
    double s = 0;
    for (int64_t c = 0; c < n; c++) s += inv[r + c * n] * ybar[c];
    alpha[r] = s;
  }
  for (int64_t c = 0; c < n; c++)
    for (int64_t r = 0; r < n; r++) T[r + c * n] = inv[r + c * n] - alpha[r] * alpha[c];
  /* sigma */
  double tr = 0;
  for (int64_t r = 0; r < n; r++) tr += T[r + r * n];
  grad[0] = -0.5 * tr * exp(theta[0]);
  /* lambda: -0.5 trace(T K_b) */
  for (int b = 0; b < B; b++) {
    const double *Kb = Kel + (int64_t)b * n * n;
    double s = 0;
    for (int64_t c = 0; c < n; c++)
      for (int64_t r = 0; r < n; r++) s += T[r + c * n] * Kb[c + r * n];
    grad[2 + b] = -0.5 * s;
  }
  if (kind == 1) {
    /* evid_scale_Matern32_gradients: cube of gradient-indexed distances */
    F = (double *)calloc((size_t)(n * n * B), sizeof(double));
    if (!F) return -1;
    for (int i = 0; i < p; i++)
      for (int64_t r = 0; r < n; r++)
        for (int b = 0; b < B; b++) {
          double e = exp(-theta[2 + B + b + B * i]);
          for (int64_t c = 0; c < n; c++) {
            double d = X[r + i * n] - X[c + i * n];
            F[r + c * n + (int64_t)b * n * n] += (d * d) * e;
          }
        }
    for (int b = 0; b < B; b++)
      for (int64_t j = 0; j < n * n; j++) {
        int64_t o = j + (int64_t)b * n * n;
        F[o] = Kel[o] / (1 + sqrt(3 * F[o]));
      }
  }
  for (int i = 0; i < p; i++) {
    for (int64_t r = 0; r < n; r++)
      for (int64_t c = 0; c < n; c++) {
        double d = X[r + i * n] - X[c + i * n];
        D2[c + r * n] = d * d;
      }
    for (int b = 0; b < B; b++) {
      double L = theta[2 + B + b + B * i];
      const double *Kb = (kind == 0 ? Kel : F) + (int64_t)b * n * n;
      double s = 0;
      if (kind == 0) {
        double e = exp(-L);
        for (int64_t c = 0; c < n; c++)
          for (int64_t r = 0; r < n; r++)
            s += T[r + c * n] * ((Kb[c + r * n] * D2[c + r * n]) * e);
        grad[2 + B + b + B * i] = -0.5 * s;
      } else {
        for (int64_t c = 0; c < n; c++)
          for (int64_t r = 0; r < n; r++) s += T[r + c * n] * (Kb[c + r * n] * D2[c + r * n]);
        grad[2 + B + b + B * i] = -0.25 * 9 * s * exp(-L);
      }
    }
  }
  if (kind == 0) {
    double s = 0;
    for (int64_t r = 0; r < n; r++) s += alpha[r];
    grad[1] = s;
  }
  /* stats (in place) */
  double ss = 0, ya = 0;
  for (int64_t r = 0; r < n; r++) {
    double kr = 0;
    for (int64_t c = 0; c < n; c++) kr += Kfull[r + c * n] * alpha[c];
    double e = ybar[r] - kr;
    ss += e * e;
    ya += y[r] * alpha[r];
  }
  stats[0] = std_y * sqrt(ss) / sqrt((double)n);
  stats[1] = -0.5 * (n * log(2.0 * M_PI) + logdet + ya);
  free(ybar);
  free(alpha);
  free(T);
  free(D2);
  free(F);
  return 0;
}

/* mu_solution_cpp: src/utilities_cpp.cpp:6-10 (Q4) */
double ref_mu_solution(int64_t n, const double *y, const double *inv) {
  double s = 0, a = 0;
  for (int64_t r = 0; r < n; r++) {
    double t = 0;
    for (int64_t c = 0; c < n; c++) {
      t += inv[r + c * n] * y[c];
      a += inv[r + c * n];
    }
    s += t;
  }
  return 0.5 * s / a;
}
