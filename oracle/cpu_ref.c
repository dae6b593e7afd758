/* cpu_ref.c -- CPU restatement of the PPLS_simult EM iteration -- TEST INFRASTRUCTURE ONLY.
 *
 * Used (a) as the timed CPU baseline of bench.py (cpu_baseline.kind = "port") and (b) as a second
 * oracle beside oracle/ppls_oracle.py.  The product never links it.
 *
 * It keeps the reference's pass structure over the data (paths relative to /root/reference):
 *   pass 1  Xw = X W, Yc = Y C, mu_T, mu_U, crossprods       Package/PPLS/R/EM_W_multi.R:689-701
 *   pass 2  ssq(mu_E), ssq(mu_F), streamed row by row         EM_W_multi.R:703-709 (R materialises)
 *   pass 3  X' mu_T, Y' mu_U                                  EM_W_multi.R:732-733
 *   pass 4  loglC_fast: X W, Y C, ||X||^2, ||Y||^2 (every call) src/loglC.cpp:318-338
 * with the coefficient block of EM_W_multi.R:670-686 / :312-320, Chh :711-712, the M-step scalars
 * :734-738 and orth(type="SVD") = U V' by Householder QR + one-sided Jacobi (OmicsPLS::orth,
 * semantics Package/functions.R:252-260).  Row-major X (n x p), Y (n x q); W, C column-major.
 * OpenMP over rows (static schedule); every thread accumulates its own partial sums, which are
 * then added in thread-index order: the result is deterministic for a fixed thread count.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define RM 16

#ifdef _OPENMP
static int max_threads(void) { return omp_get_max_threads(); }
static int thread_id(void) { return omp_get_thread_num(); }
#else
static int max_threads(void) { return 1; }
static int thread_id(void) { return 0; }
#endif

/* part[T][len] -> out[len]: the per-thread partials summed in thread-index order */
static void sum_ordered(const double* part, int T, int len, double* out) {
  for (int j = 0; j < len; ++j) out[j] = 0.0;
  for (int t = 0; t < T; ++t)
    for (int j = 0; j < len; ++j) out[j] += part[(size_t)t * len + j];
}

static void coef_estep(double t, double b, double sE, double sF, double sH, double* c1, double* c2,
                       double* c3, double* Kc_out, int logl_variant) {
  const double t2 = t * t, t4 = t2 * t2, t6 = t4 * t2, b2 = b * b, sE2 = sE * sE, sF2 = sF * sF;
  double g = t2 * b2 + sH * sH;
  if (logl_variant) { double gs = sqrt(g); g = gs * gs; }   /* logl_W :312 takes sqrt then squares */
  const double Kw = t2 - t4 * b2 / sF2 + t4 * b2 * g / (sF2 * (g + sF2));
  const double Kc = g - t4 * b2 / sE2 + t6 * b2 / (sE2 * (t2 + sE2));
  const double Kwc = t2 * b / (sE2 * sF2) - Kc * t2 * b / (sE2 * sF2 * (Kc + sF2)) -
                     t4 * b / (sE2 * sF2 * (t2 + sE2)) + Kc * t4 * b / (sE2 * sF2 * (Kc + sF2) * (t2 + sE2));
  *c1 = Kw / (sE2 * (Kw + sE2));
  *c3 = Kc / (sF2 * (Kc + sF2));
  *c2 = Kwc;
  if (Kc_out) *Kc_out = Kc;
}

/* U V' of the p x r matrix S (column-major), Householder QR + Jacobi on R. */
static int polar(const double* S, int p, int r, double* out) {
  double* A = (double*)malloc(sizeof(double) * p * r);
  double* E = (double*)calloc((size_t)p * r, sizeof(double));
  double vtv[RM], R[RM * RM], V[RM * RM], Ac[RM * RM], sv[RM];
  memcpy(A, S, sizeof(double) * p * r);
  memset(R, 0, sizeof R);
  for (int k = 0; k < r; ++k) {
    double s2 = 0;
    for (int i = k; i < p; ++i) s2 += A[k * p + i] * A[k * p + i];
    const double sig = sqrt(s2), akk = A[k * p + k], alpha = akk >= 0 ? -sig : sig;
    if (!(sig > 0)) { free(A); free(E); return -1; }
    vtv[k] = 2 * sig * (sig + fabs(akk));
    A[k * p + k] = akk - alpha;
    R[k * r + k] = alpha;
    for (int j = k + 1; j < r; ++j) {
      double d = 0;
      for (int i = k; i < p; ++i) d += A[k * p + i] * A[j * p + i];
      const double f = 2 * d / vtv[k];
      for (int i = k; i < p; ++i) A[j * p + i] -= f * A[k * p + i];
      R[j * r + k] = A[j * p + k];
    }
  }
  for (int j = 0; j < r; ++j) E[j * p + j] = 1.0;
  for (int k = r - 1; k >= 0; --k)
    for (int j = 0; j < r; ++j) {
      double d = 0;
      for (int i = k; i < p; ++i) d += A[k * p + i] * E[j * p + i];
      const double f = 2 * d / vtv[k];
      for (int i = k; i < p; ++i) E[j * p + i] -= f * A[k * p + i];
    }
  memcpy(Ac, R, sizeof R);
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) V[j * r + i] = i == j;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int i = 0; i < r - 1; ++i)
      for (int j = i + 1; j < r; ++j) {
        double a = 0, b = 0, g = 0;
        for (int k = 0; k < r; ++k) {
          a += Ac[i * r + k] * Ac[i * r + k];
          b += Ac[j * r + k] * Ac[j * r + k];
          g += Ac[i * r + k] * Ac[j * r + k];
        }
        if (g == 0) continue;
        const double rel = fabs(g) / sqrt(a * b);
        if (rel > off) off = rel;
        if (rel < 1e-17) continue;
        const double z = (b - a) / (2 * g), t = (z >= 0 ? 1.0 : -1.0) / (fabs(z) + sqrt(1 + z * z));
        const double c = 1 / sqrt(1 + t * t), s = c * t;
        for (int k = 0; k < r; ++k) {
          const double x = Ac[i * r + k], y = Ac[j * r + k];
          Ac[i * r + k] = c * x - s * y;
          Ac[j * r + k] = s * x + c * y;
          const double vx = V[i * r + k], vy = V[j * r + k];
          V[i * r + k] = c * vx - s * vy;
          V[j * r + k] = s * vx + c * vy;
        }
      }
    if (off < 1e-15) break;
  }
  for (int i = 0; i < r; ++i) {
    double nr = 0;
    for (int k = 0; k < r; ++k) nr += Ac[i * r + k] * Ac[i * r + k];
    sv[i] = sqrt(nr);
    for (int k = 0; k < r; ++k) Ac[i * r + k] /= sv[i];
  }
  double P[RM * RM];
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) {
      double a = 0;
      for (int k = 0; k < r; ++k) a += Ac[k * r + i] * V[k * r + j];
      P[j * r + i] = a;
    }
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < p; ++i) {
      double a = 0;
      for (int k = 0; k < r; ++k) a += E[k * p + i] * P[j * r + k];
      out[j * p + i] = a;
    }
  free(A);
  free(E);
  return 0;
}

/* loglC_fast, src/loglC.cpp:318-338, over (row-major) data. */
static double loglc(const double* X, const double* Y, int64_t n, int p, int q, int r, const double* W,
                    const double* C, double sE, double sF, double sH, const double* b, const double* t) {
  double c1[RM], c2[RM], c3[RM], Kc[RM];
  for (int k = 0; k < r; ++k) coef_estep(t[k], b[k], sE, sF, sH, &c1[k], &c2[k], &c3[k], &Kc[k], 1);
  const double sX2 = sE * sE, sY2 = sF * sF;
  double a1 = 0, a2 = 0;
  for (int k = 0; k < r; ++k) { a1 += log(sX2 + t[k] * t[k]); a2 += log(sY2 + Kc[k]); }
  const double logdet = a1 + (p - r) * log(sX2) + a2 + (q - r) * log(sY2);
  const int T = max_threads();
  double* part = (double*)calloc((size_t)T * 3, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double ssx = 0, ssy = 0, quad = 0;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double* x = X + i * p;
      const double* y = Y + i * q;
      double xw[RM] = {0}, yc[RM] = {0}, sx = 0, sy = 0;
      for (int j = 0; j < p; ++j) {
        sx += x[j] * x[j];
        for (int k = 0; k < r; ++k) xw[k] += x[j] * W[k * p + j];
      }
      for (int j = 0; j < q; ++j) {
        sy += y[j] * y[j];
        for (int k = 0; k < r; ++k) yc[k] += y[j] * C[k * q + j];
      }
      ssx += sx;
      ssy += sy;
      for (int k = 0; k < r; ++k) quad += c1[k] * xw[k] * xw[k] + 2 * c2[k] * xw[k] * yc[k] + c3[k] * yc[k] * yc[k];
    }
    double* mine = part + 3 * (size_t)thread_id();
    mine[0] = ssx;
    mine[1] = ssy;
    mine[2] = quad;
  }
  double tot[3];
  sum_ordered(part, T, 3, tot);
  free(part);
  const double ssx = tot[0], ssy = tot[1], quad = tot[2];
  const double traceL = ssx / sX2 + ssy / sY2 - quad;
  return -0.5 * (double)n * (p + q) * log(2 * M_PI) - 0.5 * (double)n * logdet - 0.5 * traceL;
}

/* One EM iteration (Expect_M closed form %>% Maximiz_M, then logl_W) in place on theta.
 * Returns 0 and writes the log-likelihood of the new theta. */
int cpu_ref_em_step(const double* X, const double* Y, int64_t n, int p, int q, int r, double* W, double* C,
                    double* b, double* t, double* sig /* sE, sF, sH */, double* loglik, int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  if (r < 1 || r > RM) return -1;
  const double sE = sig[0], sF = sig[1], sH = sig[2];
  const double sE2 = sE * sE, sF2 = sF * sF, sH2 = sH * sH;
  double c1[RM], c2[RM], c3[RM], al[RM], be[RM], ga[RM], de[RM];
  for (int k = 0; k < r; ++k) {
    coef_estep(t[k], b[k], sE, sF, sH, &c1[k], &c2[k], &c3[k], 0, 0);
    const double t2 = t[k] * t[k], v = t2 * b[k] * b[k] + sH2;
    al[k] = t2 / sE2 - c1[k] * t2 - c2[k] * t2 * b[k];
    be[k] = t2 * b[k] / sF2 - c2[k] * t2 - c3[k] * b[k] * t2;
    ga[k] = t2 * b[k] / sE2 - c1[k] * t2 * b[k] - c2[k] * v;
    de[k] = v / sF2 - c2[k] * t2 * b[k] - c3[k] * v;
  }
  double* muT = (double*)malloc(sizeof(double) * n * r);
  double* muU = (double*)malloc(sizeof(double) * n * r);
  double* Xw = (double*)malloc(sizeof(double) * n * r);
  double* Yc = (double*)malloc(sizeof(double) * n * r);
  double tt[RM] = {0}, uu[RM] = {0}, ut[RM] = {0}, hh[RM * RM] = {0};   /* uu: Cuu, not used by the M-step */
  (void)uu;
  double h1[RM], h2[RM];
  for (int k = 0; k < r; ++k) { h1[k] = sH2 / sF2 - sH2 * c3[k]; h2[k] = -sH2 * c2[k]; }
  /* pass 1: Xw, Yc, mu_T, mu_U and their crossprods (:689-701), mu_H crossprod (:711-712) */
  const int T = max_threads();
  const int L1 = 3 * RM + RM * RM;
  double* part1 = (double*)calloc((size_t)T * L1, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double* mine = part1 + (size_t)thread_id() * L1;
    double *ltt = mine, *luu = mine + RM, *lut = mine + 2 * RM, *lhh = mine + 3 * RM;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double* x = X + i * p;
      const double* y = Y + i * q;
      double a[RM] = {0}, c[RM] = {0}, h[RM];
      for (int j = 0; j < p; ++j)
        for (int k = 0; k < r; ++k) a[k] += x[j] * W[k * p + j];
      for (int j = 0; j < q; ++j)
        for (int k = 0; k < r; ++k) c[k] += y[j] * C[k * q + j];
      for (int k = 0; k < r; ++k) {
        Xw[i * r + k] = a[k];
        Yc[i * r + k] = c[k];
        const double mt = al[k] * a[k] + be[k] * c[k], mu = ga[k] * a[k] + de[k] * c[k];
        muT[i * r + k] = mt;
        muU[i * r + k] = mu;
        ltt[k] += mt * mt;
        luu[k] += mu * mu;
        lut[k] += mu * mt;
        h[k] = h1[k] * c[k] + h2[k] * a[k];
      }
      for (int k = 0; k < r; ++k)
        for (int l = 0; l < r; ++l) lhh[l * r + k] += h[k] * h[l];
    }
  }
  {
    double tot1[3 * RM + RM * RM];
    sum_ordered(part1, T, L1, tot1);
    for (int k = 0; k < r; ++k) { tt[k] = tot1[k]; uu[k] = tot1[RM + k]; ut[k] = tot1[2 * RM + k]; }
    for (int k = 0; k < r * r; ++k) hh[k] = tot1[3 * RM + k];
    free(part1);
  }
  /* pass 2: ssq(mu_E), ssq(mu_F) streamed (:703-709) */
  double* part2 = (double*)calloc((size_t)T * 2, sizeof(double));
#pragma omp parallel num_threads(T)
  {
  double sse = 0, ssf = 0;
#pragma omp for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    const double* x = X + i * p;
    const double* y = Y + i * q;
    double z[RM], zf[RM];
    for (int k = 0; k < r; ++k) {
      z[k] = sE2 * (Xw[i * r + k] * c1[k] + Yc[i * r + k] * c2[k]);
      zf[k] = sF2 * (Yc[i * r + k] * c3[k] + Xw[i * r + k] * c2[k]);
    }
    for (int j = 0; j < p; ++j) {
      double e = x[j];
      for (int k = 0; k < r; ++k) e -= z[k] * W[k * p + j];
      sse += e * e;
    }
    for (int j = 0; j < q; ++j) {
      double f = y[j];
      for (int k = 0; k < r; ++k) f -= zf[k] * C[k * q + j];
      ssf += f * f;
    }
  }
  part2[2 * (size_t)thread_id()] = sse;
  part2[2 * (size_t)thread_id() + 1] = ssf;
  }
  double tot2[2];
  sum_ordered(part2, T, 2, tot2);
  free(part2);
  const double sse = tot2[0], ssf = tot2[1];
  const double N = (double)n;
  double Ctt[RM], Cut[RM], trChh = 0, sc1 = 0, sc3 = 0;
  for (int k = 0; k < r; ++k) {
    const double t2 = t[k] * t[k], t4 = t2 * t2, bb = b[k], b2 = bb * bb, v = t2 * b2 + sH2;
    Ctt[k] = fabs(t2 - t4 / sE2 - t4 * b2 / sF2 + t4 * c1[k] + 2 * t4 * bb * c2[k] + t4 * b2 * c3[k] + tt[k] / N);
    Cut[k] = t2 * bb - t4 * bb / sE2 - t2 * bb * v / sF2 + t4 * bb * c1[k] + t2 * v * c2[k] + t4 * b2 * c2[k] +
             t2 * bb * v * c3[k] + ut[k] / N;
    trChh += fabs(sH2 - sH2 * sH2 / sF2 + sH2 * sH2 * c3[k] + hh[k * r + k] / N);
    sc1 += c1[k];
    sc3 += c3[k];
  }
  const double Cee = (sE2 * sE2 * sc1 + sse / N) / p, Cff = (sF2 * sF2 * sc3 + ssf / N) / q;
  /* pass 3: X' mu_T, Y' mu_U (:732-733) */
  double* SX = (double*)calloc((size_t)p * r, sizeof(double));
  double* SY = (double*)calloc((size_t)q * r, sizeof(double));
  const int L3 = (p + q) * r;
  double* part3 = (double*)calloc((size_t)T * L3, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double* lx = part3 + (size_t)thread_id() * L3;
    double* ly = lx + (size_t)p * r;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double* x = X + i * p;
      const double* y = Y + i * q;
      for (int k = 0; k < r; ++k) {
        const double mt = muT[i * r + k], mu = muU[i * r + k];
        for (int j = 0; j < p; ++j) lx[k * p + j] += x[j] * mt;
        for (int j = 0; j < q; ++j) ly[k * q + j] += y[j] * mu;
      }
    }
  }
  for (int t = 0; t < T; ++t) {   /* thread-index order */
    const double* lx = part3 + (size_t)t * L3;
    for (int j = 0; j < p * r; ++j) SX[j] += lx[j];
    for (int j = 0; j < q * r; ++j) SY[j] += lx[(size_t)p * r + j];
  }
  free(part3);
  int rc = polar(SX, p, r, W);
  if (rc == 0) rc = polar(SY, q, r, C);
  for (int k = 0; k < r; ++k) {
    b[k] = Cut[k] * (1.0 / Ctt[k]);
    t[k] = sqrt(Ctt[k]);
  }
  sig[0] = sqrt(Cee);
  sig[1] = sqrt(Cff);
  sig[2] = sqrt(trChh / r);
  /* pass 4: logl_W of the new theta (loglC_fast recomputes X W, Y C, ||X||^2, ||Y||^2) */
  if (loglik) *loglik = loglc(X, Y, n, p, q, r, W, C, sig[0], sig[1], sig[2], b, t);
  free(SX); free(SY); free(muT); free(muU); free(Xw); free(Yc);
  return rc;
}

int cpu_ref_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
