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
 * cpu_ref_ppls_simult restates the whole PPLS_simult call the same way: the sequential initialiser
 * PPLS(X, Y, a, 20, 1e-4) (EMstepC_fast steps on explicitly deflated copies of X, Y, as R does),
 * the EM loop with its stop rule, and Eout.
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
/* The process's default OpenMP thread count, captured before the first omp_set_num_threads: a
 * call with nthreads <= 0 restores it (a 1-thread run must not leave later runs on one thread). */
static int def_threads = 0;
static void set_threads(int nthreads) {
  if (!def_threads) def_threads = omp_get_max_threads();
  omp_set_num_threads(nthreads > 0 ? nthreads : def_threads);
}
static int max_threads(void) { return omp_get_max_threads(); }
static int thread_id(void) { return omp_get_thread_num(); }
static double omp_wtime_or_clock(void) { return omp_get_wtime(); }
#else
#include <time.h>
static void set_threads(int nthreads) { (void)nthreads; }
static int max_threads(void) { return 1; }
static int thread_id(void) { return 0; }
static double omp_wtime_or_clock(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
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

/* Expect_M's closed form (EM_W_multi.R:668-716) over row-major data: pass 1 (X W, Y C, mu_T, mu_U
 * and their crossprods, :689-701; crossprod(mu_H), :711-712) and pass 2 (ssq(mu_E), ssq(mu_F)
 * streamed row by row, :703-709).  mu_T, mu_U: n x r row-major (caller's buffers).  Writes the
 * moments Ctt, Cuu, Cut (r), Cee, Cff, trChh and the coefficients the M-step needs. */
typedef struct {
  double c1[RM], c2[RM], c3[RM], al[RM], be[RM], ga[RM], de[RM];
  double Ctt[RM], Cuu[RM], Cut[RM], Cee, Cff, trChh;
} Moments;

static void estep_passes(const double* X, const double* Y, int64_t n, int p, int q, int r, const double* W,
                         const double* C, const double* b, const double* t, const double* sig, double* muT,
                         double* muU, Moments* m) {
  const double sE = sig[0], sF = sig[1], sH = sig[2];
  const double sE2 = sE * sE, sF2 = sF * sF, sH2 = sH * sH;
  double *c1 = m->c1, *c2 = m->c2, *c3 = m->c3, *al = m->al, *be = m->be, *ga = m->ga, *de = m->de;
  for (int k = 0; k < r; ++k) {
    coef_estep(t[k], b[k], sE, sF, sH, &c1[k], &c2[k], &c3[k], 0, 0);
    const double t2 = t[k] * t[k], v = t2 * b[k] * b[k] + sH2;
    al[k] = t2 / sE2 - c1[k] * t2 - c2[k] * t2 * b[k];
    be[k] = t2 * b[k] / sF2 - c2[k] * t2 - c3[k] * b[k] * t2;
    ga[k] = t2 * b[k] / sE2 - c1[k] * t2 * b[k] - c2[k] * v;
    de[k] = v / sF2 - c2[k] * t2 * b[k] - c3[k] * v;
  }
  double* Xw = (double*)malloc(sizeof(double) * n * r);
  double* Yc = (double*)malloc(sizeof(double) * n * r);
  double tt[RM] = {0}, uu[RM] = {0}, ut[RM] = {0}, hh[RM * RM] = {0};
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
  free(Xw);
  free(Yc);
  const double sse = tot2[0], ssf = tot2[1];
  const double N = (double)n;
  double sc1 = 0, sc3 = 0;
  m->trChh = 0;
  for (int k = 0; k < r; ++k) {
    const double t2 = t[k] * t[k], t4 = t2 * t2, bb = b[k], b2 = bb * bb, v = t2 * b2 + sH2;
    m->Ctt[k] = fabs(t2 - t4 / sE2 - t4 * b2 / sF2 + t4 * c1[k] + 2 * t4 * bb * c2[k] + t4 * b2 * c3[k] + tt[k] / N);
    m->Cuu[k] = fabs(v - t4 * b2 / sE2 - v * v / sF2 + t4 * b2 * c1[k] + 2 * t2 * bb * v * c2[k] + v * v * c3[k] +
                     uu[k] / N);
    m->Cut[k] = t2 * bb - t4 * bb / sE2 - t2 * bb * v / sF2 + t4 * bb * c1[k] + t2 * v * c2[k] + t4 * b2 * c2[k] +
                t2 * bb * v * c3[k] + ut[k] / N;
    m->trChh += fabs(sH2 - sH2 * sH2 / sF2 + sH2 * sH2 * c3[k] + hh[k * r + k] / N);
    sc1 += c1[k];
    sc3 += c3[k];
  }
  m->Cee = (sE2 * sE2 * sc1 + sse / N) / p;
  m->Cff = (sF2 * sF2 * sc3 + ssf / N) / q;
}

/* One EM iteration (Expect_M closed form %>% Maximiz_M, then logl_W) in place on theta.
 * Returns 0 and writes the log-likelihood of the new theta. */
int cpu_ref_em_step(const double* X, const double* Y, int64_t n, int p, int q, int r, double* W, double* C,
                    double* b, double* t, double* sig /* sE, sF, sH */, double* loglik, int nthreads) {
  set_threads(nthreads);
  if (r < 1 || r > RM) return -1;
  double* muT = (double*)malloc(sizeof(double) * n * r);
  double* muU = (double*)malloc(sizeof(double) * n * r);
  Moments m;
  estep_passes(X, Y, n, p, q, r, W, C, b, t, sig, muT, muU, &m);
  /* pass 3: X' mu_T, Y' mu_U (:732-733) */
  const int T = max_threads();
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
  for (int th = 0; th < T; ++th) {   /* thread-index order */
    const double* lx = part3 + (size_t)th * L3;
    for (int j = 0; j < p * r; ++j) SX[j] += lx[j];
    for (int j = 0; j < q * r; ++j) SY[j] += lx[(size_t)p * r + j];
  }
  free(part3);
  int rc = polar(SX, p, r, W);
  if (rc == 0) rc = polar(SY, q, r, C);
  for (int k = 0; k < r; ++k) {   /* :734-738 */
    b[k] = m.Cut[k] * (1.0 / m.Ctt[k]);
    t[k] = sqrt(m.Ctt[k]);
  }
  sig[0] = sqrt(m.Cee);
  sig[1] = sqrt(m.Cff);
  sig[2] = sqrt(m.trChh / r);
  /* pass 4: logl_W of the new theta (loglC_fast recomputes X W, Y C, ||X||^2, ||Y||^2) */
  if (loglik) *loglik = loglc(X, Y, n, p, q, r, W, C, sig[0], sig[1], sig[2], b, t);
  free(SX); free(SY); free(muT); free(muU);
  return rc;
}

/* ------------------------------------------------------------------ the whole PPLS_simult call
 * EMstepC_fast (src/loglC.cpp:340-397) with EMstep_W's coefficients (EM_W_multi.R:51-73) on
 * row-major Xc, Yc, in the reference's passes: Xw = X w, Yc = Y c (:351); X'mu_T, Y'mu_U (:355,
 * :360); ssq(X), ssq(Y) (:365, :369).  th = {B, sigX, sigY, sigH, sigT} and w, c in/out. */
static void rank1_step(const double* X, const double* Y, int64_t n, int p, int q, double* w, double* c, double* th) {
  const double B = th[0], sX = th[1], sY = th[2], sH = th[3], sT = th[4];
  const double s2X = sX * sX, s2Y = sY * sY, s2H = sH * sH, s2T = sT * sT;
  double c1, c2, c3;
  coef_estep(sT, B, sX, sY, sH, &c1, &c2, &c3, 0, 0);
  const double v = s2T * B * B + s2H;
  const double al = s2T * (-c1 + -c2 * B + 1 / s2X), be = s2T * (-c2 + -c3 * B + 1 / s2Y * B);
  const double ga = -s2T * B * c1 + -c2 * v + 1 / s2X * B * s2T, de = -c2 * B * s2T + -c3 * v + 1 / s2Y * v;
  const int T = max_threads();
  double* xw = (double*)malloc(sizeof(double) * n);
  double* yc = (double*)malloc(sizeof(double) * n);
  /* pass 1: Xw, Yc and the crossprods of mu_T, mu_U, mu_H */
  double* part = (double*)calloc((size_t)T * 8, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double* mine = part + 8 * (size_t)thread_id();
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double* x = X + i * p;
      const double* y = Y + i * q;
      double a = 0, d = 0;
      for (int j = 0; j < p; ++j) a += x[j] * w[j];
      for (int j = 0; j < q; ++j) d += y[j] * c[j];
      xw[i] = a;
      yc[i] = d;
      const double mt = a * al + d * be, mu = a * ga + d * de, mh = -c2 * s2H * a - (c3 - 1 / s2Y) * s2H * d;
      mine[0] += mt * mt;
      mine[1] += mu * mu;
      mine[2] += mu * mt;
      mine[3] += a * a;
      mine[4] += d * d;
      mine[5] += a * d;
      mine[6] += mh * mh;
    }
  }
  double tot[8];
  sum_ordered(part, T, 8, tot);
  /* pass 2: Cxt = X' mu_T, Cyu = Y' mu_U */
  const int L = p + q;
  double* part2 = (double*)calloc((size_t)T * L, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double* lx = part2 + (size_t)thread_id() * L;
    double* ly = lx + p;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      const double* x = X + i * p;
      const double* y = Y + i * q;
      const double mt = xw[i] * al + yc[i] * be, mu = xw[i] * ga + yc[i] * de;
      for (int j = 0; j < p; ++j) lx[j] += x[j] * mt;
      for (int j = 0; j < q; ++j) ly[j] += y[j] * mu;
    }
  }
  double* cxy = (double*)malloc(sizeof(double) * L);
  sum_ordered(part2, T, L, cxy);
  free(part2);
  /* pass 3: ssq(X), ssq(Y) (EMstepC_fast recomputes them on every call) */
  double* part3 = (double*)calloc((size_t)T * 2, sizeof(double));
#pragma omp parallel num_threads(T)
  {
    double ssx = 0, ssy = 0;
#pragma omp for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      for (int j = 0; j < p; ++j) ssx += X[i * p + j] * X[i * p + j];
      for (int j = 0; j < q; ++j) ssy += Y[i * q + j] * Y[i * q + j];
    }
    part3[2 * (size_t)thread_id()] = ssx;
    part3[2 * (size_t)thread_id() + 1] = ssy;
  }
  double ss[2];
  sum_ordered(part3, T, 2, ss);
  free(part3);
  free(part);
  free(xw);
  free(yc);
  const double N = (double)n;
  const double Ctt = s2T - s2T * s2T * (-c1 - 2 * B * c2 - B * B * (c3 - 1 / s2Y) + 1 / s2X) + tot[0] / N;
  const double Cut = s2T * B - (-s2T * s2T * B * (c1 - 1 / s2X) - s2T * s2T * B * B * c2 - s2T * v * c2 -
                                v * s2T * B * (c3 - 1 / s2Y)) + tot[2] / N;
  const double xw2 = tot[3], yc2 = tot[4], xy = tot[5];
  const double Ceetmp = c1 * c1 * s2X * s2X * xw2 + ss[0] + c2 * c2 * s2X * s2X * yc2 - 2 * c1 * s2X * xw2 +
                        2 * c1 * c2 * s2X * s2X * xy - 2 * c2 * s2X * xy;
  const double Cee = s2X - (-s2X * s2X * c1 + p * s2X) / p + Ceetmp / N / p;
  const double Cfftmp = c3 * c3 * s2Y * s2Y * yc2 + ss[1] + c2 * c2 * s2Y * s2Y * xw2 - 2 * c3 * s2Y * yc2 +
                        2 * c3 * c2 * s2Y * s2Y * xy - 2 * c2 * s2Y * xy;
  const double Cff = s2Y - (-s2Y * s2Y * c3 + q * s2Y) / q + Cfftmp / N / q;
  const double Chh = s2H - (-s2H * s2H * (c3 - 1 / s2Y)) + tot[6] / N;
  double nx = 0, ny = 0;
  for (int j = 0; j < p; ++j) nx += cxy[j] * cxy[j];
  for (int j = 0; j < q; ++j) ny += cxy[p + j] * cxy[p + j];
  nx = sqrt(nx);
  ny = sqrt(ny);
  for (int j = 0; j < p; ++j) w[j] = cxy[j] / nx;        /* Cxt.normalized() (the 1/N cancels) */
  for (int j = 0; j < q; ++j) c[j] = cxy[p + j] / ny;
  free(cxy);
  th[0] = Cut / Ctt;
  th[1] = sqrt(Cee);
  th[2] = sqrt(Cff);
  th[3] = sqrt(Chh);
  th[4] = sqrt(Ctt);
}

static double logl_rank1(const double* X, const double* Y, int64_t n, int p, int q, const double* w, const double* c,
                         const double* th) {
  return loglc(X, Y, n, p, q, 1, w, c, th[1], th[2], th[3], &th[0], &th[4]);
}

/* X <- X - (X w) w' in place (EM_W_multi.R:270-271), row-major n x p */
static void deflate_rows(double* X, int64_t n, int p, const double* w) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double* x = X + i * p;
    double a = 0;
    for (int j = 0; j < p; ++j) a += x[j] * w[j];
    for (int j = 0; j < p; ++j) x[j] -= a * w[j];
  }
}

/* canonical order of EM_W_multi.R:773-778 / :794-799 on column-major W (p x r), C, b, t */
static void canonicalize(double* W, double* C, double* b, double* t, int p, int q, int r) {
  double sg[RM], key[RM], W0[RM], b0[RM], t0[RM];
  int rot[RM];
  for (int k = 0; k < r; ++k) {
    const double d = t[k] * b[k];
    sg[k] = d > 0 ? 1.0 : d < 0 ? -1.0 : 0.0;
    key[k] = d * sg[k];
    rot[k] = k;
  }
  for (int i = 1; i < r; ++i)   /* stable insertion sort, decreasing (order(..., decreasing = TRUE)) */
    for (int j = i; j > 0 && key[rot[j]] > key[rot[j - 1]]; --j) { const int tmp = rot[j]; rot[j] = rot[j - 1]; rot[j - 1] = tmp; }
  double* Wc = (double*)malloc(sizeof(double) * p * r);
  double* Cc = (double*)malloc(sizeof(double) * q * r);
  for (int k = 0; k < r; ++k) {
    for (int i = 0; i < p; ++i) Wc[k * p + i] = W[rot[k] * p + i] * sg[k];
    for (int i = 0; i < q; ++i) Cc[k * q + i] = C[rot[k] * q + i] * sg[k];
    b0[k] = b[rot[k]] * sg[rot[k]];
    t0[k] = t[rot[k]];
  }
  (void)W0;
  memcpy(W, Wc, sizeof(double) * p * r);
  memcpy(C, Cc, sizeof(double) * q * r);
  memcpy(b, b0, sizeof(double) * r);
  memcpy(t, t0, sizeof(double) * r);
  free(Wc);
  free(Cc);
}

/* PPLS_simult(X, Y, a, EMsteps, atol) (EM_W_multi.R:758-807) on row-major X, Y: f0 = PPLS(X, Y, a,
 * init_steps, init_atol) from the given starting values (inits: a x 5 {B, sigX, sigY, sigH, sigT},
 * init_w p x a, init_c q x a column-major -- the 'random' draws, :126-140), then the EM loop with
 * the stop rule (:780-793), the canonical order (:794-799) and Eout = Expect_M (:802).  Outputs:
 * W, C (column-major), b, t (r), sig {sE, sF, sH}, loglik (EMsteps), *steps, comp_steps (a),
 * secs = {init, loop, Eout} wall seconds.  Returns 0, -1 on a rank collapse (fewer than a
 * components, as R would fail at W.[, rotLoad]). */
int cpu_ref_ppls_simult(const double* X, const double* Y, int64_t n, int p, int q, int a, const double* inits,
                        const double* init_w, const double* init_c, int init_steps, double init_atol, int EMsteps,
                        double atol, double* W, double* C, double* b, double* t, double* sig, double* loglik,
                        int* steps, int* comp_steps, double* secs, int nthreads) {
  set_threads(nthreads);
  if (a < 1 || a > RM) return -2;
  double t0 = omp_wtime_or_clock();
  double* Xc = (double*)malloc(sizeof(double) * n * p);
  double* Yc = (double*)malloc(sizeof(double) * n * q);
  memcpy(Xc, X, sizeof(double) * n * p);
  memcpy(Yc, Y, sizeof(double) * n * q);
  double sigE_last = 0, sigF_last = 0, sigH_last = 0;
  int rc = 0;
  for (int k = 0; k < a && rc == 0; ++k) {   /* PPLS (:254-275), PPLSi (:116-180) */
    double* w = W + (size_t)k * p;
    double* c = C + (size_t)k * q;
    memcpy(w, init_w + (size_t)k * p, sizeof(double) * p);
    memcpy(c, init_c + (size_t)k * q, sizeof(double) * q);
    double th[5];
    memcpy(th, inits + 5 * k, sizeof th);
    double lprev = logl_rank1(Xc, Yc, n, p, q, w, c, th);   /* logvalue[1], :149 */
    int i = 0;
    for (i = 1; i <= init_steps; ++i) {
      if (th[1] < 100 * 2.220446049250313e-16 || th[2] < 100 * 2.220446049250313e-16) { rc = -1; break; }
      rank1_step(Xc, Yc, n, p, q, w, c, th);
      const double l = logl_rank1(Xc, Yc, n, p, q, w, c, th);   /* :172 */
      const double inc = l - lprev;
      lprev = l;
      if (inc < init_atol) break;   /* :173 */
    }
    if (i > init_steps) i = init_steps;
    comp_steps[k] = i;
    b[k] = th[0];
    t[k] = th[4];
    sigE_last = th[1];
    sigF_last = th[2];
    sigH_last = th[3];
    deflate_rows(Xc, n, p, w);   /* :270-271 */
    deflate_rows(Yc, n, q, c);
    /* Other_output$Loglikelihoods[i] = logl_W(X, Y, components 1..k) (:274) */
    double bb[RM], tt2[RM];
    for (int j = 0; j <= k; ++j) { bb[j] = b[j]; tt2[j] = t[j]; }
    (void)loglc(X, Y, n, p, q, k + 1, W, C, th[1], th[2], th[3], bb, tt2);
  }
  free(Xc);
  free(Yc);
  double t1 = omp_wtime_or_clock();
  if (secs) secs[0] = t1 - t0;
  if (rc != 0) return rc;
  /* theta0 (:764-771) in the canonical order (:773-778) */
  sig[0] = sigE_last;
  sig[1] = sigF_last;
  sig[2] = sigH_last;
  canonicalize(W, C, b, t, p, q, a);
  int i = 0;
  for (i = 1; i <= EMsteps; ++i) {   /* :780-793 */
    rc = cpu_ref_em_step(X, Y, n, p, q, a, W, C, b, t, sig, &loglik[i - 1], nthreads);
    if (rc != 0) return rc;
    if (i > 1 && loglik[i - 1] - loglik[i - 2] < atol) break;
  }
  if (i > EMsteps) i = EMsteps;
  *steps = i;
  /* Eout = Expect_M of the un-canonicalised final theta (:802), then the canonical estimates */
  double t2 = omp_wtime_or_clock();
  double* muT = (double*)malloc(sizeof(double) * n * a);
  double* muU = (double*)malloc(sizeof(double) * n * a);
  Moments m;
  estep_passes(X, Y, n, p, q, a, W, C, b, t, sig, muT, muU, &m);
  free(muT);
  free(muU);
  canonicalize(W, C, b, t, p, q, a);
  double t3 = omp_wtime_or_clock();
  if (secs) { secs[1] = t2 - t1; secs[2] = t3 - t2; }
  return 0;
}

int cpu_ref_max_threads(void) {
#ifdef _OPENMP
  return def_threads ? def_threads : omp_get_max_threads();
#else
  return 1;
#endif
}
