// ppls_math.h -- O(r) / O(r^2) scalar algebra of one PPLS_simult EM step, shared verbatim by the
// device finalize kernel and the host-side (CPU-testable) entry points.
//
// Everything here is derived from the one-pass sufficient statistics of a sweep:
//   G  = [Xw Yc]'[Xw Yc]    (2r x 2r, column-major, ld = 2r)
//   ssqX = ||X||^2, ssqY = ||Y||^2, N = total number of samples,
//   WtW = W'W, CtC = C'C    (r x r) of the parameters the sweep used.
// Reference lines restated (paths relative to /root/reference):
//   coefficients          Package/PPLS/R/EM_W_multi.R:669-686 (Expect_M) and :312-320 (logl_W)
//   mu coefficients       EM_W_multi.R:691-694
//   E-step moments        EM_W_multi.R:696-716
//   M-step scalars        EM_W_multi.R:734-738, tr() Package/PPLS/R/PJSC.R:1-5
//   log-likelihood        Package/PPLS/src/loglC.cpp:318-338
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define PPLS_HD __host__ __device__ inline __attribute__((always_inline))
#else
#define PPLS_HD inline
#endif

#define PPLS_RMAX 16

// Scalar parameters of theta plus the derived per-component coefficients the sweep consumes.
struct PplsScalars {
  double b[PPLS_RMAX];      // diag(B)
  double t[PPLS_RMAX];      // diag(sigT)  (standard deviations, as in the reference)
  double sigE, sigF, sigH;  // sigE == sigX, sigF == sigY
  double pad0;
  // mu_T[:,k] = alpha_k Xw_k + beta_k Yc_k ; mu_U[:,k] = gamma_k Xw_k + delta_k Yc_k
  double alpha[PPLS_RMAX], beta[PPLS_RMAX], gamma[PPLS_RMAX], delta[PPLS_RMAX];
};

// Expectations returned by Expect_M (EM_W_multi.R:715-716); Ctt/Cuu/Cut are diagonal there.
struct PplsMoments {
  double Ctt[PPLS_RMAX], Cuu[PPLS_RMAX], Cut[PPLS_RMAX];
  double Cee, Cff;
  double Chh[PPLS_RMAX * PPLS_RMAX];  // full r x r, column-major, abs() applied
};

// Expect_M coefficient block, EM_W_multi.R:670-686.
PPLS_HD void ppls_coef_estep(double t, double b, double sigE, double sigF, double sigH,
                             double* c1, double* c2, double* c3, double* Kc_out) {
  const double t2 = t * t, t4 = t2 * t2, t6 = t4 * t2, b2 = b * b;
  const double sE2 = sigE * sigE, sF2 = sigF * sigF;
  const double g = t2 * b2 + sigH * sigH;
  const double Kw = t2 - t4 * b2 / sF2 + t4 * b2 * g / (sF2 * (g + sF2));
  const double Kc = g - t4 * b2 / sE2 + t6 * b2 / (sE2 * (t2 + sE2));
  const double Kwc = t2 * b / (sE2 * sF2) - Kc * t2 * b / (sE2 * sF2 * (Kc + sF2)) -
                     t4 * b / (sE2 * sF2 * (t2 + sE2)) +
                     Kc * t4 * b / (sE2 * sF2 * (Kc + sF2) * (t2 + sE2));
  *c1 = Kw / (sE2 * (Kw + sE2));
  *c3 = Kc / (sF2 * (Kc + sF2));
  *c2 = Kwc;
  if (Kc_out) *Kc_out = Kc;
}

// logl_W coefficient block, EM_W_multi.R:312-320: identical except g = sqrt(.) then squared.
PPLS_HD void ppls_coef_logl(double t, double b, double sigX, double sigY, double sigH,
                            double* c1, double* c2, double* c3, double* Kc_out) {
  const double t2 = t * t, t4 = t2 * t2, t6 = t4 * t2, b2 = b * b;
  const double sX2 = sigX * sigX, sY2 = sigY * sigY;
  const double gs = sqrt(t2 * b2 + sigH * sigH);
  const double g2 = gs * gs;
  const double Kw = t2 - t4 * b2 / sY2 + t4 * b2 * g2 / (sY2 * (g2 + sY2));
  const double Kc = g2 - t4 * b2 / sX2 + t6 * b2 / (sX2 * (t2 + sX2));
  const double Kwc = t2 * b / (sX2 * sY2) - Kc * t2 * b / (sX2 * sY2 * (Kc + sY2)) -
                     t4 * b / (sX2 * sY2 * (t2 + sX2)) +
                     Kc * t4 * b / (sX2 * sY2 * (Kc + sY2) * (t2 + sX2));
  *c1 = Kw / (sX2 * (Kw + sX2));
  *c3 = Kc / (sY2 * (Kc + sY2));
  *c2 = Kwc;
  *Kc_out = Kc;
}

// alpha..delta of the per-row posterior means, EM_W_multi.R:691-694 collected per column.
PPLS_HD void ppls_mu_coef_k(double t, double b, double sigE, double sigF, double sigH, double* al,
                            double* be, double* ga, double* de) {
  double c1, c2, c3;
  ppls_coef_estep(t, b, sigE, sigF, sigH, &c1, &c2, &c3, nullptr);
  const double t2 = t * t;
  const double v = t2 * b * b + sigH * sigH;   // varU, :688
  const double iE = 1.0 / (sigE * sigE), iF = 1.0 / (sigF * sigF);
  *al = iE * t2 - c1 * t2 - c2 * t2 * b;
  *be = iF * t2 * b - c2 * t2 - c3 * b * t2;
  *ga = iE * t2 * b - c1 * t2 * b - c2 * v;
  *de = iF * v - c2 * t2 * b - c3 * v;
}

PPLS_HD void ppls_mu_coef(PplsScalars* s, int r) {
  for (int k = 0; k < r; ++k)
    ppls_mu_coef_k(s->t[k], s->b[k], s->sigE, s->sigF, s->sigH, &s->alpha[k], &s->beta[k],
                   &s->gamma[k], &s->delta[k]);
}

// Gram accessors: G is 2r x 2r column-major; A = Xw'Xw, D = Xw'Yc, Bm = Yc'Yc.
#define PPLS_GA(G, r, k, l) (G)[(size_t)(l) * (2 * (r)) + (k)]
#define PPLS_GD(G, r, k, l) (G)[(size_t)((r) + (l)) * (2 * (r)) + (k)]
#define PPLS_GB(G, r, k, l) (G)[(size_t)((r) + (l)) * (2 * (r)) + (r) + (k)]

// Expect_M second moments (EM_W_multi.R:696-716) from the sufficient statistics of a sweep that
// used theta = (W, C, s).  ssq(mu_E) and ssq(mu_F) are expanded exactly:
//   ||X - sE^2 Z W'||^2 = ||X||^2 - 2 sE^2 tr(Z'Xw) + sE^4 tr(Z'Z W'W),  Z = Xw c1 + Yc c2.
// The pieces below are shared by the serial form (ppls_estep_moments, host and tests) and the
// lane-parallel device form (one lane per component / per component pair).

// Component k: diagonal Ctt, Cuu, Cut (:696-701, abs() of :715) and its terms of tr(Z'Xw), tr(Z_F'Yc).
PPLS_HD void ppls_moment_diag(const double* G, int r, int k, const PplsScalars* s, double c1, double c2,
                              double c3, double N, double* Ctt_o, double* Cuu_o, double* Cut_o,
                              double* xz_o, double* yz_o) {
  const double sE2 = s->sigE * s->sigE, sF2 = s->sigF * s->sigF, sH2 = s->sigH * s->sigH;
  const double iE = 1.0 / sE2, iF = 1.0 / sF2;
  const double t2 = s->t[k] * s->t[k], t4 = t2 * t2, b = s->b[k], b2 = b * b;
  const double v = t2 * b2 + sH2;
  const double A = PPLS_GA(G, r, k, k), D = PPLS_GD(G, r, k, k), Bm = PPLS_GB(G, r, k, k);
  const double al = s->alpha[k], be = s->beta[k], ga = s->gamma[k], de = s->delta[k];
  const double tt = al * al * A + 2.0 * al * be * D + be * be * Bm;   // crossprod(mu_T)_kk
  const double uu = ga * ga * A + 2.0 * ga * de * D + de * de * Bm;   // crossprod(mu_U)_kk
  const double ut = ga * al * A + (ga * be + de * al) * D + de * be * Bm;
  const double Ctt = t2 - iE * t4 - iF * (t4 * b2) + t4 * c1 + 2.0 * (t4 * b * c2) +
                     t4 * b2 * c3 + tt / N;                                       // :696-697
  const double Cuu = v - iE * (t4 * b2) - iF * (v * v) + t4 * b2 * c1 +
                     2.0 * (t2 * b * v * c2) + v * v * c3 + uu / N;            // :698-699
  const double Cut = t2 * b - iE * (t4 * b) - iF * (t2 * b * v) + t4 * b * c1 +
                     t2 * v * c2 + t4 * b2 * c2 + t2 * b * v * c3 + ut / N;  // :700-701
  *Ctt_o = fabs(Ctt);   // abs(Ctt)*I, :715
  *Cuu_o = fabs(Cuu);
  *Cut_o = Cut;
  *xz_o = c1 * A + c2 * D;
  *yz_o = c3 * Bm + c2 * D;
}

// Component pair (k, l): (Z'Z)_kl W'W_lk, (Z_F'Z_F)_kl C'C_lk (:703-709) and Chh_kl (:711-712, abs).
PPLS_HD void ppls_moment_pair(const double* G, int r, int k, int l, double c1k, double c2k, double c3k,
                              double c1l, double c2l, double c3l, double WtW_lk, double CtC_lk,
                              const PplsScalars* s, double N, double* zz_o, double* ww_o, double* Chh_o) {
  const double sF2 = s->sigF * s->sigF, sH2 = s->sigH * s->sigH, iF = 1.0 / sF2;
  // (Z'Z)_kl with Z_k = c1_k a_k + c2_k b_k ; D(k,l) = sum a_k b_l
  const double zkl = c1k * c1l * PPLS_GA(G, r, k, l) + c1k * c2l * PPLS_GD(G, r, k, l) +
                     c2k * c1l * PPLS_GD(G, r, l, k) + c2k * c2l * PPLS_GB(G, r, k, l);
  // (Z'_F Z_F)_kl with Z_F,k = c3_k b_k + c2_k a_k
  const double fkl = c3k * c3l * PPLS_GB(G, r, k, l) + c3k * c2l * PPLS_GD(G, r, l, k) +
                     c2k * c3l * PPLS_GD(G, r, k, l) + c2k * c2l * PPLS_GA(G, r, k, l);
  *zz_o = zkl * WtW_lk;
  *ww_o = fkl * CtC_lk;
  // mu_H,k = h1_k Yc_k + h2_k Xw_k
  const double h1k = iF * sH2 - sH2 * c3k, h2k = -sH2 * c2k;
  const double h1l = iF * sH2 - sH2 * c3l, h2l = -sH2 * c2l;
  const double hh = h1k * h1l * PPLS_GB(G, r, k, l) + h1k * h2l * PPLS_GD(G, r, l, k) +
                    h2k * h1l * PPLS_GD(G, r, k, l) + h2k * h2l * PPLS_GA(G, r, k, l);
  double v = hh / N;
  if (k == l) v = (sH2 - sH2 * sH2 / sF2) + sH2 * sH2 * c3k + v;
  *Chh_o = fabs(v);   // abs(Chh), :716
}

// Cee, Cff (:706, :709) from the reduced traces.
PPLS_HD void ppls_moment_noise(double ssqX, double ssqY, double N, int64_t p, int64_t q, const PplsScalars* s,
                               double xz, double yz, double zz, double ww, double sc1, double sc3,
                               double* Cee, double* Cff) {
  const double sE2 = s->sigE * s->sigE, sF2 = s->sigF * s->sigF;
  const double ssqE = ssqX - 2.0 * sE2 * xz + sE2 * sE2 * zz;
  const double ssqF = ssqY - 2.0 * sF2 * yz + sF2 * sF2 * ww;
  const double pd = (double)p, qd = (double)q;
  *Cee = (pd * sE2 - pd * sE2 + sE2 * sE2 * sc1 + ssqE / N) / pd;   // :706
  *Cff = (qd * sF2 - qd * sF2 + sF2 * sF2 * sc3 + ssqF / N) / qd;   // :709
}

PPLS_HD void ppls_estep_moments(const double* G, const double* WtW, const double* CtC,
                                double ssqX, double ssqY, double N, int64_t p, int64_t q, int r,
                                const PplsScalars* s, PplsMoments* m) {
  double c1[PPLS_RMAX], c2[PPLS_RMAX], c3[PPLS_RMAX];
  for (int k = 0; k < r; ++k)
    ppls_coef_estep(s->t[k], s->b[k], s->sigE, s->sigF, s->sigH, &c1[k], &c2[k], &c3[k], nullptr);
  double xz = 0.0, zz = 0.0, yz = 0.0, ww = 0.0, sc1 = 0.0, sc3 = 0.0;
  for (int k = 0; k < r; ++k) {
    double xk, yk;
    ppls_moment_diag(G, r, k, s, c1[k], c2[k], c3[k], N, &m->Ctt[k], &m->Cuu[k], &m->Cut[k], &xk, &yk);
    xz += xk;
    yz += yk;
    sc1 += c1[k];
    sc3 += c3[k];
  }
  for (int l = 0; l < r; ++l)
    for (int k = 0; k < r; ++k) {
      double z, w;
      ppls_moment_pair(G, r, k, l, c1[k], c2[k], c3[k], c1[l], c2[l], c3[l], WtW[l * r + k],
                       CtC[l * r + k], s, N, &z, &w, &m->Chh[l * r + k]);
      zz += z;
      ww += w;
    }
  ppls_moment_noise(ssqX, ssqY, N, p, q, s, xz, yz, zz, ww, sc1, sc3, &m->Cee, &m->Cff);
}

// loglC_fast (loglC.cpp:318-338) for theta = (W, C, s) from the Gram of the sweep that used W, C.
// Component k's log-determinant terms (:331) and trace term (:335).
PPLS_HD void ppls_logl_k(const double* G, int r, int k, const PplsScalars* s, double* logs, double* trk) {
  const double sX2 = s->sigE * s->sigE, sY2 = s->sigF * s->sigF;
  double c1, c2, c3, Kc;
  ppls_coef_logl(s->t[k], s->b[k], s->sigE, s->sigF, s->sigH, &c1, &c2, &c3, &Kc);
  *logs = log(sX2 + s->t[k] * s->t[k]) + log(sY2 + Kc);
  *trk = -c1 * PPLS_GA(G, r, k, k) - 2.0 * c2 * PPLS_GD(G, r, k, k) - c3 * PPLS_GB(G, r, k, k);
}

PPLS_HD double ppls_logl_total(double logs, double trk, double ssqX, double ssqY, double N, int64_t p,
                               int64_t q, int r, const PplsScalars* s) {
  const double sX2 = s->sigE * s->sigE, sY2 = s->sigF * s->sigF;
  const double logdet = logs + (double)(p - r) * log(sX2) + (double)(q - r) * log(sY2);   // :331
  const double traceL = 1.0 / sX2 * ssqX + 1.0 / sY2 * ssqY + trk;                       // :334-335
  return -0.5 * N * (double)(p + q) * log(2.0 * M_PI) - 0.5 * N * logdet - 0.5 * traceL;  // :336
}

PPLS_HD double ppls_loglik_from_gram(const double* G, double ssqX, double ssqY, double N, int64_t p,
                                     int64_t q, int r, const PplsScalars* s) {
  double logs = 0.0, trk = 0.0;
  for (int k = 0; k < r; ++k) {
    double a, b;
    ppls_logl_k(G, r, k, s, &a, &b);
    logs += a;
    trk += b;
  }
  return ppls_logl_total(logs, trk, ssqX, ssqY, N, p, q, r, s);
}

// Generic loglC_fast from explicit coefficient vectors (the drop-in for the .Call boundary).
PPLS_HD double ppls_loglc_fast_from_gram(const double* G, double ssqX, double ssqY, double N,
                                         int64_t p, int64_t q, int r, double sigX, double sigY,
                                         const double* sig2T, const double* c1, const double* c2,
                                         const double* c3, const double* Kc) {
  const double sX2 = sigX * sigX, sY2 = sigY * sigY;
  double a1 = 0.0, a2 = 0.0;
  for (int k = 0; k < r; ++k) { a1 += log(sX2 + sig2T[k]); a2 += log(sY2 + Kc[k]); }
  const double logdet = a1 + (double)(p - r) * log(sX2) + a2 + (double)(q - r) * log(sY2);
  double traceL = 1.0 / sX2 * ssqX + 1.0 / sY2 * ssqY;
  for (int k = 0; k < r; ++k)
    traceL += -c1[k] * PPLS_GA(G, r, k, k) - 2.0 * c2[k] * PPLS_GD(G, r, k, k) -
              c3[k] * PPLS_GB(G, r, k, k);
  return -0.5 * N * (double)(p + q) * log(2.0 * M_PI) - 0.5 * N * logdet - 0.5 * traceL;
}

// Maximiz_M scalar updates, EM_W_multi.R:734-738.
PPLS_HD void ppls_mstep_scalars(const PplsMoments* m, int r, PplsScalars* nx) {
  double trChh = 0.0;
  for (int k = 0; k < r; ++k) {
    nx->b[k] = m->Cut[k] * (1.0 / m->Ctt[k]);   // Cut %*% solve(Ctt) * I
    nx->t[k] = sqrt(m->Ctt[k]);                 // sqrt(Ctt * I)
    trChh += m->Chh[k * r + k];
  }
  nx->sigE = sqrt(m->Cee / 1.0);
  nx->sigF = sqrt(m->Cff / 1.0);
  nx->sigH = sqrt(trChh / (double)r);
  ppls_mu_coef(nx, r);
}

// ---- rank-1 EM step of the sequential initialiser (EMstep_W EM_W_multi.R:51-73 ->
// EMstepC_fast src/loglC.cpp:340-397; meta_Estep / meta_Mstep loglC.cpp:399-474 restate the same
// formulas).  Scalars of one component; the loadings live beside them.
struct PplsRank1 {
  double B, sigE, sigF, sigH, sigT;
};

// EMstep_W's coefficients (:60-70) and EMstepC_fast's mu coefficients (:354, :358).
PPLS_HD void ppls_rank1_coefs(const PplsRank1* t, double* c1, double* c2, double* c3, double* al, double* be,
                              double* ga, double* de) {
  ppls_coef_estep(t->sigT, t->B, t->sigE, t->sigF, t->sigH, c1, c2, c3, nullptr);
  const double s2X = t->sigE * t->sigE, s2Y = t->sigF * t->sigF, s2H = t->sigH * t->sigH;
  const double s2T = t->sigT * t->sigT, B = t->B, v = s2T * B * B + s2H;
  *al = s2T * (-*c1 + -*c2 * B + 1 / s2X);
  *be = s2T * (-*c2 + -*c3 * B + 1 / s2Y * B);
  *ga = -s2T * B * *c1 + -*c2 * v + 1 / s2X * B * s2T;
  *de = -*c2 * B * s2T + -*c3 * v + 1 / s2Y * v;
}

// PplsScalars (r = 1) the sweep consumes for component t.
PPLS_HD void ppls_rank1_sweep_scalars(const PplsRank1* t, PplsScalars* s) {
  for (int k = 0; k < PPLS_RMAX; ++k) s->b[k] = s->t[k] = s->alpha[k] = s->beta[k] = s->gamma[k] = s->delta[k] = 0.0;
  s->b[0] = t->B;
  s->t[0] = t->sigT;
  s->sigE = t->sigE;
  s->sigF = t->sigF;
  s->sigH = t->sigH;
  s->pad0 = 0.0;
  double c1, c2, c3;
  ppls_rank1_coefs(t, &c1, &c2, &c3, &s->alpha[0], &s->beta[0], &s->gamma[0], &s->delta[0]);
}

// logl_W(Xc, Yc, w, c, B, sigE, sigF, sigH, sigT) from the sweep's 2 x 2 Gram (:297-323, r = 1).
PPLS_HD double ppls_rank1_loglik(const PplsRank1* t, const double G[4], double ssqX, double ssqY, double N,
                                 int64_t p, int64_t q) {
  PplsScalars s;
  ppls_rank1_sweep_scalars(t, &s);
  return ppls_loglik_from_gram(G, ssqX, ssqY, N, p, q, 1, &s);
}

// The rank-1 E-step moments and M-step scalars from one sweep's Gram G = [||Xw||^2, <Xw,Yc>, ., ||Yc||^2]:
// B = Cut/Ctt, sighat = (sqrt(Cee), sqrt(Cff)), siglathat = (sqrt(Chh), sqrt(Ctt)).
PPLS_HD void ppls_rank1_scalars(const PplsRank1* t, const double G[4], double ssqX, double ssqY, double N,
                                int64_t p, int64_t q, PplsRank1* n) {
  double c1, c2, c3, al, be, ga, de;
  ppls_rank1_coefs(t, &c1, &c2, &c3, &al, &be, &ga, &de);
  const double s2X = t->sigE * t->sigE, s2Y = t->sigF * t->sigF, s2H = t->sigH * t->sigH;
  const double s2T = t->sigT * t->sigT, B = t->B, v = s2T * B * B + s2H;
  const double A = G[0], D = G[1], Bm = G[3];   // ||Xw||^2, <Xw, Yc>, ||Yc||^2
  const double mt2 = al * al * A + 2.0 * al * be * D + be * be * Bm;
  const double mut = ga * al * A + (ga * be + de * al) * D + de * be * Bm;
  const double Ctt = s2T - s2T * s2T * (-c1 - 2 * B * c2 - B * B * (c3 - 1 / s2Y) + 1 / s2X) + mt2 / N;   // :356
  const double Cut = s2T * B - (-s2T * s2T * B * (c1 - 1 / s2X) - s2T * s2T * B * B * c2 - s2T * v * c2 -
                                v * s2T * B * (c3 - 1 / s2Y)) + mut / N;                              // :363
  const double Ceetmp = c1 * c1 * s2X * s2X * A + ssqX + c2 * c2 * s2X * s2X * Bm - 2 * c1 * s2X * A +
                        2 * c1 * c2 * s2X * s2X * D - 2 * c2 * s2X * D;                                // :365-366
  const double Cee = s2X - (-s2X * s2X * c1 + (double)p * s2X) / (double)p + Ceetmp / N / (double)p;   // :367
  const double Cfftmp = c3 * c3 * s2Y * s2Y * Bm + ssqY + c2 * c2 * s2Y * s2Y * A - 2 * c3 * s2Y * Bm +
                        2 * c3 * c2 * s2Y * s2Y * D - 2 * c2 * s2Y * D;                                // :369-370
  const double Cff = s2Y - (-s2Y * s2Y * c3 + (double)q * s2Y) / (double)q + Cfftmp / N / (double)q;   // :371
  const double hx = -c2 * s2H, hy = -(c3 - 1 / s2Y) * s2H;
  const double Chh = s2H - (-s2H * s2H * (c3 - 1 / s2Y)) + (hx * hx * A + 2 * hx * hy * D + hy * hy * Bm) / N;  // :373
  n->B = Cut / Ctt;         // :385
  n->sigE = sqrt(Cee);      // sighat (:376)
  n->sigF = sqrt(Cff);
  n->sigH = sqrt(Chh);      // siglathat (:377)
  n->sigT = sqrt(Ctt);
}

// Polar factor U_R V_R' of a small r x r matrix R (column-major, ld r) by one-sided (Hestenes)
// Jacobi: R V = U S.  Returns 0 on success, -1 if R is numerically rank deficient.
// P (r x r, column-major) receives U_R V_R'.
template <int RC>
PPLS_HD int ppls_small_polar_n(const double* R, int r, double* P) {
  // RC: compile-time capacity (arrays stay in registers when RC == r is a constant)
  double A[RC * RC], V[RC * RC];
  for (int i = 0; i < r * r; ++i) A[i] = R[i];
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) V[j * r + i] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int i = 0; i < r - 1; ++i)
      for (int j = i + 1; j < r; ++j) {
        double a = 0.0, b = 0.0, g = 0.0;
        for (int k = 0; k < r; ++k) {
          a += A[i * r + k] * A[i * r + k];
          b += A[j * r + k] * A[j * r + k];
          g += A[i * r + k] * A[j * r + k];
        }
        if (g == 0.0) continue;
        const double rel = fabs(g) / sqrt(a * b);
        if (rel > off) off = rel;
        if (rel < 1e-17) continue;
        const double zeta = (b - a) / (2.0 * g);
        const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + tt * tt), sn = c * tt;
        for (int k = 0; k < r; ++k) {
          const double x = A[i * r + k], y = A[j * r + k];
          A[i * r + k] = c * x - sn * y;
          A[j * r + k] = sn * x + c * y;
          const double vx = V[i * r + k], vy = V[j * r + k];
          V[i * r + k] = c * vx - sn * vy;
          V[j * r + k] = sn * vx + c * vy;
        }
      }
    if (off < 1e-15) break;
  }
  double smax = 0.0, sv[RC];
  for (int i = 0; i < r; ++i) {
    double nrm = 0.0;
    for (int k = 0; k < r; ++k) nrm += A[i * r + k] * A[i * r + k];
    sv[i] = sqrt(nrm);
    if (sv[i] > smax) smax = sv[i];
  }
  int rc = 0;
  for (int i = 0; i < r; ++i) {
    if (!(sv[i] > smax * 1e-14)) { rc = -1; sv[i] = 1.0; }
    for (int k = 0; k < r; ++k) A[i * r + k] /= sv[i];   // U_R column i
  }
  // P = U V'
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) {
      double acc = 0.0;
      for (int k = 0; k < r; ++k) acc += A[k * r + i] * V[k * r + j];
      P[j * r + i] = acc;
    }
  return rc;
}

// Same algorithm with caller-provided workspace A, V (r*r each; e.g. LDS on the device).
template <int RC>
PPLS_HD int ppls_small_polar_ws(const double* R, int r, double* P, double* A, double* V) {
  for (int i = 0; i < r * r; ++i) A[i] = R[i];
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) V[j * r + i] = (i == j) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0;
    for (int i = 0; i < r - 1; ++i)
      for (int j = i + 1; j < r; ++j) {
        double a = 0.0, b = 0.0, g = 0.0;
        for (int k = 0; k < r; ++k) {
          a += A[i * r + k] * A[i * r + k];
          b += A[j * r + k] * A[j * r + k];
          g += A[i * r + k] * A[j * r + k];
        }
        if (g == 0.0) continue;
        const double rel = fabs(g) / sqrt(a * b);
        if (rel > off) off = rel;
        if (rel < 1e-17) continue;
        const double zeta = (b - a) / (2.0 * g);
        const double tt = (zeta >= 0.0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
        const double c = 1.0 / sqrt(1.0 + tt * tt), sn = c * tt;
        for (int k = 0; k < r; ++k) {
          const double x = A[i * r + k], y = A[j * r + k];
          A[i * r + k] = c * x - sn * y;
          A[j * r + k] = sn * x + c * y;
          const double vx = V[i * r + k], vy = V[j * r + k];
          V[i * r + k] = c * vx - sn * vy;
          V[j * r + k] = sn * vx + c * vy;
        }
      }
    if (off < 1e-15) break;
  }
  double smax = 0.0, sv[RC];
  for (int i = 0; i < r; ++i) {
    double nrm = 0.0;
    for (int k = 0; k < r; ++k) nrm += A[i * r + k] * A[i * r + k];
    sv[i] = sqrt(nrm);
    if (sv[i] > smax) smax = sv[i];
  }
  int rc = 0;
  for (int i = 0; i < r; ++i) {
    if (!(sv[i] > smax * 1e-14)) { rc = -1; sv[i] = 1.0; }
    for (int k = 0; k < r; ++k) A[i * r + k] /= sv[i];   // U_R column i
  }
  // P = U V'
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < r; ++i) {
      double acc = 0.0;
      for (int k = 0; k < r; ++k) acc += A[k * r + i] * V[k * r + j];
      P[j * r + i] = acc;
    }
  return rc;
}

PPLS_HD int ppls_small_polar(const double* R, int r, double* P) {
  return ppls_small_polar_n<PPLS_RMAX>(R, r, P);
}

// Sign/order canonicalisation, EM_W_multi.R:773-778 / :794-799.  Produces the permutation rot
// (stable decreasing order of |t_k b_k|) and the signs sign(t_k b_k).
PPLS_HD void ppls_canonical_order(const double* t, const double* b, int r, int* rot, double* sgn) {
  double key[PPLS_RMAX];
  for (int k = 0; k < r; ++k) {
    const double sb = t[k] * b[k];
    sgn[k] = (sb > 0.0) ? 1.0 : ((sb < 0.0) ? -1.0 : 0.0);
    key[k] = t[k] * (b[k] * sgn[k]);
    rot[k] = k;
  }
  // stable insertion sort, decreasing
  for (int i = 1; i < r; ++i) {
    const int cur = rot[i];
    int j = i - 1;
    while (j >= 0 && key[rot[j]] < key[cur]) { rot[j + 1] = rot[j]; --j; }
    rot[j + 1] = cur;
  }
}
