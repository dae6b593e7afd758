/* ppls.h -- C ABI of the MI355X-native PPLS_simult EM inner loop (libppls_amd.so).
 *
 * Drop-in boundary for the hot path of selbouhaddani/PPLS (paths relative to the reference):
 *   - the only native call on the loop today is
 *       .Call('PPLS_loglC_fast', PACKAGE='PPLS', W, C, X, Y, sigX, sigY, sig2T, c1, c2, c3, Kc)
 *     Package/PPLS/R/RcppExports.R:32-34 -> Package/PPLS/src/RcppExports.cpp:79-99
 *     -> Package/PPLS/src/loglC.cpp:318-338;              replaced by ppls_loglC_fast()
 *   - the R closures on the loop have no native boundary; their C-ABI counterparts are
 *       Expect_M   Package/PPLS/R/EM_W_multi.R:637-717      -> ppls_estep()
 *       Maximiz_M  Package/PPLS/R/EM_W_multi.R:729-742      -> ppls_mstep()
 *       Expect_M %>% Maximiz_M (one loop body, :782)         -> ppls_em_step()
 *       logl_W     Package/PPLS/R/EM_W_multi.R:297-323      -> ppls_loglik()
 *       PPLS_simult loop :780-807 (given theta0)             -> ppls_em_run()
 *
 * Conventions: all matrices crossing the ABI are column-major fp64 (R's layout), sizes are
 * int64_t for the sample dimension, the caller owns every host buffer, the context owns every
 * device buffer.  No exception crosses the ABI: every call returns PPLS_OK (0) or a negative
 * PPLS_E_* code, with a message in ppls_last_error(ctx).  A context is bound to one GPU and one
 * host thread; it is not re-entrant.
 */
#ifndef PPLS_AMD_PPLS_H
#define PPLS_AMD_PPLS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PPLS_OK 0
#define PPLS_E_ARG (-1)     /* invalid argument (R: stop()) */
#define PPLS_E_HIP (-2)     /* HIP runtime / device error */
#define PPLS_E_NUMERIC (-3) /* rank-deficient X'mu_T / Y'mu_U, non-finite update */
#define PPLS_E_STATE (-4)   /* no data loaded / wrong call order */
#define PPLS_E_COMM (-5)    /* RCCL error */
#define PPLS_E_NOMEM (-6)   /* device allocation failed */

#define PPLS_ORTH_SVD 0 /* orth(., type = "SVD"): polar factor U V' (default of PPLS_simult) */
#define PPLS_ORTH_QR 1  /* orth(., type = "QR"):  qr.Q(qr(.)) */

#define PPLS_LAYOUT_COLMAJOR 0 /* R matrices */
#define PPLS_LAYOUT_ROWMAJOR 1

typedef struct ppls_ctx ppls_ctx;

/* theta = (W, C, B, sigE, sigF, sigH, sigT) of Expect_M's argument list (EM_W_multi.R:637). */
typedef struct {
  double* W;    /* p x r column-major */
  double* C;    /* q x r column-major */
  double* B;    /* r: diag(B) */
  double* sigT; /* r: diag(sigT) (standard deviations) */
  double sigE;  /* == sigX */
  double sigF;  /* == sigY */
  double sigH;
} ppls_theta;

/* Expect_M's return list (EM_W_multi.R:715-716).  Ctt, Cuu, Cut are diagonal r x r matrices in the
 * reference; only their diagonals are exchanged.  mu_T / mu_U may be NULL (not requested). */
typedef struct {
  double* mu_T; /* n_local x r column-major (this rank's rows) */
  double* mu_U; /* n_local x r column-major */
  double* Ctt;  /* r */
  double* Cuu;  /* r */
  double* Cut;  /* r */
  double Cee;
  double Cff;
  double* Chh;  /* r x r column-major */
} ppls_expect;

int ppls_version(void);
const char* ppls_strerror(int code);

/* ---- context ---------------------------------------------------------------------------- */
int ppls_ctx_create(int device, ppls_ctx** out);
void ppls_ctx_destroy(ppls_ctx* ctx);
const char* ppls_last_error(const ppls_ctx* ctx);
/* keys: "sweep" (0 auto: the single-pass split sweep where W, C and the X'mu accumulators fit in
 *                registers, else the panel sweep; 3 panel (wide p, two passes)),
 *       "rows_per_step" (split sweep: 0 auto, 1, 2), "pipe" (split sweep software pipelining, 0/1),
 *       "grid" (workgroups, 0 = auto),
 *       "polar1" (finalize polar factor: 1 (default) one Cholesky-QR pass when
 *                 ||R1||_F ||R1^-1||_F <= k (R1 = chol(S'S)), else Cholesky-QR2; 0 always Cholesky-QR2),
 *       "polar1_kappa" (that bound k: 0 = the default min(8 r, 40); up to 255),
 *       "exact_gram" (finalize: 1 (default) the Gram W'W, C'C of the new loadings exactly, 0 the
 *                     identity -- faster, less accurate at small sigma_E),
 *       "team_rows" (finalize polar factor: rows of S per workgroup of a team; 0 = default 2048),
 *       "dtype" (storage of X, Y: 0 fp64, 1 fp32; arithmetic stays fp64; set before loading data),
 *       "nt" (sweep loads with the non-temporal cache policy: -1 auto (default: when X, Y exceed
 *             the 256 MB MALL), 0 off, 1 on),
 *       "timing" (N > 0: record HIP events around every N-th sweep launch; 0 off),
 *       "balance" (split sweep row partition: 0 (default) the even split -- bitwise reproducible
 *                  across processes; 1 per-XCD weights calibrated once per context and data shape
 *                  with 8 timed launches, from 2048 rows per workgroup: ~0.5 % faster at C3, but
 *                  the row grouping of the sums, hence the last bits, then vary between contexts),
 *       "xprod" (statistics of ppls_em_run / ppls_em_iterate: 0 (default) one streaming sweep over X, Y
 *                per iteration; 1 from the cross-products S = [X Y]'[X Y], formed once per data set
 *                on MFMA and all-reduced once, after which an iteration reads S (8 (p+q)^2 bytes) and
 *                needs no collective; -1 auto: S when a cost model of max_steps iterations says so
 *                and S with its Gram partials fits the smallest free HBM over all ranks (measured when
 *                the data were loaded; falls back to streaming, on every rank alike, if S cannot be
 *                allocated); S stays resident (8 (p+q)^2 bytes) until the data change, xprod goes from
 *                non-zero to 0 (not for an S of ppls_xprod_prepare), or ppls_xprod_release; setting 0
 *                ends an ppls_em_begin session that reads S: ppls_em_iterate then returns
 *                PPLS_E_STATE until the next ppls_em_begin -- never a silent switch to streaming),
 *       "meta_device" (ppls_meta_ppls: 1, default, the whole loop on the device -- the statistics of
 *                      every population from one read of X, Y per EM step (the split sweep: one
 *                      segmented launch; fp32 storage / wide p, the panel sweep: one launch per
 *                      population); 0 the per-population loop driven by the host),
 *       "gram_int8" (the Gram that forms S and ppls_variances' X'X: 0, default, fp64 MFMA; 1 the
 *                    int8-MFMA Chinese-remainder form when the columns' spread allows it -- else the
 *                    fp64 one; ppls_gram_info.  Its residue planes (17 x n x (p + q) bytes at C3's
 *                    spread) are a workspace kept between formations -- also across
 *                    ppls_xprod_release and new data -- until gram_int8 = 0 or ppls_ctx_destroy; a
 *                    device allocation of the library that fails frees them and tries again),
 *       "vorth" (the finalize re-orthonormalises the Jacobi warm start it carries between
 *                iterations every vorth-th iteration: 1 .. 255, default 8),
 *       "xprod_rw" (rows of S per wave of the cross-product tile kernel: 0 auto, 1, 2, 4, 8),
 *       "xprod_fuse" (1, default: the finalize after a cross-product step forms the 2r x 2r Gram
 *                     itself when r <= 8 and p + q <= 6144; 0: a separate Gram kernel),
 *       "dots_rows" (panel sweep dots: rows per wave, 0 auto (64 from 32768 rows, else 32), 32, 64),
 *       "dots_pair" (panel sweep dots: a wave pair per row tile, -1 auto (when row tiles are fewer
 *                    than resident wave slots), 0, 1),
 *       "acc_chunks" (panel sweep accumulation: row chunks, 0 auto, else that many),
 *       "var_chol" (ppls_variances' inverse of the observed information: 1, default, the
 *                   hand-written batched Cholesky + inverse (ppls_linalg.hip); 2 rocSOLVER
 *                   potrf/potri; 0 rocSOLVER LU getrf/getri; a matrix that is not positive definite
 *                   sends the batch to LU, as R's solve() would) */
int ppls_set_option(ppls_ctx* ctx, const char* key, int64_t value);

/* ---- multi-GPU: samples are sharded over ranks; one RCCL all-reduce per EM iteration ---- */
void ppls_shard_range(int64_t n_total, int nranks, int rank, int64_t* row0, int64_t* n_local);
int ppls_comm_unique_id(char id[128]);
int ppls_comm_init(ppls_ctx* ctx, int nranks, int rank, const char id[128]);
/* Host-side reduction in place of RCCL (MPI, gloo, a test harness, k contexts on one GPU, ...):
 * fn(user, buf, count) must replace buf[0..count) by its element-wise sum over all ranks and return
 * 0 (non-zero -> PPLS_E_COMM).  Every collective of the library (per-iteration sufficient statistics,
 * ||X||^2 and ||Y||^2, population and deflation sums, variances) then runs device -> host -> fn ->
 * device, synchronously, in the same order on every rank.  fn = NULL restores RCCL (or no
 * reduction).  Collective when data is resident (||X||^2, ||Y||^2 are re-reduced). */
typedef int (*ppls_reduce_fn)(void* user, double* buf, int64_t count);
int ppls_set_reducer(ppls_ctx* ctx, ppls_reduce_fn fn, void* user);

/* ---- data (X: n_local x p, Y: n_local x q; this rank's rows of an n_total-sample problem) ----
 * A NaN or Inf anywhere in X or Y (on any rank) -> PPLS_E_ARG on every rank, with the data dropped:
 * the reference's svd() in orth() stops on non-finite data (EM_W_multi.R:732-733).  It is detected
 * from the all-reduced sums of squares, so all ranks return together (no rank waits alone in a
 * collective).  Fits (ppls_em_run, ppls_em_begin, ppls_ppls*, ppls_meta_ppls) refuse an all-zero X
 * or Y with PPLS_E_ARG: the reference's fit stops on the NA increment that data produce. */
int ppls_set_data(ppls_ctx* ctx, const double* X, const double* Y, int64_t n_local, int p, int q,
                  int layout, int64_t n_total);
/* simulC-model synthetic data generated on the device (src/loglC.cpp:268-315, r >= 1):
 * X = T W' + sigE E, Y = U C' + sigF F, U = T B + H, T = N(0,1) diag(sigT), H = sigH N(0,1);
 * counter-based Philox4x32-10 normals keyed by (seed, element index): independent of sharding. */
int ppls_generate_synthetic(ppls_ctx* ctx, int64_t n_total, int64_t row0, int64_t n_local, int p,
                            int q, int r, const ppls_theta* truth, uint64_t seed);
int ppls_get_data(ppls_ctx* ctx, double* X, double* Y, int64_t row_begin, int64_t nrows);
/* The same rows in row-major layout (X: nrows x p, Y: nrows x q, C order), streamed without a
 * device-side transpose: what a row-oriented host consumer (the CPU baseline) reads. */
int ppls_get_data_rows(ppls_ctx* ctx, double* X, double* Y, int64_t row_begin, int64_t nrows);
int ppls_data_ssq(ppls_ctx* ctx, double* ssqX, double* ssqY);   /* global (all ranks) */

/* ---- the hot path ------------------------------------------------------------------------ */
int ppls_estep(ppls_ctx* ctx, const ppls_theta* th, int r, ppls_expect* out);
int ppls_mstep(ppls_ctx* ctx, const ppls_expect* fit, int r, int type, ppls_theta* out);
int ppls_em_step(ppls_ctx* ctx, const ppls_theta* in, int r, int type, ppls_theta* out,
                 ppls_expect* fit /* nullable: Expect_M of `in` */);
int ppls_loglik(ppls_ctx* ctx, const ppls_theta* th, int r, double* out);
/* PPLS_simult's loop and tail (EM_W_multi.R:773-806) from an explicit theta0 (in `th`).
 * On return `th` holds the canonicalised estimates (:794-799), loglik[0..*steps_done-1] the
 * log-likelihood trace, and eout (nullable) Expect_M at the un-canonicalised final theta (:802).
 * Returns PPLS_OK; *negative_increment = 1 where the reference warns (:801).  A NaN log-likelihood
 * increment under a finite atol is R's `if (NA < atol)` error (:792): the run stops there and
 * returns PPLS_E_NUMERIC, as it does for any non-finite trace entry or estimate -- never PPLS_OK. */
int ppls_em_run(ppls_ctx* ctx, ppls_theta* th, int r, int max_steps, double atol, int type,
                double* loglik, int* steps_done, int* negative_increment, ppls_expect* eout);

/* Device-resident iteration (benchmark / long runs): ppls_em_begin uploads theta0 (canonicalised as
 * :773-778); ppls_em_iterate enqueues exactly `nsteps` EM iterations (sweep + reduce + all-reduce +
 * finalize each, no host synchronisation, no stop rule); ppls_em_state downloads the current theta
 * (un-canonicalised) and the log-likelihood history logl(theta_1..theta_{k-1}) after k iterations. */
int ppls_em_begin(ppls_ctx* ctx, const ppls_theta* theta0, int r);
int ppls_em_iterate(ppls_ctx* ctx, int nsteps, int type);
int ppls_em_state(ppls_ctx* ctx, ppls_theta* out, double* loglik, int loglik_cap, int* n_loglik);

/* ---- sequential initialiser: PPLS(X, Y, a, EMsteps, atol, initialGuess) -------------------------
 * Replaces the R functions PPLS (Package/PPLS/R/EM_W_multi.R:229-279), PPLSi (:116-180) and
 * EMstep_W (:51-73) -> .Call('PPLS_EMstepC_fast') (R/RcppExports.R:36-38, src/loglC.cpp:340-397),
 * i.e. the f0 = PPLS(X, Y, a, 20, 1e-4, 'random') that PPLS_simult starts from (:762).
 * a rank-1 EM fits, component k on X, Y deflated by components 1..k-1 (:270-271; implicit here).
 * init: a starting values (theta with r = 1: W p, C q, B[1], sigT[1], sigE, sigF, sigH), i.e. the
 * initialGuess draws the R side makes (:126-145).  Stop rule per component: increment < atol
 * (critfunc = identity), no constraints.  If a component's sigE or sigF falls below
 * 100 * DBL_EPSILON the fit stops there (:152-154, :258-263): ncomp < a. */
/* scores.PPLS (Package/PPLS/R/EM_W_multi.R:411-420): T = X W (n_local x k), U = Y C (n_local x k),
 * column-major, for this rank's rows; one pass over the resident data.  T or U may be NULL. */
int ppls_scores(ppls_ctx* ctx, const double* W, const double* C, int k, double* T, double* U);

typedef struct {
  double* W;               /* p x a, column-major (R's W) */
  double* C;               /* q x a */
  double* B;               /* a */
  double* sig;             /* a x 4, column-major: sigX, sigY, sigH, sigT (R's sig) */
  double* logvalue;        /* nullable: a x (EMsteps + 1), row k = component k's logvalue, NaN padded */
  double* last_increment;  /* nullable: a (Other_output$Last_increment) */
  int* number_steps;       /* nullable: a (Other_output$Number_steps) */
  double* loglikelihoods;  /* nullable: a (Other_output$Loglikelihoods: logl_W of X, Y, comps 1..k) */
  int ncomp;               /* out: components fitted */
  int not_monotone;        /* out: bit k set if component k's logvalue decreased (warning, :177) */
} ppls_seq_fit;
int ppls_ppls(ppls_ctx* ctx, int a, int max_steps, double atol, const ppls_theta* init, ppls_seq_fit* out);
/* PPLS / PPLSi with the reference's optional arguments: critfunc (crit_abs 0 = identity, 1 = abs)
 * and constraints = list(fconstraint(...)) per component (Package/PPLS/R/EM_W_multi.R:85-92,
 * :141-145, :165-169): each non-NULL pointer fixes that parameter (W: p, C: q, the rest: 1 value)
 * at the start and after every EM step.  cons: a entries, or NULL (no constraints). */
typedef struct {
  const double* W;
  const double* C;
  const double* B;
  const double* sigE;
  const double* sigF;
  const double* sigH;
  const double* sigT;
} ppls_constraint;
int ppls_ppls_ex(ppls_ctx* ctx, int a, int max_steps, double atol, int crit_abs, const ppls_theta* init,
                 const ppls_constraint* cons, ppls_seq_fit* out);
int ppls_synchronize(ppls_ctx* ctx);

/* ---- multi-population rank-1 fits: meta_EMstep / meta_PPLSi ----------------------------------
 * Replace the R functions meta_EMstep (Package/PPLS/R/EM_W_multi.R:446-485) -> .Call meta_Estep /
 * meta_Mstep (R/RcppExports.R:40-46, src/loglC.cpp:399-474) and meta_PPLSi (:509-589): one shared
 * loading pair (W., C.) and per-population scalars (B_T, sigX, sigY, sigH, sigT).
 * Populations are contiguous row blocks in level order: population j is global rows
 * [N_1 + .. + N_{j-1}, N_1 + .. + N_j), exactly the reference's X[popui, ] with popui from
 * cumsum(table(Ipopu)) (:451-458, :537-541).  pop_local[j] = rows of population j in this rank's
 * shard (contiguous, in order; they sum to n_local), pop_total[j] = N_j over all ranks.
 * params: npop x 5 column-major, columns B_T, sigX, sigY, sigH, sigT (params[[j]] of the reference).
 * Each population is one r = 1 sweep over its rows (one all-reduce when sharded). */
int ppls_meta_emstep(ppls_ctx* ctx, int npop, const int64_t* pop_local, const int64_t* pop_total,
                     const double* W, const double* C, const double* params_in, double* W_out,
                     double* C_out, double* params_out, double* Cxt /* p x npop, nullable */,
                     double* Cyu /* q x npop, nullable */);
typedef struct {
  double* W;       /* p (out): c(Wnw) */
  double* C;       /* q (out) */
  double* params;  /* npop x 5 (out) */
  double* log;     /* nullable: (EMsteps + 1) x npop column-major logvalue; row 0 = the initial
                      rep(logl_W(X, Y, theta0), npop) (:544), rows 1..steps the EM steps; NaN padded */
  int steps;       /* out: EM steps made (the reference's i) */
} ppls_meta_fit;
/* crit_abs: 0 critfunc = identity (default), 1 critfunc = abs.  init: theta with r = 1. */
int ppls_meta_ppls(ppls_ctx* ctx, int npop, const int64_t* pop_local, const int64_t* pop_total,
                   int max_steps, double atol, int crit_abs, const ppls_theta* init, ppls_meta_fit* out);

/* loglC_fast (src/loglC.cpp:318-338) with the reference's argument list.  X, Y (column-major
 * n x p / n x q host matrices) are uploaded into ctx like Rcpp's input_parameter copies them;
 * pass X = Y = NULL to evaluate on the data already resident in ctx (zero-copy). */
int ppls_loglC_fast(ppls_ctx* ctx, const double* W, const double* C, const double* X, const double* Y,
                    int64_t n, int p, int q, int a, double sigX, double sigY, const double* sig2T,
                    const double* c1, const double* c2, const double* c3, const double* Kc,
                    double* out);

/* ---- variances.PPLS_simult(fit, data, XorY) (Package/PPLS/R/EM_W_multi.R:830-860) ---------------
 * mu: this rank's rows of fit$Expectations$mu_T (xory 0, "X") or $mu_U (xory 1, "Y"), n_local x a
 * column-major; Cdiag: diag of $Ctt (or $Cuu), a; sigE: fit$estimates$sigE (the reference uses sigE
 * for both XorY).  Outputs (p = ncol(data)): W = orth(t(data) %*% mu, "SVD") p x a; B_exp[i]: the
 * reference's B_exp of component i is B_exp[i] * diag(p); varMatrix, SSt_exp, SSt_star (each a
 * consecutive p x p column-major matrices, nullable) and seLoad (p x a).  t(data) diag(Ctt) data is
 * Ctt * data'data: one MFMA Gram for all components. */
int ppls_variances(ppls_ctx* ctx, const double* mu, const double* Cdiag, double sigE, int a, int xory,
                   double* W, double* B_exp, double* varMatrix, double* SSt_exp, double* SSt_star,
                   double* seLoad);

/* ---- cross-product form (option "xprod") ----------------------------------------------------
 * Form S = [X Y]'[X Y] now (*ms = the MFMA Gram kernel time, *total_ms = with the all-reduce and
 * allocation; both nullable) -- otherwise the first run that reads S forms it.  Collective when the
 * rows are sharded: every rank calls it (one all-reduce of (p+q)^2 doubles). */
int ppls_xprod_prepare(ppls_ctx* ctx, double* ms, double* total_ms);
/* Free S (and its scratch) now; the next run that reads S forms it again.  (The int8 Gram's
 * residue planes stay: see option "gram_int8".) */
int ppls_xprod_release(ppls_ctx* ctx);

/* ---- host-side algebra (no GPU; the same code the device finalize runs) ------------------------ */
/* From the all-reduced sufficient statistics of one sweep with theta (stats = [X'mu_T p x r |
 * Y'mu_U q x r | Gram 2r x 2r], all column-major) compute Expect_M's moments, logl_W(theta) and
 * the M-step scalars.  W_next/C_next (nullable) receive orth(X'mu_T)/orth(Y'mu_U). */
int ppls_finalize_host(const double* SX, const double* SY, const double* G, double ssqX, double ssqY,
                       double N, int p, int q, int r, const ppls_theta* th, int type,
                       ppls_theta* next, ppls_expect* moments, double* loglik);
/* alpha, beta, gamma, delta (4r) with mu_T = Xw diag(alpha) + Yc diag(beta) and
 * mu_U = Xw diag(gamma) + Yc diag(delta) (EM_W_multi.R:691-694). */
int ppls_mu_coefficients(const ppls_theta* th, int r, double* coef4r);

#ifdef __cplusplus
}
#endif
#endif /* PPLS_AMD_PPLS_H */
