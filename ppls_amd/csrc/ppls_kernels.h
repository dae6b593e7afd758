// ppls_kernels.h -- internal launch interface between the host runtime and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_math.h"

#define PPLS_SWEEP_SLOTS 4       // LDS-DMA ring depth (rows)
#define PPLS_FUSED_RMAX 8

struct PplsSweepArgs {
  const double* X;
  const double* Y;
  int64_t n_local;
  int p, q;               // columns of X, Y (ldx, ldy include padding)
  int ldx, ldy;          // leading dimensions (doubles, even)
  const double* Wp;      // ldx x r column-major (padded rows are 0)
  const double* Cp;      // ldy x r
  const PplsScalars* sc; // device scalars (alpha..delta)
  double* part;          // grid x part_ld partials
  int64_t part_ld;       // r*ldx + r*ldy + 4 r^2
  double* mu;            // n_local x 2r column-major [mu_T | mu_U] or nullptr
  int write_mu;
  int r;
  int ns;                // split sweep: column pairs per thread
  int threads;           // split sweep workgroup size (512)
  int rp;                // split sweep rows per pipeline step (0 auto, 1 or 2)
  int pipe;              // split kernel: 1 = dots(g+1) before update(g), 0 = after
  int* occ_out;          // split kernel: if set, report resident WGs per CU instead of launching
  int grid;              // workgroups (split) / row chunks (accumulation, panel accumulation)
  int nt;                // non-temporal loads of X, Y (data larger than the MALL)
  int dots_grid;         // panel dots workgroups (0 = enough for every row tile, capped)
  int dots_rows;         // panel dots rows per wave: 0 auto (64 from 32768 rows, else 32), 32, 64
  int dots_pair;         // panel dots wave pair per row tile: -1 auto (when tiles < wave slots), 0, 1
  int dots_only;         // panel: the dots pass only (Z and mu; scores)
  int num_cus;           // compute units of the device (panel dots: wave pairs on small shards)
  const int* stop;       // device stop flag (em_run's convergence test) or nullptr: kernels exit if set
  long long* trace;      // split sweep diagnostics: 4 wall-clock stamps per workgroup, or nullptr
  const int64_t* row_bounds;   // split sweep: grid + 1 row boundaries (workgroup g owns rows
                               // [b[g], b[g+1])), or nullptr for the even split
  const int* wg_seg;           // split sweep: per workgroup the index of its scalars (sc[wg_seg[g]]:
                               // meta_PPLSi's populations), or nullptr (sc for all)
  const int64_t* seg_ends;     // panel sweep, meta_PPLSi: nseg cumulative row ends of the populations;
  int nseg;                    // row i uses sc[j], j the first segment with i < seg_ends[j] (or nullptr)
  const int64_t* chunk_bounds; // panel accumulation: grid + 1 row boundaries of its chunks (each inside
                               // one population), or nullptr for the guided default
};

struct PplsFinalizeArgs {
  const double* stats;   // reduced [SX][SY][G]
  const double* ssq;     // {||X||^2, ||Y||^2}
  double N;
  int p, q, r, ldx, ldy;
  const double* Wc;
  const double* Cc;
  const PplsScalars* sc_cur;
  double* Wn;
  double* Cn;
  PplsScalars* sc_nxt;
  PplsMoments* mom;
  double* loglik;
  int logl_index;        // <0: do not write
  double* work;          // 2 (p+q) r doubles
  int* status;
  int qr;                // orth type: 0 SVD (polar), 1 QR
  int mode;              // bit0: W/C update (polar), bit1: scalars (moments, loglik, M-step),
                         // bit2: Cholesky-QR1 fast path allowed for well-conditioned X'mu
  const double* gram_cur;   // [W'W | C'C] (2 r^2) of Wc, Cc, or nullptr (finalize computes it)
  double* gram_nxt;         // receives [Wn'Wn | Cn'Cn], or nullptr
  double* vstate;           // [V_W | V_C] (2 r^2) Jacobi warm start carried across iterations, or nullptr
  long long* trace;      // diagnostics: per-block phase timestamps (16 per block) or nullptr
  int* stop;             // device stop flag or nullptr: the kernel exits if set; sets it (= stop_step)
                         // when stop_check and loglik[logl_index] - loglik[logl_index - 1] < atol
  int* stop_mirror;      // host-mapped copy of the flag the host polls (or nullptr)
  int stop_check, stop_step;
  double atol;
  unsigned* team_bar;    // wide-p polar teams: 8 zero-initialised counters, or nullptr (one block each)
  double* team_part;     // 2 x 3 x PPLS_TEAM_MAX x 64 doubles
  int team_rows;         // rows of S per team member (0: PPLS_TEAM_ROWS)
  const double* xpM;     // cross-product form (ppls_xprod.hip): M = S blockdiag(Wc, Cc), (ldx + ldy) x 2r
                         // column-major, or nullptr; when set, the scalar block forms the Gram B'M itself
                         // (in the slack of the polar blocks) and writes it to stats' Gram slot
};

#define PPLS_TEAM_ROWS 2048   // rows of S per polar team member (tools/team_rows_ab.py: p = 2000 in one block is 4 us faster than a team of 2; C5 equal at 1024 and 2048)
#define PPLS_TEAM_MAX 32
// finalize polar: Cholesky-QR1 (one pass, no second team barrier) when ||R1||_F ||R1^-1||_F <= this x r
// (a bound on kappa_2(X'mu); ||R||_F ||R^-1||_F >= r for any R)
#define PPLS_POLAR1_KAPPA 2.0

// One EM step of the sequential initialiser's rank-1 fit on the device (ppls_rank1_step_kernel).
struct PplsRank1StepArgs {
  const double* stats;     // the sweep's reduced statistics [SX ldx][SY ldy][G 4]
  int p, q, ldx, ldy;
  double N, ssqX, ssqY;    // ssq of the deflated data
  const double* Wp;        // deflation vectors w_1..w_m (p x m) and c_1..c_m (q x m)
  const double* Cp;
  int m;
  PplsRank1* st;           // the component's scalars (in/out)
  double* tw;              // its unit loadings w (p), c (q) (in/out)
  double* tc;
  const double* consW;     // fixed loadings (fconstraint) or nullptr
  const double* consC;
  PplsRank1 cons_val;      // fixed scalars, selected by cons_mask bits 0 B, 1 sigE, 2 sigF, 3 sigH, 4 sigT
  int cons_mask;
  double* Wdst;            // the next sweep's weight P_0..P_{m-1} w (ldx), P_0..P_{m-1} c (ldy), scalars
  double* Cdst;
  PplsScalars* scdst;
  double* lv;              // logvalue[0..max_steps]
  double* Gkeep;           // 4: the Gram of the last sweep that was not skipped
  int step, max_steps, crit_abs;
  double atol;
  int* stop;               // [0] step the stop rule fired at, [1] rank collapse (sigma < 100 eps)
  int* stop_mirror;        // host-mapped: nonzero once the fit ended
};

// One EM step of meta_PPLSi on the device (ppls_meta_step_kernel): log-likelihoods and stop rule of
// the step's sweep, then meta_EMstep's M-step for the next sweep.
#define PPLS_META_KMAX 1024
#define PPLS_OZ_MAXMOD 20   // int8 Gram (ppls_ozaki.hip): at most this many CRT moduli
#define PPLS_OZ_KS 64       // int8 Gram: rows per residue-plane stage (planes are [n / KS][Pp][KS] int8)
struct PplsMetaStepArgs {
  const double* stats;     // K x part_ld: per population [X_j'mu_T ldx][Y_j'mu_U ldy][Gram 4] (r = 1)
  int64_t part_ld;
  int K, p, q, ldx, ldy;
  const double* N;         // K: rows of each population (all ranks)
  const double* ssq;       // 2K: ssq(X_j), ssq(Y_j)
  PplsRank1* st;           // K population scalars (in/out)
  PplsScalars* sc;         // K: the next sweep's mu coefficients (out)
  double* W;               // the next sweep's shared loadings (ldx, ldy; out)
  double* C;
  double* log;             // logvalue: population j's column at j log_ld, rows 0 .. max_steps
  int64_t log_ld;
  int step, max_steps, crit_abs;
  double atol;
  int* stop;               // [0] the step the fit ended at, [1] 2 = NaN increment
  int* stop_mirror;        // host-mapped copy of stop[0], or nullptr
  double ssqX, ssqY, Ntot; // the whole data's: step 0 writes logvalue[1, ] = rep(logl_W(theta0), K)
                           // from the sum of the populations' Grams (theta0 is every population's)
};

extern "C" {
hipError_t ppls_launch_meta_step(const PplsMetaStepArgs* a, hipStream_t st);
int ppls_split_supported(int r, int ldx, int ldy);
hipError_t ppls_launch_sweep_split(const PplsSweepArgs* a, hipStream_t st);
int ppls_split_describe(const PplsSweepArgs* a, char* buf, int len);
// Maximiz_M on caller-supplied moments: X'mu_T, Y'mu_U partials from Z = [mu_T | mu_U] (row-major)
hipError_t ppls_launch_accumulate(const PplsSweepArgs* a, const double* Z, hipStream_t st);
int ppls_acc_groups(int64_t n_local, int grid);
// Wide-p panel sweep (two GEMM-shaped passes); Z: n_local x 4r doubles; chunks = partial groups.
int ppls_panel_chunks(int64_t n_local, int ldx, int ldy, int num_cus, int dtype_f32, int r);
int64_t ppls_panel_z_len(int64_t n_local, int ldx, int ldy, int r);   // doubles of Z (+ transposed W, C)
hipError_t ppls_launch_sweep_panel(const PplsSweepArgs* a, int dtype_f32, double* Z, int chunks, hipStream_t st);
// dots pass only: Z = [Xw | Yc | mu_T | mu_U] and (if a->write_mu) mu (n x 2r column-major)
hipError_t ppls_launch_panel_dots(const PplsSweepArgs* a, int dtype_f32, double* Z, hipStream_t st);
hipError_t ppls_launch_reduce(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                              int accumulate, hipStream_t st);
hipError_t ppls_launch_finalize(const PplsFinalizeArgs* f, hipStream_t st);
int64_t ppls_reduce_tmp_len(int ngroups, int64_t len);
hipError_t ppls_launch_reduce2(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                               double* tmp, const int* stop, hipStream_t st);
hipError_t ppls_launch_loglc(const double* G, const double* ssq, double N, int p, int q, int r,
                             double sigX, double sigY, const double* coefs, double* out, hipStream_t st);
hipError_t ppls_launch_sumsq(const double* a, int64_t len, double* part, int nblocks, double* out,
                             int out_accumulate, hipStream_t st);
hipError_t ppls_launch_deflated_ssq(const void* X, int f32, int64_t n, int ld, int p, const double* Wd, int m,
                                    double* part, int nblocks, double* out, hipStream_t st);
hipError_t ppls_launch_sumsq_f32(const float* a, int64_t len, double* part, int nblocks, double* out,
                                 hipStream_t st);
// element conversion fp64 <-> fp32 (same type: device copy)
hipError_t ppls_launch_convert(const void* src, int src_f32, void* dst, int dst_f32, int64_t len, hipStream_t st);
hipError_t ppls_launch_generate(int64_t n_local, int64_t row0, int p, int q, int ldx, int ldy, int r,
                                const PplsScalars* truth, const double* Wt, const double* Ct,
                                uint64_t seed, double* TU, double* X, double* Y, hipStream_t st);
hipError_t ppls_launch_rank1_step(const PplsRank1StepArgs* a, hipStream_t st);
hipError_t ppls_launch_philox(const uint32_t* ctr, int64_t count, uint64_t key, uint32_t* out, hipStream_t st);
hipError_t ppls_launch_to_rowmajor(const double* src, int64_t n, int p, int ld, double* dst,
                                   hipStream_t st);
// variances.PPLS_simult (ppls_variances.hip)
// The MFMA Gram.  xreal, xcols, yreal: the joint columns that can be non-zero ([0, xreal) of X and
// [xcols, xcols + yreal) of Y; for one block xcols = its ld, xreal = p, yreal = 0).
int ppls_gram_tiles(int p);
int ppls_gram_occupancy(int f32);
// row splits for n rows (nsplit_req > 0: equal splits; 0: halving) and their bounds (nsplit + 1, nullable)
int ppls_gram_plan(int p, int xreal, int xcols, int yreal, int64_t n, int wave_slots, int nsplit_req, int64_t* bounds);
int64_t ppls_gram_part_doubles(int p, int nsplit);   // the per-item partials a launch writes
int64_t ppls_gram_queue_ints(int p, int nsplit);
hipError_t ppls_gram_queue_prepare(int* queue, int p, int xreal, int xcols, int yreal, int64_t n, int wave_slots,
                                   int nsplit_req, hipStream_t st);
hipError_t ppls_launch_gram(const void* X, int f32, int64_t n, int ld, int p, int nsplit, double* part, int* queue,
                            hipStream_t st);
hipError_t ppls_launch_gram_finish(const double* part, int nsplit, int p, int xreal, int xcols, int yreal, double* G,
                                   hipStream_t st);
int ppls_xtmu_chunks(int64_t n, int ld, int f32);
hipError_t ppls_launch_xtmu(const void* X, int f32, int64_t n, int ld, const double* mu, int a, int chunks,
                            double* part, int64_t part_ld, hipStream_t st);
hipError_t ppls_launch_varmat(const double* G, const double* cxt, const double* w, int p, double ctt, double k1,
                              double k2, double bstar, double s4, double N, double* M, double* sst_exp,
                              double* sst_star, hipStream_t st);
hipError_t ppls_launch_negdiag(double* M, int p, double* se, hipStream_t st);
hipError_t ppls_launch_negate(double* M, int64_t len, hipStream_t st);
hipError_t ppls_launch_symdiag(double* M, int p, double* se, hipStream_t st);
// ppls_linalg.hip: batched inverse of SPD matrices (blocked Cholesky + inverse of the factor; the
// inverse's lower triangle in place), scratch and per-matrix pivot info (0, or the first bad pivot + 1)
int64_t ppls_spd_inverse_work(int p, int a);
hipError_t ppls_spd_inverse_batched(double* A, int p, int a, double* work, int* info, hipStream_t st);
hipError_t ppls_launch_to_colmajor(const double* src, int64_t n, int p, int ld, double* dst,
                                   hipStream_t st);
// ppls_ozaki.hip: the cross-product Gram D'D on int8 MFMA (Chinese-remainder form): column statistics
// (out = [max |D| | sum D^2] per joint column, Pp of each), residue planes [nkb][Pp][128] per modulus,
// the per-modulus SYRK of the lower 256 x 256 tiles (uint8 residues), and the CRT into G (P x P)
int ppls_oz_modulus(int l);
hipError_t ppls_launch_oz_colstats(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int yreal,
                                   int f32, int Pp, int64_t n, int chunks, double* part, double* out, hipStream_t st);
hipError_t ppls_launch_oz_residues(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int yreal,
                                   int f32, int Pp, int64_t n, int64_t nkb, const int* shift, int nmod, int8_t* planes,
                                   int64_t pstride, hipStream_t st);
int ppls_oz_splits(int64_t nkb);   // row splits of the SYRK (65,536 rows each: exact int32 sums)
hipError_t ppls_launch_oz_syrk(const int8_t* planes, int64_t pstride, int Pp, int64_t nkb, int nmod, uint8_t* part,
                               hipStream_t st);
hipError_t ppls_launch_oz_finish(const uint8_t* part, int nmod, int nsplit, int Pp, int xcols, int xreal, int yreal,
                                 int P, const int* shift, double* G, hipStream_t st);
}
