// ppls_capi.cpp -- host runtime + C ABI (include/ppls.h) of the MI355X PPLS_simult EM inner loop.
//
// One context = one GPU = one process rank.  Per EM iteration the host enqueues, on one HIP
// stream and without synchronising: sweep (1 pass over X, Y) -> deterministic reduction of the
// workgroup partials -> [RCCL all-reduce of (p+q) r + 4 r^2 doubles] -> finalize (E-step moments,
// log-likelihood, M-step incl. the polar factor).  The host only reads back the log-likelihood
// when the convergence test of PPLS_simult (EM_W_multi.R:792) needs it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ppls.h"
#include "../../include/ppls_debug.h"
#include "ppls_kernels.h"
#include "ppls_math.h"
#include "ppls_xprod.h"

struct ppls_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  int num_cus = 256;
  // options
  int sweep_mode = 0;      // 0 auto, 3 panel
  int grid_opt = 0;
  int rp_opt = 0;   // rows per pipeline step: 0 auto (2 where the kernel fits in registers)
  int pipe_opt = 1;     // split kernel: software-pipelined order
  int dots_rows = 0;   // panel dots rows per wave: 0 auto, 32, 64 (tests of both forms)
  int dots_pair = -1;  // panel dots wave pair per row tile: -1 auto, 0, 1
  int acc_chunks = 0;  // panel accumulation row chunks: 0 auto (ppls_panel_chunks), else forced
  int team_rows = 0;   // finalize polar team: rows of S per member (0: PPLS_TEAM_ROWS)
  int polar1 = 1;   // finalize polar: Cholesky-QR1 fast path when kappa(X'mu) <= PPLS_POLAR1_KAPPA
  int polar1_kappa = 0;   // its bound on ||R1||_F ||R1^-1||_F (0 = min(8 r, 40))
  int exact_gram = 1;     // finalize: compute W'W, C'C of the new loadings (1, default) or use I (0):
                          // I saves ~0.5 % at the C4/C5 shares but, through the cancellation in
                          // Cee at small sigma_E, moved mu_T by 1e-8 (golden stress_sig005)
  int ldpad = 1;   // row padding of the panel sweep's rows (ld_of); 0 = 16-B rows (experiment)
  int dtype = 0;           // storage of X, Y: 0 fp64, 1 fp32 (arithmetic is fp64 either way)
  int nt_loads = -1;       // sweep LDS-DMA non-temporal: -1 auto (when X, Y exceed the MALL), 0 off, 1 on
  int timing = 0;          // 0 off; N > 0: bracket every N-th sweep launch with HIP events
  int64_t sweep_count = 0;
  // row segment the next sweeps cover (meta_* per-population sweeps); seg_rows < 0 = all rows
  int64_t seg_row0 = 0, seg_rows = -1;
  // communicator: RCCL, or a caller-supplied host reduction (ppls_set_reducer)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  ppls_reduce_fn reducer = nullptr;
  void* reducer_user = nullptr;
  std::vector<double> reduce_host;
  // data
  bool have_data = false;
  int64_t n_local = 0, n_total = 0;
  int p = 0, q = 0, ldx = 0, ldy = 0;
  double* X = nullptr;
  double* Y = nullptr;
  double* ssq = nullptr;       // {||X||^2, ||Y||^2} (global)
  double ssq_host[2] = {0, 0};
  // the smallest free HBM over all ranks when the data were loaded (all-reduced beside ||X||^2,
  // ||Y||^2, so every rank sees the same value): the cross-product form's memory gate
  double mem_free_min = 0.0;
  double* flag = nullptr;      // 8 doubles for small agreement all-reduces (allocated with the data)
  // per-r state
  int r_alloc = 0;
  double* W[2] = {nullptr, nullptr};
  double* C[2] = {nullptr, nullptr};
  PplsScalars* sc[2] = {nullptr, nullptr};
  double* gram[2] = {nullptr, nullptr};   // [W'W | C'C] of W[i], C[i]
  double* vstate = nullptr;   // polar Jacobi warm start [V_W | V_C], reset on every theta upload
  PplsMoments* mom = nullptr;
  double* stats = nullptr;
  double* part = nullptr;
  int64_t part_ld = 0;
  int part_groups = 0;
  double* Z = nullptr;
  int z_cols = 0;          // columns allocated in Z (2r two-pass, 4r panel)
  double* mu = nullptr;
  double* loglik = nullptr;
  int loglik_cap = 0;
  double* work = nullptr;
  int* status = nullptr;
  long long* ftrace = nullptr;   // finalize phase timestamps (diagnostics)
  unsigned* team_bar = nullptr;  // finalize polar teams (wide p): counters (self-resetting) + partials
  double* team_part = nullptr;
  long long* strace = nullptr;   // split sweep per-workgroup stamps (diagnostics, PPLS_STRACE_MAX_WG x 4)
  // split-sweep load balance: the XCDs of one MI355X stream rows at rates that differ by up to ~3 %,
  // the same way every iteration (profiles/r3_sweep_balance_*.txt), so the even row split leaves a
  // tail.  The first full split sweep of the data is timed per workgroup (untimed calibration
  // launches), workgroup g then owns a row block proportional to the measured rate of its class
  // g % 8 (the XCD under round-robin dispatch); fixed afterwards, so results stay deterministic.
  int balance = 0;                 // option "balance": 1 calibrate, 0 the even split (default: bitwise
                                   // reproducible across processes; the calibrated split regroups the sums)
  bool bal_done = false;           // calibrated for (bal_n, bal_grid)
  int64_t bal_n = -1;
  int bal_grid = -1;
  double bal_w[8] = {1, 1, 1, 1, 1, 1, 1, 1};
  int64_t* bal_bounds = nullptr;   // device: grid + 1 row boundaries
  double* coefs = nullptr;     // loglC_fast coefficient block (5r)
  double* scratch = nullptr;   // generic device scratch
  size_t scratch_bytes = 0;
  // ppls_em_run's device-side stop rule: a device flag every kernel of the run checks, set by the
  // finalize that sees logl[i] - logl[i-1] < atol, and its host-mapped mirror the host polls
  int* stop_d = nullptr;
  int* stop_mirror = nullptr;       // host pointer (hipHostMalloc, mapped, coherent)
  int* stop_mirror_dev = nullptr;   // its device address
  const int* sweep_stop = nullptr;  // non-null only inside ppls_em_run with a finite atol
  double stop_atol = 0.0;
  // device-resident iteration state (ppls_em_begin / ppls_em_iterate)
  int em_r = 0, em_cur = 0, em_iter = 0;
  bool em_active = false;
  // cross-product form of the iteration (ppls_xprod.hip): S = [X Y]'[X Y] (P x P, P = ldx + ldy)
  // formed once per data set, then every statistics step reads S instead of X and Y
  int xprod = 0;            // option "xprod": 0 stream X, Y (default), 1 cross-products, -1 auto (cost model)
  int xprod_rw = 0;         // option "xprod_rw": rows of S per wave of the tile kernel (0 auto)
  int gram_int8 = 0;        // option "gram_int8": S by the int8-MFMA CRT form (1, when the column spread
                            // allows; else the fp64 MFMA Gram) or the fp64 MFMA Gram (0)
  int oz_used = 0, oz_nmod = 0, oz_L = 0;   // the last formation of S: which Gram, moduli, bits
  std::vector<int> oz_shift;                 // its per-column scalings x' = rint(D 2^shift)
  double oz_ms[4] = {0, 0, 0, 0};           // its phases (HIP events): stats+residues, SYRK, CRT, total
  // the int8 Gram's residue planes and SYRK output, kept between formations (allocating and freeing
  // tens of GB per call made later calls' hipMalloc / hipFree take ~1 s each after a dozen calls,
  // tools/oz_repeat_probe.py); freed with ppls_xprod_release, new data, gram_int8 = 0 or the context
  int8_t* oz_planes = nullptr;
  uint8_t* oz_res = nullptr;
  size_t oz_planes_len = 0, oz_res_len = 0;
  bool xp_ready = false;    // S holds the (all-reduced) cross-products of the current data
  bool xp_active = false;   // statistics steps of the current run read S
  bool xp_pending_gram = false;   // the last statistics step left the Gram B'M to the next finalize
  int xprod_fuse = 1;       // option "xprod_fuse": the finalize forms the Gram (r <= 8, P <= 6144)
  bool xp_explicit = false; // S was formed by ppls_xprod_prepare: kept until ppls_xprod_release / new data
  int meta_path = 0;        // the last ppls_meta_ppls: 1 host loop, 2 device split, 3 device panel
  int meta_device = 1;      // option "meta_device": meta_PPLSi's loop on the device (1) or per population
                            // from the host (0; also where the split sweep does not apply)
  int vorth = 8;            // option "vorth": the finalize re-orthonormalises its carried Jacobi V every
                            // vorth-th iteration (1 = every iteration)
  double* xp_S = nullptr;
  double* xp_M = nullptr;   // M = S blockdiag(W, C), P x 2r scratch
  double xp_setup_ms = 0.0; // last formation of S: Gram kernel (HIP events), and with the all-reduce
  double xp_setup_total_ms = 0.0;
  double xp_setup_ar_ms = 0.0;   // the all-reduce of S (wall clock around it and its stream sync)
  int xp_nsplit = 0;
  // the MFMA Gram's work queue (S, variances' X'X), prepared for one shape
  int* gram_q = nullptr;
  // (p, xreal, xcols, yreal, n, nsplit_req, nsplit, wave slots) of gram_q: the queue layout depends
  // on the split count and the slot count, which follow the storage dtype's occupancy
  int64_t gq_key[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
  rocblas_handle blas = nullptr;   // rocSOLVER (variances.PPLS_simult's p x p inverse), created lazily
  int var_chol = 1;                // option "var_chol": that inverse by Cholesky when positive definite: 1 hand-written
                                   // (ppls_linalg.hip), 2 rocSOLVER potrf/potri; 0 LU (rocSOLVER getrf/getri)
  // timing
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
  size_t ev_used = 0;
  double timed_ms = 0.0;
  int64_t timed_launches = 0;
  // the statistics all-reduce of the timed sweeps (RCCL only), same bookkeeping
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_ar;
  size_t ev_ar_used = 0;
  double ar_ms = 0.0;
  int64_t ar_calls = 0;
};

namespace {

int fail(ppls_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIPCHK(c, call)                                                                   \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail((c), PPLS_E_HIP, "%s: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                  __LINE__);                                                              \
  } while (0)

#define RCCLCHK(c, call)                                                                  \
  do {                                                                                    \
    ncclResult_t e_ = (call);                                                             \
    if (e_ != ncclSuccess)                                                                \
      return fail((c), PPLS_E_COMM, "%s: %s", #call, ncclGetErrorString(e_));            \
  } while (0)

void oz_free(ppls_ctx* c);
bool oz_held(const ppls_ctx* c);

template <typename T>
int dalloc(ppls_ctx* c, T** p, size_t count) {
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
  }
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e == hipErrorOutOfMemory && oz_held(c) && (void*)p != (void*)&c->oz_planes && (void*)p != (void*)&c->oz_res) {
    // the int8 Gram's kept workspace gives way first
    (void)hipGetLastError();
    (void)hipStreamSynchronize(c->stream);
    oz_free(c);
    e = hipMalloc((void**)p, count * sizeof(T));
  }
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(c, PPLS_E_NOMEM, "hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
  }
  return PPLS_OK;
}

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// Row stride (elements) of the resident X or Y.  16-B rows for narrow data and for the fp64 rows of
// the split sweep (p <= 2048: its DMA ring streams whole row ranges, alignment beyond 16 B is moot,
// and C3's 16,000-B rows stay unpadded).  Rows the panel sweep reads (fp32 storage, wider fp64) are
// padded to 128 B (one cache line per dots tile) and from 16 KB to 4 KB: the accumulation pass reads
// 4-KB column segments of every row, and 4-KB-aligned segments stream faster -- 5e5 x 40 KB rows,
// no arithmetic: 16-B-aligned stride 3.24 ms, 128-B 3.07 ms, 4-KB 2.93 ms
// (tools/acc_pattern_probe.hip, profiles/r2_row_alignment_probe.txt).  Padding columns are zero.
int ld_of(int p, int f32 = 0, int pad = 1) {
  const int es = f32 ? 4 : 8;
  const long bytes = (long)p * es;
  if (!pad || bytes < 1024 || (!f32 && p <= 2048)) return f32 ? (p + 3) & ~3 : (p + 1) & ~1;
  const long al = bytes >= 16384 ? 4096 : 128;
  return (int)(((bytes + al - 1) / al * al) / es);
}

int check_theta(ppls_ctx* c, const ppls_theta* th, int r) {
  if (!th || !th->W || !th->C || !th->B || !th->sigT) return fail(c, PPLS_E_ARG, "theta has NULL fields");
  if (r < 1 || r > PPLS_RMAX) return fail(c, PPLS_E_ARG, "r=%d outside [1,%d]", r, PPLS_RMAX);
  if (!(th->sigE > 0) || !(th->sigF > 0) || !(th->sigH >= 0))
    return fail(c, PPLS_E_ARG, "variances must be positive");
  bool fin = std::isfinite(th->sigE) && std::isfinite(th->sigF) && std::isfinite(th->sigH);
  for (int k = 0; k < r; ++k) fin = fin && std::isfinite(th->B[k]) && std::isfinite(th->sigT[k]);
  if (!fin) return fail(c, PPLS_E_ARG, "theta has non-finite B, sigT or variances");
  // PPLS: stopifnot(ncol(X) >= nr_comp, ncol(Y) >= nr_comp)  (EM_W_multi.R:245)
  if (c && c->p > 0 && (c->p < r || c->q < r))
    return fail(c, PPLS_E_ARG, "ncol(X)=%d, ncol(Y)=%d must be >= number of components %d", c->p, c->q, r);
  return PPLS_OK;
}

PplsScalars scalars_of(const ppls_theta* th, int r) {
  PplsScalars s;
  memset(&s, 0, sizeof s);
  for (int k = 0; k < r; ++k) {
    s.b[k] = th->B[k];
    s.t[k] = th->sigT[k];
  }
  s.sigE = th->sigE;
  s.sigF = th->sigF;
  s.sigH = th->sigH;
  ppls_mu_coef(&s, r);
  return s;
}

int ensure_r(ppls_ctx* c, int r, int max_steps) {
  int rc;
  c->em_active = false;   // every entry point that (re)stages theta ends an ppls_em_begin session
  c->xp_active = false;
  if (r != c->r_alloc) {
    for (int i = 0; i < 2; ++i) {
      if ((rc = dalloc(c, &c->W[i], (size_t)c->ldx * r))) return rc;
      if ((rc = dalloc(c, &c->C[i], (size_t)c->ldy * r))) return rc;
      if ((rc = dalloc(c, &c->sc[i], 1))) return rc;
      if ((rc = dalloc(c, &c->gram[i], (size_t)2 * r * r))) return rc;
    }
    if ((rc = dalloc(c, &c->mom, 1))) return rc;
    if ((rc = dalloc(c, &c->vstate, (size_t)2 * r * r))) return rc;
    c->part_ld = (int64_t)r * c->ldx + (int64_t)r * c->ldy + 4 * (int64_t)r * r;
    if ((rc = dalloc(c, &c->stats, (size_t)c->part_ld))) return rc;
    if ((rc = dalloc(c, &c->work, (size_t)2 * (c->p + c->q) * r + 16))) return rc;
    if ((rc = dalloc(c, &c->status, 1))) return rc;
    if ((rc = dalloc(c, &c->coefs, (size_t)5 * r))) return rc;
    dfree(c->part);
    dfree(c->Z);
    c->z_cols = 0;
    dfree(c->mu);
    c->part_groups = 0;
    c->r_alloc = r;
  }
  if (max_steps + 2 > c->loglik_cap) {
    if ((rc = dalloc(c, &c->loglik, (size_t)max_steps + 2))) return rc;
    c->loglik_cap = max_steps + 2;
  }
  return PPLS_OK;
}

int upload_theta(ppls_ctx* c, const ppls_theta* th, int r, int slot) {
  // W, C: p x r column-major -> ldx x r padded
  std::vector<double> buf((size_t)std::max(c->ldx, c->ldy) * r, 0.0);
  for (int k = 0; k < r; ++k)
    for (int i = 0; i < c->ldx; ++i) buf[(size_t)k * c->ldx + i] = i < c->p ? th->W[(size_t)k * c->p + i] : 0.0;
  HIPCHK(c, hipMemcpyAsync(c->W[slot], buf.data(), sizeof(double) * c->ldx * r, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < r; ++k)
    for (int i = 0; i < c->ldy; ++i) buf[(size_t)k * c->ldy + i] = i < c->q ? th->C[(size_t)k * c->q + i] : 0.0;
  HIPCHK(c, hipMemcpyAsync(c->C[slot], buf.data(), sizeof(double) * c->ldy * r, hipMemcpyHostToDevice, c->stream));
  PplsScalars s = scalars_of(th, r);
  HIPCHK(c, hipMemcpyAsync(c->sc[slot], &s, sizeof s, hipMemcpyHostToDevice, c->stream));
  // [W'W | C'C] for the finalize's scalar block (later iterations get it from the polar blocks)
  std::vector<double> g((size_t)2 * r * r);
  for (int a = 0; a < r; ++a)
    for (int b = 0; b < r; ++b) {
      double w = 0.0, cc = 0.0;
      for (int i = 0; i < c->p; ++i) w += th->W[(size_t)a * c->p + i] * th->W[(size_t)b * c->p + i];
      for (int i = 0; i < c->q; ++i) cc += th->C[(size_t)a * c->q + i] * th->C[(size_t)b * c->q + i];
      g[(size_t)b * r + a] = w;
      g[(size_t)r * r + (size_t)b * r + a] = cc;
    }
  HIPCHK(c, hipMemcpyAsync(c->gram[slot], g.data(), sizeof(double) * g.size(), hipMemcpyHostToDevice, c->stream));
  // identity warm start for the polar Jacobi: a run's result depends only on its own theta0
  std::vector<double> eye(g.size());
  for (size_t e = 0; e < eye.size(); ++e) eye[e] = ((e % ((size_t)r * r)) % (size_t)(r + 1)) == 0 ? 1.0 : 0.0;
  HIPCHK(c, hipMemcpyAsync(c->vstate, eye.data(), sizeof(double) * eye.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PPLS_OK;
}

int download_theta(ppls_ctx* c, int r, int slot, ppls_theta* th) {
  std::vector<double> buf((size_t)std::max(c->ldx, c->ldy) * r);
  HIPCHK(c, hipMemcpy(buf.data(), c->W[slot], sizeof(double) * c->ldx * r, hipMemcpyDeviceToHost));
  for (int k = 0; k < r; ++k)
    for (int i = 0; i < c->p; ++i) th->W[(size_t)k * c->p + i] = buf[(size_t)k * c->ldx + i];
  HIPCHK(c, hipMemcpy(buf.data(), c->C[slot], sizeof(double) * c->ldy * r, hipMemcpyDeviceToHost));
  for (int k = 0; k < r; ++k)
    for (int i = 0; i < c->q; ++i) th->C[(size_t)k * c->q + i] = buf[(size_t)k * c->ldy + i];
  PplsScalars s;
  HIPCHK(c, hipMemcpy(&s, c->sc[slot], sizeof s, hipMemcpyDeviceToHost));
  for (int k = 0; k < r; ++k) {
    th->B[k] = s.b[k];
    th->sigT[k] = s.t[k];
  }
  th->sigE = s.sigE;
  th->sigF = s.sigF;
  th->sigH = s.sigH;
  return PPLS_OK;
}

int download_moments(ppls_ctx* c, int r, ppls_expect* e) {
  if (!e) return PPLS_OK;
  PplsMoments m;
  HIPCHK(c, hipMemcpy(&m, c->mom, sizeof m, hipMemcpyDeviceToHost));
  for (int k = 0; k < r; ++k) {
    if (e->Ctt) e->Ctt[k] = m.Ctt[k];
    if (e->Cuu) e->Cuu[k] = m.Cuu[k];
    if (e->Cut) e->Cut[k] = m.Cut[k];
  }
  e->Cee = m.Cee;
  e->Cff = m.Cff;
  if (e->Chh)
    for (int i = 0; i < r * r; ++i) e->Chh[i] = m.Chh[i];
  return PPLS_OK;
}

int download_mu(ppls_ctx* c, int r, ppls_expect* e) {
  if (!e || (!e->mu_T && !e->mu_U) || c->n_local == 0) return PPLS_OK;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t blk = sizeof(double) * (size_t)c->n_local * r;
  if (e->mu_T) HIPCHK(c, hipMemcpy(e->mu_T, c->mu, blk, hipMemcpyDeviceToHost));
  if (e->mu_U) HIPCHK(c, hipMemcpy(e->mu_U, c->mu + (size_t)c->n_local * r, blk, hipMemcpyDeviceToHost));
  return PPLS_OK;
}

// The finalize's Cholesky-QR1 acceptance bound on ||R1||_F ||R1^-1||_F (>= kappa_2): CholQR1 loses
// ~eps kappa^2 of orthogonality, so the default keeps kappa <= 40 (<= 1e-13); at C3/C4 it lets
// Y'mu_U (kappa ~ 20) skip the second Cholesky-QR pass (profiles/r3_polar1_kappa_ab.txt).
int polar1_bound(const ppls_ctx* c, int r) {
  if (c->polar1_kappa > 0) return c->polar1_kappa;
  return std::min(8 * r, 40);
}

int grid_of(ppls_ctx* c) { return c->grid_opt > 0 ? c->grid_opt : c->num_cus; }

// Allreduce in place (sum) over ranks, on the context stream: RCCL, or the caller's host
// reduction (ppls_set_reducer: device -> host, fn sums over the caller's ranks, host -> device).
int allreduce(ppls_ctx* c, double* buf, size_t count) {
  if (c->reducer) {
    if (c->reduce_host.size() < count) c->reduce_host.resize(count);
    double* h = c->reduce_host.data();
    HIPCHK(c, hipMemcpyAsync(h, buf, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const int rc = c->reducer(c->reducer_user, h, (int64_t)count);
    if (rc != 0) return fail(c, PPLS_E_COMM, "host reducer returned %d", rc);
    HIPCHK(c, hipMemcpyAsync(buf, h, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PPLS_OK;
  }
  if (!c->comm) return PPLS_OK;   // a 1-rank communicator still takes the RCCL path
  RCCLCHK(c, ncclAllReduce(buf, buf, count, ncclDouble, ncclSum, c->comm, c->stream));
  return PPLS_OK;
}

// Per-group partials plus, behind them, the two-stage reduction's chunk sums (sized for the largest
// group count seen, so the tail pointer part + part_groups * part_ld is always in bounds).
int ensure_part(ppls_ctx* c, int groups) {
  if (groups <= c->part_groups && c->part) return PPLS_OK;
  const size_t tmp = (size_t)ppls_reduce_tmp_len(groups, c->part_ld);
  int rc = dalloc(c, &c->part, (size_t)groups * c->part_ld + tmp);
  c->part_groups = rc ? 0 : groups;
  return rc;
}

// Which sweep kernel runs for this shape: 3 = split ownership (default), 4 = panel (wide p, large r
// or fp32 storage, or option sweep = 3); a->grid is the workgroup count.
int64_t sweep_rows(const ppls_ctx* c) { return c->seg_rows >= 0 ? c->seg_rows : c->n_local; }

int sweep_plan(ppls_ctx* c, int r, PplsSweepArgs* a) {
  const int64_t nrows = sweep_rows(c);
  const int nsplit = ppls_split_supported(r, c->ldx, c->ldy);
  memset(a, 0, sizeof *a);
  a->ldx = c->ldx;
  a->ldy = c->ldy;
  a->p = c->p;
  a->q = c->q;
  a->r = r;
  a->threads = 512;
  a->num_cus = c->num_cus;
  a->dots_rows = c->dots_rows;
  a->dots_pair = c->dots_pair;
  if (c->sweep_mode != 3 && !c->dtype && nsplit > 0) {
    a->ns = nsplit;
    a->pipe = c->pipe_opt;
    a->rp = c->rp_opt;             // 0 = auto: two rows per step wherever instantiated
    int occ = 0;
    a->occ_out = &occ;
    if (ppls_launch_sweep_split(a, c->stream) != hipSuccess || occ < 1) occ = 1;
    a->occ_out = nullptr;
    a->grid = c->grid_opt > 0 ? c->grid_opt : c->num_cus * occ;
    return 3;
  }
  // wide data / large r / fp32 storage: the panel sweep (two GEMM-shaped passes)
  a->grid = c->acc_chunks > 0 ? c->acc_chunks
          : c->grid_opt > 0 ? c->grid_opt : ppls_panel_chunks(nrows, c->ldx, c->ldy, c->num_cus, c->dtype, r);
  a->dots_grid = c->grid_opt;   // the grid option also sets the dots grid (tests: grid-stride path)
  return 4;
}

// Split-sweep row balance (see the context's bal_* fields).  For a full sweep of n_local rows on
// `grid` workgroups, the first call runs PPLS_BAL_CAL calibration launches with per-workgroup
// stamps (host syncs; their partials are overwritten by the real launch that follows): each times
// when every workgroup's row loop ends under the current partition, and the rows of XCD class x
// (g % 8) are rescaled by sqrt(mean end time / class end time) -- a damped fixed-point iteration
// (the first launch only warms up), since a class that finishes early hands its HBM share to the
// others, so the rates move with the partition.  Later calls reuse the boundaries, so results are
// deterministic for the context.  Shapes with fewer than PPLS_BAL_MIN_ROWS rows per workgroup keep
// the even split.
#define PPLS_BAL_CAL 8
#define PPLS_BAL_MIN_ROWS 2048   // C3: 3,906 rows per workgroup; at 488 (one GPU's C4 share) the calibration noise costs more than the tail
namespace {
void bal_bounds_of(const double* w, int grid, int64_t n, std::vector<int64_t>& bnd) {
  bnd.assign((size_t)grid + 1, 0);
  double tot = 0.0;
  for (int g = 0; g < grid; ++g) tot += w[g % 8];
  double cum = 0.0;
  for (int g = 0; g < grid; ++g) {
    cum += w[g % 8];
    int64_t b = g + 1 == grid ? n : std::min<int64_t>(n, (int64_t)std::llround(cum / tot * (double)n));
    bnd[(size_t)g + 1] = std::max(b, bnd[g]);
  }
}
}  // namespace

int balance_rows(ppls_ctx* c, PplsSweepArgs* a) {
  const int grid = a->grid;
  const int64_t n = a->n_local;
  if (grid < 16 || grid > PPLS_STRACE_MAX_WG || n < (int64_t)PPLS_BAL_MIN_ROWS * grid) return PPLS_OK;
  if (!(c->bal_done && c->bal_n == n && c->bal_grid == grid)) {
    int rc;
    struct OwnTrace {   // a stamp buffer of our own unless tracing is on; freed on every exit path
      ppls_ctx* c;
      bool own;
      ~OwnTrace() {
        if (own && c->strace) { (void)hipFree(c->strace); c->strace = nullptr; }
      }
    } tg{c, c->strace == nullptr};
    if (tg.own) HIPCHK(c, hipMalloc(&c->strace, (size_t)PPLS_STRACE_MAX_WG * 4 * sizeof(long long)));
    if ((rc = dalloc(c, &c->bal_bounds, (size_t)grid + 1))) return rc;
    PplsSweepArgs b = *a;
    b.trace = c->strace;
    b.row_bounds = c->bal_bounds;
    b.stop = nullptr;
    b.mu = nullptr;
    b.write_mu = 0;
    double w[8] = {1, 1, 1, 1, 1, 1, 1, 1};
    std::vector<int64_t> bnd;
    std::vector<long long> st((size_t)grid * 4);
    for (int k = 0; k < PPLS_BAL_CAL; ++k) {
      bal_bounds_of(w, grid, n, bnd);
      HIPCHK(c, hipMemcpyAsync(c->bal_bounds, bnd.data(), sizeof(int64_t) * bnd.size(), hipMemcpyHostToDevice,
                               c->stream));
      HIPCHK(c, ppls_launch_sweep_split(&b, c->stream));
      HIPCHK(c, hipMemcpyAsync(st.data(), c->strace, st.size() * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      long long t0 = st[0];
      for (int g = 1; g < grid; ++g) t0 = std::min(t0, st[(size_t)g * 4]);
      double cls[8] = {0}, cnt[8] = {0}, mean = 0.0;
      for (int g = 0; g < grid; ++g) {
        cls[g % 8] += (double)(st[(size_t)g * 4 + 2] - t0);   // this workgroup's row loop ends
        cnt[g % 8] += 1.0;
      }
      bool ok = true;
      for (int x = 0; x < 8; ++x) {
        cls[x] = cnt[x] > 0 ? cls[x] / cnt[x] : 0.0;
        ok = ok && cls[x] > 0.0;
        mean += cls[x] / 8.0;
      }
      if (!ok) break;
      if (k == 0) continue;   // the first launch warms caches and clocks; its times are not used
      for (int x = 0; x < 8; ++x) w[x] *= std::sqrt(mean / cls[x]);   // damped: the rates move with the load
      double wm = 0.0;
      for (int x = 0; x < 8; ++x) wm += w[x] / 8.0;
      for (int x = 0; x < 8; ++x) w[x] = std::min(1.1, std::max(0.9, w[x] / wm));   // a mis-measurement
    }                                                                                 // cannot starve an XCD
    for (int x = 0; x < 8; ++x) c->bal_w[x] = std::round(w[x] * 4096.0) / 4096.0;
    bal_bounds_of(c->bal_w, grid, n, bnd);
    HIPCHK(c, hipMemcpy(c->bal_bounds, bnd.data(), sizeof(int64_t) * bnd.size(), hipMemcpyHostToDevice));
    c->bal_done = true;
    c->bal_n = n;
    c->bal_grid = grid;
  }
  a->row_bounds = c->bal_bounds;
  return PPLS_OK;
}

// The next pair of timing events for a statistics launch, when option "timing" selects this one.
int timing_pair(ppls_ctx* c, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  if (!(c->timing > 0 && (c->sweep_count++ % c->timing) == 0)) return PPLS_OK;
  if (c->ev_used == c->ev.size()) {
    std::pair<hipEvent_t, hipEvent_t> pr;
    HIPCHK(c, hipEventCreate(&pr.first));
    HIPCHK(c, hipEventCreate(&pr.second));
    c->ev.push_back(pr);
  }
  *e0 = c->ev[c->ev_used].first;
  *e1 = c->ev[c->ev_used].second;
  ++c->ev_used;
  return PPLS_OK;
}

// One sweep with theta[slot] -> c->stats (all-reduced).  mu_only: just this rank's mu rows (the
// statistics are not reduced: no collective).
int sweep(ppls_ctx* c, int r, int slot, bool write_mu, bool mu_only = false) {
  int rc;
  PplsSweepArgs a;
  const int plan = sweep_plan(c, r, &a);
  const int64_t nrows = sweep_rows(c);
  if (c->seg_rows >= 0 && write_mu) return fail(c, PPLS_E_STATE, "mu write-out is not available for row segments");
  const int groups = a.grid;
  if ((rc = ensure_part(c, groups))) return rc;
  if (write_mu && !c->mu)
    if ((rc = dalloc(c, &c->mu, (size_t)std::max<int64_t>(c->n_local, 1) * 2 * r))) return rc;
  if (plan == 4 && c->z_cols < 4 * r) {
    dfree(c->Z);
    c->z_cols = 0;
    if ((rc = dalloc(c, &c->Z, (size_t)ppls_panel_z_len(c->n_local, c->ldx, c->ldy, r)))) return rc;
    c->z_cols = 4 * r;
  }
  if (nrows == 0) {
    if (mu_only) return PPLS_OK;
    HIPCHK(c, hipMemsetAsync(c->stats, 0, sizeof(double) * c->part_ld, c->stream));
  } else {
    const size_t esz = c->dtype ? sizeof(float) : sizeof(double);
    a.X = (const double*)((const char*)c->X + (size_t)c->seg_row0 * c->ldx * esz);
    a.Y = (const double*)((const char*)c->Y + (size_t)c->seg_row0 * c->ldy * esz);
    a.n_local = nrows;
    a.Wp = c->W[slot];
    a.Cp = c->C[slot];
    a.sc = c->sc[slot];
    a.part = c->part;
    a.part_ld = c->part_ld;
    a.mu = write_mu ? c->mu : nullptr;
    a.write_mu = write_mu ? 1 : 0;
    // once-read streams bigger than the 256 MB MALL: the non-temporal policy lands 3-9 % faster
    // (6.53 vs 6.34 TB/s at C3); smaller X, Y stay MALL-resident across iterations by default
    const bool nt = c->nt_loads > 0 ||
                    (c->nt_loads < 0 && 8.0 * nrows * (double)(c->ldx + c->ldy) > 256.0 * (1 << 20));
    a.nt = nt ? 1 : 0;
    a.stop = c->sweep_stop;
    a.trace = (plan == 3 && a.grid <= PPLS_STRACE_MAX_WG) ? c->strace : nullptr;
    // the row partition (its one-time calibration launches stay outside the timed events)
    if (plan == 3 && c->balance && c->seg_rows < 0 && (rc = balance_rows(c, &a))) return rc;
    if (mu_only) {   // the rows' mu only (untimed): the panel sweep's dots pass, or the split sweep
      if (plan == 4) HIPCHK(c, ppls_launch_panel_dots(&a, c->dtype, c->Z, c->stream));
      else HIPCHK(c, ppls_launch_sweep_split(&a, c->stream));
      return PPLS_OK;
    }
    hipEvent_t e0, e1;
    if ((rc = timing_pair(c, &e0, &e1))) return rc;
    const bool timed = e0 != nullptr;
    if (timed) HIPCHK(c, hipEventRecord(e0, c->stream));
    if (plan == 3) HIPCHK(c, ppls_launch_sweep_split(&a, c->stream));
    else HIPCHK(c, ppls_launch_sweep_panel(&a, c->dtype, c->Z, a.grid, c->stream));
    if (timed) HIPCHK(c, hipEventRecord(e1, c->stream));
    HIPCHK(c, ppls_launch_reduce2(c->part, groups, c->part_ld, c->part_ld, c->stats,
                                  c->part + (size_t)c->part_groups * c->part_ld, c->sweep_stop, c->stream));
    if (timed && c->comm && !c->reducer) {   // time this iteration's RCCL all-reduce as well
      if (c->ev_ar_used == c->ev_ar.size()) {
        std::pair<hipEvent_t, hipEvent_t> pr;
        HIPCHK(c, hipEventCreate(&pr.first));
        HIPCHK(c, hipEventCreate(&pr.second));
        c->ev_ar.push_back(pr);
      }
      const auto& pr = c->ev_ar[c->ev_ar_used++];
      HIPCHK(c, hipEventRecord(pr.first, c->stream));
      const int rc = allreduce(c, c->stats, (size_t)c->part_ld);
      HIPCHK(c, hipEventRecord(pr.second, c->stream));
      return rc;
    }
  }
  return allreduce(c, c->stats, (size_t)c->part_ld);
}

int finalize(ppls_ctx* c, int r, int cur, int nxt, int logl_index, int type, int stop_step = 0) {
  PplsFinalizeArgs f;
  f.stats = c->stats;
  f.ssq = c->ssq;
  f.N = (double)c->n_total;
  f.p = c->p;
  f.q = c->q;
  f.r = r;
  f.ldx = c->ldx;
  f.ldy = c->ldy;
  f.Wc = c->W[cur];
  f.Cc = c->C[cur];
  f.sc_cur = c->sc[cur];
  f.Wn = c->W[nxt];
  f.Cn = c->C[nxt];
  f.sc_nxt = c->sc[nxt];
  f.mom = c->mom;
  f.loglik = c->loglik;
  f.logl_index = logl_index;
  f.work = c->work;
  f.status = c->status;
  f.qr = type == PPLS_ORTH_QR ? 1 : 0;
  f.mode = 3 | (c->polar1 ? 4 : 0) | (c->exact_gram ? 16 : 0) | (polar1_bound(c, r) << 8) | (c->vorth << 16);
  f.trace = c->ftrace;
  f.gram_cur = c->gram[cur];
  f.gram_nxt = c->gram[nxt];
  f.vstate = c->vstate;
  if (!c->team_bar) {
    int rc;
    if ((rc = dalloc(c, &c->team_bar, 8)) || (rc = dalloc(c, &c->team_part, (size_t)2 * 3 * PPLS_TEAM_MAX * 64)))
      return rc;
    HIPCHK(c, hipMemsetAsync(c->team_bar, 0, 8 * sizeof(unsigned), c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  f.team_bar = c->team_bar;
  f.team_rows = c->team_rows;
  f.team_part = c->team_part;
  f.stop = c->sweep_stop ? c->stop_d : nullptr;
  f.stop_mirror = c->sweep_stop ? c->stop_mirror_dev : nullptr;
  f.stop_check = stop_step > 0 ? 1 : 0;
  f.stop_step = stop_step;
  f.atol = c->stop_atol;
  f.xpM = c->xp_pending_gram ? c->xp_M : nullptr;   // the Gram of a cross-product step, formed here
  c->xp_pending_gram = false;
  HIPCHK(c, ppls_launch_finalize(&f, c->stream));
  return PPLS_OK;
}

// The column space of one MFMA Gram (ppls_variances.hip): joint = S = [X Y]'[X Y] over the padded
// rows (X's p real columns of ldx, then Y's q of ldy), else D'D for D = X (xory 0) or Y.
struct GramShape {
  int p, xreal, xcols, yreal;
  const void* X;
  int ldx;
  const void* Y;
  int ldy, ycols;
};

GramShape gram_shape(const ppls_ctx* c, bool joint, int xory) {
  if (joint) return GramShape{c->ldx + c->ldy, c->p, c->ldx, c->q, c->X, c->ldx, c->Y, c->ldy, c->ldy};
  const int p = xory ? c->q : c->p, ld = xory ? c->ldy : c->ldx;
  return GramShape{p, p, ld, 0, xory ? (const void*)c->Y : (const void*)c->X, ld, nullptr, 0, 0};
}

int gram_wave_slots(const ppls_ctx* c) { return c->num_cus * ppls_gram_occupancy(c->dtype) * 4; }

// Row splits of a Gram over n rows (0 = auto: halving splits, ppls_gram_plan).
int gram_nsplit(const ppls_ctx* c, const GramShape& g, int64_t n, int req) {
  return ppls_gram_plan(g.p, g.xreal, g.xcols, g.yreal, n, gram_wave_slots(c), req, nullptr);
}

// The Gram's work queue for (shape, n, req, split plan, wave slots), prepared once and kept while
// all of them repeat.
int gram_queue(ppls_ctx* c, const GramShape& g, int64_t n, int req, int** q) {
  const int nsplit = gram_nsplit(c, g, n, req);
  const int64_t key[8] = {g.p, g.xreal, g.xcols, g.yreal, n, req, nsplit, gram_wave_slots(c)};
  if (c->gram_q && !memcmp(key, c->gq_key, sizeof key)) {
    *q = c->gram_q;
    return PPLS_OK;
  }
  *q = nullptr;
  int rc;
  c->gq_key[0] = -1;
  if ((rc = dalloc(c, &c->gram_q, (size_t)ppls_gram_queue_ints(g.p, nsplit)))) return rc;
  HIPCHK(c, ppls_gram_queue_prepare(c->gram_q, g.p, g.xreal, g.xcols, g.yreal, n, gram_wave_slots(c), req, c->stream));
  memcpy(c->gq_key, key, sizeof key);
  *q = c->gram_q;
  return PPLS_OK;
}

// G (device, p x p column-major) = the Gram of this rank's n rows: the MFMA kernel into per-item
// partials, then the finish (sum over splits, mirrored).  ms: the MFMA kernel's duration (HIP
// events), if not null.  The partials are allocated here and freed, unless the caller passes them
// (part_in, ppls_gram_part_doubles(g.p, nsplit) doubles; the caller frees them).
int gram_run(ppls_ctx* c, const GramShape& g, int64_t n, int req, double* G, float* ms, double* part_in = nullptr) {
  int rc;
  const int nsplit = gram_nsplit(c, g, n, req);
  double* part = part_in;
  int* q = nullptr;
  if (!part_in && (rc = dalloc(c, &part, (size_t)ppls_gram_part_doubles(g.p, nsplit)))) return rc;
  if ((rc = gram_queue(c, g, n, req, &q))) { if (!part_in) dfree(part); return rc; }
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipError_t e = hipSuccess;
  if (ms) {
    e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipEventRecord(e0, c->stream);
  }
  if (e == hipSuccess)
    e = ppls_launch_gram_joint(g.X, g.ldx, g.xcols, g.xreal, g.Y, g.ldy, g.ycols, g.yreal, c->dtype, n, g.p, nsplit, part,
                               q, c->stream);
  if (e == hipSuccess && ms) e = hipEventRecord(e1, c->stream);
  if (e == hipSuccess) e = ppls_launch_gram_finish(part, nsplit, g.p, g.xreal, g.xcols, g.yreal, G, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess && ms) e = hipEventElapsedTime(ms, e0, e1);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (!part_in) dfree(part);
  if (e != hipSuccess) return fail(c, PPLS_E_HIP, "MFMA Gram: %s", hipGetErrorString(e));
  return PPLS_OK;
}

// The int8-MFMA (Chinese-remainder) form of the same Gram (ppls_ozaki.hip).  Plan from the column
// statistics: e_j with max_k |D_kj| < 2^e_j, c_j = 2^e_j sqrt(n / sum_k D_kj^2) (>= 1; about 8 for
// Gaussian columns), L_j = 53 + ceil(log2 c_j) + 2 bits for column j's integers x' = rint(D 2^s_j),
// s_j = L_j - e_j -- the rounding error of every S_ij is then
// <= 2^-(s_i+1) sum|D_kj| + 2^-(s_j+1) sum|D_ki| <= 2^-55 sqrt(S_ii S_jj), under the fp64 GEMM's own
// bound u sum_k |D_ki D_kj| wherever sum |D_ki D_kj| >= sqrt(S_ii S_jj) / 4 (tests/test_gpu_ozaki.py
// checks both on sampled entries against double-double sums) -- and the fewest moduli with
// prod m_l > 2 max_j sum_k x'_kj^2 (>= |sum_k x'_ki x'_kj| by Cauchy-Schwarz).  Per-column widths keep
// every column's sum_k x'^2 below n 2^112 (one shared L = max_j L_j put up to 2 more bits on columns of
// small c_j).  Returns 1 (not an error) when L = max_j L_j > 62, more than PPLS_OZ_MAXMOD moduli are
// needed or the residue planes do not fit: the caller then runs the fp64 MFMA Gram.
bool oz_held(const ppls_ctx* c) { return c->oz_planes || c->oz_res; }

void oz_free(ppls_ctx* c) {
  dfree(c->oz_planes);
  dfree(c->oz_res);
  c->oz_planes = nullptr;
  c->oz_res = nullptr;
  c->oz_planes_len = c->oz_res_len = 0;
}

int gram_run_oz(ppls_ctx* c, const GramShape& g, int64_t n, double* G, float* ms) {
  const int P = g.p, Pp = (P + 255) / 256 * 256;
  const int64_t nkb = (n + PPLS_OZ_KS - 1) / PPLS_OZ_KS;
  const int dtype = c->dtype;
  struct Bufs {
    double* part = nullptr;
    double* st = nullptr;
    int* shift = nullptr;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    ~Bufs() {
      dfree(part); dfree(st); dfree(shift);
      for (auto e : ev) if (e) (void)hipEventDestroy(e);
    }
  } b;
  int rc;
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(256, n / 2048));
  if ((rc = dalloc(c, &b.part, (size_t)chunks * 2 * Pp)) || (rc = dalloc(c, &b.st, (size_t)2 * Pp)) ||
      (rc = dalloc(c, &b.shift, (size_t)Pp)))
    return rc;
  for (auto& e : b.ev) HIPCHK(c, hipEventCreate(&e));
  HIPCHK(c, hipEventRecord(b.ev[0], c->stream));
  HIPCHK(c, ppls_launch_oz_colstats(g.X, g.ldx, g.xcols, g.xreal, g.Y, g.ldy, g.yreal, dtype, Pp, n, chunks, b.part,
                                    b.st, c->stream));
  std::vector<double> st((size_t)2 * Pp);
  HIPCHK(c, hipMemcpyAsync(st.data(), b.st, sizeof(double) * st.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  auto live = [&](int j) { return j < g.xreal || (j >= g.xcols && j - g.xcols < g.yreal); };
  int L = 55;
  std::vector<int> shift((size_t)Pp, 0);
  double qmax = 0.0;   // max_j sum_k x'_kj^2 <= (2^s_j ||D_j|| + sqrt(n) / 2)^2
  for (int j = 0; j < P; ++j) {
    if (!live(j) || !(st[(size_t)j] > 0.0)) continue;
    int ex = 0;
    (void)std::frexp(st[(size_t)j], &ex);   // max = f 2^ex, f in [0.5, 1): max < 2^ex
    const double cj = std::max(1.0, std::ldexp(1.0, ex) * std::sqrt((double)n / st[(size_t)Pp + j]));
    const int Lj = 53 + (int)std::ceil(std::log2(cj)) + 2;
    L = std::max(L, Lj);
    shift[(size_t)j] = Lj - ex;
    const double q = std::ldexp(std::sqrt(st[(size_t)Pp + j]), Lj - ex) + 0.5 * std::sqrt((double)n);
    qmax = std::max(qmax, q * q);
  }
  c->oz_L = L;
  c->oz_shift.assign(shift.begin(), shift.begin() + P);
  if (L > 62) return 1;
  // M > 2 max |sum| (the CRT's range (-M/2, M/2)); qmax is an upper bound up to the rounding of the
  // device's sum of squares (relative <= n u ~ 1e-10 at 1e6 rows), covered by the 1e-7 bit
  const double need = std::log2(std::max(qmax, 1.0)) + 1.0 + 1e-7;
  double bits = 0.0;
  int nmod = 0;
  while (nmod < PPLS_OZ_MAXMOD && bits < need) bits += std::log2((double)ppls_oz_modulus(nmod++));
  if (bits < need) return 1;
  nmod = std::max(nmod, 12);
  c->oz_nmod = nmod;
  const int T = Pp / 256, ntiles = T * (T + 1) / 2, nsplit = ppls_oz_splits(nkb);
  const int64_t pstride = nkb * Pp * PPLS_OZ_KS;
  const size_t need_planes = (size_t)nmod * pstride, need_res = (size_t)nmod * nsplit * ntiles * 65536;
  if (need_planes > c->oz_planes_len || need_res > c->oz_res_len) {   // (re)allocate the kept buffers
    HIPCHK(c, hipStreamSynchronize(c->stream));
    oz_free(c);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 1;
    const double want = (double)need_planes + (double)need_res;
    if (want > (double)fr - std::max(1073741824.0, 0.05 * (double)fr)) return 1;
    if (dalloc(c, &c->oz_planes, need_planes) || dalloc(c, &c->oz_res, need_res)) {
      c->err.clear();
      oz_free(c);
      return 1;
    }
    c->oz_planes_len = need_planes;
    c->oz_res_len = need_res;
  }
  int8_t* planes = c->oz_planes;
  uint8_t* res = c->oz_res;
  HIPCHK(c, hipMemcpyAsync(b.shift, shift.data(), sizeof(int) * Pp, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, ppls_launch_oz_residues(g.X, g.ldx, g.xcols, g.xreal, g.Y, g.ldy, g.yreal, dtype, Pp, n, nkb, b.shift,
                                    nmod, planes, pstride, c->stream));
  HIPCHK(c, hipEventRecord(b.ev[1], c->stream));
  HIPCHK(c, ppls_launch_oz_syrk(planes, pstride, Pp, nkb, nmod, res, c->stream));
  HIPCHK(c, hipEventRecord(b.ev[2], c->stream));
  HIPCHK(c, ppls_launch_oz_finish(res, nmod, nsplit, Pp, g.xcols, g.xreal, g.yreal, P, b.shift, G, c->stream));
  HIPCHK(c, hipEventRecord(b.ev[3], c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  float t01 = 0.f, t12 = 0.f, t23 = 0.f, t03 = 0.f;
  HIPCHK(c, hipEventElapsedTime(&t01, b.ev[0], b.ev[1]));
  HIPCHK(c, hipEventElapsedTime(&t12, b.ev[1], b.ev[2]));
  HIPCHK(c, hipEventElapsedTime(&t23, b.ev[2], b.ev[3]));
  HIPCHK(c, hipEventElapsedTime(&t03, b.ev[0], b.ev[3]));
  c->oz_ms[0] = t01;
  c->oz_ms[1] = t12;
  c->oz_ms[2] = t23;
  c->oz_ms[3] = t03;
  if (ms) *ms = t03;
  return PPLS_OK;
}

// The Gram of the joint columns for S: the int8 form when option gram_int8 asks for it and the data
// allow it, else (or on its fallback) the fp64 MFMA Gram; c->oz_used records which ran.
int gram_run_s(ppls_ctx* c, const GramShape& g, int64_t n, double* G, float* ms, double* part) {
  c->oz_used = 0;
  if (c->gram_int8) {
    const int rc = gram_run_oz(c, g, n, G, ms);
    if (rc == PPLS_OK) {
      c->oz_used = 1;
      return PPLS_OK;
    }
    if (rc < 0) return rc;
  }
  return gram_run(c, g, n, 0, G, ms, part);
}

int xprod_setup(ppls_ctx* c);
bool xprod_choose(ppls_ctx* c, int max_steps, int r);

// Rows per rank the cross-product setup is sized for: the same on every rank (ceil(n_total / nranks)).
int64_t xprod_rows(const ppls_ctx* c) { return (c->n_total + c->nranks - 1) / c->nranks; }

// HBM the cross-product form allocates: S (8 P^2 B), the Gram partials while S is formed (32 KB
// per quadrant item and split; a rank with fewer rows plans no more splits) and M (P x 2 RMAX doubles).
double xprod_bytes(ppls_ctx* c) {
  const GramShape g = gram_shape(c, true, 0);
  const double PP = (double)g.p * g.p;
  return 8.0 * PP + 8.0 * (double)ppls_gram_part_doubles(g.p, gram_nsplit(c, g, xprod_rows(c), 0)) +
         16.0 * g.p * PPLS_RMAX;
}

// Start a run (or session) on the cross-products when the policy picks them.  In auto mode (-1) a
// failed allocation of S -- which xprod_setup reports on every rank alike -- falls back to streaming.
int xprod_begin(ppls_ctx* c, int steps, int r) {
  c->xp_active = c->seg_rows < 0 && xprod_choose(c, steps, r);
  if (!c->xp_active) return PPLS_OK;
  const int rc = xprod_setup(c);
  if (rc == PPLS_OK) return PPLS_OK;
  c->xp_active = false;
  if (rc == PPLS_E_NOMEM && c->xprod < 0) {
    c->err.clear();
    return PPLS_OK;
  }
  return rc;
}

// Cross-product form (ppls_xprod.hip): S = [X Y]'[X Y] over the local rows on MFMA (fp64 products
// of the stored values, exact for fp32 storage), summed over ranks by ONE all-reduce of P^2 doubles;
// afterwards an iteration needs no collective at all (every rank holds the same S and theta).
int xprod_setup(ppls_ctx* c) {
  if (c->xp_ready) return PPLS_OK;
  const int P = c->ldx + c->ldy;
  const size_t PP = (size_t)P * P;
  int rc;
  const auto t0 = std::chrono::steady_clock::now();
  // S, the Gram partials and the Gram's work queue; with collectives every rank must know that all
  // ranks allocated them before anyone enters the all-reduce of S (a rank that returned here alone
  // would leave the others waiting in it), so the allocation outcome is all-reduced first, and the
  // partials and queue allocated here are the ones gram_run uses (no allocation after the agreement)
  const GramShape g = gram_shape(c, true, 0);
  double* part = nullptr;
  int rc_alloc = dalloc(c, &c->xp_S, PP);
  if (!rc_alloc && c->n_local > 0) {
    int* q = nullptr;
    rc_alloc = dalloc(c, &part, (size_t)ppls_gram_part_doubles(P, gram_nsplit(c, g, c->n_local, 0)));
    if (!rc_alloc) rc_alloc = gram_queue(c, g, c->n_local, 0, &q);
  }
  if (c->nranks > 1 || c->reducer) {
    const double f = rc_alloc ? 1.0 : 0.0;
    double tot = 0.0;
    HIPCHK(c, hipMemcpyAsync(c->flag, &f, sizeof f, hipMemcpyHostToDevice, c->stream));
    if ((rc = allreduce(c, c->flag, 1))) { dfree(c->xp_S); dfree(part); return rc; }
    HIPCHK(c, hipMemcpyAsync(&tot, c->flag, sizeof tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (tot > 0.0) {
      dfree(c->xp_S);
      dfree(part);
      return fail(c, PPLS_E_NOMEM, "cross-products S: %d rank(s) could not allocate %.3g GB of S and Gram partials",
                  (int)tot, xprod_bytes(c) / 1e9);
    }
  } else if (rc_alloc) {
    dfree(c->xp_S);
    dfree(part);
    return rc_alloc;
  }
  c->xp_setup_ms = 0.0;
  if (c->n_local > 0) {
    c->xp_nsplit = gram_nsplit(c, g, c->n_local, 0);
    float ms = 0.f;
    rc = gram_run_s(c, g, c->n_local, c->xp_S, &ms, part);
    dfree(part);
    if (rc) { dfree(c->xp_S); return rc; }
    c->xp_setup_ms = ms;
  } else {
    HIPCHK(c, hipMemsetAsync(c->xp_S, 0, sizeof(double) * PP, c->stream));
  }
  const auto ta = std::chrono::steady_clock::now();
  if ((rc = allreduce(c, c->xp_S, PP))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->xp_setup_ar_ms = c->nranks > 1 || c->reducer ? std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count() : 0.0;
  c->xp_setup_total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->xp_ready = true;
  return PPLS_OK;
}

// Whether a run of max_steps iterations reads S: option xprod = 1 always, 0 never, -1 when the
// modelled cost of forming S plus max_steps + 1 passes over it undercuts max_steps + 1 streaming
// sweeps and S fits.  The model and the memory gate use only values every rank shares (n_total /
// nranks, P, and the smallest free HBM over all ranks, all-reduced when the data were loaded), so
// every rank of a sharded run takes the same path and issues the same collectives.  Memory gate:
// S, its Gram partials and M (xprod_bytes) within the smallest free HBM less max(1 GiB, 5 %).
bool xprod_choose(ppls_ctx* c, int max_steps, int r) {
  if (c->xprod == 0) return false;
  if (c->xprod == 1) return true;   // forced: xprod_setup reports a failed allocation (all ranks alike)
  if (!c->xp_ready && xprod_bytes(c) > c->mem_free_min - std::max(1073741824.0, 0.05 * c->mem_free_min))
    return false;
  const double P = (double)(c->ldx + c->ldy);
  const double n = (double)((c->n_total + c->nranks - 1) / c->nranks);
  const double esz = c->dtype ? 4.0 : 8.0;
  // the split sweep reads X, Y once; the panel sweep (wide p, r > 8, fp32 storage) twice -- also
  // at r = 1 (C5's initialiser steps: 7.3 ms each, like its r = 10 iterations)
  const bool split = c->sweep_mode != 3 && !c->dtype && ppls_split_supported(r, c->ldx, c->ldy) > 0;
  const double t_sweep = (split ? 1.0 : 2.0) * esz * n * P / 6.5e12 + 5e-6;
  const double t_pass = 8.0 * P * P / 6.5e12 + 5e-6;
  // the Gram's rate in n P^2 per second: fp64 MFMA ~55e12 (C3 226 ms); the int8 CRT form ~1e14
  const double gram_rate = c->gram_int8 ? 1.0e14 : 55e12;
  const double t_setup = c->xp_ready ? 0.0 : n * P * P / gram_rate + (c->nranks > 1 ? 16.0 * P * P / 100e9 : 0.0);
  return ((double)max_steps + 1.0) * (t_sweep - t_pass) > t_setup;
}

// One statistics step from S: c->stats for theta[slot] (no collective: S is global).  fuse: a
// finalize follows, which may form the Gram itself (its scalar block runs in the polar blocks'
// slack: C3 ~2 us of it against the Gram kernel's 4 us + a launch boundary).
int xprod_stats(ppls_ctx* c, int r, int slot, bool fuse = false) {
  int rc;
  const int P = c->ldx + c->ldy;
  if (!c->xp_ready && (rc = xprod_setup(c))) return rc;
  if (!c->xp_M) {
    if ((rc = dalloc(c, &c->xp_M, (size_t)P * 2 * PPLS_RMAX))) return rc;
  }
  hipEvent_t e0, e1;
  if ((rc = timing_pair(c, &e0, &e1))) return rc;
  if (e0) HIPCHK(c, hipEventRecord(e0, c->stream));
  const int rw = ppls_xprod_tile_rows(P, r, c->xprod_rw, c->num_cus);
  const bool defer = fuse && c->xprod_fuse && r <= 8 && P <= 6144;
  HIPCHK(c, ppls_launch_xprod_tile(c->xp_S, c->ldx, c->ldy, r, rw, c->W[slot], c->C[slot], c->sc[slot], c->stats,
                                   c->xp_M, c->sweep_stop, defer ? 0 : 1, c->stream));
  c->xp_pending_gram = defer;
  if (e1) HIPCHK(c, hipEventRecord(e1, c->stream));
  return PPLS_OK;
}

// The statistics of theta[slot] for an EM iteration: from S when the run reads the cross-products
// (not for the mu write-out, which needs the rows), else one streaming sweep.
int stats_step(ppls_ctx* c, int r, int slot, bool write_mu, bool finalize_next = false) {
  c->xp_pending_gram = false;
  if (c->xp_active && !write_mu && c->seg_rows < 0) return xprod_stats(c, r, slot, finalize_next);
  return sweep(c, r, slot, write_mu);
}

// The device stop flag (2 ints) and its host-mapped mirror, allocated on first use.
int ensure_stop(ppls_ctx* c) {
  if (c->stop_d) return PPLS_OK;
  int rc;
  if ((rc = dalloc(c, &c->stop_d, 2))) return rc;
  HIPCHK(c, hipHostMalloc((void**)&c->stop_mirror, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
  HIPCHK(c, hipHostGetDevicePointer((void**)&c->stop_mirror_dev, c->stop_mirror, 0));
  return PPLS_OK;
}

int reset_stop(ppls_ctx* c) {
  HIPCHK(c, hipMemsetAsync(c->stop_d, 0, 2 * sizeof(int), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  __atomic_store_n(c->stop_mirror, 0, __ATOMIC_SEQ_CST);
  return PPLS_OK;
}

int check_status(ppls_ctx* c) {
  int st = 0;
  HIPCHK(c, hipMemcpy(&st, c->status, sizeof st, hipMemcpyDeviceToHost));
  if (st == -7) {   // a polar team member waited too long: clear the team counters, report
    if (c->team_bar) HIPCHK(c, hipMemset(c->team_bar, 0, 8 * sizeof(unsigned)));
    return fail(c, PPLS_E_HIP, "finalize polar team barrier timed out (status -7)");
  }
  if (st != 0) return fail(c, PPLS_E_NUMERIC, "rank-deficient X'mu_T or Y'mu_U in the M-step (status %d)", st);
  return PPLS_OK;
}

void xprod_free(ppls_ctx* c) {
  c->xp_ready = false;
  c->xp_explicit = false;
  c->xp_active = false;
  dfree(c->xp_S);
  dfree(c->xp_M);
  // (the int8 Gram's residue planes are a workspace, not S: kept until gram_int8 = 0, the context's
  // end or an allocation that needs the room -- freeing and re-allocating tens of GB per formation
  // cost 1-5 s per call on some boxes, profiles/r6_gram_int8_percol_c3.jsonl)
}

int compute_ssq(ppls_ctx* c) {
  int rc;
  xprod_free(c);   // data or communicator changed: the cross-products are stale

  const int nb = 1024;
  const int nred = 2 + c->nranks;   // {||X||^2, ||Y||^2, free HBM of rank 0, 1, ...}
  if ((rc = dalloc(c, &c->scratch, (size_t)nb + nred))) return rc;
  HIPCHK(c, hipMemsetAsync(c->ssq, 0, 2 * sizeof(double), c->stream));
  if (c->n_local > 0 && c->dtype) {
    HIPCHK(c, ppls_launch_sumsq_f32((const float*)c->X, c->n_local * c->ldx, c->scratch, nb, c->ssq, c->stream));
    HIPCHK(c, ppls_launch_sumsq_f32((const float*)c->Y, c->n_local * c->ldy, c->scratch, nb, c->ssq + 1, c->stream));
  } else if (c->n_local > 0) {
    HIPCHK(c, ppls_launch_sumsq(c->X, c->n_local * c->ldx, c->scratch, nb, c->ssq, 0, c->stream));
    HIPCHK(c, ppls_launch_sumsq(c->Y, c->n_local * c->ldy, c->scratch, nb, c->ssq + 1, 0, c->stream));
  }
  // one all-reduce carries the sums of squares and every rank's free HBM (in its own slot), so the
  // cross-product form's memory gate (xprod_choose) is the same on every rank
  size_t mfree = 0, mtot = 0;
  HIPCHK(c, hipMemGetInfo(&mfree, &mtot));
  std::vector<double> slots((size_t)c->nranks, 0.0);
  slots[(size_t)c->rank] = (double)mfree;
  double* red = c->scratch + nb;
  HIPCHK(c, hipMemcpyAsync(red, c->ssq, 2 * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(red + 2, slots.data(), sizeof(double) * slots.size(), hipMemcpyHostToDevice, c->stream));
  if ((rc = allreduce(c, red, (size_t)nred))) return rc;
  HIPCHK(c, hipMemcpyAsync(c->ssq, red, 2 * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
  std::vector<double> h((size_t)nred);
  HIPCHK(c, hipMemcpyAsync(h.data(), red, sizeof(double) * nred, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->ssq_host[0] = h[0];
  c->ssq_host[1] = h[1];
  c->mem_free_min = h[2];
  for (int k = 1; k < c->nranks; ++k) c->mem_free_min = std::min(c->mem_free_min, h[(size_t)2 + k]);
  dfree(c->scratch);
  return PPLS_OK;
}

// Non-finite data: R's svd() in orth() refuses X'mu_T with NaN/Inf entries (EM_W_multi.R:732-733),
// so the reference stops on such data.  Detected from the all-reduced sums of squares (a NaN or Inf
// element -- or values past ~1.3e154, whose squares overflow -- makes the global sum non-finite), so
// every rank of a sharded run reaches the same verdict and none is left waiting in a collective.
int check_finite_data(ppls_ctx* c) {
  for (int m = 0; m < 2; ++m)
    if (!std::isfinite(c->ssq_host[m])) {
      c->have_data = false;
      xprod_free(c);
      return fail(c, PPLS_E_ARG,
                  "%c contains NaN or Inf (its sum of squares over all ranks is %g; values beyond 1.3e154 "
                  "also overflow it): the reference's svd() in orth() stops on non-finite data "
                  "(EM_W_multi.R:732-733)",
                  m ? 'Y' : 'X', c->ssq_host[m]);
    }
  return PPLS_OK;
}

// A fit needs ssq(X) > 0 and ssq(Y) > 0: on an all-zero block the reference's first EM step
// divides 0 by 0 (EMstepC_fast's loading normalisation, loglC.cpp:357,385), its log-likelihood
// increment is NA and `if (NA < atol)` stops the fit (EM_W_multi.R:173, :792).
int check_fit_data(ppls_ctx* c) {
  for (int m = 0; m < 2; ++m)
    if (!(c->ssq_host[m] > 0.0))
      return fail(c, PPLS_E_ARG,
                  "%c is all zero (sum of squares over all ranks = 0): the PPLS model is degenerate and the "
                  "reference's fit stops on the NA log-likelihood increment it produces (EM_W_multi.R:173,792)",
                  m ? 'Y' : 'X');
  return PPLS_OK;
}

int alloc_data(ppls_ctx* c, int64_t n_local, int p, int q, int64_t n_total) {
  int rc;
  c->em_active = false;
  if (n_local < 0 || p < 1 || q < 1) return fail(c, PPLS_E_ARG, "bad shape n=%lld p=%d q=%d", (long long)n_local, p, q);
  c->n_local = n_local;
  c->n_total = n_total > 0 ? n_total : n_local;
  c->p = p;
  c->q = q;
  c->ldx = ld_of(p, c->dtype, c->ldpad);
  c->ldy = ld_of(q, c->dtype, c->ldpad);
  // X, Y storage (fp64, or fp32 packed into the double allocation)
  const size_t es = c->dtype ? 4 : 8;
  // + 64 doubles of slack: the panel dots kernel reads whole 128-B column tiles, so the last row's
  // partial tile may run past the end (those values meet zero rows of the transposed W, so the
  // slack must hold finite values: it is zeroed here -- reused device memory can hold NaN patterns)
  const size_t xb = (size_t)std::max<int64_t>(n_local, 1) * c->ldx * es, yb = (size_t)std::max<int64_t>(n_local, 1) * c->ldy * es;
  if ((rc = dalloc(c, &c->X, (xb + 7) / 8 + 64))) return rc;
  if ((rc = dalloc(c, &c->Y, (yb + 7) / 8 + 64))) return rc;
  HIPCHK(c, hipMemsetAsync((char*)c->X + xb, 0, ((xb + 7) / 8 + 64) * 8 - xb, c->stream));
  HIPCHK(c, hipMemsetAsync((char*)c->Y + yb, 0, ((yb + 7) / 8 + 64) * 8 - yb, c->stream));
  if (!c->ssq && (rc = dalloc(c, &c->ssq, 2))) return rc;
  if (!c->flag && (rc = dalloc(c, &c->flag, 8))) return rc;
  c->r_alloc = 0;   // force per-r buffers to be re-sized for the new shape
  dfree(c->part);
  dfree(c->Z);
  c->z_cols = 0;
  dfree(c->mu);
  c->part_groups = 0;
  c->have_data = false;
  return PPLS_OK;
}

// Canonicalisation of EM_W_multi.R:773-778 / :794-799 applied to a host theta.
void canonicalize(ppls_theta* th, int p, int q, int r) {
  int rot[PPLS_RMAX];
  double sgn[PPLS_RMAX];
  ppls_canonical_order(th->sigT, th->B, r, rot, sgn);
  std::vector<double> W((size_t)p * r), C((size_t)q * r);
  double B[PPLS_RMAX], T[PPLS_RMAX];
  for (int j = 0; j < r; ++j) {
    // W.[,rotLoad] %*% diag(signLoad): column j <- old column rot[j] scaled by signLoad[j]
    for (int i = 0; i < p; ++i) W[(size_t)j * p + i] = th->W[(size_t)rot[j] * p + i] * sgn[j];
    for (int i = 0; i < q; ++i) C[(size_t)j * q + i] = th->C[(size_t)rot[j] * q + i] * sgn[j];
    B[j] = th->B[rot[j]] * sgn[rot[j]];   // diag(B %*% diag(signLoad))[rotLoad]
    T[j] = th->sigT[rot[j]];
  }
  memcpy(th->W, W.data(), sizeof(double) * W.size());
  memcpy(th->C, C.data(), sizeof(double) * C.size());
  for (int j = 0; j < r; ++j) {
    th->B[j] = B[j];
    th->sigT[j] = T[j];
  }
}

bool theta_finite(const ppls_theta* th, int p, int q, int r) {
  bool ok = std::isfinite(th->sigE) && std::isfinite(th->sigF) && std::isfinite(th->sigH);
  for (int k = 0; k < r && ok; ++k) ok = std::isfinite(th->B[k]) && std::isfinite(th->sigT[k]);
  for (size_t e = 0; e < (size_t)p * r && ok; ++e) ok = std::isfinite(th->W[e]);
  for (size_t e = 0; e < (size_t)q * r && ok; ++e) ok = std::isfinite(th->C[e]);
  return ok;
}

// Host polar factor / QR factor of the p x r matrix S (ld p): sequential Householder QR, then the
// same small Jacobi polar as the device.  out: p x r.
int host_orth(const double* S, int p, int r, int type, double* out) {
  std::vector<double> A(S, S + (size_t)p * r), E((size_t)p * r, 0.0), vtv(r);
  double R[PPLS_RMAX * PPLS_RMAX] = {0}, P[PPLS_RMAX * PPLS_RMAX];
  for (int k = 0; k < r; ++k) {
    double s2 = 0.0;
    for (int i = k; i < p; ++i) s2 += A[(size_t)k * p + i] * A[(size_t)k * p + i];
    const double sig = std::sqrt(s2), akk = A[(size_t)k * p + k];
    if (!(sig > 0.0)) return PPLS_E_NUMERIC;
    const double alpha = akk >= 0.0 ? -sig : sig;
    vtv[k] = 2.0 * sig * (sig + std::fabs(akk));
    A[(size_t)k * p + k] = akk - alpha;
    R[k * r + k] = alpha;
    for (int j = k + 1; j < r; ++j) {
      double d = 0.0;
      for (int i = k; i < p; ++i) d += A[(size_t)k * p + i] * A[(size_t)j * p + i];
      const double f = 2.0 * d / vtv[k];
      for (int i = k; i < p; ++i) A[(size_t)j * p + i] -= f * A[(size_t)k * p + i];
      R[j * r + k] = A[(size_t)j * p + k];
    }
  }
  for (int j = 0; j < r; ++j) E[(size_t)j * p + j] = 1.0;
  for (int k = r - 1; k >= 0; --k)
    for (int j = 0; j < r; ++j) {
      double d = 0.0;
      for (int i = k; i < p; ++i) d += A[(size_t)k * p + i] * E[(size_t)j * p + i];
      const double f = 2.0 * d / vtv[k];
      for (int i = k; i < p; ++i) E[(size_t)j * p + i] -= f * A[(size_t)k * p + i];
    }
  if (type == PPLS_ORTH_QR) {   // sign_e * qr.Q(qr(S)), sign_e = sign(<e_1, S_1>) = sign(R_11) (functions.R:257-259)
    const double sg = R[0] < 0.0 ? -1.0 : 1.0;
    for (size_t e = 0; e < E.size(); ++e) out[e] = sg * E[e];
    return PPLS_OK;
  }
  if (ppls_small_polar(R, r, P) != 0) return PPLS_E_NUMERIC;
  for (int j = 0; j < r; ++j)
    for (int i = 0; i < p; ++i) {
      double s = 0.0;
      for (int k = 0; k < r; ++k) s += E[(size_t)k * p + i] * P[j * r + k];
      out[(size_t)j * p + i] = s;
    }
  return PPLS_OK;
}

}  // namespace

extern "C" {

int ppls_version(void) { return 100; }

const char* ppls_strerror(int code) {
  switch (code) {
    case PPLS_OK: return "ok";
    case PPLS_E_ARG: return "invalid argument";
    case PPLS_E_HIP: return "HIP runtime error";
    case PPLS_E_NUMERIC: return "numerical failure";
    case PPLS_E_STATE: return "invalid state";
    case PPLS_E_COMM: return "RCCL error";
    case PPLS_E_NOMEM: return "out of device memory";
    default: return "unknown error";
  }
}

int ppls_ctx_create(int device, ppls_ctx** out) {
  if (!out) return PPLS_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PPLS_E_HIP;
  if (device < 0 || device >= ndev) return PPLS_E_ARG;
  ppls_ctx* c = new ppls_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return PPLS_E_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->num_cus = prop.multiProcessorCount;
  *out = c;
  return PPLS_OK;
}

void ppls_ctx_destroy(ppls_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  dfree(c->X); dfree(c->Y); dfree(c->ssq); dfree(c->flag);
  for (int i = 0; i < 2; ++i) { dfree(c->W[i]); dfree(c->C[i]); dfree(c->sc[i]); dfree(c->gram[i]); }
  dfree(c->vstate);
  dfree(c->mom); dfree(c->stats); dfree(c->part); dfree(c->Z); dfree(c->mu); dfree(c->loglik);
  c->z_cols = 0;
  dfree(c->work); dfree(c->status); dfree(c->coefs); dfree(c->scratch);
  if (c->ftrace) (void)hipFree(c->ftrace);
  if (c->strace) (void)hipFree(c->strace);
  dfree(c->stop_d);
  dfree(c->xp_S);
  dfree(c->xp_M);
  oz_free(c);
  dfree(c->bal_bounds);
  dfree(c->team_bar);
  dfree(c->team_part);
  dfree(c->gram_q);
  if (c->stop_mirror) (void)hipHostFree(c->stop_mirror);
  for (auto& e : c->ev) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  for (auto& e : c->ev_ar) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  if (c->blas) (void)rocblas_destroy_handle(c->blas);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* ppls_last_error(const ppls_ctx* c) { return c ? c->err.c_str() : "null context"; }

int ppls_set_option(ppls_ctx* c, const char* key, int64_t value) {
  if (!c || !key) return PPLS_E_ARG;
  if (!strcmp(key, "sweep")) {
    if (value != 0 && value != 3) return fail(c, PPLS_E_ARG, "sweep must be 0 (auto) or 3 (panel)");
    c->sweep_mode = (int)value;
  } else if (!strcmp(key, "grid")) {
    if (value < 0 || value > 65535) return fail(c, PPLS_E_ARG, "grid out of range");
    c->grid_opt = (int)value;
    c->part_groups = 0;
    dfree(c->part);
  } else if (!strcmp(key, "rows_per_step")) {
    if (value < 0 || value > 2) return fail(c, PPLS_E_ARG, "rows_per_step must be 0 (auto), 1 or 2");
    c->rp_opt = (int)value;
  } else if (!strcmp(key, "team_rows")) {
    if (value < 0 || value > (1 << 30)) return fail(c, PPLS_E_ARG, "team_rows must be >= 0");
    c->team_rows = (int)value;
  } else if (!strcmp(key, "polar1")) {
    c->polar1 = value ? 1 : 0;
  } else if (!strcmp(key, "exact_gram")) {
    c->exact_gram = value ? 1 : 0;
  } else if (!strcmp(key, "balance")) {
    c->balance = value ? 1 : 0;
  } else if (!strcmp(key, "polar1_kappa")) {
    if (value < 0 || value > 255) return fail(c, PPLS_E_ARG, "polar1_kappa must be in [0, 255]");
    c->polar1_kappa = (int)value;
  } else if (!strcmp(key, "pipe")) {
    c->pipe_opt = value ? 1 : 0;
  } else if (!strcmp(key, "ldpad")) {   // applies to data set or generated afterwards
    c->ldpad = value ? 1 : 0;
  } else if (!strcmp(key, "dots_rows")) {
    if (value != 0 && value != 32 && value != 64) return fail(c, PPLS_E_ARG, "dots_rows must be 0 (auto), 32 or 64");
    c->dots_rows = (int)value;
  } else if (!strcmp(key, "dots_pair")) {
    if (value < -1 || value > 1) return fail(c, PPLS_E_ARG, "dots_pair must be -1 (auto), 0 or 1");
    c->dots_pair = (int)value;
  } else if (!strcmp(key, "acc_chunks")) {
    if (value < 0 || value > 65535) return fail(c, PPLS_E_ARG, "acc_chunks must be in [0, 65535]");
    c->acc_chunks = (int)value;
  } else if (!strcmp(key, "strace")) {
    if (value && !c->strace) {
      HIPCHK(c, hipMalloc(&c->strace, (size_t)PPLS_STRACE_MAX_WG * 4 * sizeof(long long)));
      HIPCHK(c, hipMemset(c->strace, 0, (size_t)PPLS_STRACE_MAX_WG * 4 * sizeof(long long)));
    } else if (!value && c->strace) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      (void)hipFree(c->strace);
      c->strace = nullptr;
    }
  } else if (!strcmp(key, "ftrace")) {
    if (value && !c->ftrace) {
      HIPCHK(c, hipMalloc(&c->ftrace, PPLS_FTRACE_LEN * sizeof(long long)));
      HIPCHK(c, hipMemset(c->ftrace, 0, PPLS_FTRACE_LEN * sizeof(long long)));
    } else if (!value && c->ftrace) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      (void)hipFree(c->ftrace);
      c->ftrace = nullptr;
    }
  } else if (!strcmp(key, "dtype")) {
    if (value != 0 && value != 1) return fail(c, PPLS_E_ARG, "dtype must be 0 (fp64) or 1 (fp32 storage)");
    if (c->dtype != (int)value) {
      c->dtype = (int)value;
      c->have_data = false;   // the data must be (re)loaded in the new storage type
    }
  } else if (!strcmp(key, "nt")) {
    if (value < -1 || value > 1) return fail(c, PPLS_E_ARG, "nt must be -1 (auto), 0 or 1");
    c->nt_loads = (int)value;
  } else if (!strcmp(key, "xprod")) {
    if (value < -1 || value > 1) return fail(c, PPLS_E_ARG, "xprod must be -1 (auto), 0 (stream X, Y) or 1 (cross-products)");
    // the path of an ppls_em_begin session is fixed at em_begin: a session on S does not switch to
    // streaming under it -- xprod = 0 ends it (ppls_em_iterate then asks for ppls_em_begin)
    if (value == 0 && c->em_active && c->xp_active) {
      c->em_active = false;
      c->xp_active = false;
    }
    const int was = c->xprod;
    c->xprod = (int)value;
    // streaming from now on: S's 8 (p+q)^2 bytes go back -- unless S came from ppls_xprod_prepare
    // (kept for variances() and later runs until ppls_xprod_release)
    if (value == 0 && was != 0 && !c->xp_explicit) {
      HIPCHK(c, hipStreamSynchronize(c->stream));
      xprod_free(c);
    }
  } else if (!strcmp(key, "meta_device")) {
    c->meta_device = value ? 1 : 0;
  } else if (!strcmp(key, "vorth")) {
    if (value < 1 || value > 255) return fail(c, PPLS_E_ARG, "vorth must be in [1, 255]");
    c->vorth = (int)value;
  } else if (!strcmp(key, "xprod_fuse")) {
    c->xprod_fuse = value ? 1 : 0;
  } else if (!strcmp(key, "var_chol")) {
    if (value < 0 || value > 2) return fail(c, PPLS_E_ARG, "var_chol must be 0 (LU), 1 (Cholesky) or 2 (rocSOLVER Cholesky)");
    c->var_chol = (int)value;
  } else if (!strcmp(key, "gram_int8")) {
    if (value < 0 || value > 1) return fail(c, PPLS_E_ARG, "gram_int8 must be 0 (fp64 MFMA Gram) or 1 (int8 CRT form)");
    if ((int)value != c->gram_int8) {
      c->gram_int8 = (int)value;
      if (c->xp_ready && !c->xp_explicit) {   // a different Gram: S is formed again when next needed
        dfree(c->xp_S);
        c->xp_ready = false;
      }
      if (!c->gram_int8) {
        HIPCHK(c, hipStreamSynchronize(c->stream));
        oz_free(c);
      }
    }
  } else if (!strcmp(key, "xprod_rw")) {
    if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
      return fail(c, PPLS_E_ARG, "xprod_rw must be 0, 1, 2, 4 or 8");
    c->xprod_rw = (int)value;
  } else if (!strcmp(key, "timing")) {
    if (value < 0) return fail(c, PPLS_E_ARG, "timing must be >= 0");
    c->timing = (int)value;
    c->sweep_count = 0;
  } else {
    return fail(c, PPLS_E_ARG, "unknown option '%s'", key);
  }
  return PPLS_OK;
}

void ppls_shard_range(int64_t n_total, int nranks, int rank, int64_t* row0, int64_t* n_local) {
  if (nranks < 1) nranks = 1;
  const int64_t b = n_total * rank / nranks, e = n_total * (rank + 1) / nranks;
  if (row0) *row0 = b;
  if (n_local) *n_local = e - b;
}

int ppls_comm_unique_id(char id[128]) {
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return PPLS_E_COMM;
  static_assert(sizeof(u.internal) == 128, "unexpected ncclUniqueId size");
  memcpy(id, u.internal, 128);
  return PPLS_OK;
}

int ppls_comm_init(ppls_ctx* c, int nranks, int rank, const char id[128]) {
  if (!c || nranks < 1 || rank < 0 || rank >= nranks) return PPLS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
  if (nranks > 1 && !id) return fail(c, PPLS_E_ARG, "nranks=%d needs the root's unique id", nranks);
  c->nranks = nranks;
  c->rank = rank;
  if (id) {
    ncclUniqueId u;
    memcpy(u.internal, id, 128);
    RCCLCHK(c, ncclCommInitRank(&c->comm, nranks, u, rank));
  }
  if (c->have_data) return compute_ssq(c);
  return PPLS_OK;
}

int ppls_set_reducer(ppls_ctx* c, ppls_reduce_fn fn, void* user) {
  if (!c) return PPLS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  c->reducer = fn;
  c->reducer_user = user;
  if (c->have_data) return compute_ssq(c);   // ||X||^2, ||Y||^2 summed by the new reduction
  return PPLS_OK;
}

int ppls_set_data(ppls_ctx* c, const double* X, const double* Y, int64_t n_local, int p, int q,
                  int layout, int64_t n_total) {
  if (!c || (n_local > 0 && (!X || !Y))) return c ? fail(c, PPLS_E_ARG, "NULL data") : PPLS_E_ARG;
  if (layout != PPLS_LAYOUT_COLMAJOR && layout != PPLS_LAYOUT_ROWMAJOR)
    return fail(c, PPLS_E_ARG, "layout must be 0 (column-major) or 1 (row-major)");
  HIPCHK(c, hipSetDevice(c->device));
  int rc = alloc_data(c, n_local, p, q, n_total);
  if (rc) return rc;
  if (n_local > 0 && c->dtype) {   // fp32 storage: build fp64 row-major chunks, then convert
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n_local, (int64_t)(256 << 20) / (8LL * (c->ldx + p))));
    double *tmp = nullptr, *tcm = nullptr;
    const int wmax = std::max(c->ldx, c->ldy), cmax = std::max(p, q);
    if ((rc = dalloc(c, &tmp, (size_t)chunk * wmax))) return rc;
    if ((rc = dalloc(c, &tcm, (size_t)chunk * cmax))) { dfree(tmp); return rc; }
    for (int m = 0; m < 2 && !rc; ++m) {
      const double* src = m == 0 ? X : Y;
      const int cols = m == 0 ? p : q, ld = m == 0 ? c->ldx : c->ldy;
      float* dst = (float*)(m == 0 ? c->X : c->Y);
      for (int64_t r0 = 0; r0 < n_local && !rc; r0 += chunk) {
        const int64_t nc = std::min(chunk, n_local - r0);
        hipError_t e;
        if (layout == PPLS_LAYOUT_ROWMAJOR) {
          e = hipMemset2DAsync(tmp, sizeof(double) * ld, 0, sizeof(double) * ld, nc, c->stream);
          if (e == hipSuccess)
            e = hipMemcpy2DAsync(tmp, sizeof(double) * ld, src + r0 * cols, sizeof(double) * cols,
                                 sizeof(double) * cols, nc, hipMemcpyHostToDevice, c->stream);
        } else {   // column-major n_local x cols: rows [r0, r0 + nc) of every column
          e = hipMemcpy2DAsync(tcm, sizeof(double) * nc, src + r0, sizeof(double) * n_local, sizeof(double) * nc,
                               cols, hipMemcpyHostToDevice, c->stream);
          if (e == hipSuccess) e = ppls_launch_to_rowmajor(tcm, nc, cols, ld, tmp, c->stream);
        }
        if (e == hipSuccess) e = ppls_launch_convert(tmp, 0, dst + r0 * ld, 1, nc * ld, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = fail(c, PPLS_E_HIP, "fp32 upload: %s", hipGetErrorString(e));
      }
    }
    dfree(tmp);
    dfree(tcm);
    if (rc) return rc;
  } else if (n_local > 0) {
    for (int m = 0; m < 2; ++m) {
      const double* src = m == 0 ? X : Y;
      const int cols = m == 0 ? p : q, ld = m == 0 ? c->ldx : c->ldy;
      double* dst = m == 0 ? c->X : c->Y;
      if (layout == PPLS_LAYOUT_ROWMAJOR) {
        HIPCHK(c, hipMemset2DAsync(dst, sizeof(double) * ld, 0, sizeof(double) * ld, n_local, c->stream));
        HIPCHK(c, hipMemcpy2DAsync(dst, sizeof(double) * ld, src, sizeof(double) * cols, sizeof(double) * cols,
                                   n_local, hipMemcpyHostToDevice, c->stream));
      } else {
        double* tmp = nullptr;
        if ((rc = dalloc(c, &tmp, (size_t)n_local * cols))) return rc;
        HIPCHK(c, hipMemcpyAsync(tmp, src, sizeof(double) * n_local * cols, hipMemcpyHostToDevice, c->stream));
        HIPCHK(c, ppls_launch_to_rowmajor(tmp, n_local, cols, ld, dst, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        dfree(tmp);
      }
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_data = true;
  if ((rc = compute_ssq(c))) return rc;
  return check_finite_data(c);
}

int ppls_generate_synthetic(ppls_ctx* c, int64_t n_total, int64_t row0, int64_t n_local, int p, int q,
                            int r, const ppls_theta* truth, uint64_t seed) {
  if (!c) return PPLS_E_ARG;
  int rc;
  if ((rc = check_theta(c, truth, r))) return rc;
  if (row0 < 0 || n_local < 0 || row0 + n_local > n_total) return fail(c, PPLS_E_ARG, "bad row range");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = alloc_data(c, n_local, p, q, n_total))) return rc;
  double *Wt = nullptr, *Ct = nullptr, *TU = nullptr;
  if ((rc = dalloc(c, &Wt, (size_t)p * r))) return rc;
  if ((rc = dalloc(c, &Ct, (size_t)q * r))) { dfree(Wt); return rc; }
  if ((rc = dalloc(c, &TU, (size_t)std::max<int64_t>(n_local, 1) * 2 * r))) { dfree(Wt); dfree(Ct); return rc; }
  PplsScalars s = scalars_of(truth, r);
  hipError_t e = hipMemcpy(Wt, truth->W, sizeof(double) * p * r, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(Ct, truth->C, sizeof(double) * q * r, hipMemcpyHostToDevice);
  if (e == hipSuccess && !c->dtype)
    e = ppls_launch_generate(n_local, row0, p, q, c->ldx, c->ldy, r, &s, Wt, Ct, seed, TU, c->X, c->Y, c->stream);
  if (e == hipSuccess && c->dtype) {   // fp32 storage: generate fp64 row chunks, convert
    const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(std::max<int64_t>(n_local, 1),
                                                                 (int64_t)(512 << 20) / (8LL * (c->ldx + c->ldy))));
    double *gx = nullptr, *gy = nullptr;
    if (dalloc(c, &gx, (size_t)chunk * c->ldx) || dalloc(c, &gy, (size_t)chunk * c->ldy)) e = hipErrorOutOfMemory;
    for (int64_t o = 0; o < n_local && e == hipSuccess; o += chunk) {
      const int64_t nc = std::min(chunk, n_local - o);
      e = ppls_launch_generate(nc, row0 + o, p, q, c->ldx, c->ldy, r, &s, Wt, Ct, seed, TU, gx, gy, c->stream);
      if (e == hipSuccess) e = ppls_launch_convert(gx, 0, (float*)c->X + o * c->ldx, 1, nc * c->ldx, c->stream);
      if (e == hipSuccess) e = ppls_launch_convert(gy, 0, (float*)c->Y + o * c->ldy, 1, nc * c->ldy, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    dfree(gx);
    dfree(gy);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  dfree(Wt); dfree(Ct); dfree(TU);
  if (e != hipSuccess) return fail(c, PPLS_E_HIP, "synthetic generation: %s", hipGetErrorString(e));
  c->have_data = true;
  if ((rc = compute_ssq(c))) return rc;
  return check_finite_data(c);
}

int ppls_philox4x32_10(ppls_ctx* c, const uint32_t* ctr, int64_t count, uint64_t key, uint32_t* out) {
  if (!c) return PPLS_E_ARG;
  if (count < 0 || (count > 0 && (!ctr || !out))) return fail(c, PPLS_E_ARG, "bad counter array");
  if (count == 0) return PPLS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t* d = nullptr;
  HIPCHK(c, hipMalloc(&d, sizeof(uint32_t) * 8 * count));
  hipError_t e = hipMemcpy(d, ctr, sizeof(uint32_t) * 4 * count, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = ppls_launch_philox(d, count, key, d + 4 * count, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = hipMemcpy(out, d + 4 * count, sizeof(uint32_t) * 4 * count, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(c, PPLS_E_HIP, "philox: %s", hipGetErrorString(e));
  return PPLS_OK;
}

int ppls_get_data_rows(ppls_ctx* c, double* X, double* Y, int64_t row_begin, int64_t nrows) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (row_begin < 0 || nrows < 0 || row_begin + nrows > c->n_local) return fail(c, PPLS_E_ARG, "bad row range");
  if (nrows == 0) return PPLS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(nrows, (int64_t)(256 << 20) / (8LL * std::max(c->ldx, c->ldy))));
  double* wide = nullptr;
  if (c->dtype && (rc = dalloc(c, &wide, (size_t)chunk * std::max(c->ldx, c->ldy)))) return rc;
  for (int m = 0; m < 2; ++m) {
    double* dst = m == 0 ? X : Y;
    if (!dst) continue;
    const int cols = m == 0 ? c->p : c->q, ld = m == 0 ? c->ldx : c->ldy;
    for (int64_t r0 = 0; r0 < nrows; r0 += chunk) {
      const int64_t nc = std::min(chunk, nrows - r0), g0 = row_begin + r0;
      const double* src = (m == 0 ? c->X : c->Y) + g0 * ld;
      hipError_t e = hipSuccess;
      if (c->dtype) {   // fp32 storage: widen the rows first
        e = ppls_launch_convert((const float*)(m == 0 ? c->X : c->Y) + g0 * ld, 1, wide, 0, nc * ld, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        src = wide;
      }
      if (e == hipSuccess)
        e = hipMemcpy2D(dst + r0 * cols, sizeof(double) * cols, src, sizeof(double) * ld, sizeof(double) * cols, nc,
                        hipMemcpyDeviceToHost);
      if (e != hipSuccess) {
        dfree(wide);
        return fail(c, PPLS_E_HIP, "copy back: %s", hipGetErrorString(e));
      }
    }
  }
  dfree(wide);
  return PPLS_OK;
}

int ppls_get_data(ppls_ctx* c, double* X, double* Y, int64_t row_begin, int64_t nrows) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (row_begin < 0 || nrows < 0 || row_begin + nrows > c->n_local) return fail(c, PPLS_E_ARG, "bad row range");
  if (nrows == 0) return PPLS_OK;
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  for (int m = 0; m < 2; ++m) {
    double* dst = m == 0 ? X : Y;
    if (!dst) continue;
    const int cols = m == 0 ? c->p : c->q, ld = m == 0 ? c->ldx : c->ldy;
    const double* src = (m == 0 ? c->X : c->Y) + row_begin * ld;
    double *tmp = nullptr, *wide = nullptr;
    if ((rc = dalloc(c, &tmp, (size_t)nrows * cols))) return rc;
    if (c->dtype) {   // fp32 storage: widen the rows first
      if ((rc = dalloc(c, &wide, (size_t)nrows * ld))) { dfree(tmp); return rc; }
      HIPCHK(c, ppls_launch_convert((const float*)(m == 0 ? c->X : c->Y) + row_begin * ld, 1, wide, 0, nrows * ld,
                                    c->stream));
      src = wide;
    }
    HIPCHK(c, ppls_launch_to_colmajor(src, nrows, cols, ld, tmp, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    hipError_t e = hipMemcpy(dst, tmp, sizeof(double) * nrows * cols, hipMemcpyDeviceToHost);
    dfree(tmp);
    dfree(wide);
    if (e != hipSuccess) return fail(c, PPLS_E_HIP, "copy back: %s", hipGetErrorString(e));
  }
  return PPLS_OK;
}

int ppls_data_ssq(ppls_ctx* c, double* ssqX, double* ssqY) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (ssqX) *ssqX = c->ssq_host[0];
  if (ssqY) *ssqY = c->ssq_host[1];
  return PPLS_OK;
}

int ppls_estep(ppls_ctx* c, const ppls_theta* th, int r, ppls_expect* out) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, th, r))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, 1))) return rc;
  if ((rc = upload_theta(c, th, r, 0))) return rc;
  HIPCHK(c, hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  const bool wm = out && (out->mu_T || out->mu_U);
  if ((rc = sweep(c, r, 0, wm))) return rc;
  if ((rc = finalize(c, r, 0, 1, -1, PPLS_ORTH_SVD))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = download_moments(c, r, out))) return rc;
  return download_mu(c, r, out);
}

int ppls_em_step(ppls_ctx* c, const ppls_theta* in, int r, int type, ppls_theta* out, ppls_expect* fit) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, in, r))) return rc;
  if (!out || !out->W || !out->C || !out->B || !out->sigT) return fail(c, PPLS_E_ARG, "NULL output theta");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, 1))) return rc;
  if ((rc = upload_theta(c, in, r, 0))) return rc;
  HIPCHK(c, hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  const bool wm = fit && (fit->mu_T || fit->mu_U);
  if ((rc = sweep(c, r, 0, wm))) return rc;
  if ((rc = finalize(c, r, 0, 1, -1, type))) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_status(c))) return rc;
  if ((rc = download_moments(c, r, fit))) return rc;
  if ((rc = download_mu(c, r, fit))) return rc;
  return download_theta(c, r, 1, out);
}

int ppls_mstep(ppls_ctx* c, const ppls_expect* fit, int r, int type, ppls_theta* out) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (!fit || !fit->mu_T || !fit->mu_U || !fit->Ctt || !fit->Cut || !fit->Chh)
    return fail(c, PPLS_E_ARG, "Maximiz_M needs mu_T, mu_U, Ctt, Cut, Cee, Cff, Chh");
  if (!out || !out->W || !out->C || !out->B || !out->sigT) return fail(c, PPLS_E_ARG, "NULL output theta");
  if (r < 1 || r > PPLS_RMAX) return fail(c, PPLS_E_ARG, "bad r");
  if (c->dtype) return fail(c, PPLS_E_ARG, "Maximiz_M from caller-supplied moments needs fp64 storage (dtype 0)");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_r(c, r, 1))) return rc;
  const int grid = grid_of(c);
  const int groups = ppls_acc_groups(std::max<int64_t>(c->n_local, 1), grid);
  if ((rc = ensure_part(c, groups))) return rc;
  if (c->z_cols < 2 * r) {
    dfree(c->Z);
    c->z_cols = 2 * r;
    if ((rc = dalloc(c, &c->Z, (size_t)std::max<int64_t>(c->n_local, 1) * 2 * r))) return rc;
  }
  // Z = [mu_T | mu_U] row-major, coefficients alpha = delta = 1, beta = gamma = 0:
  // the accumulate pass then computes exactly X'mu_T and Y'mu_U (EM_W_multi.R:732-733).
  PplsScalars s;
  memset(&s, 0, sizeof s);
  for (int k = 0; k < r; ++k) { s.alpha[k] = 1.0; s.delta[k] = 1.0; }
  HIPCHK(c, hipMemcpy(c->sc[0], &s, sizeof s, hipMemcpyHostToDevice));
  if (c->n_local > 0) {
    double* tmp = nullptr;
    if ((rc = dalloc(c, &tmp, (size_t)c->n_local * 2 * r))) return rc;
    HIPCHK(c, hipMemcpy(tmp, fit->mu_T, sizeof(double) * c->n_local * r, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(tmp + (size_t)c->n_local * r, fit->mu_U, sizeof(double) * c->n_local * r, hipMemcpyHostToDevice));
    HIPCHK(c, ppls_launch_to_rowmajor(tmp, c->n_local, 2 * r, 2 * r, c->Z, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dfree(tmp);
    PplsSweepArgs a;
    memset(&a, 0, sizeof a);
    a.X = c->X; a.Y = c->Y; a.n_local = c->n_local; a.ldx = c->ldx; a.ldy = c->ldy;
    a.sc = c->sc[0]; a.part = c->part; a.part_ld = c->part_ld; a.r = r; a.grid = grid;
    HIPCHK(c, ppls_launch_accumulate(&a, c->Z, c->stream));
    HIPCHK(c, ppls_launch_reduce(c->part, groups, c->part_ld, c->part_ld, c->stats, 0, c->stream));
  } else {
    HIPCHK(c, hipMemsetAsync(c->stats, 0, sizeof(double) * c->part_ld, c->stream));
  }
  if ((rc = allreduce(c, c->stats, (size_t)c->part_ld))) return rc;
  HIPCHK(c, hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  PplsFinalizeArgs f;
  memset(&f, 0, sizeof f);
  f.stats = c->stats; f.ssq = c->ssq; f.N = (double)c->n_total; f.p = c->p; f.q = c->q; f.r = r;
  f.ldx = c->ldx; f.ldy = c->ldy; f.Wn = c->W[1]; f.Cn = c->C[1]; f.work = c->work; f.status = c->status;
  f.logl_index = -1; f.qr = type == PPLS_ORTH_QR ? 1 : 0; f.mode = 1 | (c->polar1 ? 4 : 0) | (polar1_bound(c, r) << 8);   // polar only
  HIPCHK(c, ppls_launch_finalize(&f, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_status(c))) return rc;
  // scalar updates on the given moments (EM_W_multi.R:734-738)
  PplsMoments m;
  memset(&m, 0, sizeof m);
  for (int k = 0; k < r; ++k) { m.Ctt[k] = fit->Ctt[k]; m.Cut[k] = fit->Cut[k]; m.Cuu[k] = fit->Cuu ? fit->Cuu[k] : 0.0; }
  m.Cee = fit->Cee;
  m.Cff = fit->Cff;
  for (int i = 0; i < r * r; ++i) m.Chh[i] = fit->Chh[i];
  PplsScalars nx;
  memset(&nx, 0, sizeof nx);
  ppls_mstep_scalars(&m, r, &nx);
  HIPCHK(c, hipMemcpy(c->sc[1], &nx, sizeof nx, hipMemcpyHostToDevice));
  return download_theta(c, r, 1, out);
}

int ppls_loglik(ppls_ctx* c, const ppls_theta* th, int r, double* out) {
  if (!c || !out) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, th, r))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, 1))) return rc;
  if ((rc = upload_theta(c, th, r, 0))) return rc;
  if ((rc = sweep(c, r, 0, false))) return rc;
  if ((rc = finalize(c, r, 0, 1, 0, PPLS_ORTH_SVD))) return rc;
  HIPCHK(c, hipMemcpyAsync(out, c->loglik, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PPLS_OK;
}

int ppls_em_run(ppls_ctx* c, ppls_theta* th, int r, int max_steps, double atol, int type, double* loglik,
                int* steps_done, int* negative_increment, ppls_expect* eout) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, th, r))) return rc;
  if (max_steps < 1) return fail(c, PPLS_E_ARG, "EMsteps must be >= 1");
  if (type != PPLS_ORTH_SVD && type != PPLS_ORTH_QR) return fail(c, PPLS_E_ARG, "type must be SVD (0) or QR (1)");
  if ((rc = check_fit_data(c))) return rc;
  if (!theta_finite(th, c->p, c->q, r)) return fail(c, PPLS_E_ARG, "theta0 has non-finite entries");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, max_steps))) return rc;
  // :773-778 canonicalise theta0 (on a copy; th is overwritten with the estimates at the end)
  {
    std::vector<double> W(th->W, th->W + (size_t)c->p * r), C(th->C, th->C + (size_t)c->q * r);
    std::vector<double> B(th->B, th->B + r), T(th->sigT, th->sigT + r);
    ppls_theta t0 = {W.data(), C.data(), B.data(), T.data(), th->sigE, th->sigF, th->sigH};
    canonicalize(&t0, c->p, c->q, r);
    if ((rc = upload_theta(c, &t0, r, 0))) return rc;
  }
  HIPCHK(c, hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  const bool want_mu = eout && (eout->mu_T || eout->mu_U);
  const bool do_check = !(atol == -INFINITY);   // atol = -Inf: the stop rule never fires
  // statistics from the cross-products S (option xprod; formed here if needed, outside the loop)
  if ((rc = xprod_begin(c, max_steps, r))) return rc;
  // The stop rule (EM_W_multi.R:792) runs on the device: the finalize that sees
  // logl[i] - logl[i-1] < atol sets a flag, and every later kernel of the run exits at once, so the
  // host enqueues iterations without a per-iteration read-back.  It polls the flag's host-mapped
  // mirror and stays at most EM_LOOKAHEAD iterations ahead of the device (events), so a long
  // EMsteps stops launching soon after convergence.  With collectives (RCCL or a host reducer) the
  // break must be the same on every rank: the mirror holds the iteration the rule fired at, which
  // every rank computes from the same all-reduced statistics, and a rank breaks at iteration s
  // iff that iteration is <= s - EM_LOOKAHEAD -- the iteration whose event it has just synced, so
  // the answer does not depend on how far each device has run.
  if (do_check) {
    if ((rc = ensure_stop(c)) || (rc = reset_stop(c))) return rc;
    c->sweep_stop = c->stop_d;
    c->stop_atol = atol;
  }
  struct StopGuard {   // the flag applies to this run only
    ppls_ctx* c;
    std::vector<hipEvent_t> evs;
    ~StopGuard() {
      c->sweep_stop = nullptr;
      c->xp_active = false;
      for (auto e : evs) (void)hipEventDestroy(e);
    }
  } guard{c, {}};
  constexpr int EM_LOOKAHEAD = 8;
  std::vector<hipEvent_t>& evs = guard.evs;
  int cur = 0;
  for (int s = 1; s <= max_steps + 1; ++s) {
    if (do_check && s > EM_LOOKAHEAD) {
      HIPCHK(c, hipEventSynchronize(evs[(size_t)(s - 1 - EM_LOOKAHEAD) % EM_LOOKAHEAD]));
      const int fired = __atomic_load_n(c->stop_mirror, __ATOMIC_ACQUIRE);
      if (fired != 0 && fired <= s - EM_LOOKAHEAD) break;   // converged: stop launching
    }
    const int nxt = cur ^ 1;
    const bool wm = want_mu && !c->xp_active && (do_check || s == max_steps + 1);
    if ((rc = stats_step(c, r, cur, wm, true))) return rc;
    if ((rc = finalize(c, r, cur, nxt, s >= 2 ? s - 2 : -1, type, do_check && s >= 3 ? s : 0))) return rc;
    if (do_check) {
      const size_t k = (size_t)(s - 1) % EM_LOOKAHEAD;
      if (evs.size() <= k) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        evs.push_back(e);
      }
      HIPCHK(c, hipEventRecord(evs[k], c->stream));
    }
    cur = nxt;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // the iteration the run ended at: the finalize of sweep s_stop saw the stop rule fire, so
  // theta_{s_stop - 1} (slot (s_stop - 1) & 1) is the estimate and logl[1 .. s_stop - 1] the trace
  int stopv[2] = {0, 0};   // {sweep the stop rule fired at, 1 if its increment was NaN}
  if (do_check) HIPCHK(c, hipMemcpy(stopv, c->stop_d, sizeof stopv, hipMemcpyDeviceToHost));
  const int s_stop = stopv[0];
  const int i_final = s_stop > 0 ? s_stop - 1 : max_steps;
  cur = i_final & 1;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_status(c))) return rc;
  if (stopv[1])   // every rank saw the same all-reduced increment, so every rank returns this
    return fail(c, PPLS_E_NUMERIC,
                "the log-likelihood increment of EM iteration %d is NaN: the reference stops PPLS_simult with "
                "an error there (`if (NA < atol)`, EM_W_multi.R:792)", i_final);
  if (c->xp_active && want_mu) {
    // Eout's mu_T, mu_U (:802) need the rows: one sweep of theta_{i_final} that only writes this
    // rank's mu rows (mu = a_i diag(alpha) + b_i diag(beta), ... from the rank's own rows and
    // theta's scalars: no collective, so ranks may ask for mu or not independently).  Eout's
    // moments are those the loop's finalize computed from S for theta_{i_final}.
    c->sweep_stop = nullptr;
    if ((rc = sweep(c, r, cur, true, true))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  std::vector<double> l(i_final);
  HIPCHK(c, hipMemcpy(l.data(), c->loglik, sizeof(double) * i_final, hipMemcpyDeviceToHost));
  if (loglik) std::copy(l.begin(), l.end(), loglik);
  if (negative_increment) {
    int neg = 0;
    for (int i = 1; i < i_final; ++i) neg |= (l[i] - l[i - 1] < 0);
    *negative_increment = neg;   // warning("Negative increments of likelihood"), :801
  }
  if (steps_done) *steps_done = i_final;
  if ((rc = download_theta(c, r, cur, th))) return rc;
  // never PPLS_OK with a non-finite trace or estimate (with atol = -Inf no stop rule looks at them)
  for (int i = 0; i < i_final; ++i)
    if (!std::isfinite(l[i]))
      return fail(c, PPLS_E_NUMERIC, "non-finite log-likelihood %g at EM iteration %d", l[i], i + 1);
  if (!theta_finite(th, c->p, c->q, r)) return fail(c, PPLS_E_NUMERIC, "non-finite estimates after %d EM iterations", i_final);
  canonicalize(th, c->p, c->q, r);   // :794-799
  if ((rc = download_moments(c, r, eout))) return rc;
  return download_mu(c, r, eout);
}

// ============================================================================ sequential initialiser
// PPLS (EM_W_multi.R:229-279) -> PPLSi (:116-180) -> EMstep_W (:51-73) -> EMstepC_fast
// (loglC.cpp:340-397).  Component k is fitted on Xc = X P_1 ... P_{k-1}, P_j = I - w_j w_j'
// (:270-271; Yc likewise with c_j) without forming Xc: the r = 1 sweep runs on X with the weight
// P_1..P_{k-1} w (so Xw of the sweep is Xc w), Xc' mu_T = P_{k-1}..P_1 X' mu_T, and
// ||Xc||^2 = ||X||^2 - sum_j ||Xc_j w_j||^2 (w_j unit).  The sweeps (all the data traffic) run on
// the device; the O((p+q) k) rank-1 update between them runs here on the host.
}  // extern "C"

namespace {

// v <- P_{m-1} ... P_0 v (first_last = true: P_0 applied first) or P_0 ... P_{m-1} v.
void deflate(const std::vector<double>& Wp, int m, int n, double* v, bool first_last) {
  for (int jj = 0; jj < m; ++jj) {
    const int j = first_last ? jj : m - 1 - jj;
    const double* w = Wp.data() + (size_t)j * n;
    double d = 0.0;
    for (int i = 0; i < n; ++i) d += w[i] * v[i];
    for (int i = 0; i < n; ++i) v[i] -= d * w[i];
  }
}

struct Rank1 {
  std::vector<double> w, c;   // unit loadings (the estimates)
  double B, sigE, sigF, sigH, sigT;
};

PplsRank1 r1_of(const Rank1& t) { return PplsRank1{t.B, t.sigE, t.sigF, t.sigH, t.sigT}; }

// EMstep_W's coefficients (:60-70) and EMstepC_fast's mu coefficients (:354, :358) (ppls_math.h).
void rank1_coefs(const Rank1& t, double* c1, double* c2, double* c3, double* al, double* be, double* ga,
                 double* de) {
  const PplsRank1 s = r1_of(t);
  ppls_rank1_coefs(&s, c1, c2, c3, al, be, ga, de);
}

// Stage component t for an r = 1 sweep over the deflated data: weights P_0..P_{m-1} w, P_0..P_{m-1} c
// (so the sweep over X, Y computes Xc w, Yc c) and the sweep scalars.
int rank1_stage(ppls_ctx* c, const Rank1& t, const std::vector<double>& Wp, const std::vector<double>& Cp, int m) {
  std::vector<double> wv(c->ldx, 0.0), cv(c->ldy, 0.0);
  std::copy(t.w.begin(), t.w.end(), wv.begin());
  std::copy(t.c.begin(), t.c.end(), cv.begin());
  deflate(Wp, m, c->p, wv.data(), false);   // X P_0 .. P_{m-1} w
  deflate(Cp, m, c->q, cv.data(), false);
  PplsScalars s;
  const PplsRank1 r1 = r1_of(t);
  ppls_rank1_sweep_scalars(&r1, &s);
  HIPCHK(c, hipMemcpyAsync(c->W[0], wv.data(), sizeof(double) * c->ldx, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->C[0], cv.data(), sizeof(double) * c->ldy, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->sc[0], &s, sizeof s, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));   // the host vectors go out of scope
  return PPLS_OK;
}

// One r = 1 sweep of theta t over the deflated data: stats -> host (SX p, SY q, G 2 x 2).
int rank1_sweep(ppls_ctx* c, const Rank1& t, const std::vector<double>& Wp, const std::vector<double>& Cp,
                int m, std::vector<double>& SX, std::vector<double>& SY, double G[4]) {
  int rc;
  if ((rc = rank1_stage(c, t, Wp, Cp, m))) return rc;
  if ((rc = stats_step(c, 1, 0, false))) return rc;
  std::vector<double> st((size_t)c->part_ld);
  HIPCHK(c, hipMemcpyAsync(st.data(), c->stats, sizeof(double) * c->part_ld, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  SX.assign(st.begin(), st.begin() + c->p);
  SY.assign(st.begin() + c->ldx, st.begin() + c->ldx + c->q);
  for (int e = 0; e < 4; ++e) G[e] = st[(size_t)c->ldx + c->ldy + e];
  return PPLS_OK;
}

// logl_W(Xc, Yc, w, c, B, sigE, sigF, sigH, sigT) from the sweep's Gram (:297-323, r = 1).
double rank1_loglik(const Rank1& t, const double G[4], double ssqX, double ssqY, double N, int p, int q) {
  const PplsRank1 s = r1_of(t);
  return ppls_rank1_loglik(&s, G, ssqX, ssqY, N, p, q);
}

// The rank-1 E-step moments and M-step scalars from one sweep's Gram (ppls_rank1_scalars, shared
// with the device step kernel): the arithmetic of EMstepC_fast (loglC.cpp:353-387) and meta_Estep /
// meta_Mstep (loglC.cpp:399-474).
void rank1_scalars(const Rank1& t, const double G[4], double ssqX, double ssqY, double N, int p, int q,
                   Rank1* n) {
  const PplsRank1 s = r1_of(t);
  PplsRank1 o;
  ppls_rank1_scalars(&s, G, ssqX, ssqY, N, p, q, &o);
  n->B = o.B;
  n->sigE = o.sigE;
  n->sigF = o.sigF;
  n->sigH = o.sigH;
  n->sigT = o.sigT;
}

// Device buffers of one PPLSi fit (ppls_rank1_step_kernel's state).
struct Rank1Dev {
  double* Wp = nullptr;   // deflation vectors (p x a), (q x a)
  double* Cp = nullptr;
  double* tw = nullptr;   // the component's loadings (p), (q)
  double* tc = nullptr;
  double* consW = nullptr;
  double* consC = nullptr;
  double* lv = nullptr;   // logvalue (EMsteps + 1) and the last Gram (4)
  PplsRank1* st = nullptr;
  ~Rank1Dev() { dfree(Wp); dfree(Cp); dfree(tw); dfree(tc); dfree(consW); dfree(consC); dfree(lv); dfree(st); }
};

// PPLSi's EM loop for component m (EM_W_multi.R:147-173) entirely on the device: per step one r = 1
// sweep and one ppls_rank1_step_kernel (loglik, stop rule, EMstepC_fast update, constraints, next
// weights), no host round trip.  The host enqueues up to EMsteps steps, at most EM_LOOKAHEAD ahead
// of the device, and stops launching once the step kernel reports the end of the fit (host-mapped
// flag = the step it ended at + 1; a rank breaks at step s iff that step is <= s - LOOKAHEAD, whose
// event it has synced, so all ranks break at the same step and their collectives stay matched).
// t: in = the constrained initial component, out = the fit.  lv: logvalue[0..i]; G: the last Gram.
int rank1_fit_device(ppls_ctx* c, Rank1Dev& d, Rank1& t, const ppls_constraint* ck, int m, double ssqX,
                     double ssqY, int max_steps, double atol, int crit_abs, const std::vector<double>& Wp,
                     const std::vector<double>& Cp, std::vector<double>& lv, int* steps, bool* na, double G[4]) {
  int rc;
  const int p = c->p, q = c->q;
  if ((rc = rank1_stage(c, t, Wp, Cp, m))) return rc;
  const PplsRank1 r1 = r1_of(t);
  HIPCHK(c, hipMemcpyAsync(d.tw, t.w.data(), sizeof(double) * p, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d.tc, t.c.data(), sizeof(double) * q, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(d.st, &r1, sizeof r1, hipMemcpyHostToDevice, c->stream));
  PplsRank1StepArgs a;
  memset(&a, 0, sizeof a);
  if (ck) {
    if (ck->W) HIPCHK(c, hipMemcpyAsync(d.consW, ck->W, sizeof(double) * p, hipMemcpyHostToDevice, c->stream));
    if (ck->C) HIPCHK(c, hipMemcpyAsync(d.consC, ck->C, sizeof(double) * q, hipMemcpyHostToDevice, c->stream));
    a.consW = ck->W ? d.consW : nullptr;
    a.consC = ck->C ? d.consC : nullptr;
    if (ck->B) { a.cons_mask |= 1; a.cons_val.B = ck->B[0]; }
    if (ck->sigE) { a.cons_mask |= 2; a.cons_val.sigE = ck->sigE[0]; }
    if (ck->sigF) { a.cons_mask |= 4; a.cons_val.sigF = ck->sigF[0]; }
    if (ck->sigH) { a.cons_mask |= 8; a.cons_val.sigH = ck->sigH[0]; }
    if (ck->sigT) { a.cons_mask |= 16; a.cons_val.sigT = ck->sigT[0]; }
  }
  if ((rc = ensure_stop(c)) || (rc = reset_stop(c))) return rc;
  a.stats = c->stats;
  a.p = p; a.q = q; a.ldx = c->ldx; a.ldy = c->ldy;
  a.N = (double)c->n_total; a.ssqX = ssqX; a.ssqY = ssqY;
  a.Wp = d.Wp; a.Cp = d.Cp; a.m = m;
  a.st = d.st; a.tw = d.tw; a.tc = d.tc;
  a.Wdst = c->W[0]; a.Cdst = c->C[0]; a.scdst = c->sc[0];
  a.lv = d.lv; a.Gkeep = d.lv + max_steps + 1;
  a.max_steps = max_steps; a.crit_abs = crit_abs; a.atol = atol;
  a.stop = c->stop_d; a.stop_mirror = c->stop_mirror_dev;
  struct Guard {
    ppls_ctx* c;
    std::vector<hipEvent_t> evs;
    ~Guard() {
      c->sweep_stop = nullptr;
      for (auto e : evs) (void)hipEventDestroy(e);
    }
  } guard{c, {}};
  c->sweep_stop = c->stop_d;
  constexpr int LOOKAHEAD = 8;
  for (int step = 0; step <= max_steps; ++step) {
    if (step >= LOOKAHEAD) {
      HIPCHK(c, hipEventSynchronize(guard.evs[(size_t)(step - LOOKAHEAD) % LOOKAHEAD]));
      const int ended = __atomic_load_n(c->stop_mirror, __ATOMIC_ACQUIRE);
      if (ended != 0 && ended - 1 <= step - LOOKAHEAD) break;   // the fit ended
    }
    if ((rc = stats_step(c, 1, 0, false))) return rc;
    a.step = step;
    HIPCHK(c, ppls_launch_rank1_step(&a, c->stream));
    {
      const size_t k = (size_t)step % LOOKAHEAD;
      if (guard.evs.size() <= k) {
        hipEvent_t e;
        HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        guard.evs.push_back(e);
      }
      HIPCHK(c, hipEventRecord(guard.evs[k], c->stream));
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int stop[2] = {0, 0};
  HIPCHK(c, hipMemcpy(stop, c->stop_d, sizeof stop, hipMemcpyDeviceToHost));
  if (stop[1] == 2)   // every rank computed the same all-reduced increment
    return fail(c, PPLS_E_NUMERIC,
                "PPLSi component %d: the log-likelihood increment of EM step %d is NaN; the reference stops with "
                "an error there (`if (critfunc(NA) < atol)`, EM_W_multi.R:173)", m + 1, stop[0]);
  *na = stop[1] != 0;
  *steps = stop[0] > 0 ? stop[0] : stop[0] < 0 ? -stop[0] : max_steps;   // < 0: sigma collapse at step -stop[0]-1
  std::vector<double> buf((size_t)max_steps + 5);
  HIPCHK(c, hipMemcpy(buf.data(), d.lv, sizeof(double) * buf.size(), hipMemcpyDeviceToHost));
  lv.assign(buf.begin(), buf.begin() + (*steps + 1));
  for (int e = 0; e < 4; ++e) G[e] = buf[(size_t)max_steps + 1 + e];
  PplsRank1 o;
  HIPCHK(c, hipMemcpy(&o, d.st, sizeof o, hipMemcpyDeviceToHost));
  t.B = o.B; t.sigE = o.sigE; t.sigF = o.sigF; t.sigH = o.sigH; t.sigT = o.sigT;
  HIPCHK(c, hipMemcpy(t.w.data(), d.tw, sizeof(double) * p, hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(t.c.data(), d.tc, sizeof(double) * q, hipMemcpyDeviceToHost));
  return PPLS_OK;
}

// ||X P_0..P_{m-1}||^2 (and the Y analogue) by an exact residual pass over the resident data,
// all-reduced over ranks.  Used when the running ||X||^2 - sum ||Xc_j w_j||^2 has cancelled to
// below 1e-6 ||X||^2, where its absolute error (~eps ||X||^2) would hide a rank collapse.
int deflated_ssq(ppls_ctx* c, const std::vector<double>& Wp, int m, bool isx, double* out) {
  int rc;
  const int n = isx ? c->p : c->q;
  const int nb = 1024;
  double* Wd = nullptr;
  double* buf = nullptr;
  if ((rc = dalloc(c, &Wd, (size_t)n * std::max(m, 1)))) return rc;
  if ((rc = dalloc(c, &buf, (size_t)nb + 1))) { dfree(Wd); return rc; }
  double res = 0.0;
  hipError_t e = hipMemcpyAsync(Wd, Wp.data(), sizeof(double) * n * m, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = ppls_launch_deflated_ssq(isx ? c->X : c->Y, c->dtype, c->n_local, isx ? c->ldx : c->ldy, n, Wd, m, buf,
                                 nb, buf + nb, c->stream);
  if (e == hipSuccess && c->n_local == 0) e = hipMemsetAsync(buf + nb, 0, sizeof(double), c->stream);
  rc = e == hipSuccess ? allreduce(c, buf + nb, 1) : fail(c, PPLS_E_HIP, "deflated ssq: %s", hipGetErrorString(e));
  if (!rc) {
    e = hipMemcpyAsync(&res, buf + nb, sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc = fail(c, PPLS_E_HIP, "deflated ssq: %s", hipGetErrorString(e));
  }
  dfree(Wd);
  dfree(buf);
  *out = res;
  return rc;
}

}  // namespace

extern "C" {

int ppls_ppls(ppls_ctx* c, int a, int max_steps, double atol, const ppls_theta* init, ppls_seq_fit* out) {
  return ppls_ppls_ex(c, a, max_steps, atol, 0, init, nullptr, out);
}

int ppls_ppls_ex(ppls_ctx* c, int a, int max_steps, double atol, int crit_abs, const ppls_theta* init,
                 const ppls_constraint* cons, ppls_seq_fit* out) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (!init || !out || !out->W || !out->C || !out->B || !out->sig) return fail(c, PPLS_E_ARG, "NULL argument");
  if (a < 1 || a > PPLS_RMAX) return fail(c, PPLS_E_ARG, "nr_comp=%d outside [1,%d]", a, PPLS_RMAX);
  if (c->p < a || c->q < a)   // stopifnot(ncol(X) >= nr_comp, ncol(Y) >= nr_comp) (:245)
    return fail(c, PPLS_E_ARG, "ncol(X)=%d, ncol(Y)=%d must be >= number of components %d", c->p, c->q, a);
  if (max_steps < 1) return fail(c, PPLS_E_ARG, "EMsteps must be >= 1");
  int rc;
  if ((rc = check_fit_data(c))) return rc;
  for (int k = 0; k < a; ++k)
    if (!init[k].W || !init[k].C || !init[k].B || !init[k].sigT)
      return fail(c, PPLS_E_ARG, "init[%d] has NULL fields", k);
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, 1, max_steps))) return rc;
  // the rank-1 steps' statistics from the cross-products S (option xprod): the sweep's weights are
  // the deflated P_0..P_{m-1} w, so S blockdiag(P w, P c) gives exactly the sweep's X'mu_T and Gram
  if ((rc = xprod_begin(c, a * max_steps, 1))) return rc;
  struct XpGuard {
    ppls_ctx* c;
    ~XpGuard() { c->xp_active = false; }
  } xp_guard{c};
  const int p = c->p, q = c->q;
  const double N = (double)c->n_total;
  double ssqX = c->ssq_host[0], ssqY = c->ssq_host[1];   // ||Xc||^2, ||Yc||^2 of the current deflation
  std::vector<double> Wp, Cp;                            // w_1..w_k, c_1..c_k (column-major)
  std::vector<double> gA, gD, gB;                        // ||X w_j||^2, <X w_j, Y c_j>, ||Y c_j||^2
  bool fixed_wc = false;                                 // some component had W or C fixed
  Rank1Dev dev;
  if ((rc = dalloc(c, &dev.Wp, (size_t)p * a)) || (rc = dalloc(c, &dev.Cp, (size_t)q * a)) ||
      (rc = dalloc(c, &dev.tw, (size_t)p)) || (rc = dalloc(c, &dev.tc, (size_t)q)) ||
      (rc = dalloc(c, &dev.consW, (size_t)p)) || (rc = dalloc(c, &dev.consC, (size_t)q)) ||
      (rc = dalloc(c, &dev.lv, (size_t)max_steps + 5)) || (rc = dalloc(c, &dev.st, 1)))
    return rc;
  out->ncomp = 0;
  out->not_monotone = 0;
  if (out->logvalue)
    for (size_t e = 0; e < (size_t)a * (max_steps + 1); ++e) out->logvalue[e] = NAN;
  for (int k = 0; k < a; ++k) {
    Rank1 t;
    t.w.assign(init[k].W, init[k].W + p);
    t.c.assign(init[k].C, init[k].C + q);
    t.B = init[k].B[0];
    t.sigT = init[k].sigT[0];
    t.sigE = init[k].sigE;
    t.sigF = init[k].sigF;
    t.sigH = init[k].sigH;
    // PPLSi's constraints (fconstraint, :85-92): fixed values replace the estimates at the start
    // (:141-145) and after every EM step (:165-169)
    const ppls_constraint* ck = cons ? &cons[k] : nullptr;
    auto constrain = [&](Rank1& u) {
      if (!ck) return;
      if (ck->W) u.w.assign(ck->W, ck->W + p);
      if (ck->C) u.c.assign(ck->C, ck->C + q);
      if (ck->B) u.B = ck->B[0];
      if (ck->sigE) u.sigE = ck->sigE[0];
      if (ck->sigF) u.sigF = ck->sigF[0];
      if (ck->sigH) u.sigH = ck->sigH[0];
      if (ck->sigT) u.sigT = ck->sigT[0];
    };
    if (ck && (ck->W || ck->C)) fixed_wc = true;
    constrain(t);
    if (k > 0) {   // deflation vectors w_1..w_k, c_1..c_k on the device
      HIPCHK(c, hipMemcpyAsync(dev.Wp, Wp.data(), sizeof(double) * Wp.size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(dev.Cp, Cp.data(), sizeof(double) * Cp.size(), hipMemcpyHostToDevice, c->stream));
    }
    // PPLSi's EM loop (:147-173) on the device; i = the reference's final i (steps made)
    double G[4];
    std::vector<double> lv;
    int i = 0;
    bool na = false;
    if ((rc = rank1_fit_device(c, dev, t, ck, k, ssqX, ssqY, max_steps, atol, crit_abs, Wp, Cp, lv, &i, &na, G)))
      return rc;
    if (na) break;   // PPLS: "residuals are of rank < 1e-14", keep components 1..k-1 (:258-263)
    if (i > max_steps) i = max_steps;
    for (int e = 0; e < p; ++e) out->W[(size_t)k * p + e] = t.w[e];
    for (int e = 0; e < q; ++e) out->C[(size_t)k * q + e] = t.c[e];
    out->B[k] = t.B;
    out->sig[k] = t.sigE;             // cbind(sigX, sigY, sigH, sigT), a x 4
    out->sig[a + k] = t.sigF;
    out->sig[2 * a + k] = t.sigH;
    out->sig[3 * a + k] = t.sigT;
    if (out->logvalue)
      for (int e = 0; e <= i; ++e) out->logvalue[(size_t)k * (max_steps + 1) + e] = lv[e];
    if (out->last_increment) out->last_increment[k] = lv[i] - lv[i - 1];   // :176
    if (out->number_steps) out->number_steps[k] = i;
    for (int e = 1; e <= i; ++e)
      if (lv[e] - lv[e - 1] < 0) out->not_monotone |= 1 << k;              // warning("Not monotone") :177
    // deflation (:270-271): the last sweep used theta_final, so its Gram holds ||Xc_k w_k||^2
    gA.push_back(G[0]);
    gD.push_back(G[1]);
    gB.push_back(G[3]);
    // ||Xc (I - w w')||^2 = ||Xc||^2 - (2 - w'w) ||Xc w||^2 (w'w = 1 unless W is a fixed constraint)
    if (ck && ck->W) {
      double ww = 0.0;
      for (int e = 0; e < p; ++e) ww += t.w[e] * t.w[e];
      ssqX -= (2.0 - ww) * G[0];
    } else {
      ssqX -= G[0];
    }
    if (ck && ck->C) {
      double cc = 0.0;
      for (int e = 0; e < q; ++e) cc += t.c[e] * t.c[e];
      ssqY -= (2.0 - cc) * G[3];
    } else {
      ssqY -= G[3];
    }
    Wp.insert(Wp.end(), t.w.begin(), t.w.end());
    Cp.insert(Cp.end(), t.c.begin(), t.c.end());
    if (k + 1 < a && ssqX < 1e-6 * c->ssq_host[0])
      if ((rc = deflated_ssq(c, Wp, k + 1, true, &ssqX))) return rc;
    if (k + 1 < a && ssqY < 1e-6 * c->ssq_host[1])
      if ((rc = deflated_ssq(c, Cp, k + 1, false, &ssqY))) return rc;
    out->ncomp = k + 1;
    // Other_output$Loglikelihoods[k] = logl_W(X, Y, W[,1:k], C[,1:k], diag(B[1:k]), sigX_k, sigY_k,
    // sigH_k, diag(sigT[1:k])) (:274).  loglC_fast only reads the Gram diagonal, and X w_j = Xc_j w_j
    // because w_j is orthogonal to w_1..w_{j-1}, so the per-component Grams above suffice.
    if (out->loglikelihoods) {
      const int r = k + 1;
      if (fixed_wc) {   // fixed W / C need not be orthogonal: X w_j from undeflated sweeps
        for (int j = 0; j < r; ++j) {
          Rank1 u = t;
          u.w.assign(Wp.begin() + (size_t)j * p, Wp.begin() + (size_t)(j + 1) * p);
          u.c.assign(Cp.begin() + (size_t)j * q, Cp.begin() + (size_t)(j + 1) * q);
          double Gj[4];
          std::vector<double> sx, sy;
          static const std::vector<double> none;
          if ((rc = rank1_sweep(c, u, none, none, 0, sx, sy, Gj))) return rc;
          gA[j] = Gj[0];
          gD[j] = Gj[1];
          gB[j] = Gj[3];
        }
      }
      std::vector<double> Gf((size_t)4 * r * r, 0.0);
      PplsScalars s;
      memset(&s, 0, sizeof s);
      for (int j = 0; j < r; ++j) {
        PPLS_GA(Gf.data(), r, j, j) = gA[j];
        PPLS_GD(Gf.data(), r, j, j) = gD[j];
        PPLS_GB(Gf.data(), r, j, j) = gB[j];
        s.b[j] = out->B[j];
        s.t[j] = out->sig[3 * a + j];
      }
      s.sigE = t.sigE;
      s.sigF = t.sigF;
      s.sigH = t.sigH;
      out->loglikelihoods[k] = ppls_loglik_from_gram(Gf.data(), c->ssq_host[0], c->ssq_host[1], N, p, q, r, &s);
    }
  }
  return PPLS_OK;
}

}  // extern "C"

namespace {

// Sums of squares of the rows [row0, row0 + nrows) of X and Y on this rank, all-reduced -> out[2].
int segment_ssq(ppls_ctx* c, int64_t row0, int64_t nrows, double out[2]) {
  int rc;
  const int nb = 1024;
  double* buf = nullptr;
  if ((rc = dalloc(c, &buf, (size_t)nb + 2))) return rc;
  hipError_t e = hipMemsetAsync(buf + nb, 0, 2 * sizeof(double), c->stream);
  for (int m = 0; m < 2 && e == hipSuccess && nrows > 0; ++m) {
    const int64_t ld = m ? c->ldy : c->ldx;
    const void* base = m ? (const void*)c->Y : (const void*)c->X;
    if (c->dtype)
      e = ppls_launch_sumsq_f32((const float*)base + row0 * ld, nrows * ld, buf, nb, buf + nb + m, c->stream);
    else
      e = ppls_launch_sumsq((const double*)base + row0 * ld, nrows * ld, buf, nb, buf + nb + m, 0, c->stream);
  }
  rc = e == hipSuccess ? allreduce(c, buf + nb, 2) : fail(c, PPLS_E_HIP, "segment ssq: %s", hipGetErrorString(e));
  if (!rc) {
    e = hipMemcpyAsync(out, buf + nb, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) rc = fail(c, PPLS_E_HIP, "segment ssq: %s", hipGetErrorString(e));
  }
  dfree(buf);
  return rc;
}

// rank1_sweep restricted to this rank's rows of one population.
int segment_sweep(ppls_ctx* c, int64_t row0, int64_t nrows, const Rank1& t, std::vector<double>& SX,
                  std::vector<double>& SY, double G[4]) {
  static const std::vector<double> none;
  c->seg_row0 = row0;
  c->seg_rows = nrows;
  const int rc = rank1_sweep(c, t, none, none, 0, SX, SY, G);
  c->seg_row0 = 0;
  c->seg_rows = -1;
  return rc;
}

struct MetaPop {
  int64_t row0 = 0, nloc = 0;   // this rank's rows of the population
  double N = 0.0;               // rows over all ranks (nrow(X[popui, ]))
  double ssq[2] = {0.0, 0.0};   // ssq(X[popui, ]), ssq(Y[popui, ])
  Rank1 t;                      // params[[j]] with the shared W., C.
  std::vector<double> SX, SY;   // X[popui, ]' mu_T, Y[popui, ]' mu_U of the last sweep
  double G[4] = {0, 0, 0, 0};
};

int meta_setup(ppls_ctx* c, int npop, const int64_t* pop_local, const int64_t* pop_total,
               std::vector<MetaPop>& pops) {
  if (npop < 1 || !pop_local || !pop_total) return fail(c, PPLS_E_ARG, "need npop >= 1 populations with row counts");
  pops.assign(npop, MetaPop());
  int64_t r0 = 0, tot = 0;
  for (int j = 0; j < npop; ++j) {
    if (pop_local[j] < 0 || pop_total[j] < 1) return fail(c, PPLS_E_ARG, "population %d has no rows", j + 1);
    pops[j].row0 = r0;
    pops[j].nloc = pop_local[j];
    pops[j].N = (double)pop_total[j];
    r0 += pop_local[j];
    tot += pop_total[j];
  }
  if (r0 != c->n_local) return fail(c, PPLS_E_ARG, "population rows on this rank sum to %lld, not n_local = %lld",
                                    (long long)r0, (long long)c->n_local);
  if (tot != c->n_total)   // stopifnot(nrow(X) == length(Ipopu)) (:448, :511)
    return fail(c, PPLS_E_ARG, "population sizes sum to %lld, not nrow(X) = %lld", (long long)tot,
                (long long)c->n_total);
  int rc;
  for (auto& pp : pops)
    if ((rc = segment_ssq(c, pp.row0, pp.nloc, pp.ssq))) return rc;
  return PPLS_OK;
}

// The M-step half of meta_EMstep (:453-484) from each population's last sweep: meta_Mstep per
// population, then W. = orth(sum_j sign(<Cxt_1, Cxt_j>) Cxt_j), C. likewise with Cyu_j.  orth of one
// column is v / ||v|| (OmicsPLS::orth semantics of Package/functions.R:252-260; unpinned).
void meta_mstep(std::vector<MetaPop>& pops, int p, int q, std::vector<double>& w, std::vector<double>& cv,
                std::vector<double>* Cxt, std::vector<double>* Cyu) {
  const int npop = (int)pops.size();
  std::vector<Rank1> nt(npop);
  for (int j = 0; j < npop; ++j) rank1_scalars(pops[j].t, pops[j].G, pops[j].ssq[0], pops[j].ssq[1], pops[j].N, p, q, &nt[j]);
  w.assign(p, 0.0);
  cv.assign(q, 0.0);
  if (Cxt) Cxt->assign((size_t)p * npop, 0.0);
  if (Cyu) Cyu->assign((size_t)q * npop, 0.0);
  const std::vector<double>& x1 = pops[0].SX;
  const double N1 = pops[0].N;
  for (int j = 0; j < npop; ++j) {
    const MetaPop& pp = pops[j];
    double d = 0.0;   // crossprod(Cxt_1, Cxt_j) = <SX_1, SX_j> / (N_1 N_j)
    for (int i = 0; i < p; ++i) d += (x1[i] / N1) * (pp.SX[i] / pp.N);
    const double sg = d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0);   // R's sign()
    for (int i = 0; i < p; ++i) w[i] += sg * (pp.SX[i] / pp.N);     // Cxt = X' mu_T / N (loglC.cpp:416)
    for (int i = 0; i < q; ++i) cv[i] += sg * (pp.SY[i] / pp.N);    // Cyu (:421)
    if (Cxt) for (int i = 0; i < p; ++i) (*Cxt)[(size_t)j * p + i] = pp.SX[i] / pp.N;
    if (Cyu) for (int i = 0; i < q; ++i) (*Cyu)[(size_t)j * q + i] = pp.SY[i] / pp.N;
  }
  double nw = 0.0, nc = 0.0;
  for (double v : w) nw += v * v;
  for (double v : cv) nc += v * v;
  nw = std::sqrt(nw);
  nc = std::sqrt(nc);
  for (double& v : w) v /= nw;
  for (double& v : cv) v /= nc;
  for (int j = 0; j < npop; ++j) {
    pops[j].t.B = nt[j].B;
    pops[j].t.sigE = nt[j].sigE;
    pops[j].t.sigF = nt[j].sigF;
    pops[j].t.sigH = nt[j].sigH;
    pops[j].t.sigT = nt[j].sigT;
  }
}

void meta_params_out(const std::vector<MetaPop>& pops, double* params) {
  const int npop = (int)pops.size();
  for (int j = 0; j < npop; ++j) {
    params[j] = pops[j].t.B;
    params[npop + j] = pops[j].t.sigE;
    params[2 * npop + j] = pops[j].t.sigF;
    params[3 * npop + j] = pops[j].t.sigH;
    params[4 * npop + j] = pops[j].t.sigT;
  }
}

int meta_sweep_all(ppls_ctx* c, std::vector<MetaPop>& pops, const std::vector<double>& w,
                   const std::vector<double>& cv) {
  int rc;
  for (auto& pp : pops) {
    pp.t.w = w;
    pp.t.c = cv;
    if ((rc = segment_sweep(c, pp.row0, pp.nloc, pp.t, pp.SX, pp.SY, pp.G))) return rc;
  }
  return PPLS_OK;
}

// meta_PPLSi on the device (ppls_meta_step_kernel) for every storage and shape: one segmented
// sweep per EM step -- the split sweep (fp64, p and q within its register budget) or, round 6, the
// panel sweep (fp32 storage, wide p).  Option meta_device = 0 keeps the per-population host loop.
bool meta_device_ok(const ppls_ctx* c, int npop) {
  return c->meta_device && npop >= 1 && npop <= PPLS_META_KMAX;
}

// The whole meta_PPLSi loop (EM_W_multi.R:544-578) on the device.  Per EM step the statistics of
// every population from ONE segmented sweep over X and Y -- the split sweep: workgroups partitioned
// over the populations in proportion to their rows (each workgroup's rows in one population, using
// that population's scalars); the panel sweep (fp32 storage, wide p): the dots give every row its
// population's mu, and the accumulation's row chunks are partitioned like those workgroups -- then per
// population a reduction of its workgroups' partials, one all-reduce of the K statistics blocks when
// sharded, and ppls_meta_step_kernel (log-likelihoods, stop rule, M-step, the next sweep's loadings
// and scalars).  No host round trip per step: the host enqueues at most LOOKAHEAD steps ahead and
// stops launching once the step kernel reports the end of the fit (all ranks at the same step).
// logvalue[1, ] comes from the first sweep (theta0 is every population's, so the full-data Gram is
// the sum of theirs): no separate full-data sweep.
int meta_ppls_device(ppls_ctx* c, const std::vector<MetaPop>& pops, const Rank1& t0, int max_steps, double atol,
                     int crit_abs, ppls_meta_fit* out) {
  const int K = (int)pops.size();
  const int p = c->p, q = c->q;
  int rc;
  PplsSweepArgs a;
  const int plan = sweep_plan(c, 1, &a);
  if (plan != 3 && plan != 4) return fail(c, PPLS_E_STATE, "meta device path: no sweep for this shape");
  const bool panel = plan == 4;
  c->meta_path = panel ? 3 : 2;
  // workgroups per population: proportional to its local rows, at least one if it has any.  A rank
  // with no local rows (nz = 0) gets no workgroups: it launches no sweep, zeroes its K statistics
  // blocks and still joins every all-reduce (the remainder loop below never ended there).
  // Panel: the same partition of the accumulation's row chunks (a.grid: the chunk policy of a sweep of
  // every local row), so each chunk lies in one population.
  int nz = 0;
  for (const auto& pp : pops) nz += pp.nloc > 0 ? 1 : 0;
  std::vector<int> gk((size_t)K, 0);
  int G = 0;
  if (nz > 0) {
    G = std::max(a.grid, nz);
    int left = G;
    for (int j = 0; j < K; ++j) gk[(size_t)j] = pops[j].nloc > 0 ? 1 : 0;
    left -= nz;
    const double nrows = (double)std::max<int64_t>(c->n_local, 1);
    for (int j = 0; j < K && left > 0; ++j) {
      if (pops[j].nloc <= 0) continue;
      const int extra = std::min(left, (int)std::floor((double)(G - nz) * (double)pops[j].nloc / nrows));
      gk[(size_t)j] += extra;
      left -= extra;
    }
    for (int j = 0; left > 0; j = (j + 1) % K)   // the rounding remainder, one at a time (nz > 0: ends)
      if (pops[j].nloc > 0) { ++gk[(size_t)j]; --left; }
  }
  std::vector<int64_t> bnd((size_t)G + 1);
  std::vector<int> seg((size_t)G), g0((size_t)K + 1, 0);
  {
    int g = 0;
    for (int j = 0; j < K; ++j) {
      g0[(size_t)j] = g;
      for (int u = 0; u < gk[(size_t)j]; ++u, ++g) {
        bnd[(size_t)g] = pops[j].row0 + pops[j].nloc * u / gk[(size_t)j];
        seg[(size_t)g] = j;
      }
    }
    g0[(size_t)K] = g;
    bnd[(size_t)G] = c->n_local;
  }
  if ((rc = ensure_part(c, std::max(G, 1)))) return rc;
  if (panel && c->z_cols < 4) {   // Z = [Xw | Yc | mu_T | mu_U] rows + the transposed W, C
    dfree(c->Z);
    c->z_cols = 0;
    if ((rc = dalloc(c, &c->Z, (size_t)ppls_panel_z_len(c->n_local, c->ldx, c->ldy, 1)))) return rc;
    c->z_cols = 4;
  }
  if ((rc = ensure_stop(c)) || (rc = reset_stop(c))) return rc;
  struct Dev {
    int64_t* bnd = nullptr;
    int64_t* segend = nullptr;
    int* seg = nullptr;
    double* stats = nullptr;
    double* N = nullptr;
    double* ssq = nullptr;
    double* log = nullptr;
    PplsRank1* st = nullptr;
    PplsScalars* sc = nullptr;
    ppls_ctx* c = nullptr;
    std::vector<hipEvent_t> evs;
    ~Dev() {
      dfree(bnd); dfree(segend); dfree(seg); dfree(stats); dfree(N); dfree(ssq); dfree(log); dfree(st); dfree(sc);
      if (c) c->sweep_stop = nullptr;
      for (auto e : evs) (void)hipEventDestroy(e);
    }
  } d;
  d.c = c;
  const int64_t pld = c->part_ld, lld = (int64_t)max_steps + 1;
  if ((rc = dalloc(c, &d.bnd, (size_t)G + 1)) || (rc = dalloc(c, &d.seg, (size_t)std::max(G, 1))) ||
      (rc = dalloc(c, &d.segend, (size_t)K)) ||
      (rc = dalloc(c, &d.stats, (size_t)K * pld)) || (rc = dalloc(c, &d.N, (size_t)K)) ||
      (rc = dalloc(c, &d.ssq, (size_t)2 * K)) || (rc = dalloc(c, &d.log, (size_t)K * lld)) ||
      (rc = dalloc(c, &d.st, (size_t)K)) || (rc = dalloc(c, &d.sc, (size_t)K)))
    return rc;
  {
    std::vector<double> hN((size_t)K), hs((size_t)2 * K), hl((size_t)K * lld, NAN);
    std::vector<PplsRank1> hst((size_t)K, r1_of(t0));
    std::vector<PplsScalars> hsc((size_t)K);
    for (int j = 0; j < K; ++j) {
      hN[(size_t)j] = pops[j].N;
      hs[(size_t)2 * j] = pops[j].ssq[0];
      hs[(size_t)2 * j + 1] = pops[j].ssq[1];
      ppls_rank1_sweep_scalars(&hst[(size_t)j], &hsc[(size_t)j]);
    }
    std::vector<double> wv((size_t)c->ldx, 0.0), cv((size_t)c->ldy, 0.0);
    std::copy(t0.w.begin(), t0.w.end(), wv.begin());
    std::copy(t0.c.begin(), t0.c.end(), cv.begin());
    HIPCHK(c, hipMemcpyAsync(d.bnd, bnd.data(), sizeof(int64_t) * bnd.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.seg, seg.data(), sizeof(int) * seg.size(), hipMemcpyHostToDevice, c->stream));
    std::vector<int64_t> se((size_t)K);
    for (int j = 0; j < K; ++j) se[(size_t)j] = pops[j].row0 + pops[j].nloc;
    HIPCHK(c, hipMemcpyAsync(d.segend, se.data(), sizeof(int64_t) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.N, hN.data(), sizeof(double) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.ssq, hs.data(), sizeof(double) * 2 * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.log, hl.data(), sizeof(double) * hl.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.st, hst.data(), sizeof(PplsRank1) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d.sc, hsc.data(), sizeof(PplsScalars) * K, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->W[0], wv.data(), sizeof(double) * wv.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->C[0], cv.data(), sizeof(double) * cv.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));   // the host vectors go out of scope
  }
  a.X = c->X;
  a.Y = c->Y;
  a.n_local = c->n_local;
  a.Wp = c->W[0];
  a.Cp = c->C[0];
  a.sc = d.sc;
  a.part = c->part;
  a.part_ld = pld;
  a.mu = nullptr;
  a.write_mu = 0;
  a.grid = G;
  a.row_bounds = d.bnd;
  a.wg_seg = d.seg;
  a.nt = (c->nt_loads > 0 || (c->nt_loads < 0 && 8.0 * c->n_local * (double)(c->ldx + c->ldy) > 256.0 * (1 << 20))) ? 1 : 0;
  a.stop = c->stop_d;
  a.trace = nullptr;
  c->sweep_stop = c->stop_d;
  PplsMetaStepArgs m;
  memset(&m, 0, sizeof m);
  m.stats = d.stats; m.part_ld = pld; m.K = K; m.p = p; m.q = q; m.ldx = c->ldx; m.ldy = c->ldy;
  m.N = d.N; m.ssq = d.ssq; m.st = d.st; m.sc = d.sc; m.W = c->W[0]; m.C = c->C[0];
  m.log = d.log; m.log_ld = lld; m.max_steps = max_steps; m.crit_abs = crit_abs; m.atol = atol;
  m.stop = c->stop_d; m.stop_mirror = c->stop_mirror_dev;
  m.ssqX = c->ssq_host[0]; m.ssqY = c->ssq_host[1]; m.Ntot = (double)c->n_total;
  double* tmp = c->part + (size_t)c->part_groups * pld;
  // one segmented sweep of the current parameters -> d.stats (K blocks, all-reduced)
  if (panel) {   // the dots use each row's population scalars; the accumulation's chunks are bnd
    a.row_bounds = nullptr;
    a.wg_seg = nullptr;
    a.seg_ends = d.segend;
    a.nseg = K;
    a.chunk_bounds = d.bnd;
  }
  auto seg_sweep = [&]() -> int {
    if (G > 0) {
      if (panel) HIPCHK(c, ppls_launch_sweep_panel(&a, c->dtype, c->Z, G, c->stream));
      else HIPCHK(c, ppls_launch_sweep_split(&a, c->stream));
    }
    for (int j = 0; j < K; ++j) {
      const int ng = g0[(size_t)j + 1] - g0[(size_t)j];
      if (ng > 0)
        HIPCHK(c, ppls_launch_reduce2(c->part + (size_t)g0[(size_t)j] * pld, ng, pld, pld, d.stats + (size_t)j * pld,
                                      tmp, c->stop_d, c->stream));
      else
        HIPCHK(c, hipMemsetAsync(d.stats + (size_t)j * pld, 0, sizeof(double) * pld, c->stream));
    }
    return allreduce(c, d.stats, (size_t)K * pld);
  };
  constexpr int LOOKAHEAD = 8;
  for (int step = 0; step <= max_steps; ++step) {
    if (step >= LOOKAHEAD) {
      HIPCHK(c, hipEventSynchronize(d.evs[(size_t)(step - LOOKAHEAD) % LOOKAHEAD]));
      const int ended = __atomic_load_n(c->stop_mirror, __ATOMIC_ACQUIRE);
      if (ended != 0 && ended <= step - LOOKAHEAD) break;   // the same break step on every rank
    }
    if ((rc = seg_sweep())) return rc;
    m.step = step;
    HIPCHK(c, ppls_launch_meta_step(&m, c->stream));
    const size_t k = (size_t)step % LOOKAHEAD;
    if (d.evs.size() <= k) {
      hipEvent_t e;
      HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      d.evs.push_back(e);
    }
    HIPCHK(c, hipEventRecord(d.evs[k], c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int stop[2] = {0, 0};
  HIPCHK(c, hipMemcpy(stop, c->stop_d, sizeof stop, hipMemcpyDeviceToHost));
  if (stop[1] == 2)
    return fail(c, PPLS_E_NUMERIC, "meta_PPLSi: the log-likelihood increment of EM step %d is NaN", stop[0]);
  out->steps = stop[0] > 0 ? stop[0] : max_steps;
  std::vector<double> hl((size_t)K * lld), hw((size_t)c->ldx), hc((size_t)c->ldy);
  std::vector<PplsRank1> hst((size_t)K);
  HIPCHK(c, hipMemcpy(hl.data(), d.log, sizeof(double) * hl.size(), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(hw.data(), c->W[0], sizeof(double) * hw.size(), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(hc.data(), c->C[0], sizeof(double) * hc.size(), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(hst.data(), d.st, sizeof(PplsRank1) * K, hipMemcpyDeviceToHost));
  if (out->log) std::copy(hl.begin(), hl.end(), out->log);
  std::copy(hw.begin(), hw.begin() + p, out->W);
  std::copy(hc.begin(), hc.begin() + q, out->C);
  for (int j = 0; j < K; ++j) {
    out->params[j] = hst[(size_t)j].B;
    out->params[K + j] = hst[(size_t)j].sigE;
    out->params[2 * K + j] = hst[(size_t)j].sigF;
    out->params[3 * K + j] = hst[(size_t)j].sigH;
    out->params[4 * K + j] = hst[(size_t)j].sigT;
  }
  return PPLS_OK;
}

}  // namespace

extern "C" {

int ppls_meta_emstep(ppls_ctx* c, int npop, const int64_t* pop_local, const int64_t* pop_total, const double* W,
                     const double* C, const double* params_in, double* W_out, double* C_out, double* params_out,
                     double* Cxt, double* Cyu) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (!W || !C || !params_in || !W_out || !C_out || !params_out) return fail(c, PPLS_E_ARG, "NULL argument");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_r(c, 1, 1))) return rc;
  std::vector<MetaPop> pops;
  if ((rc = meta_setup(c, npop, pop_local, pop_total, pops))) return rc;
  std::vector<double> w(W, W + c->p), cv(C, C + c->q);
  for (int j = 0; j < npop; ++j) {
    Rank1& t = pops[j].t;
    t.B = params_in[j];
    t.sigE = params_in[npop + j];
    t.sigF = params_in[2 * npop + j];
    t.sigH = params_in[3 * npop + j];
    t.sigT = params_in[4 * npop + j];
  }
  if ((rc = meta_sweep_all(c, pops, w, cv))) return rc;
  std::vector<double> cx, cy;
  meta_mstep(pops, c->p, c->q, w, cv, Cxt ? &cx : nullptr, Cyu ? &cy : nullptr);
  std::copy(w.begin(), w.end(), W_out);
  std::copy(cv.begin(), cv.end(), C_out);
  meta_params_out(pops, params_out);
  if (Cxt) std::copy(cx.begin(), cx.end(), Cxt);
  if (Cyu) std::copy(cy.begin(), cy.end(), Cyu);
  return PPLS_OK;
}

int ppls_meta_ppls(ppls_ctx* c, int npop, const int64_t* pop_local, const int64_t* pop_total, int max_steps,
                   double atol, int crit_abs, const ppls_theta* init, ppls_meta_fit* out) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (!init || !init->W || !init->C || !init->B || !init->sigT || !out || !out->W || !out->C || !out->params)
    return fail(c, PPLS_E_ARG, "NULL argument");
  if (max_steps < 1) return fail(c, PPLS_E_ARG, "EMsteps must be >= 1");
  int rc;
  if ((rc = check_fit_data(c))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, 1, max_steps))) return rc;
  std::vector<MetaPop> pops;
  if ((rc = meta_setup(c, npop, pop_local, pop_total, pops))) return rc;
  const int p = c->p, q = c->q;
  std::vector<double> w(init->W, init->W + p), cv(init->C, init->C + q);
  Rank1 t0;
  t0.w = w;
  t0.c = cv;
  t0.B = init->B[0];
  t0.sigE = init->sigE;
  t0.sigF = init->sigF;
  t0.sigH = init->sigH;
  t0.sigT = init->sigT[0];
  for (auto& pp : pops) pp.t = t0;   // params = lapply(.., list(B_T = Bnw, sigX = signw[1], ...)) (:545)
  auto crit = [&](double x) { return crit_abs ? std::fabs(x) : x; };
  const size_t ld = (size_t)max_steps + 1;
  if (out->log)
    for (size_t e = 0; e < ld * npop; ++e) out->log[e] = NAN;
  if (meta_device_ok(c, npop)) return meta_ppls_device(c, pops, t0, max_steps, atol, crit_abs, out);
  c->meta_path = 1;
  // logvalue[1, ] = rep(logl_W(X, Y, Wnw, Cnw, Bnw, ...), K) (:544): one full-data sweep
  {
    std::vector<double> SX, SY;
    double G[4];
    if ((rc = rank1_sweep(c, t0, std::vector<double>(), std::vector<double>(), 0, SX, SY, G))) return rc;
    const double l0 = rank1_loglik(t0, G, c->ssq_host[0], c->ssq_host[1], (double)c->n_total, p, q);
    if (out->log)
      for (int j = 0; j < npop; ++j) out->log[(size_t)j * ld] = l0;
    out->steps = 0;
    std::vector<double> prev(npop, l0);
    if ((rc = meta_sweep_all(c, pops, w, cv))) return rc;   // meta_EMstep's E-step of step 1
    int i;
    for (i = 1; i <= max_steps; ++i) {                           // :551
      meta_mstep(pops, p, q, w, cv, nullptr, nullptr);         // fit = meta_EMstep(...) (:555-570)
      if ((rc = meta_sweep_all(c, pops, w, cv))) return rc;   // next E-step; its Gram gives logl_W
      double s_new = 0.0, s_old = 0.0;
      for (int j = 0; j < npop; ++j) {                          // logvalue[i+1, j] (:571-573)
        const double lj = rank1_loglik(pops[j].t, pops[j].G, pops[j].ssq[0], pops[j].ssq[1], pops[j].N, p, q);
        if (out->log) out->log[(size_t)j * ld + i] = lj;
        s_old += prev[j];
        s_new += lj;
        prev[j] = lj;
      }
      out->steps = i;
      if (std::isnan(s_new - s_old))                            // `if (NA < atol)` stops meta_PPLSi (:575)
        return fail(c, PPLS_E_NUMERIC, "meta_PPLSi: the log-likelihood increment of EM step %d is NaN", i);
      if (crit(s_new - s_old) < atol) break;                    // :575-578
    }
  }
  std::copy(w.begin(), w.end(), out->W);
  std::copy(cv.begin(), cv.end(), out->C);
  meta_params_out(pops, out->params);
  return PPLS_OK;
}

// variances.PPLS_simult (EM_W_multi.R:830-860).  X'X (or Y'Y) once on MFMA for all components,
// Cxt = X' mu in one HBM pass, then per component the p x p B_exp - SSt_exp on the device and its
// inverse by rocSOLVER: Cholesky potrf/potri of -(B_exp - SSt_exp), or getrf/getri (R's solve())
// when one is not positive definite.  Data-dependent sums are all-reduced over ranks.
int ppls_variances(ppls_ctx* c, const double* mu, const double* Cdiag, double sigE, int a, int xory, double* W,
                   double* B_exp, double* varMatrix, double* SSt_exp, double* SSt_star, double* seLoad) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if ((!mu && c->n_local > 0) || !Cdiag || !W || !B_exp || !seLoad) return fail(c, PPLS_E_ARG, "NULL argument");
  if (a < 1 || a > 16) return fail(c, PPLS_E_ARG, "number of components %d outside [1, 16]", a);
  if (xory != 0 && xory != 1) return fail(c, PPLS_E_ARG, "XorY must be 0 (\"X\") or 1 (\"Y\")");
  HIPCHK(c, hipSetDevice(c->device));
  const int f32 = c->dtype;
  const int p = xory ? c->q : c->p, ld = xory ? c->ldy : c->ldx;
  const void* D = xory ? (const void*)c->Y : (const void*)c->X;
  const int64_t n = c->n_local;
  const double N = (double)c->n_total;
  if (a > p) return fail(c, PPLS_E_ARG, "more components (%d) than columns (%d)", a, p);
  int rc = PPLS_OK;
  double *dmu = nullptr, *dpart = nullptr, *dS = nullptr, *dG = nullptr, *dM = nullptr, *dv = nullptr, *dMc = nullptr;
  double *dexp = nullptr, *dstar = nullptr, *dse = nullptr;
  rocblas_int *ipiv = nullptr, *info = nullptr;
  hipEvent_t evS = nullptr;
  auto done = [&](int code) {
    if (evS) (void)hipEventDestroy(evS);
    dfree(dmu); dfree(dpart); dfree(dS); dfree(dG); dfree(dM); dfree(dMc); dfree(dv); dfree(dexp); dfree(dstar); dfree(dse);
    if (ipiv) (void)hipFree(ipiv);
    if (info) (void)hipFree(info);
    return code;
  };
#define VCHK(call)                                                                              \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) return done(fail(c, PPLS_E_HIP, "%s: %s", #call, hipGetErrorString(e_))); \
  } while (0)
#define VRC(call)                  \
  do {                             \
    if ((rc = (call))) return done(rc); \
  } while (0)
  const size_t pp = (size_t)p * p;
  // ---- Cxt = D' mu (a x ld, column k contiguous) and ||mu_k||^2 (all-reduced) ----------------
  const int chunks = ppls_xtmu_chunks(std::max<int64_t>(n, 1), ld, f32);
  const int64_t sld = (int64_t)a * ld;
  VRC(dalloc(c, &dS, (size_t)sld + 16));
  std::vector<double> mu2(a, 0.0);
  if (n > 0) {
    VRC(dalloc(c, &dmu, (size_t)n * a));
    VRC(dalloc(c, &dpart, (size_t)chunks * sld + (size_t)ppls_reduce_tmp_len(chunks, sld)));
    VCHK(hipMemcpyAsync(dmu, mu, sizeof(double) * n * a, hipMemcpyHostToDevice, c->stream));
    VCHK(ppls_launch_xtmu(D, f32, n, ld, dmu, a, chunks, dpart, sld, c->stream));
    VCHK(ppls_launch_reduce2(dpart, chunks, sld, sld, dS, dpart + (size_t)chunks * sld, nullptr, c->stream));
    for (int k = 0; k < a; ++k)
      for (int64_t i = 0; i < n; ++i) mu2[k] += mu[(size_t)k * n + i] * mu[(size_t)k * n + i];   // crossprod(mu_T)
    dfree(dpart);
  } else {
    VCHK(hipMemsetAsync(dS, 0, sizeof(double) * sld, c->stream));
  }
  VCHK(hipMemcpyAsync(dS + sld, mu2.data(), sizeof(double) * a, hipMemcpyHostToDevice, c->stream));
  VRC(allreduce(c, dS, (size_t)sld + a));
  std::vector<double> S((size_t)sld + a);
  VCHK(hipMemcpyAsync(S.data(), dS, sizeof(double) * S.size(), hipMemcpyDeviceToHost, c->stream));
  VCHK(hipEventCreateWithFlags(&evS, hipEventDisableTiming));
  VCHK(hipEventRecord(evS, c->stream));   // the host's orth below overlaps the Gram
  // ---- G = D'D on MFMA, split over row ranges, all-reduced -- or, when the cross-product form
  // has formed S = [X Y]'[X Y] for this data (ppls_xprod.hip), its X'X or Y'Y block as it stands
  // (already summed over ranks; symmetric, so its row-major block is the column-major G) ------
  VRC(dalloc(c, &dG, pp));
  if (c->xp_ready) {
    const size_t P = (size_t)c->ldx + c->ldy, off = xory ? (size_t)c->ldx : 0;
    VCHK(hipMemcpy2DAsync(dG, sizeof(double) * p, c->xp_S + off * P + off, sizeof(double) * P, sizeof(double) * p, p,
                          hipMemcpyDeviceToDevice, c->stream));
  } else {
    if (n > 0) {   // (option gram_int8: the int8 CRT form, else / on its fallback the fp64 MFMA Gram)
      VRC(gram_run_s(c, gram_shape(c, false, xory), n, dG, nullptr, nullptr));
    } else {
      VCHK(hipMemsetAsync(dG, 0, sizeof(double) * pp, c->stream));
    }
    VRC(allreduce(c, dG, pp));
  }
  VCHK(hipEventSynchronize(evS));
  std::vector<double> Sp((size_t)p * a);   // t(data) %*% mu (p x a, column-major)
  for (int k = 0; k < a; ++k)
    for (int i = 0; i < p; ++i) Sp[(size_t)k * p + i] = S[(size_t)k * ld + i];
  for (int k = 0; k < a; ++k) mu2[k] = S[(size_t)sld + k];
  // W = orth(t(data) %*% mu, type = "SVD") (:831-832)
  if ((rc = host_orth(Sp.data(), p, a, PPLS_ORTH_SVD, W)))
    return done(fail(c, rc, "orth(t(data) %%*%% mu): rank-deficient"));
  // ---- per component: M = B_exp - SSt_exp, varMatrix = -solve(M), seLoad --------------------
  if (!c->blas) {
    if (rocblas_create_handle(&c->blas) != rocblas_status_success) return done(fail(c, PPLS_E_HIP, "rocblas_create_handle failed"));
  }
  if (rocblas_set_stream(c->blas, c->stream) != rocblas_status_success) return done(fail(c, PPLS_E_HIP, "rocblas_set_stream failed"));
  // all a matrices at once: one strided-batched LU and inverse (rocSOLVER's panel factorisation is
  // thousands of small launches per matrix; batching shares them -- profiles/r3_variances_*.txt)
  VRC(dalloc(c, &dM, pp * (size_t)a));
  VRC(dalloc(c, &dv, (size_t)2 * p));
  VRC(dalloc(c, &dse, (size_t)p));
  if (SSt_exp) VRC(dalloc(c, &dexp, pp));
  if (SSt_star) VRC(dalloc(c, &dstar, pp));
  VCHK(hipMalloc((void**)&ipiv, sizeof(rocblas_int) * p * a));
  VCHK(hipMalloc((void**)&info, sizeof(rocblas_int) * a));
  const double s2 = sigE * sigE, s4 = s2 * s2;
  std::vector<double> v2((size_t)2 * p);
  for (int i = 0; i < a; ++i) {
    const double ctt = N * Cdiag[i];                         // Ctt = N * t(Ctt[i, i]) (:840)
    const double Vt = ctt - mu2[i];                          // Vt = Ctt - crossprod(mu_T) (:842)
    const double k1 = ctt + 2.0 * Vt;
    const double k2 = ctt * ctt + 4.0 * mu2[i] * Vt + 2.0 * Vt * Vt;
    const double bstar = ctt / s2 / N;                       // B_star = c(Ctt)/(sigE^2) * I / nrow(X) (:844)
    B_exp[i] = bstar;
    for (int e = 0; e < p; ++e) {
      v2[e] = Sp[(size_t)i * p + e];                         // Cxt = t(X) %*% mu_T (:843)
      v2[(size_t)p + e] = W[(size_t)i * p + e];
    }
    VCHK(hipMemcpyAsync(dv, v2.data(), sizeof(double) * 2 * p, hipMemcpyHostToDevice, c->stream));
    VCHK(ppls_launch_varmat(dG, dv, dv + p, p, ctt, k1, k2, bstar, s4, N, dM + pp * i, dexp, dstar, c->stream));
    if (SSt_exp) VCHK(hipMemcpyAsync(SSt_exp + (size_t)i * pp, dexp, sizeof(double) * pp, hipMemcpyDeviceToHost, c->stream));
    if (SSt_star) VCHK(hipMemcpyAsync(SSt_star + (size_t)i * pp, dstar, sizeof(double) * pp, hipMemcpyDeviceToHost, c->stream));
    VCHK(hipStreamSynchronize(c->stream));   // dv is reused by the next component
  }
  // varMatrix = -solve(M) = (-M)^-1, and -M = SSt_exp - B_exp is the observed information: symmetric
  // and, at a proper fit, positive definite.  Cholesky potrf + potri (half the flops of LU + inverse)
  // on a copy of -M; if any matrix is not positive definite, the batch takes R's solve() route, LU
  // getrf + getri, from the untouched M.  Either inverse is backward stable: they agree to ~kappa eps.
  std::vector<rocblas_int> inf(a, 0);
  bool chol = c->var_chol != 0;
  int chol_mode = c->var_chol;
  if (chol_mode == 1) {   // the hand-written inverse needs a p^2 scratch per matrix more than rocSOLVER
    const size_t need = sizeof(double) * (pp * (size_t)a + (size_t)ppls_spd_inverse_work(p, a));
    if (hipMalloc((void**)&dMc, need) != hipSuccess) {
      (void)hipGetLastError();   // (clear it) not enough HBM: rocSOLVER's in-place potrf/potri instead
      dMc = nullptr;
      chol_mode = 2;
    }
  }
  if (chol && chol_mode == 1) {
    // hand-written (ppls_linalg.hip): blocked Cholesky of every matrix of the batch in the same
    // launches, then T = L^-1 and T'T -- 3 nb launches (nb = p / 64) where rocSOLVER's potrf + potri
    // took 1,400 (profiles/r4_variances_c3_timeline.txt)
    VCHK(hipMemcpyAsync(dMc, dM, sizeof(double) * pp * a, hipMemcpyDeviceToDevice, c->stream));
    VCHK(ppls_launch_negate(dMc, (int64_t)pp * a, c->stream));
    VCHK(ppls_spd_inverse_batched(dMc, p, a, dMc + pp * (size_t)a, (int*)info, c->stream));
    VCHK(hipMemcpyAsync(inf.data(), info, sizeof(rocblas_int) * a, hipMemcpyDeviceToHost, c->stream));
    VCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < a; ++i) chol = chol && inf[i] == 0;
  } else if (chol) {
    VRC(dalloc(c, &dMc, pp * (size_t)a));
    VCHK(hipMemcpyAsync(dMc, dM, sizeof(double) * pp * a, hipMemcpyDeviceToDevice, c->stream));
    VCHK(ppls_launch_negate(dMc, (int64_t)pp * a, c->stream));
    if (rocsolver_dpotrf_strided_batched(c->blas, rocblas_fill_lower, p, dMc, p, (rocblas_stride)pp, info, a) !=
        rocblas_status_success)
      return done(fail(c, PPLS_E_HIP, "rocsolver potrf (strided batched) failed"));
    VCHK(hipMemcpyAsync(inf.data(), info, sizeof(rocblas_int) * a, hipMemcpyDeviceToHost, c->stream));
    VCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < a; ++i) chol = chol && inf[i] == 0;
    if (chol && rocsolver_dpotri_strided_batched(c->blas, rocblas_fill_lower, p, dMc, p, (rocblas_stride)pp, info, a) !=
                    rocblas_status_success)
      return done(fail(c, PPLS_E_HIP, "rocsolver potri (strided batched) failed"));
  }
  if (!chol) {
    if (rocsolver_dgetrf_strided_batched(c->blas, p, p, dM, p, (rocblas_stride)pp, ipiv, p, info, a) !=
            rocblas_status_success ||
        rocsolver_dgetri_strided_batched(c->blas, p, dM, p, (rocblas_stride)pp, ipiv, p, info, a) !=
            rocblas_status_success)
      return done(fail(c, PPLS_E_HIP, "rocsolver getrf/getri (strided batched) failed"));
  }
  VCHK(hipMemcpyAsync(inf.data(), info, sizeof(rocblas_int) * a, hipMemcpyDeviceToHost, c->stream));
  VCHK(hipStreamSynchronize(c->stream));
  for (int i = 0; i < a; ++i)
    if (inf[i] != 0)   // solve(): "Lapack routine dgesv: system is exactly singular"
      return done(fail(c, PPLS_E_NUMERIC, "component %d: B_exp - SSt_exp is exactly singular (U[%d,%d] = 0)", i + 1,
                       (int)inf[i], (int)inf[i]));
  if (chol) std::swap(dM, dMc);   // the inverse to copy out
  for (int i = 0; i < a; ++i) {
    if (chol) VCHK(ppls_launch_symdiag(dM + pp * i, p, dse, c->stream));
    else VCHK(ppls_launch_negdiag(dM + pp * i, p, dse, c->stream));
    if (varMatrix) VCHK(hipMemcpyAsync(varMatrix + (size_t)i * pp, dM + pp * i, sizeof(double) * pp, hipMemcpyDeviceToHost, c->stream));
    VCHK(hipMemcpyAsync(seLoad + (size_t)i * p, dse, sizeof(double) * p, hipMemcpyDeviceToHost, c->stream));
    VCHK(hipStreamSynchronize(c->stream));   // dse is reused by the next component
  }
  VCHK(hipStreamSynchronize(c->stream));
#undef VCHK
#undef VRC
  return done(PPLS_OK);
}

// Diagnostics / tests: the batched SPD inverse of variances.PPLS_simult on host matrices.
int ppls_spd_inverse(ppls_ctx* c, const double* A, int p, int a, int method, double* out, int* info, double* ms) {
  if (!c || !A || !out || !info || p < 1 || a < 1 || (method != 1 && method != 2)) return PPLS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t pp = (size_t)p * p;
  double *dA = nullptr, *dse = nullptr;
  int* dinfo = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int rc = PPLS_OK;
  auto done = [&](int code) {
    dfree(dA); dfree(dse);
    if (dinfo) (void)hipFree(dinfo);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return code;
  };
  const size_t work = method == 1 ? (size_t)ppls_spd_inverse_work(p, a) : 0;
  if ((rc = dalloc(c, &dA, pp * a + work)) || (rc = dalloc(c, &dse, (size_t)p))) return done(rc);
  if (hipMalloc((void**)&dinfo, sizeof(int) * 2 * a) != hipSuccess) return done(fail(c, PPLS_E_HIP, "hipMalloc failed"));
  if (hipMemcpy(dA, A, sizeof(double) * pp * a, hipMemcpyHostToDevice) != hipSuccess ||
      hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    return done(fail(c, PPLS_E_HIP, "spd_inverse: setup failed"));
  if (method == 2) {
    if (!c->blas && rocblas_create_handle(&c->blas) != rocblas_status_success)
      return done(fail(c, PPLS_E_HIP, "rocblas_create_handle failed"));
    if (rocblas_set_stream(c->blas, c->stream) != rocblas_status_success)
      return done(fail(c, PPLS_E_HIP, "rocblas_set_stream failed"));
  }
  (void)hipEventRecord(e0, c->stream);
  if (method == 1) {
    if (ppls_spd_inverse_batched(dA, p, a, dA + pp * a, dinfo, c->stream) != hipSuccess)
      return done(fail(c, PPLS_E_HIP, "spd_inverse: launch failed"));
  } else if (rocsolver_dpotrf_strided_batched(c->blas, rocblas_fill_lower, p, dA, p, (rocblas_stride)pp, dinfo, a) !=
                 rocblas_status_success ||
             rocsolver_dpotri_strided_batched(c->blas, rocblas_fill_lower, p, dA, p, (rocblas_stride)pp, dinfo + a, a) !=
                 rocblas_status_success) {   // (info: potrf's)
    return done(fail(c, PPLS_E_HIP, "rocsolver potrf/potri failed"));
  }
  (void)hipEventRecord(e1, c->stream);
  for (int z = 0; z < a; ++z)
    if (ppls_launch_symdiag(dA + pp * z, p, dse, c->stream) != hipSuccess)
      return done(fail(c, PPLS_E_HIP, "spd_inverse: symdiag failed"));
  if (hipStreamSynchronize(c->stream) != hipSuccess ||   // (the context stream does not block with stream 0)
      hipMemcpy(out, dA, sizeof(double) * pp * a, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(info, dinfo, sizeof(int) * a, hipMemcpyDeviceToHost) != hipSuccess)
    return done(fail(c, PPLS_E_HIP, "spd_inverse: copy-out failed"));
  float t = 0.f;
  (void)hipEventElapsedTime(&t, e0, e1);
  if (ms) *ms = t;
  return done(PPLS_OK);
}

// Diagnostics / benchmark: G = D'D (D = X for xory 0, Y for 1) on the MFMA Gram kernel only, with
// nsplit equal row splits (0 = the automatic halving splits, as in ppls_variances); G (p x p,
// column-major) may be NULL.
// *ms receives the Gram kernel's duration (HIP events on the context stream).
int ppls_gram(ppls_ctx* c, int xory, int nsplit, double* G, double* ms) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (xory < 0 || xory > 2) return fail(c, PPLS_E_ARG, "xory must be 0 (X'X), 1 (Y'Y) or 2 ([X Y]'[X Y])");
  HIPCHK(c, hipSetDevice(c->device));
  const GramShape g = xory == 2 ? gram_shape(c, true, 0) : gram_shape(c, false, xory);
  const size_t pp = (size_t)g.p * g.p;
  if (c->n_local <= 0) return fail(c, PPLS_E_STATE, "no rows on this rank");
  int rc;
  double* dG = nullptr;
  if ((rc = dalloc(c, &dG, pp))) return rc;
  float t = 0.f;
  rc = gram_run(c, g, c->n_local, nsplit > 0 ? nsplit : 0, dG, &t);
  if (!rc && G) {
    if (xory < 2) {
      if (hipMemcpy(G, dG, sizeof(double) * pp, hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail(c, PPLS_E_HIP, "gram: copy-out failed");
    } else {   // the joint Gram without the row padding between X's and Y's columns: (p + q)^2
      std::vector<double> full(pp);
      if (hipMemcpy(full.data(), dG, sizeof(double) * pp, hipMemcpyDeviceToHost) != hipSuccess) {
        rc = fail(c, PPLS_E_HIP, "gram: copy-out failed");
      } else {
        const int P = c->p + c->q;
        auto src = [&](int k) { return k < c->p ? k : c->ldx + (k - c->p); };
        for (int b = 0; b < P; ++b)
          for (int a = 0; a < P; ++a) G[(size_t)b * P + a] = full[(size_t)src(b) * g.p + src(a)];
      }
    }
  }
  dfree(dG);
  if (!rc && ms) *ms = t;
  return rc;
}

// scores.PPLS (EM_W_multi.R:411-420): T = X W, U = Y C (local rows, column-major n_local x k) in
// one pass -- the panel dots kernel with mu coefficients (1, 0; 0, 1), whose mu write-out is then
// exactly [X W | Y C].
int ppls_scores(ppls_ctx* c, const double* W, const double* C, int k, double* T, double* U) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (!W || !C || k < 1 || k > PPLS_RMAX) return fail(c, PPLS_E_ARG, "W, C must be given with 1 <= k <= %d", PPLS_RMAX);
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  if ((rc = ensure_r(c, k, 1))) return rc;
  std::vector<double> B(k, 1.0), sT(k, 1.0);
  ppls_theta th = {const_cast<double*>(W), const_cast<double*>(C), B.data(), sT.data(), 1.0, 1.0, 1.0};
  if ((rc = upload_theta(c, &th, k, 0))) return rc;
  PplsScalars s;
  memset(&s, 0, sizeof s);
  for (int j = 0; j < k; ++j) { s.alpha[j] = 1.0; s.delta[j] = 1.0; }
  HIPCHK(c, hipMemcpyAsync(c->sc[0], &s, sizeof s, hipMemcpyHostToDevice, c->stream));
  if (c->z_cols < 4 * k) {
    dfree(c->Z);
    c->z_cols = 0;
    if ((rc = dalloc(c, &c->Z, (size_t)ppls_panel_z_len(c->n_local, c->ldx, c->ldy, k)))) return rc;
    c->z_cols = 4 * k;
  }
  dfree(c->mu);
  if ((rc = dalloc(c, &c->mu, (size_t)std::max<int64_t>(c->n_local, 1) * 2 * k))) return rc;
  PplsSweepArgs a;
  memset(&a, 0, sizeof a);
  a.X = c->X; a.Y = c->Y; a.n_local = c->n_local; a.p = c->p; a.q = c->q; a.ldx = c->ldx; a.ldy = c->ldy;
  a.Wp = c->W[0]; a.Cp = c->C[0]; a.sc = c->sc[0]; a.mu = c->mu; a.write_mu = 1; a.r = k;
  a.num_cus = c->num_cus; a.dots_rows = c->dots_rows; a.dots_pair = c->dots_pair;
  HIPCHK(c, ppls_launch_panel_dots(&a, c->dtype, c->Z, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const size_t blk = sizeof(double) * (size_t)c->n_local * k;
  if (c->n_local > 0 && T) HIPCHK(c, hipMemcpy(T, c->mu, blk, hipMemcpyDeviceToHost));
  if (c->n_local > 0 && U) HIPCHK(c, hipMemcpy(U, c->mu + (size_t)c->n_local * k, blk, hipMemcpyDeviceToHost));
  dfree(c->mu);   // sized for this k; the EM path re-allocates its own
  return PPLS_OK;
}

int ppls_em_begin(ppls_ctx* c, const ppls_theta* th, int r) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, th, r))) return rc;
  if ((rc = check_fit_data(c))) return rc;
  if (!theta_finite(th, c->p, c->q, r)) return fail(c, PPLS_E_ARG, "theta0 has non-finite entries");
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, 1 << 16))) return rc;
  std::vector<double> W(th->W, th->W + (size_t)c->p * r), C(th->C, th->C + (size_t)c->q * r);
  std::vector<double> B(th->B, th->B + r), T(th->sigT, th->sigT + r);
  ppls_theta t0 = {W.data(), C.data(), B.data(), T.data(), th->sigE, th->sigF, th->sigH};
  canonicalize(&t0, c->p, c->q, r);
  if ((rc = upload_theta(c, &t0, r, 0))) return rc;
  HIPCHK(c, hipMemsetAsync(c->status, 0, sizeof(int), c->stream));
  c->em_r = r;
  c->em_cur = 0;
  c->em_iter = 0;
  if ((rc = xprod_begin(c, 1 << 16, r))) return rc;
  c->em_active = true;
  return PPLS_OK;
}

int ppls_em_iterate(ppls_ctx* c, int nsteps, int type) {
  if (!c) return PPLS_E_ARG;
  if (!c->em_active || c->r_alloc != c->em_r) return fail(c, PPLS_E_STATE, "call ppls_em_begin first");
  if (nsteps < 0) return fail(c, PPLS_E_ARG, "nsteps < 0");
  if (c->em_iter + nsteps + 2 > c->loglik_cap) return fail(c, PPLS_E_ARG, "too many iterations for one run");
  HIPCHK(c, hipSetDevice(c->device));
  int rc;
  for (int s = 0; s < nsteps; ++s) {
    const int nxt = c->em_cur ^ 1;
    if ((rc = stats_step(c, c->em_r, c->em_cur, false, true))) return rc;
    if ((rc = finalize(c, c->em_r, c->em_cur, nxt, c->em_iter >= 1 ? c->em_iter - 1 : -1, type))) return rc;
    c->em_cur = nxt;
    ++c->em_iter;
  }
  return PPLS_OK;
}

int ppls_em_state(ppls_ctx* c, ppls_theta* out, double* loglik, int cap, int* n_loglik) {
  if (!c) return PPLS_E_ARG;
  if (!c->em_active) return fail(c, PPLS_E_STATE, "call ppls_em_begin first");
  int rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if ((rc = check_status(c))) return rc;
  if (out && (rc = download_theta(c, c->em_r, c->em_cur, out))) return rc;
  const int n = c->em_iter >= 1 ? c->em_iter - 1 : 0;
  if (n_loglik) *n_loglik = n;
  std::vector<double> l((size_t)n);
  if (n > 0) HIPCHK(c, hipMemcpy(l.data(), c->loglik, sizeof(double) * n, hipMemcpyDeviceToHost));
  if (loglik && n > 0) std::copy(l.begin(), l.begin() + std::min(n, cap), loglik);
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(l[i]))
      return fail(c, PPLS_E_NUMERIC, "non-finite log-likelihood %g at EM iteration %d", l[i], i + 1);
  if (out && !theta_finite(out, c->p, c->q, c->em_r))
    return fail(c, PPLS_E_NUMERIC, "non-finite estimates after %d EM iterations", c->em_iter);
  return PPLS_OK;
}

int ppls_synchronize(ppls_ctx* c) {
  if (!c) return PPLS_E_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PPLS_OK;
}

int ppls_loglC_fast(ppls_ctx* c, const double* W, const double* C, const double* X, const double* Y, int64_t n,
                    int p, int q, int a, double sigX, double sigY, const double* sig2T, const double* c1,
                    const double* c2, const double* c3, const double* Kc, double* out) {
  if (!c || !W || !C || !sig2T || !c1 || !c2 || !c3 || !Kc || !out) return c ? fail(c, PPLS_E_ARG, "NULL argument") : PPLS_E_ARG;
  if (a < 1 || a > PPLS_RMAX) return fail(c, PPLS_E_ARG, "a=%d outside [1,%d]", a, PPLS_RMAX);
  int rc;
  if (X || Y) {
    if (!X || !Y) return fail(c, PPLS_E_ARG, "X and Y must both be given or both be NULL");
    if ((rc = ppls_set_data(c, X, Y, n, p, q, PPLS_LAYOUT_COLMAJOR, n))) return rc;
  } else if (!c->have_data || c->p != p || c->q != q) {
    return fail(c, PPLS_E_STATE, "no resident data of shape p=%d q=%d", p, q);
  }
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, a, 1))) return rc;
  std::vector<double> B(a, 0.0), T(a, 1.0);
  ppls_theta th = {const_cast<double*>(W), const_cast<double*>(C), B.data(), T.data(), sigX, sigY, 0.0};
  if ((rc = upload_theta(c, &th, a, 0))) return rc;
  if ((rc = sweep(c, a, 0, false))) return rc;
  std::vector<double> cf(5 * (size_t)a);
  for (int k = 0; k < a; ++k) {
    cf[k] = sig2T[k]; cf[a + k] = c1[k]; cf[2 * a + k] = c2[k]; cf[3 * a + k] = c3[k]; cf[4 * a + k] = Kc[k];
  }
  HIPCHK(c, hipMemcpyAsync(c->coefs, cf.data(), sizeof(double) * cf.size(), hipMemcpyHostToDevice, c->stream));
  const double* G = c->stats + (int64_t)a * c->ldx + (int64_t)a * c->ldy;
  HIPCHK(c, ppls_launch_loglc(G, c->ssq, (double)c->n_total, p, q, a, sigX, sigY, c->coefs, c->loglik, c->stream));
  HIPCHK(c, hipMemcpyAsync(out, c->loglik, sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return PPLS_OK;
}

int ppls_xprod_prepare(ppls_ctx* c, double* ms, double* total_ms) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  HIPCHK(c, hipSetDevice(c->device));
  const bool was = c->xp_ready;
  int rc;
  if ((rc = xprod_setup(c))) return rc;
  c->xp_explicit = true;
  if (ms) *ms = was ? 0.0 : c->xp_setup_ms;
  if (total_ms) *total_ms = was ? 0.0 : c->xp_setup_total_ms;
  return PPLS_OK;
}

int ppls_xprod_release(ppls_ctx* c) {
  if (!c) return PPLS_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  xprod_free(c);
  return PPLS_OK;
}

int ppls_xprod_setup_times(ppls_ctx* c, double* gram_ms, double* allreduce_ms, double* total_ms) {
  if (!c) return PPLS_E_ARG;
  if (gram_ms) *gram_ms = c->xp_setup_ms;
  if (allreduce_ms) *allreduce_ms = c->xp_setup_ar_ms;
  if (total_ms) *total_ms = c->xp_setup_total_ms;
  return PPLS_OK;
}

int ppls_xprod_tile_timing(ppls_ctx* c, int reps, double* ms) {
  if (!c || reps < 1 || !ms) return PPLS_E_ARG;
  if (!c->em_active || c->r_alloc != c->em_r) return fail(c, PPLS_E_STATE, "call ppls_em_begin first");
  if (!c->xp_ready || !c->xp_M) return fail(c, PPLS_E_STATE, "the cross-products S are not formed");
  HIPCHK(c, hipSetDevice(c->device));
  const int r = c->em_r, slot = c->em_cur, P = c->ldx + c->ldy;
  const int rw = ppls_xprod_tile_rows(P, r, c->xprod_rw, c->num_cus);
  hipEvent_t e0, e1;
  HIPCHK(c, hipEventCreate(&e0));
  HIPCHK(c, hipEventCreate(&e1));
  hipError_t e = hipEventRecord(e0, c->stream);
  for (int i = 0; e == hipSuccess && i < reps; ++i)   // the statistics of the current theta, rewritten
    e = ppls_launch_xprod_tile(c->xp_S, c->ldx, c->ldy, r, rw, c->W[slot], c->C[slot], c->sc[slot], c->stats,
                               c->xp_M, nullptr, 0, c->stream);
  if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
  if (e == hipSuccess) e = hipEventSynchronize(e1);
  float t = 0.f;
  if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  HIPCHK(c, e);
  *ms = (double)t / reps;
  return PPLS_OK;
}

int ppls_xprod_info(ppls_ctx* c, int r, int* ready, int64_t* bytes_per_pass, double* flops, int* rows_per_wave) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  const int64_t P = (int64_t)c->ldx + c->ldy;
  if (ready) *ready = c->xp_ready ? 1 : 0;
  if (bytes_per_pass) *bytes_per_pass = 8 * P * P;   // S's bytes one iteration reads
  if (flops) {   // lower 128 x 128 tiles incl. the diagonal ones, 2 flops per multiply-add
    const double nb = (double)((P + 127) / 128);
    flops[0] = 2.0 * (double)c->n_local * nb * (nb + 1) / 2.0 * 128.0 * 128.0;
  }
  if (rows_per_wave) *rows_per_wave = ppls_xprod_tile_rows((int)P, r < 1 ? 1 : r, c->xprod_rw, c->num_cus);
  return PPLS_OK;
}

int ppls_xprod_stats(ppls_ctx* c, const ppls_theta* th, int r, double* stats) {
  if (!c || !stats) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  int rc;
  if ((rc = check_theta(c, th, r))) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  if ((rc = ensure_r(c, r, 1))) return rc;
  if ((rc = upload_theta(c, th, r, 0))) return rc;
  if ((rc = xprod_stats(c, r, 0))) return rc;
  std::vector<double> st((size_t)c->part_ld);
  HIPCHK(c, hipMemcpyAsync(st.data(), c->stats, sizeof(double) * st.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < r; ++k) {
    for (int i = 0; i < c->p; ++i) stats[(size_t)k * c->p + i] = st[(size_t)k * c->ldx + i];
    for (int i = 0; i < c->q; ++i)
      stats[(size_t)r * c->p + (size_t)k * c->q + i] = st[(size_t)r * c->ldx + (size_t)k * c->ldy + i];
  }
  for (int e = 0; e < 4 * r * r; ++e)
    stats[(size_t)r * (c->p + c->q) + e] = st[(size_t)r * (c->ldx + c->ldy) + e];
  return PPLS_OK;
}

int ppls_sweep_timing(ppls_ctx* c, double* total_ms, int64_t* launches, int reset) {
  if (!c) return PPLS_E_ARG;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < c->ev_used; ++i) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev[i].first, c->ev[i].second));
    c->timed_ms += ms;
    ++c->timed_launches;
  }
  c->ev_used = 0;
  if (total_ms) *total_ms = c->timed_ms;
  if (launches) *launches = c->timed_launches;
  if (reset) { c->timed_ms = 0.0; c->timed_launches = 0; }
  return PPLS_OK;
}

int ppls_sweep_balance(ppls_ctx* c, double* w8, int64_t* bounds, int cap, int* n_bounds) {
  if (!c) return PPLS_E_ARG;
  if (w8)
    for (int x = 0; x < 8; ++x) w8[x] = c->bal_done ? c->bal_w[x] : 1.0;
  const int nb = c->bal_done ? c->bal_grid + 1 : 0;
  if (n_bounds) *n_bounds = nb;
  if (bounds && cap > 0 && nb > 0)
    HIPCHK(c, hipMemcpy(bounds, c->bal_bounds, sizeof(int64_t) * (size_t)std::min(cap, nb), hipMemcpyDeviceToHost));
  return PPLS_OK;
}

int ppls_comm_info(ppls_ctx* c, int* nranks, int* rank, double* allreduce_ms, int64_t* allreduce_calls,
                   int reset) {
  if (!c) return PPLS_E_ARG;
  int nr = c->nranks, rk = c->rank;
  if (c->comm) {   // what RCCL itself reports for the communicator
    RCCLCHK(c, ncclCommCount(c->comm, &nr));
    RCCLCHK(c, ncclCommUserRank(c->comm, &rk));
  }
  if (nranks) *nranks = nr;
  if (rank) *rank = rk;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < c->ev_ar_used; ++i) {
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_ar[i].first, c->ev_ar[i].second));
    c->ar_ms += ms;
    ++c->ar_calls;
  }
  c->ev_ar_used = 0;
  if (allreduce_ms) *allreduce_ms = c->ar_ms;
  if (allreduce_calls) *allreduce_calls = c->ar_calls;
  if (reset) { c->ar_ms = 0.0; c->ar_calls = 0; }
  return PPLS_OK;
}

int ppls_sweep_info(ppls_ctx* c, int r, int64_t* bytes_per_sweep, int* variant, int* grid) {
  if (!c) return PPLS_E_ARG;
  PplsSweepArgs a;
  const int plan = sweep_plan(c, r, &a);
  if (bytes_per_sweep) *bytes_per_sweep = (int64_t)(c->dtype ? 4 : 8) * c->n_local * ((int64_t)c->p + c->q);
  if (variant) *variant = plan == 4 ? 5 : plan == 3 ? 4 : 2;
  if (grid) *grid = a.grid;
  return PPLS_OK;
}

int ppls_gram_int8(ppls_ctx* c, int which, double* G, int* nmod, int* L, double* ms) {
  if (!c) return PPLS_E_ARG;
  if (!c->have_data) return fail(c, PPLS_E_STATE, "no data");
  if (which < 0 || which > 2) return fail(c, PPLS_E_ARG, "which must be 0 (X), 1 (Y) or 2 (joint [X Y])");
  if (c->n_local <= 0) return fail(c, PPLS_E_STATE, "no rows on this rank");
  HIPCHK(c, hipSetDevice(c->device));
  const GramShape g = which == 2 ? gram_shape(c, true, 0) : gram_shape(c, false, which);
  const size_t pp = (size_t)g.p * g.p;
  int rc;
  double* dG = nullptr;
  if ((rc = dalloc(c, &dG, pp))) return rc;
  float t = 0.f;
  rc = gram_run_oz(c, g, c->n_local, dG, &t);
  if (nmod) *nmod = c->oz_nmod;
  if (L) *L = c->oz_L;
  if (rc == 1) rc = fail(c, PPLS_E_NUMERIC, "int8 Gram: the column spread needs L = %d bits or more than %d moduli, "
                         "or the residue planes do not fit", c->oz_L, PPLS_OZ_MAXMOD);
  if (!rc && G && hipMemcpy(G, dG, sizeof(double) * pp, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(c, PPLS_E_HIP, "int8 gram: copy-out failed");
  dfree(dG);
  if (!rc && ms) for (int k = 0; k < 4; ++k) ms[k] = c->oz_ms[k];
  return rc;
}

int ppls_gram_shifts(ppls_ctx* c, int* shift, int P, int* count) {
  if (!c) return PPLS_E_ARG;
  const int k = (int)c->oz_shift.size();
  if (count) *count = k;
  if (shift) for (int j = 0; j < std::min(P, k); ++j) shift[j] = c->oz_shift[(size_t)j];
  return PPLS_OK;
}

int ppls_gram_info(ppls_ctx* c, int* int8_used, int* nmod, int* L, double* ms) {
  if (!c) return PPLS_E_ARG;
  if (int8_used) *int8_used = c->oz_used;
  if (nmod) *nmod = c->oz_nmod;
  if (L) *L = c->oz_L;
  if (ms) for (int k = 0; k < 4; ++k) ms[k] = c->oz_ms[k];
  return PPLS_OK;
}

int ppls_meta_info(ppls_ctx* c, int* path) {
  if (!c || !path) return PPLS_E_ARG;
  *path = c->meta_path;
  return PPLS_OK;
}

int ppls_sweep_kernel(ppls_ctx* c, int r, char* buf, int len) {
  if (!c || !buf || len < 1) return PPLS_E_ARG;
  if (r < 1 || r > PPLS_RMAX) return fail(c, PPLS_E_ARG, "bad r");
  PplsSweepArgs a;
  const int plan = sweep_plan(c, r, &a);
  const int nt = c->nt_loads > 0 ||
                 (c->nt_loads < 0 && 8.0 * sweep_rows(c) * (double)(c->ldx + c->ldy) > 256.0 * (1 << 20));
  char k[128];
  if (plan == 3) {
    if (ppls_split_describe(&a, k, sizeof k) != 0) return fail(c, PPLS_E_STATE, "no split instantiation for r=%d", r);
  } else {
    // as ppls_kernels.hip launch_panel_t picks them
    const bool rows64 = c->dots_rows ? c->dots_rows == 64 : sweep_rows(c) >= 32768;
    const int64_t wtiles = (sweep_rows(c) + (rows64 ? 63 : 31)) / (rows64 ? 64 : 32);
    const bool pair = c->dots_pair >= 0 ? c->dots_pair == 1 : wtiles < (int64_t)c->num_cus * 4 * (rows64 ? 2 : 3);
    snprintf(k, sizeof k, "panel<%s,%d> (mfmadots %d rows/%s + acc, %d chunks)", c->dtype ? "float" : "double", r,
             rows64 ? 64 : 32, pair ? "wave pair" : "wave", a.grid);
  }
  snprintf(buf, (size_t)len, "%s%s", k, plan == 3 && nt ? " nt" : "");
  return PPLS_OK;
}

int ppls_finalize_trace(ppls_ctx* c, int64_t* stamps, double* tick_ns) {
  if (!c || !stamps) return PPLS_E_ARG;
  if (!c->ftrace) return fail(c, PPLS_E_STATE, "finalize tracing is off (set_option ftrace 1)");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(stamps, c->ftrace, PPLS_FTRACE_LEN * sizeof(long long), hipMemcpyDeviceToHost));
  if (tick_ns) {
    int khz = 0;
    HIPCHK(c, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    *tick_ns = khz > 0 ? 1e6 / khz : 0.0;
  }
  return PPLS_OK;
}

int ppls_sweep_trace(ppls_ctx* c, int64_t* stamps, int cap, int* n, double* tick_ns) {
  if (!c || !stamps || !n) return PPLS_E_ARG;
  if (!c->strace) return fail(c, PPLS_E_STATE, "sweep tracing is off (set_option strace 1)");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int m = std::min(cap, PPLS_STRACE_MAX_WG);
  HIPCHK(c, hipMemcpy(stamps, c->strace, (size_t)m * 4 * sizeof(long long), hipMemcpyDeviceToHost));
  *n = m;
  if (tick_ns) {
    int khz = 0;
    HIPCHK(c, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    *tick_ns = khz > 0 ? 1e6 / khz : 0.0;
  }
  return PPLS_OK;
}

int ppls_mu_coefficients(const ppls_theta* th, int r, double* coef) {
  if (!th || !th->B || !th->sigT || !coef || r < 1 || r > PPLS_RMAX) return PPLS_E_ARG;
  PplsScalars s = scalars_of(th, r);
  for (int k = 0; k < r; ++k) {
    coef[k] = s.alpha[k]; coef[r + k] = s.beta[k]; coef[2 * r + k] = s.gamma[k]; coef[3 * r + k] = s.delta[k];
  }
  return PPLS_OK;
}

int ppls_finalize_host(const double* SX, const double* SY, const double* G, double ssqX, double ssqY, double N,
                       int p, int q, int r, const ppls_theta* th, int type, ppls_theta* next,
                       ppls_expect* mom_out, double* loglik) {
  if (!G || !th || !th->W || !th->C || !th->B || !th->sigT || r < 1 || r > PPLS_RMAX || p < 1 || q < 1)
    return PPLS_E_ARG;
  PplsScalars s = scalars_of(th, r);
  double WtW[PPLS_RMAX * PPLS_RMAX], CtC[PPLS_RMAX * PPLS_RMAX];
  for (int a = 0; a < r; ++a)
    for (int b = 0; b < r; ++b) {
      double w = 0.0, cc = 0.0;
      for (int i = 0; i < p; ++i) w += th->W[(size_t)a * p + i] * th->W[(size_t)b * p + i];
      for (int i = 0; i < q; ++i) cc += th->C[(size_t)a * q + i] * th->C[(size_t)b * q + i];
      WtW[b * r + a] = w;
      CtC[b * r + a] = cc;
    }
  if (loglik) *loglik = ppls_loglik_from_gram(G, ssqX, ssqY, N, p, q, r, &s);
  PplsMoments m;
  ppls_estep_moments(G, WtW, CtC, ssqX, ssqY, N, p, q, r, &s, &m);
  if (mom_out) {
    for (int k = 0; k < r; ++k) {
      if (mom_out->Ctt) mom_out->Ctt[k] = m.Ctt[k];
      if (mom_out->Cuu) mom_out->Cuu[k] = m.Cuu[k];
      if (mom_out->Cut) mom_out->Cut[k] = m.Cut[k];
    }
    mom_out->Cee = m.Cee;
    mom_out->Cff = m.Cff;
    if (mom_out->Chh) memcpy(mom_out->Chh, m.Chh, sizeof(double) * r * r);
  }
  if (next) {
    PplsScalars nx = s;
    ppls_mstep_scalars(&m, r, &nx);
    if (next->B) for (int k = 0; k < r; ++k) next->B[k] = nx.b[k];
    if (next->sigT) for (int k = 0; k < r; ++k) next->sigT[k] = nx.t[k];
    next->sigE = nx.sigE;
    next->sigF = nx.sigF;
    next->sigH = nx.sigH;
    if (next->W && SX && host_orth(SX, p, r, type, next->W) != PPLS_OK) return PPLS_E_NUMERIC;
    if (next->C && SY && host_orth(SY, q, r, type, next->C) != PPLS_OK) return PPLS_E_NUMERIC;
  }
  return PPLS_OK;
}

}  // extern "C"
