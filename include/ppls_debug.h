/* ppls_debug.h -- measurement and diagnostic entry points of libppls_amd.so.
 *
 * Not part of the reference's interface (include/ppls.h is the drop-in boundary): these exist for
 * bench.py's roofline and collective timings, for the parity tests that pin a production kernel by
 * name or check one statistics step in isolation, and for the tools/ trace scripts.  The same
 * library exports them; nothing on the EM path calls them.
 */
#ifndef PPLS_AMD_PPLS_DEBUG_H
#define PPLS_AMD_PPLS_DEBUG_H

#include "ppls.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Sum of HIP-event durations of the statistics launches (sweep, or the cross-product tile kernel)
 * recorded since the last reset (option "timing" = N brackets every N-th launch). */
int ppls_sweep_timing(ppls_ctx* ctx, double* total_ms, int64_t* launches, int reset);
/* The split sweep's calibrated row partition (option "balance"): the per-XCD-class weights w8[8]
 * (1.0 before calibration) and up to cap of the grid + 1 row boundaries (*n_bounds = grid + 1, or 0
 * while the even split is used). */
int ppls_sweep_balance(ppls_ctx* ctx, double* w8, int64_t* bounds, int cap, int* n_bounds);
/* The communicator as RCCL reports it (ncclCommCount / ncclCommUserRank; without RCCL the
 * context's own nranks/rank, i.e. 1/0 or the host reducer's) and the summed HIP-event durations of
 * the per-iteration statistics all-reduce on the timed sweeps (option "timing"; RCCL only). */
int ppls_comm_info(ppls_ctx* ctx, int* nranks, int* rank, double* allreduce_ms, int64_t* allreduce_calls,
                   int reset);
/* Cross-product form: *ready = S is formed for the current data, *bytes_per_pass = the bytes of S
 * one iteration reads (8 P^2, P = padded p + q), *flops = 2 n_local x the lower 128 x 128 tiles of
 * P^2 as the Gram computes them, *rows_per_wave = rows of S per wave of the tile kernel. */
int ppls_xprod_info(ppls_ctx* ctx, int r, int* ready, int64_t* bytes_per_pass, double* flops, int* rows_per_wave);
/* The last formation of S: the MFMA Gram (HIP events), the all-reduce of S over ranks (wall clock
 * around the collective and its stream synchronisation; 0 on one rank) and the whole setup. */
int ppls_xprod_setup_times(ppls_ctx* ctx, double* gram_ms, double* allreduce_ms, double* total_ms);
/* The cross-product tile kernel alone, reps launches back to back between two HIP events, for the
 * current theta of an ppls_em_begin session (S formed): *ms = the average per launch.  Rewrites the
 * session's statistics buffer with that theta's (the next ppls_em_iterate recomputes it anyway). */
int ppls_xprod_tile_timing(ppls_ctx* ctx, int reps, double* ms);
/* One statistics step from S for theta: stats = [X'mu_T p x r | Y'mu_U q x r | Gram 2r x 2r], all
 * column-major, as ppls_finalize_host takes them (unit parity against the sweep and a host S B). */
int ppls_xprod_stats(ppls_ctx* ctx, const ppls_theta* th, int r, double* stats);
/* Shape facts for the roofline: bytes of X and Y one sweep reads (algorithmic), kernel variant. */
int ppls_sweep_info(ppls_ctx* ctx, int r, int64_t* bytes_per_sweep, int* variant, int* grid);
/* The sweep kernel instantiation the next EM iteration with r components launches, as text
 * (e.g. "split<5,4,512,2,false,4,4> nt"): tests assert the production kernel is the one checked. */
int ppls_sweep_kernel(ppls_ctx* ctx, int r, char* buf, int len);
/* The Gram by the int8-MFMA Chinese-remainder form (ppls_ozaki.hip) alone, for tests and
 * benchmarks: which = 0 X'X, 1 Y'Y, 2 the joint [X Y]'[X Y] (P = ldx + ldy, padding columns 0);
 * G (column-major, nullable); *nmod moduli, *L bits of the widest column's integers; ms[4] = stats +
 * residues, SYRK, CRT, total (HIP events).  PPLS_E_NUMERIC when the columns' spread is too wide. */
int ppls_gram_int8(ppls_ctx* ctx, int which, double* G, int* nmod, int* L, double* ms);
/* The per-column scalings of the last int8 Gram (x'_kj = rint(D_kj 2^shift[j]); 0 for empty and
 * padding columns): the first min(P, *count) of them, *count = its column count. */
int ppls_gram_shifts(ppls_ctx* ctx, int* shift, int P, int* count);
/* Host copies of the int8 Gram's arithmetic (no GPU needed; tests/test_ozaki_host.py): the symmetric
 * residue of x' = rint(x 2^shift) modulo the l-th modulus (|x'| < 2^62), the l-th modulus, and the
 * CRT of nmod residues (0 <= r_l < m_l) to the nearest double of the integer in (-M/2, M/2). */
int ppls_oz_residue_host(double x, int shift, int l, int* r);
int ppls_oz_crt_host(const int* r, int nmod, double* out);
int ppls_oz_modulus(int l);
/* Which Gram ran last -- forming S, or ppls_variances' X'X / Y'Y (1 int8 CRT form, 0 fp64 MFMA) -- its
 * moduli, bits and phases (ms[4]). */
int ppls_gram_info(ppls_ctx* ctx, int* int8_used, int* nmod, int* L, double* ms);
/* The path the last ppls_meta_ppls took: 0 none yet, 1 the host loop, 2 the device loop on the split
 * sweep (one segmented launch per EM step), 3 the device loop on the panel sweep (one launch per
 * population and step). */
int ppls_meta_info(ppls_ctx* ctx, int* path);
/* The Gram D'D alone (D = X for xory 0, Y for 1, the joint [X Y] for 2; nsplit 0 = auto; this rank's
 * rows), for tests, benchmarks and the 'o2m' starting values of the Python PPLS / PPLSi /
 * meta_PPLSi: G (p x p, q x q or (p + q) x (p + q) without padding columns, column-major,
 * nullable), *ms = the MFMA kernel's duration. */
int ppls_gram(ppls_ctx* ctx, int xory, int nsplit, double* G, double* ms);
/* Inverse of a batch of symmetric positive definite matrices (host A: a x p x p, column-major, stride
 * p^2) as variances.PPLS_simult inverts the observed information: method 1 the hand-written blocked
 * Cholesky + inverse (ppls_linalg.hip), 2 rocSOLVER potrf + potri.  out: the full symmetric inverses;
 * info[z] = 0, or the 1-based column of the first non-positive pivot of matrix z (then out[z] is
 * not meaningful); *ms = device time of the factorisation and inverse. */
int ppls_spd_inverse(ppls_ctx* ctx, const double* A, int p, int a, int method, double* out, int* info, double* ms);
/* The generator's Philox4x32-10 block function on the device, for known-answer checks: out[4i..4i+3]
 * = philox4x32_10(ctr[4i..4i+3], key = {key & 0xffffffff, key >> 32}), i < count (host arrays).
 * The generator uses ctr = {pair lo, pair hi, stream, 0}, key = seed. */
int ppls_philox4x32_10(ppls_ctx* ctx, const uint32_t* ctr, int64_t count, uint64_t key, uint32_t* out);

/* Wall-clock stamps of the last finalize's phases (PPLS_FTRACE_LEN = 3 blocks x 16 slots; 0 = slot
 * not reached) and the tick length in ns.  Requires set_option("ftrace", 1). */
#define PPLS_FTRACE_LEN 48
int ppls_finalize_trace(ppls_ctx* ctx, int64_t* stamps, double* tick_ns);
/* Wall-clock stamps of the last split sweep per workgroup (entry, ring prologue done, row loop done,
 * partials written; 4 per workgroup, row-major), up to PPLS_STRACE_MAX_WG workgroups; *n =
 * workgroups copied.  Requires set_option("strace", 1). */
#define PPLS_STRACE_MAX_WG 4096
int ppls_sweep_trace(ppls_ctx* ctx, int64_t* stamps, int cap, int* n, double* tick_ns);

#ifdef __cplusplus
}
#endif
#endif /* PPLS_AMD_PPLS_DEBUG_H */
