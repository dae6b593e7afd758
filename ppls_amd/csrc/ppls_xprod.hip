// ppls_xprod.hip -- the cross-product form of one PPLS_simult EM iteration (ppls_xprod.h).
//
// The reference reads X and Y about ten times per iteration; the streaming sweep
// (ppls_kernels.hip) reads them once.  Every statistic of the iteration is a quadratic form in the
// joint cross-product S = [X Y]'[X Y] (P x P, P = ldx + ldy; formed once per data set on MFMA by
// ppls_gram_mfma_kernel), so an iteration here reads S instead: 8 P^2 bytes against
// esz n (p + q) -- 128 MB against 32 GB at C3, and 128 MB fits the 256 MiB Infinity Cache.
//
//   ppls_xprod_tile_kernel   M = S B (B = blockdiag(W, C)) by row groups of S walking 128-column
//                            tiles, B staged in LDS per tile, and from it X'mu_T (:732), Y'mu_U
//                            (:733) rows: HBM/MALL-bound, one pass over S
//   ppls_xprod_gram_kernel   Gram([Xw Yc]) = B'M (:696-712, loglC.cpp:335), one workgroup per
//                            upper-triangle entry, mirrored (exactly symmetric, as the sweep's), when
//                            the finalize does not form it itself (r > 8 or p + q > 6144)
// Row i of M needs row i of S only (S is symmetric, so rows and columns are interchangeable).
// Measured and removed: a row-group form without LDS (W, C re-read from L1/L2 per
// row group: 350 vs 210 us at C5), a lower-triangle form (half the bytes, but latency-bound tiles
// plus a partial reduction: not faster at C3 or C5), and a two-stream pipeline running the pass over
// S of iteration i beside its finalize (cross-queue waits and a 2r-wide pass: slower at C3 and C5).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_device.h"
#include "ppls_xprod.h"

#ifndef PPLS_XP_DEPTH
#define PPLS_XP_DEPTH 1   // staged tiles of S in flight per wave (1: loaded right before use; round 3: 2, 3, 4, 6
                          // equal within 1 %; round 4, with two sub-tiles per barrier at r <= 5: 1 is fastest --
                          // C3 tile 22.9 -> 21.7 us, C5 202 -> 200 us; profiles/r4_xprod_depth_ab_*.txt)
#endif
#ifndef PPLS_XP_WAVES
#define PPLS_XP_WAVES 0   // waves per tile-kernel workgroup sharing each staged B tile (0: ppls_xp_waves)
#endif
#ifndef PPLS_XP_TPB
#define PPLS_XP_TPB 0     // 128-column sub-tiles per staged B tile and workgroup barrier (0: ppls_xp_tpb)
#endif

namespace {

// Sub-tiles per staged B tile (one workgroup barrier each): 2 for r <= 5 (C3: tile 23.5 -> 22.9 us),
// else 1 (C5, r = 10: 2 is 6 % slower, 4 is slower at C3; profiles/r4_xprod_tpb_ab.txt).
constexpr int ppls_xp_tpb(int r) { return PPLS_XP_TPB > 0 ? PPLS_XP_TPB : (r <= 5 ? 2 : 1); }
// Waves per workgroup: 8 for r <= 5 (C3 tile 21.7 -> 21.5 us), else 4 (C5: 8 is 1-3 % slower, 2 is
// 25 % slower everywhere; profiles/r4_xprod_waves8_depth1_ab.txt, r4_xprod_waves2_ab.txt).
constexpr int ppls_xp_waves(int r) { return PPLS_XP_WAVES > 0 ? PPLS_XP_WAVES : (r <= 5 ? 8 : 4); }

// Values a lane holds after ppls_rs's six butterfly levels on M values (M > 64: several).
constexpr int ppls_rs_left(int m, int l) { return l == 6 ? m : (m == 1 ? 1 : ppls_rs_left((m + 1) / 2, l + 1)); }

// Row-tile form: a workgroup owns 4 RW rows of S (RW per wave) and walks the columns
// in tiles of 128 -- first the X columns, then the Y columns.  Each tile's 128 x R values of B (W on
// X columns, C on Y columns) are staged in LDS once per workgroup and read by all its rows, so W and
// C cost ~R / (4 RW) of S's traffic from L2.  S tiles are loaded into a register ring
// PPLS_XP_DEPTH - 1 staged tiles ahead of their use (default: none -- the 16 resident waves per CU
// keep enough bytes in flight, and fewer live registers measured faster), B one tile ahead through
// LDS; one barrier per staged tile of ppls_xp_tpb(R) 128-column sub-tiles.
template <int R, int RW, bool NT>
__device__ __forceinline__ void ppls_xprod_tile_phase(const double* const (&srow)[RW], const double* __restrict__ Bsrc,
                                                      int ldb, int width, int soff, double (&acc)[RW * R + 1],
                                                      double* __restrict__ sB, int lane) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  constexpr int TP = ppls_xp_tpb(R);         // 128-column sub-tiles per staged tile (one barrier each)
  constexpr int TV = TP * R * 64;            // 16-B values of B per staged tile
  constexpr int NTH = 64 * ppls_xp_waves(R);
  constexpr int NB = (TV + NTH - 1) / NTH;   // 16-B B loads per thread and tile
  constexpr int D = PPLS_XP_DEPTH;           // S tiles in flight per wave (register ring)
  const int tid = threadIdx.x;
  const int ntile = (width + 128 * TP - 1) / (128 * TP);
  if (ntile == 0) return;
  d2v bn[NB], ring[D][RW][TP];
  auto ld_s = [&](int n, d2v (&dst)[RW][TP]) {   // tile n: S values of this lane's two columns per sub-tile
#pragma unroll
    for (int sp = 0; sp < TP; ++sp) {
      const int c = (n * TP + sp) * 128 + 2 * lane;
#pragma unroll
      for (int rr = 0; rr < RW; ++rr) {
        if (c < width) {
          if constexpr (NT) dst[rr][sp] = __builtin_nontemporal_load((const d2v*)(srow[rr] + soff + c));
          else dst[rr][sp] = *(const d2v*)(srow[rr] + soff + c);
        } else {
          dst[rr][sp] = d2v{0.0, 0.0};
        }
      }
    }
  };
  auto ld_b = [&](int n) {   // tile n: this thread's share of the TP x 128 x R values of B
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int e = tid + NTH * v, sp = e / (R * 64), f = e - sp * R * 64, t = f >> 6;
      const int cb = (n * TP + sp) * 128 + 2 * (f & 63);
      bn[v] = (e < TV && cb < width) ? *(const d2v*)(Bsrc + (int64_t)t * ldb + cb) : d2v{0.0, 0.0};
    }
  };
  auto st_b = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int e = tid + NTH * v;
      if (e < TV) ((d2v*)sB)[buf * TV + e] = bn[v];
    }
  };
#pragma unroll
  for (int u = 0; u < D - 1; ++u)
    if (u < ntile) ld_s(u, ring[u]);
  ld_b(0);
  st_b(0);
  __syncthreads();
  for (int n0 = 0; n0 < ntile; n0 += D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int n = n0 + u;
      if (n >= ntile) break;
      // B of the next tile first: the wait for it before st_b (vmcnt counts in issue order) then
      // leaves the S loads issued after it in flight
      if (n + 1 < ntile) ld_b(n + 1);
      if (n + D - 1 < ntile) ld_s(n + D - 1, ring[(u + D - 1) % D]);
#pragma unroll
      for (int sp = 0; sp < TP; ++sp) {   // sub-tiles in column order: the sums equal TP = 1's
        const d2v* b = (const d2v*)sB + (n & 1) * TV + sp * R * 64 + lane;
#pragma unroll
        for (int t = 0; t < R; ++t) {
          const d2v bv = b[t * 64];
#pragma unroll
          for (int rr = 0; rr < RW; ++rr)
            acc[rr * R + t] = fma(ring[u][rr][sp].y, bv.y, fma(ring[u][rr][sp].x, bv.x, acc[rr * R + t]));
        }
      }
      if (n + 1 < ntile) st_b((n + 1) & 1);
      __syncthreads();
    }
  }
}

// The products a wave's RW rows of S give against B = blockdiag(Bx, By) (RB columns each; Bx
// lives on the X columns of S with leading dimension ldbx, By on the Y columns): on return
// smw[rr * 2 RB + b] = S[i0 + rr, X] Bx[:, b] and smw[rr * 2 RB + RB + b] = S[i0 + rr, Y] By[:, b]
// (this wave's slice of LDS; the caller synchronises before reading it).
template <int RB, int RW, bool NT>
__device__ __forceinline__ void ppls_xprod_rows(const double* __restrict__ S, int ldx, int ldy,
                                                const double* __restrict__ Bx, int ldbx,
                                                const double* __restrict__ By, int ldby, int64_t i0,
                                                double* __restrict__ sB, double* __restrict__ smw, int lane) {
  constexpr int NV = RW * RB, R2 = 2 * RB;
  constexpr int LEFT = ppls_rs_left(NV, 0);
  const int P = ldx + ldy;
  const double* srow[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) srow[rr] = S + (i0 + rr < P ? i0 + rr : (int64_t)P - 1) * P;   // rows past P: dropped
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {   // X columns with Bx, then Y columns with By
    double acc[NV + 1];
#pragma unroll
    for (int v = 0; v <= NV; ++v) acc[v] = 0.0;
    if (ph == 0) ppls_xprod_tile_phase<RB, RW, NT>(srow, Bx, ldbx, ldx, 0, acc, sB, lane);
    else ppls_xprod_tile_phase<RB, RW, NT>(srow, By, ldby, ldy, ldx, acc, sB, lane);
    int idx = 0, nreal = 0;
    bool canon = true;
    ppls_rs<NV, 0, NV + 1>(acc, lane, idx, canon, nreal);
    if (canon) {
#pragma unroll
      for (int j = 0; j < LEFT; ++j)
        if (j < nreal && idx + j < NV) {
          const int rr = (idx + j) / RB, t = idx + j - rr * RB;
          smw[rr * R2 + ph * RB + t] = acc[j];
        }
    }
  }
}

// M = S blockdiag(W, C) for a wave's RW rows, then X'mu_T / Y'mu_U of those rows (the statistics
// step of an iteration from S: EM_W_multi.R:691-694, :732-733).
template <int R, int RW, bool NT>
__device__ __forceinline__ void ppls_xprod_tile_body(const double* __restrict__ S, int ldx, int ldy,
                                                     const double* __restrict__ Wp, const double* __restrict__ Cp,
                                                     const PplsScalars* __restrict__ sc, double* __restrict__ stats,
                                                     double* __restrict__ M, double* __restrict__ sB,
                                                     double* __restrict__ smw, int64_t i0, int lane) {
  constexpr int R2 = 2 * R;
  const int P = ldx + ldy;
  ppls_xprod_rows<R, RW, NT>(S, ldx, ldy, Wp, ldx, Cp, ldy, i0, sB, smw, lane);
  __syncthreads();
  for (int e = lane; e < RW * R2; e += 64) {
    const int rr = e / R2, b = e - rr * R2;
    if (i0 + rr < P) M[(int64_t)b * P + i0 + rr] = smw[e];
  }
  for (int e = lane; e < RW * R; e += 64) {
    const int rr = e / R, t = e - rr * R;
    const int64_t i = i0 + rr;
    if (i >= P) continue;
    const double mw = smw[rr * R2 + t], mc = smw[rr * R2 + R + t];
    if (i < ldx) stats[(int64_t)t * ldx + i] = sc->alpha[t] * mw + sc->beta[t] * mc;   // X'mu_T
    else stats[(int64_t)R * ldx + (int64_t)t * ldy + (i - ldx)] = sc->gamma[t] * mw + sc->delta[t] * mc;   // Y'mu_U
  }
}

template <int R, int RW, bool NT>
__global__ __launch_bounds__(64 * ppls_xp_waves(R)) void ppls_xprod_tile_kernel(const double* __restrict__ S, int ldx, int ldy,
                                                              const double* __restrict__ Wp,
                                                              const double* __restrict__ Cp,
                                                              const PplsScalars* __restrict__ sc,
                                                              double* __restrict__ stats, double* __restrict__ M,
                                                              const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged at an earlier iteration
  __shared__ double sB[2 * R * 128 * ppls_xp_tpb(R)];
  __shared__ double sm[ppls_xp_waves(R)][RW * 2 * R];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = ((int64_t)blockIdx.x * ppls_xp_waves(R) + wave) * RW;   // this wave's first row of S
  ppls_xprod_tile_body<R, RW, NT>(S, ldx, ldy, Wp, Cp, sc, stats, M, sB, sm[wave], i0, lane);
}

// Gram entry (a, b), a <= b, of B'M: sum over the rows where column a of B lives (X rows for
// a < R, Y rows otherwise); written to (a, b) and (b, a).
__global__ __launch_bounds__(256) void ppls_xprod_gram_kernel(int ldx, int ldy, int R, const double* __restrict__ Wp,
                                                              const double* __restrict__ Cp,
                                                              const double* __restrict__ M,
                                                              double* __restrict__ stats,
                                                              const int* __restrict__ stop) {
  if (stop && *stop) return;
  __shared__ double red[4];
  const int R2 = 2 * R, P = ldx + ldy;
  const int t = blockIdx.x;
  int b = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((b + 1) * (b + 2) / 2 <= t) ++b;
  while (b * (b + 1) / 2 > t) --b;
  const int a = t - b * (b + 1) / 2;
  const double* Bcol = a < R ? Wp + (int64_t)a * ldx : Cp + (int64_t)(a - R) * ldy;
  const double* Mcol = M + (int64_t)b * P + (a < R ? 0 : ldx);
  const int rows = a < R ? ldx : ldy;
  // four independent partial sums per thread (loads of four rows in flight), added in fixed order
  double v4[4] = {0.0, 0.0, 0.0, 0.0};
  int i = threadIdx.x;
  for (; i + 3 * 256 < rows; i += 4 * 256) {
#pragma unroll
    for (int u = 0; u < 4; ++u) v4[u] = fma(Bcol[i + u * 256], Mcol[i + u * 256], v4[u]);
  }
  for (; i < rows; i += 256) v4[0] = fma(Bcol[i], Mcol[i], v4[0]);
  double v = (v4[0] + v4[1]) + (v4[2] + v4[3]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double g = (red[0] + red[1]) + (red[2] + red[3]);
    double* G = stats + (int64_t)R * ldx + (int64_t)R * ldy;
    G[(int64_t)b * R2 + a] = g;
    G[(int64_t)a * R2 + b] = g;
  }
}

template <int R, int RW>
hipError_t launch_tile(const double* S, int ldx, int ldy, const double* Wp, const double* Cp, const PplsScalars* sc,
                       double* stats, double* M, const int* stop, hipStream_t st) {
  const int P = ldx + ldy;
  constexpr int NWV = ppls_xp_waves(R);
  const unsigned blocks = (unsigned)((P + NWV * RW - 1) / (NWV * RW));
  if (8.0 * P * (double)P > 200.0 * (1 << 20))   // S beyond the Infinity Cache: non-temporal loads
    hipLaunchKernelGGL((ppls_xprod_tile_kernel<R, RW, true>), dim3(blocks), dim3(64 * NWV), 0, st, S, ldx, ldy, Wp, Cp, sc,
                       stats, M, stop);
  else
    hipLaunchKernelGGL((ppls_xprod_tile_kernel<R, RW, false>), dim3(blocks), dim3(64 * NWV), 0, st, S, ldx, ldy, Wp, Cp,
                       sc, stats, M, stop);
  return hipGetLastError();
}

template <int R>
hipError_t launch_tile_rw(int rw, const double* S, int ldx, int ldy, const double* Wp, const double* Cp,
                          const PplsScalars* sc, double* stats, double* M, const int* stop, hipStream_t st) {
  if (rw == 1) return launch_tile<R, 1>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  if (rw == 2) return launch_tile<R, 2>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  if (rw == 4) return launch_tile<R, 4>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);   // one phase's RW r accumulators live
  if constexpr (R <= 8)
    if (rw == 8) return launch_tile<R, 8>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

int ppls_xprod_tile_rows(int P, int r, int rw_opt, int num_cus) {
  if (rw_opt == 1 || rw_opt == 2 || rw_opt == 4 || (rw_opt == 8 && r <= 8)) return rw_opt;
  return P / 8 >= 2 * num_cus ? 2 : 1;   // two rows per wave while >= 2 workgroups per CU remain
}

hipError_t ppls_launch_xprod_tile(const double* S, int ldx, int ldy, int r, int rw, const double* Wp,
                                  const double* Cp, const PplsScalars* sc, double* stats, double* M, const int* stop,
                                  int with_gram, hipStream_t st) {
  if (ldx < 2 || ldy < 2 || (ldx & 1) || (ldy & 1) || r < 1 || r > PPLS_RMAX) return hipErrorInvalidValue;
  if (((uintptr_t)S | (uintptr_t)Wp | (uintptr_t)Cp) & 15) return hipErrorInvalidValue;   // 16-B loads
  hipError_t e;
  switch (r) {
#define PPLS_XP_CASE(k) \
    case k: e = launch_tile_rw<k>(rw, S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st); break;
    PPLS_XP_CASE(1) PPLS_XP_CASE(2) PPLS_XP_CASE(3) PPLS_XP_CASE(4) PPLS_XP_CASE(5) PPLS_XP_CASE(6)
    PPLS_XP_CASE(7) PPLS_XP_CASE(8) PPLS_XP_CASE(9) PPLS_XP_CASE(10) PPLS_XP_CASE(11) PPLS_XP_CASE(12)
    PPLS_XP_CASE(13) PPLS_XP_CASE(14) PPLS_XP_CASE(15) PPLS_XP_CASE(16)
#undef PPLS_XP_CASE
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  if (!with_gram) return hipSuccess;   // the finalize's scalar block forms B'M (PplsFinalizeArgs::xpM)
  const int R2 = 2 * r;
  hipLaunchKernelGGL(ppls_xprod_gram_kernel, dim3((unsigned)(R2 * (R2 + 1) / 2)), dim3(256), 0, st, ldx, ldy, r, Wp,
                     Cp, M, stats, stop);
  return hipGetLastError();
}

}  // extern "C"
