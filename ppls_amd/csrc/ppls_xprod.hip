// ppls_xprod.hip -- the cross-product form of one PPLS_simult EM iteration (ppls_xprod.h).
//
// The reference reads X and Y about ten times per iteration; the streaming sweep
// (ppls_kernels.hip) reads them once.  Every statistic of the iteration is a quadratic form in the
// joint cross-product S = [X Y]'[X Y] (P x P, P = ldx + ldy; formed once per data set on MFMA by
// ppls_gram_mfma_kernel), so an iteration here reads S instead: 8 P^2 bytes against
// esz n (p + q) -- 128 MB against 32 GB at C3, and 128 MB fits the 256 MiB Infinity Cache.
//
//   ppls_xprod_tile_kernel   M = S B (B = blockdiag(W, C)) by row groups of S walking 128-column
//                            tiles, B staged in LDS per tile (default), and from it X'mu_T (:732),
//                            Y'mu_U (:733) rows: HBM/MALL-bound, one pass over S
//   ppls_xprod_apply_kernel  the same without LDS (option xprod_kernel = 1; W, C re-read per row
//                            group from L1/L2: that traffic bounds it at wide p and large r)
//   ppls_xprod_gram_kernel   Gram([Xw Yc]) = B'M (:696-712, loglC.cpp:335), one workgroup per
//                            upper-triangle entry, mirrored (exactly symmetric, as the sweep's)
// Row i of M needs row i of S only (S is symmetric, so rows and columns are interchangeable); W and
// C are re-read from L1/L2 by every workgroup, RW rows of S share each load of them.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_device.h"
#include "ppls_xprod.h"

#ifndef PPLS_XP_DEPTH
#define PPLS_XP_DEPTH 2   // 128-column tiles of S in flight per wave in the row-tile kernel (2, 3, 4, 6: same within 1 %, 6 slower at r = 10)
#endif

namespace {

// Values a lane holds after ppls_rs's six butterfly levels on M values (M > 64: several).
constexpr int ppls_rs_left(int m, int l) { return l == 6 ? m : (m == 1 ? 1 : ppls_rs_left((m + 1) / 2, l + 1)); }

template <int R, int RW, bool NT>
__global__ __launch_bounds__(256) void ppls_xprod_apply_kernel(const double* __restrict__ S, int ldx, int ldy,
                                                               const double* __restrict__ Wp,
                                                               const double* __restrict__ Cp,
                                                               const PplsScalars* __restrict__ sc,
                                                               double* __restrict__ stats, double* __restrict__ M,
                                                               const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged at an earlier iteration
  constexpr int R2 = 2 * R, NV = RW * R2;
  __shared__ double sm[4][NV];
  const int P = ldx + ldy;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the workgroup's RW rows of S; its four waves take interleaved 128-column steps of each row
  const int64_t i0 = (int64_t)blockIdx.x * RW;
  const double* srow[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) srow[rr] = S + (i0 + rr < P ? i0 + rr : (int64_t)P - 1) * P;   // rows past P: dropped
  double acc[NV + 1];
#pragma unroll
  for (int v = 0; v <= NV; ++v) acc[v] = 0.0;
  typedef double d2v __attribute__((ext_vector_type(2)));
  auto lds2 = [](const double* a) -> d2v {
    if constexpr (NT) return __builtin_nontemporal_load((const d2v*)a);
    else return *(const d2v*)a;
  };
  const int j0 = 2 * lane + 128 * wave;
  // X columns: M[i, k] += S[i, j] W[j, k], two columns j per lane and step (16-B loads)
#pragma unroll 2
  for (int j = j0; j < ldx; j += 512) {
    d2v s[RW];
#pragma unroll
    for (int rr = 0; rr < RW; ++rr) s[rr] = lds2(srow[rr] + j);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const d2v w = *(const d2v*)(Wp + (int64_t)k * ldx + j);
#pragma unroll
      for (int rr = 0; rr < RW; ++rr) acc[rr * R2 + k] = fma(s[rr].y, w.y, fma(s[rr].x, w.x, acc[rr * R2 + k]));
    }
  }
  // Y columns: M[i, R + k] += S[i, ldx + j] C[j, k]
#pragma unroll 2
  for (int j = j0; j < ldy; j += 512) {
    d2v s[RW];
#pragma unroll
    for (int rr = 0; rr < RW; ++rr) s[rr] = lds2(srow[rr] + ldx + j);
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const d2v cv = *(const d2v*)(Cp + (int64_t)k * ldy + j);
#pragma unroll
      for (int rr = 0; rr < RW; ++rr)
        acc[rr * R2 + R + k] = fma(s[rr].y, cv.y, fma(s[rr].x, cv.x, acc[rr * R2 + R + k]));
    }
  }
  // wave sums (reduce-scatter: lane ends with value(s) idx..), then the four waves in order
  int idx = 0;
  bool canon = true;
  ppls_rs<NV, 0, NV + 1>(acc, lane, idx, canon);
  constexpr int LEFT = ppls_rs_left(NV, 0);
  if (canon) {
#pragma unroll
    for (int j = 0; j < LEFT; ++j)
      if (idx + j < NV) sm[wave][idx + j] = acc[j];
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int e = threadIdx.x;
    const double v = (sm[0][e] + sm[1][e]) + (sm[2][e] + sm[3][e]);
    const int rr = e / R2, b = e - rr * R2;
    if (i0 + rr < P) M[(int64_t)b * P + i0 + rr] = v;
    sm[0][e] = v;
  }
  __syncthreads();
  if (threadIdx.x < RW * R) {
    const int e = threadIdx.x;
    const int rr = e / R, k = e - rr * R;
    const int64_t i = i0 + rr;
    if (i < P) {
      const double mw = sm[0][rr * R2 + k], mc = sm[0][rr * R2 + R + k];
      if (i < ldx) stats[(int64_t)k * ldx + i] = sc->alpha[k] * mw + sc->beta[k] * mc;   // X'mu_T
      else stats[(int64_t)R * ldx + (int64_t)k * ldy + (i - ldx)] = sc->gamma[k] * mw + sc->delta[k] * mc;   // Y'mu_U
    }
  }
}

// Row-tile form (the default): a workgroup owns 4 RW rows of S (RW per wave) and walks the columns
// in tiles of 128 -- first the X columns, then the Y columns.  Each tile's 128 x R values of B (W on
// X columns, C on Y columns) are staged in LDS once per workgroup and read by all its rows, so W and
// C cost ~R / (4 RW) of S's traffic from L2 (the row-group kernel above re-reads them per RW rows
// from L1/L2: R / RW, which bounds it at wide p and large r).  S tiles stream through a register
// ring PPLS_XP_DEPTH tiles ahead (enough bytes in flight per CU to cover HBM/MALL latency: one
// 128-column tile is only 1 KB per wave and row), B one tile ahead through LDS; one barrier per tile.
template <int R, int RW, bool NT>
__device__ __forceinline__ void ppls_xprod_tile_phase(const double* const (&srow)[RW], const double* __restrict__ Bsrc,
                                                      int ldb, int width, int soff, double (&acc)[RW * R + 1],
                                                      double* __restrict__ sB, int lane) {
  typedef double d2v __attribute__((ext_vector_type(2)));
  constexpr int NB = (R * 64 + 255) / 256;   // 16-B B loads per thread and tile
  constexpr int D = PPLS_XP_DEPTH;           // S tiles in flight per wave (register ring)
  const int tid = threadIdx.x;
  const int ntile = (width + 127) >> 7;
  if (ntile == 0) return;
  d2v bn[NB], ring[D][RW];
  auto ld_s = [&](int n, d2v (&dst)[RW]) {   // tile n: S values of this lane's two columns
    const int c = (n << 7) + 2 * lane;
#pragma unroll
    for (int rr = 0; rr < RW; ++rr) {
      if (c < width) {
        if constexpr (NT) dst[rr] = __builtin_nontemporal_load((const d2v*)(srow[rr] + soff + c));
        else dst[rr] = *(const d2v*)(srow[rr] + soff + c);
      } else {
        dst[rr] = d2v{0.0, 0.0};
      }
    }
  };
  auto ld_b = [&](int n) {   // tile n: this thread's share of the 128 x R values of B
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int e = tid + 256 * v, t = e >> 6, cb = (n << 7) + 2 * (e & 63);
      bn[v] = (e < R * 64 && cb < width) ? *(const d2v*)(Bsrc + (int64_t)t * ldb + cb) : d2v{0.0, 0.0};
    }
  };
  auto st_b = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NB; ++v) {
      const int e = tid + 256 * v;
      if (e < R * 64) ((d2v*)sB)[buf * R * 64 + e] = bn[v];
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
      const d2v* b = (const d2v*)sB + (n & 1) * R * 64 + lane;
#pragma unroll
      for (int t = 0; t < R; ++t) {
        const d2v bv = b[t * 64];
#pragma unroll
        for (int rr = 0; rr < RW; ++rr)
          acc[rr * R + t] = fma(ring[u][rr].y, bv.y, fma(ring[u][rr].x, bv.x, acc[rr * R + t]));
      }
      if (n + 1 < ntile) st_b((n + 1) & 1);
      __syncthreads();
    }
  }
}

template <int R, int RW, bool NT>
__global__ __launch_bounds__(256) void ppls_xprod_tile_kernel(const double* __restrict__ S, int ldx, int ldy,
                                                              const double* __restrict__ Wp,
                                                              const double* __restrict__ Cp,
                                                              const PplsScalars* __restrict__ sc,
                                                              double* __restrict__ stats, double* __restrict__ M,
                                                              const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged at an earlier iteration
  constexpr int R2 = 2 * R, NV = RW * R;
  __shared__ double sB[2 * R * 128];
  __shared__ double sm[4][RW * R2];
  const int P = ldx + ldy;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + wave) * RW;   // this wave's first row of S
  const double* srow[RW];
#pragma unroll
  for (int rr = 0; rr < RW; ++rr) srow[rr] = S + (i0 + rr < P ? i0 + rr : (int64_t)P - 1) * P;   // rows past P: dropped
  constexpr int LEFT = ppls_rs_left(NV, 0);
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {   // X columns with W, then Y columns with C
    double acc[NV + 1];
#pragma unroll
    for (int v = 0; v <= NV; ++v) acc[v] = 0.0;
    if (ph == 0) ppls_xprod_tile_phase<R, RW, NT>(srow, Wp, ldx, ldx, 0, acc, sB, lane);
    else ppls_xprod_tile_phase<R, RW, NT>(srow, Cp, ldy, ldy, ldx, acc, sB, lane);
    int idx = 0;
    bool canon = true;
    ppls_rs<NV, 0, NV + 1>(acc, lane, idx, canon);
    if (canon) {
#pragma unroll
      for (int j = 0; j < LEFT; ++j)
        if (idx + j < NV) {
          const int rr = (idx + j) / R, t = idx + j - rr * R;
          sm[wave][rr * R2 + ph * R + t] = acc[j];
        }
    }
  }
  __syncthreads();
  for (int e = lane; e < RW * R2; e += 64) {
    const int rr = e / R2, b = e - rr * R2;
    if (i0 + rr < P) M[(int64_t)b * P + i0 + rr] = sm[wave][e];
  }
  for (int e = lane; e < RW * R; e += 64) {
    const int rr = e / R, t = e - rr * R;
    const int64_t i = i0 + rr;
    if (i >= P) continue;
    const double mw = sm[wave][rr * R2 + t], mc = sm[wave][rr * R2 + R + t];
    if (i < ldx) stats[(int64_t)t * ldx + i] = sc->alpha[t] * mw + sc->beta[t] * mc;   // X'mu_T
    else stats[(int64_t)R * ldx + (int64_t)t * ldy + (i - ldx)] = sc->gamma[t] * mw + sc->delta[t] * mc;   // Y'mu_U
  }
}

// Lower-triangle form (the default for r <= PPLS_XP_TRI_RMAX): S is symmetric, so each
// off-diagonal 128 x 128 tile S_IJ (J < I) is read once and used twice -- its rows give M[I] +=
// S_IJ B_J, its columns give M[J] += S_IJ' B_I -- halving the bytes per iteration.  The blocks
// I, J of the joint index space are aligned to the X/Y seam (X columns in 128-steps from 0, Y
// columns from ldx), so a tile's B rows are all W or all C.  A workgroup takes a run of tiles
// (I, J0..J1-1) of one block row: its four waves own 32 rows each, a lane two columns.
//   column contribution: per lane, cc[k] (two columns) += S[i, j] B_I[i, k], B_I rows broadcast
//     from LDS; summed over the four waves in LDS and written per tile (colpart);
//   row contribution: per lane and row, the partial S[i, j..j+1] . B_J[j..j+1, k] of its two columns,
//     G rows x r values at a time summed over the wave by a DPP reduce-scatter, accumulated over
//     the run's tiles in registers and written per run (rowpart).
// ppls_xprod_tri_reduce_kernel then sums, per row of M, its run partials and the column partials of
// the tiles below it in a fixed order (deterministic), and writes M, X'mu_T and Y'mu_U.
struct XpBlk {
  int start, len, type;   // first row / column, width (<= 128), 0 = X block (B rows of W), 1 = Y (C)
};
__device__ __forceinline__ XpBlk ppls_xp_blk(int b, int bx, int ldx, int ldy) {
  if (b < bx) {
    const int st = b << 7;
    return XpBlk{st, min(128, ldx - st), 0};
  }
  const int st = (b - bx) << 7;
  return XpBlk{ldx + st, min(128, ldy - st), 1};
}

template <int R, bool NT>
__global__ __launch_bounds__(256) void ppls_xprod_tri_kernel(const double* __restrict__ S, int ldx, int ldy,
                                                             const double* __restrict__ Wp,
                                                             const double* __restrict__ Cp,
                                                             const int4* __restrict__ items,
                                                             double* __restrict__ rowpart,
                                                             double* __restrict__ colpart,
                                                             const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged at an earlier iteration
  typedef double d2v __attribute__((ext_vector_type(2)));
  constexpr int G = 32 / R > 0 ? 32 / R : 1;   // rows per reduce-scatter batch (G r <= 32 values)
  constexpr int NVB = G * R;
  constexpr int NBATCH = (32 + G - 1) / G;     // batches over a wave's 32 rows
  __shared__ double sBI[128 * R];               // B rows of block I, [row][k]
  __shared__ double red[R * 128];               // column contributions, [k][column]
  const int P = ldx + ldy, bx = (ldx + 127) >> 7;
  const int4 it = items[blockIdx.x];
  const int I = it.x, J0 = it.y, J1 = it.z;
  const XpBlk bI = ppls_xp_blk(I, bx, ldx, ldy);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int e = tid; e < 128 * R; e += 256) {
    const int row = e / R, k = e - row * R;
    sBI[e] = row < bI.len ? (bI.type ? Cp[(int64_t)k * ldy + (bI.start - ldx) + row] : Wp[(int64_t)k * ldx + bI.start + row])
                          : 0.0;
  }
  __syncthreads();
  const int r0 = 32 * wave, rlim = bI.len - r0;   // this wave's rows r0 + rr, rr < min(32, rlim)
  const int c = 2 * lane;
  double racc[2][NBATCH];
#pragma unroll
  for (int b = 0; b < NBATCH; ++b) racc[0][b] = racc[1][b] = 0.0;
  int idx = 0;
  bool canon = true;
  for (int J = J0; J < J1; ++J) {
    const XpBlk bJ = ppls_xp_blk(J, bx, ldx, ldy);
    const bool off = J != I, cl = c < bJ.len;
    const double* bsrc = bJ.type ? Cp + (bJ.start - ldx) + c : Wp + bJ.start + c;
    const int ldb = bJ.type ? ldy : ldx;
    d2v bj[R], cc[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      bj[k] = cl ? *(const d2v*)(bsrc + (int64_t)k * ldb) : d2v{0.0, 0.0};
      cc[k] = d2v{0.0, 0.0};
    }
    const double* sb = S + (int64_t)(bI.start + r0) * P + bJ.start + c;
    auto ld = [&](int rr) -> d2v {
      if (!(cl && rr < rlim)) return d2v{0.0, 0.0};
      if constexpr (NT) return __builtin_nontemporal_load((const d2v*)(sb + (int64_t)rr * P));
      else return *(const d2v*)(sb + (int64_t)rr * P);
    };
    d2v sn[G];
#pragma unroll
    for (int g = 0; g < G; ++g) sn[g] = g < 32 ? ld(g) : d2v{0.0, 0.0};
#pragma unroll
    for (int b = 0; b < NBATCH; ++b) {
      d2v sv[G];
#pragma unroll
      for (int g = 0; g < G; ++g) sv[g] = sn[g];
      if (b + 1 < NBATCH) {   // next batch's rows in flight while this one is reduced
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int rr = (b + 1) * G + g;
          sn[g] = rr < 32 ? ld(rr) : d2v{0.0, 0.0};
        }
      }
      double pr[NVB + 1];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const int rr = b * G + g;
        if (off && rr < 32 && rr < rlim) {
          const double* bi = sBI + (r0 + rr) * R;
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const double v = bi[k];
            cc[k].x = fma(sv[g].x, v, cc[k].x);
            cc[k].y = fma(sv[g].y, v, cc[k].y);
          }
        }
#pragma unroll
        for (int k = 0; k < R; ++k) pr[g * R + k] = fma(sv[g].y, bj[k].y, sv[g].x * bj[k].x);
      }
      pr[NVB] = 0.0;
      idx = 0;
      canon = true;
      ppls_rs<NVB, 0, NVB + 1>(pr, lane, idx, canon);
      if (bJ.type) racc[1][b] += pr[0];
      else racc[0][b] += pr[0];
    }
    if (off) {   // M[J rows] += S_IJ' B_I: this tile's column partial, the four waves in order
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        if (wave == w) {
#pragma unroll
          for (int k = 0; k < R; ++k) {
            red[k * 128 + c] = (w ? red[k * 128 + c] : 0.0) + cc[k].x;
            red[k * 128 + c + 1] = (w ? red[k * 128 + c + 1] : 0.0) + cc[k].y;
          }
        }
        __syncthreads();
      }
      double* cp = colpart + ((int64_t)I * (I + 1) / 2 + J) * (R * 128);
      for (int e = tid; e < R * 128; e += 256) cp[e] = red[e];
      __syncthreads();
    }
  }
  // this run's row partial: rowpart[run][2r][128]; lane idx holds row g, component k of each batch
  double* rp = rowpart + (int64_t)blockIdx.x * (2 * R * 128);
  if (canon && idx < NVB) {
    const int g = idx / R, k = idx - g * R;
#pragma unroll
    for (int b = 0; b < NBATCH; ++b) {
      const int rr = b * G + g;
      if (rr < 32) {
        rp[k * 128 + r0 + rr] = racc[0][b];
        rp[(R + k) * 128 + r0 + rr] = racc[1][b];
      }
    }
  }
}

// Row i of M: its block's run partials (row_items[b] .. row_items[b + 1]) in run order, then the
// column partials of the tiles (I, b) below it in I order; then X'mu_T / Y'mu_U of row i.
template <int R>
__global__ __launch_bounds__(256) void ppls_xprod_tri_reduce_kernel(int ldx, int ldy, const int* __restrict__ row_items,
                                                                    const double* __restrict__ rowpart,
                                                                    const double* __restrict__ colpart,
                                                                    const PplsScalars* __restrict__ sc,
                                                                    double* __restrict__ stats,
                                                                    double* __restrict__ M,
                                                                    const int* __restrict__ stop) {
  if (stop && *stop) return;
  const int P = ldx + ldy, bx = (ldx + 127) >> 7, nb = bx + ((ldy + 127) >> 7);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)P * R) return;
  const int k = (int)(e / P), i = (int)(e - (int64_t)k * P);
  const int b = i < ldx ? i >> 7 : bx + ((i - ldx) >> 7);
  const int r = i < ldx ? i & 127 : (i - ldx) & 127;
  double m0 = 0.0, m1 = 0.0;
  for (int t = row_items[b]; t < row_items[b + 1]; ++t) {
    m0 += rowpart[(int64_t)t * (2 * R * 128) + k * 128 + r];
    m1 += rowpart[(int64_t)t * (2 * R * 128) + (R + k) * 128 + r];
  }
#pragma unroll 4
  for (int I = b + 1; I < nb; ++I) {
    const double v = colpart[((int64_t)I * (I + 1) / 2 + b) * (R * 128) + k * 128 + r];
    if (I < bx) m0 += v;
    else m1 += v;
  }
  M[(int64_t)k * P + i] = m0;
  M[(int64_t)(R + k) * P + i] = m1;
  if (i < ldx) stats[(int64_t)k * ldx + i] = sc->alpha[k] * m0 + sc->beta[k] * m1;   // X'mu_T
  else stats[(int64_t)R * ldx + (int64_t)k * ldy + (i - ldx)] = sc->gamma[k] * m0 + sc->delta[k] * m1;   // Y'mu_U
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
  double v = 0.0;
  for (int i = threadIdx.x; i < rows; i += 256) v = fma(Bcol[i], Mcol[i], v);
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
hipError_t launch_apply(const double* S, int ldx, int ldy, const double* Wp, const double* Cp, const PplsScalars* sc,
                        double* stats, double* M, const int* stop, hipStream_t st) {
  const int P = ldx + ldy;
  const unsigned blocks = (unsigned)((P + RW - 1) / RW);
  // S beyond the 256 MiB Infinity Cache is read once per iteration: non-temporal loads
  if (8.0 * P * (double)P > 200.0 * (1 << 20))
    hipLaunchKernelGGL((ppls_xprod_apply_kernel<R, RW, true>), dim3(blocks), dim3(256), 0, st, S, ldx, ldy, Wp, Cp, sc,
                       stats, M, stop);
  else
    hipLaunchKernelGGL((ppls_xprod_apply_kernel<R, RW, false>), dim3(blocks), dim3(256), 0, st, S, ldx, ldy, Wp, Cp,
                       sc, stats, M, stop);
  return hipGetLastError();
}

template <int R>
hipError_t launch_apply_rw(int rw, const double* S, int ldx, int ldy, const double* Wp, const double* Cp,
                           const PplsScalars* sc, double* stats, double* M, const int* stop, hipStream_t st) {
  if (rw == 1) return launch_apply<R, 1>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  if (rw == 2) return launch_apply<R, 2>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  if constexpr (R <= 8)
    if (rw == 4) return launch_apply<R, 4>(S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);
  return hipErrorInvalidValue;
}

template <int R, int RW>
hipError_t launch_tile(const double* S, int ldx, int ldy, const double* Wp, const double* Cp, const PplsScalars* sc,
                       double* stats, double* M, const int* stop, hipStream_t st) {
  const int P = ldx + ldy;
  const unsigned blocks = (unsigned)((P + 4 * RW - 1) / (4 * RW));
  if (8.0 * P * (double)P > 200.0 * (1 << 20))   // S beyond the Infinity Cache: non-temporal loads
    hipLaunchKernelGGL((ppls_xprod_tile_kernel<R, RW, true>), dim3(blocks), dim3(256), 0, st, S, ldx, ldy, Wp, Cp, sc,
                       stats, M, stop);
  else
    hipLaunchKernelGGL((ppls_xprod_tile_kernel<R, RW, false>), dim3(blocks), dim3(256), 0, st, S, ldx, ldy, Wp, Cp,
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

template <int R>
hipError_t launch_tri(const double* S, int ldx, int ldy, const double* Wp, const double* Cp, const PplsScalars* sc,
                      double* stats, double* M, const int* items, int nruns, const int* row_items, double* rowpart,
                      double* colpart, const int* stop, hipStream_t st) {
  const int P = ldx + ldy;
  if (4.0 * P * (double)P > 200.0 * (1 << 20))   // the lower triangle beyond the Infinity Cache: nt loads
    hipLaunchKernelGGL((ppls_xprod_tri_kernel<R, true>), dim3((unsigned)nruns), dim3(256), 0, st, S, ldx, ldy, Wp, Cp,
                       (const int4*)items, rowpart, colpart, stop);
  else
    hipLaunchKernelGGL((ppls_xprod_tri_kernel<R, false>), dim3((unsigned)nruns), dim3(256), 0, st, S, ldx, ldy, Wp, Cp,
                       (const int4*)items, rowpart, colpart, stop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int64_t n = (int64_t)P * R;
  hipLaunchKernelGGL((ppls_xprod_tri_reduce_kernel<R>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ldx, ldy,
                     row_items, rowpart, colpart, sc, stats, M, stop);
  return hipGetLastError();
}

}  // namespace

extern "C" {

int ppls_xprod_tri_plan(int ldx, int ldy, int r, int num_cus, int* items, int* row_items, int64_t* rowpart_len,
                        int64_t* colpart_len) {
  if (r < 1 || r > PPLS_XP_TRI_RMAX || ldx < 2 || ldy < 2) return -1;
  const int bx = (ldx + 127) / 128, nb = bx + (ldy + 127) / 128;
  const int64_t ntiles = (int64_t)nb * (nb + 1) / 2;
  int T = (int)(ntiles / (2 * (int64_t)(num_cus > 0 ? num_cus : 256)));   // ~2 runs per CU
  if (T < 1) T = 1;
  int nr = 0;
  for (int I = 0; I < nb; ++I) {
    if (row_items) row_items[I] = nr;
    for (int J0 = 0; J0 <= I; J0 += T) {
      if (items) {
        items[4 * nr] = I;
        items[4 * nr + 1] = J0;
        items[4 * nr + 2] = J0 + T <= I + 1 ? J0 + T : I + 1;
        items[4 * nr + 3] = 0;
      }
      ++nr;
    }
  }
  if (row_items) row_items[nb] = nr;
  if (rowpart_len) *rowpart_len = (int64_t)nr * 2 * r * 128;
  if (colpart_len) *colpart_len = ntiles * r * 128;
  return nr;
}

hipError_t ppls_launch_xprod_tri(const double* S, int ldx, int ldy, int r, const double* Wp, const double* Cp,
                                 const PplsScalars* sc, double* stats, double* M, const int* items, int nruns,
                                 const int* row_items, double* rowpart, double* colpart, const int* stop,
                                 hipStream_t st) {
  if (ldx < 2 || ldy < 2 || (ldx & 1) || (ldy & 1) || r < 1 || r > PPLS_XP_TRI_RMAX || nruns < 1)
    return hipErrorInvalidValue;
  if (((uintptr_t)S | (uintptr_t)Wp | (uintptr_t)Cp) & 15) return hipErrorInvalidValue;   // 16-B loads
  hipError_t e;
  switch (r) {
#define PPLS_XT_CASE(k) \
    case k: e = launch_tri<k>(S, ldx, ldy, Wp, Cp, sc, stats, M, items, nruns, row_items, rowpart, colpart, stop, st); break;
    PPLS_XT_CASE(1) PPLS_XT_CASE(2) PPLS_XT_CASE(3) PPLS_XT_CASE(4) PPLS_XT_CASE(5) PPLS_XT_CASE(6)
    PPLS_XT_CASE(7) PPLS_XT_CASE(8) PPLS_XT_CASE(9) PPLS_XT_CASE(10)
#undef PPLS_XT_CASE
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess) return e;
  const int R2 = 2 * r;
  hipLaunchKernelGGL(ppls_xprod_gram_kernel, dim3((unsigned)(R2 * (R2 + 1) / 2)), dim3(256), 0, st, ldx, ldy, r, Wp,
                     Cp, M, stats, stop);
  return hipGetLastError();
}


int ppls_xprod_rows_per_wave(int P, int r, int rw_opt) {
  if (rw_opt == 1 || rw_opt == 2 || (rw_opt == 4 && r <= 8)) return rw_opt;
  if (r <= 8 && P / 4 >= 1024) return 4;   // >= 4 workgroups per CU left at four rows per workgroup
  return P / 2 >= 512 ? 2 : 1;
}

int ppls_xprod_tile_rows(int P, int r, int rw_opt, int num_cus) {
  if (rw_opt == 1 || rw_opt == 2 || rw_opt == 4 || (rw_opt == 8 && r <= 8)) return rw_opt;
  return P / 8 >= 2 * num_cus ? 2 : 1;   // two rows per wave while >= 2 workgroups per CU remain
}

hipError_t ppls_launch_xprod_apply(const double* S, int ldx, int ldy, int r, int kind, int rw, const double* Wp,
                                   const double* Cp, const PplsScalars* sc, double* stats, double* M, const int* stop,
                                   int with_gram, hipStream_t st) {
  if (ldx < 2 || ldy < 2 || (ldx & 1) || (ldy & 1) || r < 1 || r > PPLS_RMAX) return hipErrorInvalidValue;
  if (((uintptr_t)S | (uintptr_t)Wp | (uintptr_t)Cp) & 15) return hipErrorInvalidValue;   // 16-B loads
  hipError_t e;
  switch (r) {
#define PPLS_XP_CASE(k)                                                                                  \
    case k:                                                                                              \
      e = kind == 0 ? launch_tile_rw<k>(rw, S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st)                  \
                    : launch_apply_rw<k>(rw, S, ldx, ldy, Wp, Cp, sc, stats, M, stop, st);               \
      break;
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
