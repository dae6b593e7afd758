// Batched inverse of symmetric positive definite matrices for variances.PPLS_simult (row f4b):
// varMatrix = -solve(B_exp - SSt_exp) (EM_W_multi.R:852-856), where -(B_exp - SSt_exp) is the observed
// information -- SPD at a proper fit.  Replaces rocSOLVER's potrf + potri (1,400 launches, 24 ms at
// C3: VERDICT r4 weak 7) with a blocked right-looking Cholesky and a blocked inverse of the factor,
// 64 x 64 blocks, every matrix of the batch in the same launch (blockIdx.y):
//
//   for k = 0 .. nb-1:                         A = L L'
//     diag(k):   L_kk = chol(A_kk), Li_k = L_kk^-1     (k > 0: inside update(k - 1)'s first tile)
//     panel(k):  L_ik = A_ik Li_k'                      for i > k
//     update(k): A_ij -= L_ik L_jk'                     for k < j <= i
//   for i = 0 .. nb-2:                          T = L^-1 (T_ii = Li_i from diag), right-looking
//     trtri(i):  B_mk -= L_mi T_ik for m > i, k <= i;  T_{i+1,k} = Li_{i+1} B_{i+1,k}
//                (B_mk = -sum_{j<=i} L_mj T_jk accumulates in T's block)
//   lauum:       A^-1 = T' T, lower blocks (i, j): sum_{m >= i} T_mi' T_mj
//
// p^3 flops per matrix (p^3/3 each for the factorisation, T and T'T), 3 nb launches.  The
// 64 x 64 x 64 block products run on fp64 VALU from LDS (each thread a 4 x 4 register tile).
// Column-major p x p storage, batch stride p^2; rows / columns past p read as the identity's.
// info[z] = 64 k + j + 1 for the first non-positive (or non-finite) pivot of matrix z, else 0.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_kernels.h"

namespace {

constexpr int NB = 64;     // block size
constexpr int SL = 66;     // LDS row stride (doubles): 16-B aligned rows, writes 4-way at worst

// LDS per workgroup: two 64 x 66 double tiles (67.6 KB; the diagonal-block kernel two 64 x 65) --
// over the 64 KB of earlier CDNA parts, within gfx950's 160 KB.  gfx950 is the only target
// (build.py's PPLS_OFFLOAD_ARCH would otherwise fail at launch, not at build).
constexpr int kLdsLimit = 160 * 1024;
static_assert(2 * NB * SL * sizeof(double) <= kLdsLimit, "ppls_linalg.hip: tile pair exceeds gfx950 LDS");
static_assert(2 * NB * (NB + 1) * sizeof(double) <= kLdsLimit, "ppls_linalg.hip: diag tiles exceed gfx950 LDS");
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "ppls_linalg.hip needs gfx950 (67.6 KB of LDS per workgroup); build with --offload-arch=gfx950"
#endif

// An op(X) block (64 x 64, element (r, m)) of a column-major matrix with leading dimension ld into
// LDS as s[m][r] (the micro-kernel's k-major image).  trans: op(X)(r, m) = X(m, r).  Elements past
// `lim` rows / cols of the stored matrix read 0 (lim = valid extent of the block's rows and cols).
__device__ __forceinline__ void stage_a(double* s, const double* X, int64_t ld, int rlim, int clim, bool trans) {
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int lo = e & 63, hi = e >> 6;
    if (!trans) {   // s[m][r] = X(r, m): lanes along r
      const int r = lo, m = hi;
      s[m * SL + r] = (r < rlim && m < clim) ? X[r + (int64_t)m * ld] : 0.0;
    } else {        // s[m][r] = X(m, r): lanes along m
      const int m = lo, r = hi;
      s[m * SL + r] = (m < rlim && r < clim) ? X[m + (int64_t)r * ld] : 0.0;
    }
  }
}

// op(Y) block (element (m, c)) into LDS as s[m][c].  trans: op(Y)(m, c) = Y(c, m).
__device__ __forceinline__ void stage_b(double* s, const double* Y, int64_t ld, int rlim, int clim, bool trans) {
  for (int e = threadIdx.x; e < NB * NB; e += 256) {
    const int lo = e & 63, hi = e >> 6;
    if (!trans) {   // s[m][c] = Y(m, c): lanes along m
      const int m = lo, c = hi;
      s[m * SL + c] = (m < rlim && c < clim) ? Y[m + (int64_t)c * ld] : 0.0;
    } else {        // s[m][c] = Y(c, m): lanes along c
      const int c = lo, m = hi;
      s[m * SL + c] = (c < rlim && m < clim) ? Y[c + (int64_t)m * ld] : 0.0;
    }
  }
}

// acc[i][j] += sum_m sA[m][4 tr + i] sB[m][4 tc + j]
__device__ __forceinline__ void mm64(double (&acc)[4][4], const double* sA, const double* sB, int tr, int tc) {
#pragma unroll 8
  for (int m = 0; m < NB; ++m) {
    const double2 a0 = *(const double2*)(sA + m * SL + 4 * tr), a1 = *(const double2*)(sA + m * SL + 4 * tr + 2);
    const double2 b0 = *(const double2*)(sB + m * SL + 4 * tc), b1 = *(const double2*)(sB + m * SL + 4 * tc + 2);
    const double a[4] = {a0.x, a0.y, a1.x, a1.y}, b[4] = {b0.x, b0.y, b1.x, b1.y};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fma(a[i], b[j], acc[i][j]);
  }
}

__device__ __forceinline__ double ppls_bcast(double v, int lane) {   // lane's v, wave-uniform lane
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// diag(k): L_kk = chol(A_kk) (lower, written back), Li_k = L_kk^-1 into Li (64 x 64 per block,
// column-major) and into T's diagonal block.  Padding beyond p: the identity.  Every thread of the
// 256-thread workgroup calls it.  Blocked by 16: for each 16-column panel J, wave 0 factors and
// inverts the 16 x 16 diagonal sub-block in registers (lane r holds row r; columns exchanged by
// readlane), then the workgroup scales the panel below it (L_IJ = A_IJ D_J^-T) and updates the
// trailing lower triangle; the inverse's off-diagonal sub-blocks follow by levels I - J = 1, 2, 3:
// Li_IJ = -Li_II sum_{K=J}^{I-1} L_IK Li_KJ (the sums parked in Li's unused upper triangle).
// L, I: LDS, 64 x 65 doubles each.
__device__ __forceinline__ void diag_block(double* __restrict__ A, int p, int64_t pp, int k, double* __restrict__ Li,
                                           int nb, double* __restrict__ T, int* __restrict__ info, int z,
                                           double* __restrict__ L, double* __restrict__ I) {
  constexpr int LS = NB + 1, SB = 16;
  const int t = threadIdx.x;
  double* Az = A + pp * z;
  const int o = NB * k, lim = p - o < NB ? p - o : NB;
  {   // the lower triangle (identity past p): thread t row t & 63, columns 4 u + (t >> 6)
    const int r = t & 63, c0 = t >> 6;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int c = 4 * u + c0;
      v[u] = (r < lim && c < lim && r >= c) ? Az[(o + r) + (int64_t)(o + c) * p] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int c = 4 * u + c0;
      L[r * LS + c] = (r < lim && c < lim) ? v[u] : (r == c ? 1.0 : 0.0);
    }
  }
  __syncthreads();
  int bad = 0;   // (wave 0, uniform)
  for (int J = 0; J < 4; ++J) {
    const int c0 = SB * J;
    if (t < 64) {   // wave 0: factor and invert the 16 x 16 diagonal sub-block (lanes >= 16 mirror 0..15)
      const int rr = t & 15;
      double row[SB];
#pragma unroll
      for (int l = 0; l < SB; ++l) row[l] = L[(c0 + rr) * LS + c0 + l];
#pragma unroll
      for (int j = 0; j < SB; ++j) {
        const double d = ppls_bcast(row[j], j);
        if (!bad && !(d > 0.0 && d < INFINITY)) bad = c0 + j + 1;   // NaN fails too
        const double sq = sqrt(d);
        row[j] = rr > j ? row[j] / sq : (rr == j ? sq : row[j]);
#pragma unroll
        for (int l = j + 1; l < SB; ++l) {
          const double clj = ppls_bcast(row[j], l);   // L[l][j], scaled
          row[l] = fma(-((rr > j && l <= rr) ? row[j] : 0.0), clj, row[l]);
        }
      }
      double x[SB];   // column rr of the sub-block's inverse
#pragma unroll
      for (int i = 0; i < SB; ++i) {
        double sacc = i == rr ? 1.0 : 0.0;
#pragma unroll
        for (int m = 0; m < i; ++m) sacc = fma(-ppls_bcast(row[m], i), x[m], sacc);
        x[i] = i >= rr ? sacc / ppls_bcast(row[i], i) : 0.0;
      }
      if (t < SB) {
#pragma unroll
        for (int l = 0; l < SB; ++l) {
          if (l <= rr) L[(c0 + rr) * LS + c0 + l] = row[l];
          I[(c0 + l) * LS + c0 + rr] = x[l];   // Li's diagonal sub-block, column rr
        }
      }
    }
    __syncthreads();
    const int nr = NB - c0 - SB;   // rows below the sub-block
    if (nr > 0) {
      // panel: L[r][c0 + c] = sum_m A[r][c0 + m] Di[c][m] for r >= c0 + 16 (thread: a row, 4 columns)
      double pv[4] = {0.0, 0.0, 0.0, 0.0};
      const int r = c0 + SB + (t >> 2), cq = 4 * (t & 3);
      const bool act = (t >> 2) < nr;
      if (act) {
        double arow[SB];
#pragma unroll
        for (int m = 0; m < SB; ++m) arow[m] = L[r * LS + c0 + m];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int m = 0; m < SB; ++m) pv[c] = fma(arow[m], I[(c0 + cq + c) * LS + c0 + m], pv[c]);
      }
      __syncthreads();
      if (act)
#pragma unroll
        for (int c = 0; c < 4; ++c) L[r * LS + c0 + cq + c] = pv[c];
      __syncthreads();
      // trailing update of the lower triangle: L[r][l] -= sum_m L[r][c0 + m] L[l][c0 + m]
      for (int e = t; e < nr * nr; e += 256) {
        const int ri = e / nr, li = e - ri * nr;
        if (li <= ri) {
          const int rA = c0 + SB + ri, lA = c0 + SB + li;
          double sacc = 0.0;
#pragma unroll
          for (int m = 0; m < SB; ++m) sacc = fma(L[rA * LS + c0 + m], L[lA * LS + c0 + m], sacc);
          L[rA * LS + lA] -= sacc;
        }
      }
      __syncthreads();
    }
  }
  // off-diagonal sub-blocks of Li by levels: S = sum_{K=J}^{I-1} L_IK Li_KJ into Li's (J, I) block,
  // then Li_IJ = -Li_II S
  for (int dl = 1; dl < 4; ++dl) {
    const int np = 4 - dl;
    for (int e = t; e < np * 256; e += 256) {
      const int J = e >> 8, Ib = J + dl, a = (e >> 4) & 15, b2 = e & 15;
      double sacc = 0.0;
      for (int K = J; K < Ib; ++K)
#pragma unroll
        for (int m = 0; m < SB; ++m) sacc = fma(L[(SB * Ib + a) * LS + SB * K + m], I[(SB * K + m) * LS + SB * J + b2], sacc);
      I[(SB * J + a) * LS + SB * Ib + b2] = sacc;
    }
    __syncthreads();
    for (int e = t; e < np * 256; e += 256) {
      const int J = e >> 8, Ib = J + dl, a = (e >> 4) & 15, b2 = e & 15;
      double sacc = 0.0;
#pragma unroll
      for (int m = 0; m < SB; ++m) sacc = fma(I[(SB * Ib + a) * LS + SB * Ib + m], I[(SB * J + m) * LS + SB * Ib + b2], sacc);
      I[(SB * Ib + a) * LS + SB * J + b2] = -sacc;
    }
    __syncthreads();
  }
  double* Lz = Li + ((int64_t)z * nb + k) * NB * NB;
  double* Tz = T + pp * z;
  {
    const int r = t & 63, c0 = t >> 6;
#pragma unroll 4
    for (int u = 0; u < 16; ++u) {
      const int c = 4 * u + c0;
      const double iv = r >= c ? I[r * LS + c] : 0.0;   // (the upper triangle held the level sums)
      Lz[r + NB * c] = iv;
      if (r < lim && c < lim) {
        if (r >= c) Az[(o + r) + (int64_t)(o + c) * p] = L[r * LS + c];
        Tz[(o + r) + (int64_t)(o + c) * p] = iv;
      }
    }
  }
  if (t == 0 && bad && info[z] == 0) info[z] = o + bad;
}

__global__ __launch_bounds__(256) void chol_diag_kernel(double* __restrict__ A, int p, int64_t pp, int k,
                                                       double* __restrict__ Li, int nb, double* __restrict__ T,
                                                       int* __restrict__ info) {
  __shared__ double L[NB * (NB + 1)], I[NB * (NB + 1)];
  diag_block(A, p, pp, k, Li, nb, T, info, blockIdx.y, L, I);
}

// panel(k): L_ik = A_ik Li_k' for block rows i = k + 1 + blockIdx.x
__global__ __launch_bounds__(256) void chol_panel_kernel(double* __restrict__ A, int p, int64_t pp, int k,
                                                        const double* __restrict__ Li, int nb) {
  __shared__ __attribute__((aligned(16))) double sA[NB * SL];
  __shared__ __attribute__((aligned(16))) double sB[NB * SL];
  const int z = blockIdx.y, t = threadIdx.x, tr = t & 15, tc = t >> 4;
  const int i = k + 1 + blockIdx.x;
  const int ro = NB * i, co = NB * k, rl = p - ro < NB ? p - ro : NB;
  double* Az = A + pp * z;
  stage_a(sA, Az + ro + (int64_t)co * p, p, rl, NB, false);
  stage_b(sB, Li + ((int64_t)z * nb + k) * NB * NB, NB, NB, NB, true);
  __syncthreads();
  double acc[4][4] = {};
  mm64(acc, sA, sB, tr, tc);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = 4 * tr + a, c = 4 * tc + b;
      if (r < rl && co + c < p) Az[(ro + r) + (int64_t)(co + c) * p] = acc[a][b];
    }
}

__device__ __forceinline__ void tri_index(int e, int& ii, int& jj) {   // e -> (ii >= jj), row by row
  ii = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
  while ((ii + 1) * (ii + 2) / 2 <= e) ++ii;
  while (ii * (ii + 1) / 2 > e) --ii;
  jj = e - ii * (ii + 1) / 2;
}

// update(k): A_ij -= L_ik L_jk' for k < j <= i (blockIdx.x enumerates the trailing lower triangle)
__global__ __launch_bounds__(256) void chol_update_kernel(double* __restrict__ A, int p, int64_t pp, int k,
                                                         double* __restrict__ Li, int nb, double* __restrict__ T,
                                                         int* __restrict__ info) {
  __shared__ __attribute__((aligned(16))) double sA[NB * SL];
  __shared__ __attribute__((aligned(16))) double sB[NB * SL];
  const int z = blockIdx.y, t = threadIdx.x, tr = t & 15, tc = t >> 4;
  int ii, jj;
  tri_index(blockIdx.x, ii, jj);
  const int i = k + 1 + ii, j = k + 1 + jj;
  const int ro = NB * i, cj = NB * j, ck = NB * k;
  const int rl = p - ro < NB ? p - ro : NB, cl = p - cj < NB ? p - cj : NB;
  double* Az = A + pp * z;
  stage_a(sA, Az + ro + (int64_t)ck * p, p, rl, NB, false);          // L_ik
  stage_b(sB, Az + cj + (int64_t)ck * p, p, cl, NB, true);           // L_jk'
  __syncthreads();
  double acc[4][4] = {};
  mm64(acc, sA, sB, tr, tc);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = 4 * tr + a, c = 4 * tc + b;
      if (r < rl && c < cl && (i != j || r >= c)) Az[(ro + r) + (int64_t)(cj + c) * p] -= acc[a][b];
    }
  // the workgroup of the first trailing diagonal block factors it at once (diag(k + 1)): its latency
  // hides behind the other tiles of this launch instead of running alone before panel(k + 1)
  if (blockIdx.x == 0) {
    __syncthreads();   // this tile's stores are visible to the workgroup; sA, sB are free
    diag_block(A, p, pp, k + 1, Li, nb, T, info, z, sA, sB);
  }
}

// trtri step i (right-looking T = L^-1), for block rows m > i and columns k <= i:
//   B_mk -= L_mi T_ik      (B_mk, held in T's block until row m is final, = -sum_{j<=i} L_mj T_jk;
//                           k == i is its first touch: B_mi = -L_mi T_ii)
// and row m = i + 1 is then complete: T_mk = Li_m B_mk  (T_mk = -L_mm^-1 sum_{j<m} L_mj T_jk).
__global__ __launch_bounds__(256) void trtri_step_kernel(const double* __restrict__ A, int p, int64_t pp, int i,
                                                        const double* __restrict__ Li, int nb,
                                                        double* __restrict__ T) {
  __shared__ __attribute__((aligned(16))) double sA[NB * SL];
  __shared__ __attribute__((aligned(16))) double sB[NB * SL];
  const int z = blockIdx.y, t = threadIdx.x, tr = t & 15, tc = t >> 4;
  const int k = blockIdx.x % (i + 1), m = i + 1 + blockIdx.x / (i + 1);
  const int rm = NB * m, ci = NB * i, ck = NB * k, ml = p - rm < NB ? p - rm : NB;
  const double* Az = A + pp * z;
  double* Tz = T + pp * z;
  stage_a(sA, Az + rm + (int64_t)ci * p, p, ml, NB, false);   // L_mi
  stage_b(sB, Tz + ci + (int64_t)ck * p, p, NB, NB, false);   // T_ik (final)
  __syncthreads();
  double acc[4][4];
  if (k == i) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = 0.0;
  } else {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int r = 4 * tr + a, c = 4 * tc + b;
        acc[a][b] = r < ml ? Tz[(rm + r) + (int64_t)(ck + c) * p] : 0.0;   // -sum so far
      }
  }
  // acc = -sum_{j<=i} L_mj T_jk: subtract this step's product
  {
    double prod[4][4] = {};
    mm64(prod, sA, sB, tr, tc);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] -= prod[a][b];
  }
  if (m == i + 1) {   // row m final: T_mk = Li_m acc
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) sB[(4 * tr + a) * SL + 4 * tc + b] = acc[a][b];
    stage_a(sA, Li + ((int64_t)z * nb + m) * NB * NB, NB, NB, NB, false);
    __syncthreads();
    double out[4][4] = {};
    mm64(out, sA, sB, tr, tc);
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) acc[a][b] = out[a][b];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = 4 * tr + a, c = 4 * tc + b;
      if (r < ml) Tz[(rm + r) + (int64_t)(ck + c) * p] = acc[a][b];
    }
}

// lauum: out lower block (i, j), j <= i: sum_{m=i}^{nb-1} T_mi' T_mj (blockIdx.x enumerates the
// lower triangle).  out may alias A (the factor is no longer read).
__global__ __launch_bounds__(256) void lauum_kernel(const double* __restrict__ T, int p, int64_t pp, int nb,
                                                   double* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) double sA[NB * SL];
  __shared__ __attribute__((aligned(16))) double sB[NB * SL];
  const int z = blockIdx.y, t = threadIdx.x, tr = t & 15, tc = t >> 4;
  int i, j;
  tri_index(blockIdx.x, i, j);
  const int ci = NB * i, cj = NB * j;
  const int il = p - ci < NB ? p - ci : NB, jl = p - cj < NB ? p - cj : NB;
  const double* Tz = T + pp * z;
  double acc[4][4] = {};
  for (int m = i; m < nb; ++m) {
    const int rm = NB * m, ml = p - rm < NB ? p - rm : NB;
    __syncthreads();
    stage_a(sA, Tz + rm + (int64_t)ci * p, p, ml, il, true);    // op(A)(r, s) = T_mi(s, r)
    stage_b(sB, Tz + rm + (int64_t)cj * p, p, ml, jl, false);   // T_mj
    __syncthreads();
    mm64(acc, sA, sB, tr, tc);
  }
  double* oz = out + pp * z;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int r = 4 * tr + a, c = 4 * tc + b;
      if (r < il && c < jl) oz[(ci + r) + (int64_t)(cj + c) * p] = acc[a][b];
    }
}

}  // namespace

extern "C" {

int64_t ppls_spd_inverse_work(int p, int a) {   // doubles of scratch: T (a p^2) + the Li blocks
  const int64_t nb = (p + NB - 1) / NB;
  return (int64_t)a * p * p + (int64_t)a * nb * NB * NB;
}

// A (a matrices p x p, column-major, stride p^2): SPD in, its inverse's lower triangle out (the
// upper triangle holds the factor's garbage: mirror it, ppls_launch_symdiag).  work: at least
// ppls_spd_inverse_work(p, a) doubles; info: a ints, zeroed here.
hipError_t ppls_spd_inverse_batched(double* A, int p, int a, double* work, int* info, hipStream_t st) {
  if (p <= 0 || a <= 0) return hipSuccess;
  const int nb = (p + NB - 1) / NB;
  const int64_t pp = (int64_t)p * p;
  double* T = work;
  double* Li = work + (int64_t)a * pp;
  hipError_t e = hipMemsetAsync(info, 0, sizeof(int) * a, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chol_diag_kernel, dim3(1, a), dim3(256), 0, st, A, p, pp, 0, Li, nb, T, info);
  for (int k = 0; k + 1 < nb; ++k) {   // (update(k) also factors block k + 1)
    const int nt = nb - 1 - k;
    hipLaunchKernelGGL(chol_panel_kernel, dim3(nt, a), dim3(256), 0, st, A, p, pp, k, Li, nb);
    hipLaunchKernelGGL(chol_update_kernel, dim3(nt * (nt + 1) / 2, a), dim3(256), 0, st, A, p, pp, k, Li, nb, T,
                       info);
  }
  // T = L^-1, right-looking: step i finishes block row i + 1 and updates the rows below it
  for (int i = 0; i + 1 < nb; ++i)
    hipLaunchKernelGGL(trtri_step_kernel, dim3((nb - 1 - i) * (i + 1), a), dim3(256), 0, st, A, p, pp, i, Li, nb, T);
  hipLaunchKernelGGL(lauum_kernel, dim3(nb * (nb + 1) / 2, a), dim3(256), 0, st, T, p, pp, nb, A);
  return hipGetLastError();
}

}  // extern "C"
