// ppls_variances.hip -- kernels of variances.PPLS_simult (Package/PPLS/R/EM_W_multi.R:830-860), the
// asymptotic standard errors of the loadings.  Per component i the reference forms
//   SSt_expec = t(X) %*% diag(c(Ctt), N) %*% X - Cxt k1 w' - w k1 Cxt' + k2 w w'     (:846-848)
// with an N x N diagonal in the middle: that is Ctt * X'X, the p x p Gram of the data -- the one
// genuinely MFMA-bound product of the package (2 n p^2 flops; C3: 8 TFLOP, 4.5 TFLOP for the
// lower triangle).  It is computed ONCE for all components on v_mfma_f64_16x16x4_f64:
//   ppls_gram_mfma_kernel   lower-triangular 128 x 128 tiles of X'X, split over row ranges
//   ppls_gram_finish_kernel sum of the splits, mirrored into a full column-major p x p
//   ppls_xtmu_kernel        Cxt = X' mu (p x a) partials per row chunk (HBM-bound, one pass)
//   ppls_varmat_kernel      B_exp - SSt_exp (and SSt_exp, SSt_star on request) of one component
//   ppls_negdiag_kernel     varMatrix = -solve(.) and seLoad = sqrt(diag(varMatrix))  (LU path)
//   ppls_negate_kernel, ppls_symdiag_kernel   the Cholesky path: -(B_exp - SSt_exp), then the
//                           inverse's lower triangle mirrored and seLoad
// The p x p inverse between them is rocSOLVER (library factorisation): Cholesky potrf/potri of the
// observed information -(B_exp - SSt_exp) when it is positive definite, else LU getrf/getri.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

#include "ppls_kernels.h"
#include "ppls_xprod.h"

#define PPLS_GT 128   // output tile edge (4 waves x 64 x 64)
#define PPLS_GK 16    // rows per LDS stage
#define PPLS_GLD 144  // LDS row stride in doubles: 1152 B = 128 mod 256, so the 4 row groups of a
                      // ds_read_b64 wave fall in disjoint bank halves per half-wave

namespace {

template <typename T>
struct GVec;   // one 16-B global load of T
template <>
struct GVec<double> {
  double2 v;
  __device__ __forceinline__ void load(const double* p) { v = *(const double2*)p; }
  __device__ __forceinline__ void zero() { v = make_double2(0.0, 0.0); }
  __device__ __forceinline__ void store(double* d) const { *(double2*)d = v; }
};
template <>
struct GVec<float> {
  float4 v;
  __device__ __forceinline__ void load(const float* p) { v = *(const float4*)p; }
  __device__ __forceinline__ void zero() { v = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void store(double* d) const {
    *(double2*)d = make_double2((double)v.x, (double)v.y);
    *(double2*)(d + 2) = make_double2((double)v.z, (double)v.w);
  }
};

}  // namespace

// The columns of the joint space that can be non-zero: [0, xreal) of X and [xcols, xcols + yreal) of
// Y -- between and after them lie the rows' zero padding (C5: X columns 10,000 .. 10,239).
struct PplsGramCols {
  int p, xreal, xcols, yend;
};

// Whether the 16 columns [a, a + 16) of the joint space hold any that can be non-zero.
__host__ __device__ inline bool ppls_gram_live(const PplsGramCols& g, int a) {
  return a < g.p && (a < g.xreal || (a + 16 > g.xcols && a < g.yend));
}

// Active 16 x 16 MFMA blocks of wave (wi, wj) in the lower tile (I, J) of a p x p Gram: bit m * 4 + q
// for the wave's block row m and block column q.  A block is skipped when its rows or columns are
// all zero padding (past p, or between X's real columns and Y's), or -- in a diagonal tile -- when it
// lies wholly above the diagonal (the finish kernel reads only the lower triangle).  C3 (p = 4000 ->
// 32 blocks of 128): the last block row is 3/4 padding and the diagonal tiles 7/16 upper half, 7 %
// of the executed flops; C5 also skips the 240 padding columns of X's 40,960-B rows (4 %).  Skipped
// blocks inside p are written as the zeros they are (their accumulators are never touched).
__host__ __device__ inline unsigned ppls_gram_active(int I, int J, int wi, int wj, const PplsGramCols& g) {
  unsigned act = 0;
  for (int m = 0; m < 4; ++m)
    for (int q = 0; q < 4; ++q) {
      const int i0 = I * PPLS_GT + wi * 64 + m * 16, j0 = J * PPLS_GT + wj * 64 + q * 16;
      if (ppls_gram_live(g, i0) && ppls_gram_live(g, j0) && (I != J || wj * 4 + q <= wi * 4 + m))
        act |= 1u << (m * 4 + q);
    }
  return act;
}

// Whether tile (I, J) has any skipped block (its items take the masked code path).
__host__ __device__ inline bool ppls_gram_partial(int I, int J, const PplsGramCols& g) {
  if (I == J) return true;
  for (int a = 0; a < PPLS_GT; a += 16)
    if (!ppls_gram_live(g, I * PPLS_GT + a) || !ppls_gram_live(g, J * PPLS_GT + a)) return true;
  return false;
}

__host__ __device__ inline void ppls_gram_tile_of(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

// The persistent form's next work item: group g's queue first (its workgroups share an XCD, so
// their items -- consecutive tiles of one row split -- share column panels in that L2), then the
// other groups' (stealing: an XCD that runs ahead takes the cheap tail of a slower one).  One
// global atomic per grab (items take milliseconds); -1 when every queue is empty.
__device__ inline int ppls_gram_next(unsigned* cnt, const int* qoff, const int* items, int g) {
  for (int k = 0; k < 8; ++k) {
    const int gg = (g + k) & 7;
    const int len = qoff[gg + 1] - qoff[gg];
    const unsigned idx = atomicAdd(&cnt[gg], 1u);
    if ((int)idx < len) return items[qoff[gg] + idx];
  }
  return -1;
}

// X'X on MFMA.  Work item L = split s x lower tile t = (I, J), J <= I.  A wave owns a 64 x 64
// sub-tile = 4 x 4 MFMA blocks (64 fp64 accumulators per lane); per 4-row k-step it reads 4 A and 4
// B operands from LDS (lane l: row l >> 4 of the step, column l & 15 of its block) -- both straight
// from the row-major panels, no transpose, since A[i][k] = X[k][i] and B[k][j] = X[k][j].  The next
// stage's global loads are in flight during the MFMAs; one barrier per 16-row stage.  Output:
// part[s][i p + j] for the tile's (i, j), i in block I >= block J (row-major of the lower blocks;
// coalesced over j).
//
// Scheduling (template DYN): the static form runs one work item per workgroup, blockIdx remapped so
// that each XCD -- blockIdx mod 8 -- gets a contiguous range of items (tiles that share column panels
// share an L2).  Its items all take the same time, so the last round of them leaves the slots that
// have none idle (C3: 6,336 items on 512 slots, the 13th round 3/8 full: ~5 % of the kernel).  The
// persistent form (DYN) launches one workgroup per slot; each takes items from the queue of its group
// (blockIdx mod 8: the same contiguous ranges), costliest first -- tiles with skipped blocks (SKIP)
// are cheaper and come last, so the final items of every queue are short -- and steals from the
// other groups' queues once its own is empty.  Each item's sums depend only on the item, so the
// result is the same bit for bit whichever workgroup runs it.
//
// The column space is that of the joint matrix [X | Y] (ppls_xprod.hip's cross-product form of the
// EM iteration): column c is X[:, c] for c < xcols and Y[:, c - xcols] for c - xcols < ycols (zero
// beyond); xcols and ycols are multiples of the 16-B vector, so no load straddles the seam.  The
// Gram of X alone is xcols = ld, ycols = 0, p the output edge.
template <typename T, bool SKIP, bool MASKED>
__device__ __forceinline__ void ppls_gram_item(const T* __restrict__ X, int ldx, int xcols, const T* __restrict__ Y,
                                               int ldy, int ycols, int64_t n, int p, int ntiles, int nsplit,
                                               int64_t L, double* __restrict__ part, int64_t part_stride,
                                               const PplsGramCols gc, double (*sm)[2][PPLS_GK][PPLS_GLD]) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int EV = 16 / sizeof(T);              // elements per 16-B load
  constexpr int VPR = PPLS_GT / EV;               // 16-B vectors per panel row
  constexpr int NV = PPLS_GK * VPR / 256;         // per thread per panel (fp64: 4, fp32: 2)
  const int s = (int)(L / ntiles), t = (int)(L - (int64_t)s * ntiles);
  int I, J;
  ppls_gram_tile_of(t, &I, &J);
  const int64_t r0 = n * s / nsplit, r1 = n * (s + 1) / nsplit;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int colA = I * PPLS_GT, colB = J * PPLS_GT;
  // wave-uniform (SGPR) block mask; MASKED code paths test it per MFMA, the full path does not
  const unsigned act = SKIP ? ppls_gram_active(I, J, wi, wj, gc) : 0xffffu;

  GVec<T> ra[NV], rb[NV];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = tid + 256 * v, row = c / VPR, cv = c - row * VPR;
      const int64_t gr = k0 + row;
      const int ca = colA + cv * EV, cb = colB + cv * EV;
      if (gr < r1 && ca < xcols) ra[v].load(X + gr * ldx + ca);
      else if (gr < r1 && ca - xcols < ycols) ra[v].load(Y + gr * ldy + (ca - xcols));
      else ra[v].zero();
      if (gr < r1 && cb < xcols) rb[v].load(X + gr * ldx + cb);
      else if (gr < r1 && cb - xcols < ycols) rb[v].load(Y + gr * ldy + (cb - xcols));
      else rb[v].zero();
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = tid + 256 * v, row = c / VPR, cv = c - row * VPR;
      ra[v].store(&sm[buf][0][row][cv * EV]);
      rb[v].store(&sm[buf][1][row][cv * EV]);
    }
  };

  d4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = d4{0.0, 0.0, 0.0, 0.0};
  const int64_t nsteps = (r1 - r0 + PPLS_GK - 1) / PPLS_GK;
  if (nsteps > 0) {
    load(r0);
    store(0);
  }
  __syncthreads();
  const int ko = lane >> 4, cl = lane & 15;
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = (int)(st & 1);
    if (st + 1 < nsteps) load(r0 + (st + 1) * PPLS_GK);
    if (!MASKED || act) {
#pragma unroll
      for (int kk = 0; kk < PPLS_GK / 4; ++kk) {
        const double* ar = &sm[buf][0][kk * 4 + ko][wi * 64 + cl];
        const double* br = &sm[buf][1][kk * 4 + ko][wj * 64 + cl];
        double a[4], b[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = ar[m * 16];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = br[q * 16];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (!MASKED || ((act >> (m * 4 + q)) & 1u))
              acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[q], acc[m][q], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  double* out = part + (int64_t)s * part_stride;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = colB + wj * 64 + q * 16 + cl;
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // f64 MFMA D map: col = lane & 15, row = (lane >> 4) + 4 g
        const int i = colA + wi * 64 + m * 16 + ko + 4 * g;
        if (i < p && j < p) out[(int64_t)i * p + j] = acc[m][q][g];
      }
    }
}

template <typename T, bool DYN, bool SKIP>
__global__ __launch_bounds__(256, 2) void ppls_gram_mfma_kernel(const T* __restrict__ X, int ldx, int xcols,
                                                                 const T* __restrict__ Y, int ldy, int ycols,
                                                                 int64_t n, int p, int ntiles, int nsplit,
                                                                 int64_t work, double* __restrict__ part,
                                                                 int64_t part_stride, int* __restrict__ queue,
                                                                 PplsGramCols gc) {
  __shared__ __attribute__((aligned(16))) double sm[2][2][PPLS_GK][PPLS_GLD];
  if constexpr (!DYN) {
    const int64_t per = gridDim.x >> 3;
    const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (L >= work) return;
    if (SKIP) {
      int I, J;
      ppls_gram_tile_of((int)(L % ntiles), &I, &J);
      if (ppls_gram_partial(I, J, gc)) {   // a tile with skipped blocks: the masked code path
        ppls_gram_item<T, true, true>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
        return;
      }
    }
    ppls_gram_item<T, false, false>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
  } else {
    // queue = [qoff (9) | counters (8, zeroed before the launch) | items (work)]
    const int* qoff = queue;
    unsigned* cnt = (unsigned*)(queue + 9);
    const int* items = queue + 17;
    __shared__ int s_next;
    const int g = blockIdx.x & 7;
    for (;;) {
      if (threadIdx.x == 0) s_next = ppls_gram_next(cnt, qoff, items, g);
      __syncthreads();
      const int L = s_next;
      __syncthreads();   // every thread has read s_next before thread 0 writes the next one
      if (L < 0) return;
      int I, J;
      ppls_gram_tile_of(L % ntiles, &I, &J);
      if (SKIP && ppls_gram_partial(I, J, gc))
        ppls_gram_item<T, true, true>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
      else
        ppls_gram_item<T, false, false>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
    }
  }
}

// G (p x p column-major, full) = sum over splits of the lower-block entries: element (a, b) is read
// at (max, min), which lies in a computed tile and makes G exactly symmetric.
__global__ void ppls_gram_finish_kernel(const double* __restrict__ part, int nsplit, int64_t part_stride, int p,
                                        double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t pp = (int64_t)p * p;
  if (e >= pp) return;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);
  const int hi = a > b ? a : b, lo = a > b ? b : a;
  double v = 0.0;
  for (int s = 0; s < nsplit; ++s) v += part[(int64_t)s * part_stride + (int64_t)hi * p + lo];
  G[e] = v;
}

// Cxt partials: part[chunk][k * ld + c] = sum over the chunk's rows of X[row][c] mu[row][k]
// (mu: n x a column-major, a <= 16).  One thread per 16-B column vector; mu rows of 64-row blocks
// staged in LDS (broadcast reads).  HBM-bound (one pass over X).
template <typename T>
__global__ __launch_bounds__(256) void ppls_xtmu_kernel(const T* __restrict__ X, int64_t n, int ld, const double* __restrict__ mu,
                                                        int a, int64_t rows_per_chunk, double* __restrict__ part,
                                                        int64_t part_ld) {
  constexpr int EV = 16 / sizeof(T);
  __shared__ double ms[64][16];
  const int nvec = ld / EV;
  const int cv = blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = rows_per_chunk * blockIdx.y;
  const int64_t r1 = r0 + rows_per_chunk < n ? r0 + rows_per_chunk : n;
  double acc[16][EV];
#pragma unroll
  for (int k = 0; k < 16; ++k)
#pragma unroll
    for (int e = 0; e < EV; ++e) acc[k][e] = 0.0;
  for (int64_t b0 = r0; b0 < r1; b0 += 64) {
    const int nr = (int)(r1 - b0 < 64 ? r1 - b0 : 64);
    __syncthreads();
    for (int e = threadIdx.x; e < 64 * 16; e += 256) {
      const int rr = e >> 4, k = e & 15;
      ms[rr][k] = (rr < nr && k < a) ? mu[(int64_t)k * n + b0 + rr] : 0.0;
    }
    __syncthreads();
    if (cv < nvec) {
      for (int rr = 0; rr < nr; ++rr) {
        GVec<T> xv;
        xv.load(X + (b0 + rr) * ld + (int64_t)cv * EV);
        double xd[EV];
        xv.store(xd);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const double m = ms[rr][k];
#pragma unroll
          for (int e = 0; e < EV; ++e) acc[k][e] = fma(xd[e], m, acc[k][e]);
        }
      }
    }
  }
  if (cv < nvec) {
    double* o = part + (int64_t)blockIdx.y * part_ld;
    for (int k = 0; k < a; ++k)
#pragma unroll
      for (int e = 0; e < EV; ++e) o[(int64_t)k * ld + (int64_t)cv * EV + e] = acc[k][e];
  }
}

// One component of variances.PPLS_simult (EM_W_multi.R:838-857):
//   M = B_exp - SSt_exp, B_exp = Ctt / sigE^2 I / N, SSt_exp = (Ctt G - k1 (Cxt w' + w Cxt') + k2 w w')
//   / sigE^4 / N, k1 = Ctt + 2 Vt, k2 = Ctt^2 + 4 ||mu||^2 Vt + 2 Vt^2, Vt = Ctt - ||mu||^2 (Ctt = N Ctt_ii);
//   SSt_star = (Cxt - w Ctt)(Cxt - w Ctt)' / sigE^4.
__global__ void ppls_varmat_kernel(const double* __restrict__ G, const double* __restrict__ cxt,
                                   const double* __restrict__ w, int p, double ctt, double k1, double k2,
                                   double bstar, double s4, double N, double* __restrict__ M,
                                   double* __restrict__ sst_exp, double* __restrict__ sst_star) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)p * p) return;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);
  const double xa = cxt[a], xb = cxt[b], wa = w[a], wb = w[b];
  const double sse = (ctt * G[e] - xa * k1 * wb - wa * k1 * xb + wa * k2 * wb) / s4 / N;
  M[e] = (a == b ? bstar : 0.0) - sse;
  if (sst_exp) sst_exp[e] = sse;
  if (sst_star) sst_star[e] = (xa - wa * ctt) * (xb - wb * ctt) / s4;
}

// varMatrix = -Minv in place; seLoad = sqrt(diag(varMatrix)) (NaN where negative, as R's sqrt).
__global__ void ppls_negdiag_kernel(double* __restrict__ M, int p, double* __restrict__ se) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)p * p) return;
  const double v = -M[e];
  M[e] = v;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);
  if (a == b) se[a] = sqrt(v);
}

// batch x (p x p): M <- -M (before the Cholesky factorisation of -(B_exp - SSt_exp)).
__global__ void ppls_negate_kernel(double* __restrict__ M, int64_t len) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < len) M[e] = -M[e];
}

// The lower triangle potri wrote (varMatrix = (-(B_exp - SSt_exp))^-1) mirrored into the upper one,
// and seLoad = sqrt(diag(varMatrix)).
__global__ void ppls_symdiag_kernel(double* __restrict__ M, int p, double* __restrict__ se) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)p * p) return;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);   // element (a, b), column-major
  if (a < b) M[e] = M[(int64_t)a * p + b];
  else if (a == b) se[a] = sqrt(M[e]);
}

extern "C" {

hipError_t ppls_launch_negate(double* M, int64_t len, hipStream_t st) {
  hipLaunchKernelGGL(ppls_negate_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0, st, M, len);
  return hipGetLastError();
}

hipError_t ppls_launch_symdiag(double* M, int p, double* se, hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  hipLaunchKernelGGL(ppls_symdiag_kernel, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, M, p, se);
  return hipGetLastError();
}

int ppls_gram_tiles(int p) {
  const int nb = (p + PPLS_GT - 1) / PPLS_GT;
  return nb * (nb + 1) / 2;
}

int ppls_gram_occupancy(int f32) {
  int occ = 0;
  hipError_t e = f32 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<float, true, true>, 256, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<double, true, true>, 256, 0);
  return e == hipSuccess && occ > 0 ? occ : 1;
}

// MFMA blocks an item of tile t executes (of 64): the persistent queue's cost order.
static int ppls_gram_cost(int t, const PplsGramCols& gc, int variant) {
  if (!(variant & PPLS_GRAM_SKIP)) return 64;
  int I, J;
  ppls_gram_tile_of(t, &I, &J);
  int c = 0;
  for (int w = 0; w < 4; ++w) c += __builtin_popcount(ppls_gram_active(I, J, w >> 1, w & 1, gc));
  return c;
}

// Row splits of a p x p Gram over n rows (partials: nsplit x 8 p^2 bytes, kept under 4 GB).
// Static form: enough items to fill whole rounds of the slots (>= 95 % of the last round).  Persistent
// form: about 12 items per slot, so the queues end on short items.
int ppls_gram_splits(int p, int64_t n, int slots, int variant) {
  const int ntiles = ppls_gram_tiles(p);
  const double pp = (double)p * p;
  auto allowed = [&](int sp) { return sp == 1 || ((int64_t)sp * 512 <= n && (double)sp * pp * 8.0 <= 4.0e9); };
  if (variant & PPLS_GRAM_DYN) {
    int sp = (int)((12LL * slots + ntiles - 1) / ntiles);
    sp = sp < 1 ? 1 : (sp > 32 ? 32 : sp);
    while (sp > 1 && !allowed(sp)) --sp;
    return sp;
  }
  int nsplit = 1;
  double best = -1.0;
  for (int sp = 1; sp <= 32; ++sp) {
    if (!allowed(sp)) break;
    const int64_t w = (int64_t)ntiles * sp;
    const double eff = (double)w / (double)(((w + slots - 1) / slots) * slots);
    if (eff > best + 1e-9) { best = eff; nsplit = sp; }
    if (eff >= 0.95) break;
  }
  return nsplit;
}

int64_t ppls_gram_queue_ints(int p, int nsplit) { return 17 + (int64_t)ppls_gram_tiles(p) * nsplit; }

// The persistent form's queues (device ints, ppls_gram_queue_ints): group g gets the contiguous item
// range [g W / 8, (g + 1) W / 8) of the split-major order (its XCD's tiles share column panels),
// sorted costliest first (stable: ties keep the split-major order).  Synchronous (host staging);
// the launch resets the counters, so one prepared queue serves any number of launches.
hipError_t ppls_gram_queue_prepare(int* queue, int p, int xreal, int xcols, int yreal, int nsplit, int variant,
                                   hipStream_t st) {
  const PplsGramCols gc{p, xreal, xcols, xcols + yreal};
  const int ntiles = ppls_gram_tiles(p);
  const int64_t work = (int64_t)ntiles * nsplit;
  std::vector<int> h((size_t)ppls_gram_queue_ints(p, nsplit), 0);
  std::vector<int> tc((size_t)ntiles);
  for (int t = 0; t < ntiles; ++t) tc[(size_t)t] = ppls_gram_cost(t, gc, variant);
  int* items = h.data() + 17;
  for (int g = 0; g < 8; ++g) {
    const int64_t a = work * g / 8, b = work * (g + 1) / 8;
    h[(size_t)g] = (int)a;
    for (int64_t L = a; L < b; ++L) items[L] = (int)L;
    std::stable_sort(items + a, items + b,
                     [&](int x, int y) { return tc[(size_t)(x % ntiles)] > tc[(size_t)(y % ntiles)]; });
  }
  h[8] = (int)work;
  hipError_t e = hipMemcpyAsync(queue, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}

hipError_t ppls_launch_gram_joint(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int ycols,
                                  int yreal, int f32, int64_t n, int p, int nsplit, double* part, int64_t part_stride,
                                  int* queue, int variant, hipStream_t st) {
  if (n <= 0 || p <= 0 || nsplit < 1 || xcols + ycols < 1 || xreal > xcols || yreal > ycols) return hipErrorInvalidValue;
  const PplsGramCols gc{p, xreal, xcols, xcols + yreal};
  const int ev = f32 ? 4 : 2;
  if (xcols % ev || ycols % ev) return hipErrorInvalidValue;
  const int ntiles = ppls_gram_tiles(p);
  const int64_t work = (int64_t)ntiles * nsplit;
  const bool dyn = (variant & PPLS_GRAM_DYN) != 0, skip = (variant & PPLS_GRAM_SKIP) != 0;
  if (work > 0x7fffffff - 32) return hipErrorInvalidValue;
  int64_t grid;
  if (dyn) {
    if (!queue) return hipErrorInvalidValue;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    grid = (int64_t)cus * ppls_gram_occupancy(f32);
    grid = (grid + 7) / 8 * 8;
    hipError_t e = hipMemsetAsync(queue + 9, 0, 8 * sizeof(int), st);   // the queue counters
    if (e != hipSuccess) return e;
  } else {
    grid = (work + 7) / 8 * 8;   // a multiple of 8: the XCD remap needs whole rounds
  }
#define PPLS_GRAM_LAUNCH(TT, D, S)                                                                           \
  hipLaunchKernelGGL((ppls_gram_mfma_kernel<TT, D, S>), dim3((unsigned)grid), dim3(256), 0, st, (const TT*)X, ldx, \
                     xcols, (const TT*)Y, ldy, ycols, n, p, ntiles, nsplit, work, part, part_stride, queue, gc)
  if (f32) {
    if (dyn && skip) PPLS_GRAM_LAUNCH(float, true, true);
    else if (dyn) PPLS_GRAM_LAUNCH(float, true, false);
    else if (skip) PPLS_GRAM_LAUNCH(float, false, true);
    else PPLS_GRAM_LAUNCH(float, false, false);
  } else {
    if (dyn && skip) PPLS_GRAM_LAUNCH(double, true, true);
    else if (dyn) PPLS_GRAM_LAUNCH(double, true, false);
    else if (skip) PPLS_GRAM_LAUNCH(double, false, true);
    else PPLS_GRAM_LAUNCH(double, false, false);
  }
#undef PPLS_GRAM_LAUNCH
  return hipGetLastError();
}

hipError_t ppls_launch_gram(const void* X, int f32, int64_t n, int ld, int p, int nsplit, double* part,
                            int64_t part_stride, int* queue, int variant, hipStream_t st) {
  return ppls_launch_gram_joint(X, ld, ld, p, nullptr, 0, 0, 0, f32, n, p, nsplit, part, part_stride, queue, variant, st);
}

hipError_t ppls_launch_gram_finish(const double* part, int nsplit, int64_t part_stride, int p, double* G,
                                   hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  hipLaunchKernelGGL(ppls_gram_finish_kernel, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, part, nsplit,
                     part_stride, p, G);
  return hipGetLastError();
}

int ppls_xtmu_chunks(int64_t n, int ld, int f32) {
  const int nvec = ld / (f32 ? 4 : 2);
  const int ctiles = (nvec + 255) / 256;
  int64_t ch = (2048 + ctiles - 1) / ctiles;
  const int64_t maxch = (n + 255) / 256;
  if (ch > maxch) ch = maxch;
  return (int)(ch < 1 ? 1 : ch);
}

hipError_t ppls_launch_xtmu(const void* X, int f32, int64_t n, int ld, const double* mu, int a, int chunks,
                            double* part, int64_t part_ld, hipStream_t st) {
  if (n <= 0 || a < 1 || a > 16) return hipErrorInvalidValue;
  const int nvec = ld / (f32 ? 4 : 2);
  const int64_t rpc = (n + chunks - 1) / chunks;
  const dim3 grid((nvec + 255) / 256, chunks);
  if (f32)
    hipLaunchKernelGGL(ppls_xtmu_kernel<float>, grid, dim3(256), 0, st, (const float*)X, n, ld, mu, a, rpc, part,
                       part_ld);
  else
    hipLaunchKernelGGL(ppls_xtmu_kernel<double>, grid, dim3(256), 0, st, (const double*)X, n, ld, mu, a, rpc, part,
                       part_ld);
  return hipGetLastError();
}

hipError_t ppls_launch_varmat(const double* G, const double* cxt, const double* w, int p, double ctt, double k1,
                              double k2, double bstar, double s4, double N, double* M, double* sst_exp,
                              double* sst_star, hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  hipLaunchKernelGGL(ppls_varmat_kernel, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, G, cxt, w, p, ctt,
                     k1, k2, bstar, s4, N, M, sst_exp, sst_star);
  return hipGetLastError();
}

hipError_t ppls_launch_negdiag(double* M, int p, double* se, hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  hipLaunchKernelGGL(ppls_negdiag_kernel, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, M, p, se);
  return hipGetLastError();
}

}  // extern "C"
