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

#define PPLS_GT 128   // output tile edge (4 quadrants of 64 x 64, one wave each)
#define PPLS_GQ 64    // quadrant edge
#define PPLS_GRING 3  // k-steps of MFMA operands in flight per wave (2-4 measured equal, 6 spills)

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

__host__ __device__ inline bool ppls_gram_col_live(const PplsGramCols& g, int c) {
  return c < g.p && (c < g.xreal || (c >= g.xcols && c < g.yend));
}

// Whether the 16 columns [a, a + 16) of the joint space hold any that can be non-zero.
__host__ __device__ inline bool ppls_gram_live(const PplsGramCols& g, int a) {
  return a < g.p && (a < g.xreal || (a + 16 > g.xcols && a < g.yend));
}

__host__ __device__ inline void ppls_gram_tile_of(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

// Whether quadrant quad = 2 wi + wj (one wave's 64 x 64 output) of the lower tile (I, J) is computed:
// not when it lies wholly above the diagonal (the finish reads only the lower triangle), nor when
// its rows or its columns are all zero padding (past p, or between X's real columns and Y's).
// C3 (p = 4000): the last tile row's lower 64 rows and the diagonal tiles' upper quadrants, 4.5 % of
// the quadrants; C5 also the quadrants of X's 240 padding columns.
__host__ __device__ inline bool ppls_gram_quad_live(const PplsGramCols& g, int I, int J, int quad) {
  const int wi = quad >> 1, wj = quad & 1;
  if (I == J && wi == 0 && wj == 1) return false;
  bool ra = false, cb = false;
  for (int a = 0; a < PPLS_GQ; a += 16) {
    ra = ra || ppls_gram_live(g, I * PPLS_GT + wi * PPLS_GQ + a);
    cb = cb || ppls_gram_live(g, J * PPLS_GT + wj * PPLS_GQ + a);
  }
  return ra && cb;
}

// The next work item of a wave: its group's queue first (blockIdx mod 8: workgroups that share an
// XCD, whose items -- the tiles of one contiguous range, split by split -- share column panels in
// that L2), then the other groups' (stealing: an XCD that runs ahead takes the tail of a slower
// one).  One global atomic per item (items take tens of microseconds to milliseconds); -1 when every
// queue is empty.
__device__ inline int ppls_gram_next(unsigned* cnt, const int* qoff, const int* items, int g) {
  for (int k = 0; k < 8; ++k) {
    const int gg = (g + k) & 7;
    const int len = qoff[gg + 1] - qoff[gg];
    const unsigned idx = atomicAdd(&cnt[gg], 1u);
    if ((int)idx < len) return items[qoff[gg] + idx];
  }
  return -1;
}

// A lane's MFMA operands of one 4-row k-step, per side (A: the quadrant's 64 output rows, B: its 64
// output columns), loaded straight from the row-major data: lane l reads row k0 + (l >> 4) and, for
// fp64, the column pairs 2 i, 2 i + 1 and 32 + 2 i, 33 + 2 i of the side's 64 (i = l & 15: each
// 16-lane group reads 256 contiguous bytes per load); for fp32 the quad 4 i .. 4 i + 3 (one 16-B
// load).  MFMA block m (16 output rows or columns) then holds the columns col(m, i).
template <typename T>
struct PplsGramOps;
template <>
struct PplsGramOps<double> {
  static constexpr int NL = 2;   // 16-B loads per side per k-step
  double2 v[2];
  __device__ __forceinline__ void load(const double* const* ptr) {
    v[0] = *(const double2*)ptr[0];
    v[1] = *(const double2*)ptr[1];
  }
  __device__ __forceinline__ double op(int m) const { return m == 0 ? v[0].x : m == 1 ? v[0].y : m == 2 ? v[1].x : v[1].y; }
  __host__ __device__ static int lcol(int l, int i) { return 32 * l + 2 * i; }
  __host__ __device__ static int col(int m, int i) { return 32 * (m >> 1) + 2 * i + (m & 1); }
};
template <>
struct PplsGramOps<float> {
  static constexpr int NL = 1;
  float4 v[1];
  __device__ __forceinline__ void load(const float* const* ptr) { v[0] = *(const float4*)ptr[0]; }
  __device__ __forceinline__ double op(int m) const {
    return (double)(m == 0 ? v[0].x : m == 1 ? v[0].y : m == 2 ? v[0].z : v[0].w);
  }
  __host__ __device__ static int lcol(int, int i) { return 4 * i; }
  __host__ __device__ static int col(int m, int i) { return 4 * i + m; }
};

// One work item = split s x lower tile t = (I, J) x quadrant, on ONE wave: its 64 x 64 output as 4 x 4
// v_mfma_f64_16x16x4_f64 blocks (64 fp64 accumulators per lane), every MFMA operand loaded by the
// lane that feeds it straight from global memory into a ring PPLS_GRING k-steps deep -- no LDS, no
// workgroup barrier: waves never wait for each other.  The round-4 form staged 16-row panels in LDS
// behind one barrier per stage; at C3 it took 271.6 ms against 240.8 ms for this one, bit for bit the
// same sums (tools/gram_lab.hip, profiles/r5_gram_lab_*.txt).  Columns past p read column 0: that
// garbage only meets its own output rows / columns, which the finish never reads, so the steady
// state needs no masks; rows past the split's end are zeros (the one partial k-step).
// Output: part[item][a][b], a quadrant-local row, b column (64 x 64 doubles per item).
template <typename T>
__device__ __forceinline__ void ppls_gram_wave_item(const T* __restrict__ X, int ldx, int xcols, const T* __restrict__ Y,
                                                    int ldy, int ycols, int p, int ntiles, int it,
                                                    const int64_t* __restrict__ bounds, double* __restrict__ part) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  typedef PplsGramOps<T> Op;
  constexpr int D = PPLS_GRING;
  const int quad = it & 3, st = it >> 2;
  const int s = st / ntiles, t = st - s * ntiles;
  int I, J;
  ppls_gram_tile_of(t, &I, &J);
  const int64_t r0 = bounds[s], r1 = bounds[s + 1];
  const int lane = threadIdx.x & 63, kr = lane >> 4, li = lane & 15;
  const T* pa[Op::NL];
  const T* pb[Op::NL];
  int64_t sa[Op::NL], sb[Op::NL];
  auto base = [&](int c, const T** pp, int64_t* step) {
    const T* b0;
    int64_t ld;
    if (c < xcols && c < p) { b0 = X + c; ld = ldx; }
    else if (c >= xcols && c - xcols < ycols && c < p) { b0 = Y + (c - xcols); ld = ldy; }
    else { b0 = X; ld = ldx; }   // padding past p
    *pp = b0 + (r0 + kr) * ld;
    *step = 4 * ld;
  };
#pragma unroll
  for (int l = 0; l < Op::NL; ++l) {
    base(I * PPLS_GT + (quad >> 1) * PPLS_GQ + Op::lcol(l, li), &pa[l], &sa[l]);
    base(J * PPLS_GT + (quad & 1) * PPLS_GQ + Op::lcol(l, li), &pb[l], &sb[l]);
  }
  Op ra[D], rb[D];
  auto ld_step = [&](int d) {
    ra[d].load(pa);
    rb[d].load(pb);
#pragma unroll
    for (int l = 0; l < Op::NL; ++l) {
      pa[l] += sa[l];
      pb[l] += sb[l];
    }
  };
  d4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = d4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](const Op& A, const Op& B) {
    double a[4], b[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) a[m] = A.op(m);
#pragma unroll
    for (int q = 0; q < 4; ++q) b[q] = B.op(q);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[q], acc[m][q], 0, 0, 0);
  };
  const int64_t nfull = (r1 - r0) / 4;   // whole 4-row k-steps
  int64_t kk = 0;
  if (nfull >= 2 * D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      ld_step(d);
      __builtin_amdgcn_sched_barrier(0);   // the ring order of the loop (its vmcnt waits rely on it)
    }
    // steady state: every prefetched k-step lies inside the split, no branch between the loads;
    // the oldest step is consumed next, so vmcnt(NL' (D - 1)) suffices
    for (; kk + 2 * D <= nfull; kk += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        mma(ra[d], rb[d]);
        ld_step(d);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) mma(ra[d], rb[d]);
    kk += D;
  }
  for (; kk < nfull; ++kk) {   // the last < D whole k-steps
    ld_step(0);
    mma(ra[0], rb[0]);
  }
  if (r1 - r0 > 4 * nfull) {   // a partial last k-step: rows past r1 are zeros
    Op A, B;
#pragma unroll
    for (int l = 0; l < Op::NL; ++l) {
      A.v[l] = {};
      B.v[l] = {};
    }
    if (r0 + 4 * nfull + kr < r1) {
      A.load(pa);
      B.load(pb);
    }
    mma(A, B);
  }
  double* out = part + (int64_t)it * (PPLS_GQ * PPLS_GQ);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int b = Op::col(q, li);
#pragma unroll
      for (int g = 0; g < 4; ++g)   // f64 MFMA D map: row (lane >> 4) + 4 g, column lane & 15
        out[Op::col(m, kr + 4 * g) * PPLS_GQ + b] = acc[m][q][g];
    }
}

// Persistent: one workgroup per resident slot (4 independent waves); every wave takes work items
// from the queues (ppls_gram_next) until they are empty.  Each item's sums depend only on the item,
// so the result is the same bit for bit whichever wave runs it.
template <typename T>
__global__ __launch_bounds__(256, 2) void ppls_gram_mfma_kernel(const T* __restrict__ X, int ldx, int xcols,
                                                                 const T* __restrict__ Y, int ldy, int ycols, int p,
                                                                 int ntiles, int nsplit, int* __restrict__ queue,
                                                                 double* __restrict__ part) {
  // queue = [qoff (9) | counters (8, zeroed before the launch) | pad | row bounds (nsplit + 1 int64) | items]
  const int* qoff = queue;
  unsigned* cnt = (unsigned*)(queue + 9);
  const int64_t* bounds = (const int64_t*)(queue + 18);
  const int* items = queue + 18 + 2 * (nsplit + 1);
  const int g = blockIdx.x & 7, lane = threadIdx.x & 63;
  for (;;) {
    int it = 0;
    if (lane == 0) it = ppls_gram_next(cnt, qoff, items, g);
    it = __builtin_amdgcn_readfirstlane(it);
    if (it < 0) return;
    ppls_gram_wave_item<T>(X, ldx, xcols, Y, ldy, ycols, p, ntiles, it, bounds, part);
  }
}

// G (p x p column-major, full) = sum over the splits' quadrant partials: element (a, b) is read at
// (max, min), which lies in a computed quadrant, so G is exactly symmetric; elements in a zero
// padding column (never computed when their whole quadrant is padding) are 0.
__global__ void ppls_gram_finish_kernel(const double* __restrict__ part, int nsplit, int ntiles, PplsGramCols gc,
                                        double* __restrict__ G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int p = gc.p;
  const int64_t pp = (int64_t)p * p;
  if (e >= pp) return;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);
  const int hi = a > b ? a : b, lo = a > b ? b : a;
  double v = 0.0;
  if (ppls_gram_col_live(gc, hi) && ppls_gram_col_live(gc, lo)) {
    const int I = hi >> 7, J = lo >> 7, t = I * (I + 1) / 2 + J;
    const int quad = (((hi & 127) >> 6) << 1) | ((lo & 127) >> 6);
    const int64_t off = ((int64_t)t * 4 + quad) * (PPLS_GQ * PPLS_GQ) + (hi & 63) * PPLS_GQ + (lo & 63);
    const int64_t stride = (int64_t)ntiles * 4 * (PPLS_GQ * PPLS_GQ);
    for (int s = 0; s < nsplit; ++s) v += part[(int64_t)s * stride + off];
  }
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
  hipError_t e = f32 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<float>, 256, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<double>, 256, 0);
  return e == hipSuccess && occ > 0 ? occ : 1;
}

static int ppls_gram_live_quads(const PplsGramCols& gc) {
  const int ntiles = ppls_gram_tiles(gc.p);
  int w = 0;
  for (int t = 0; t < ntiles; ++t) {
    int I, J;
    ppls_gram_tile_of(t, &I, &J);
    for (int qd = 0; qd < 4; ++qd) w += ppls_gram_quad_live(gc, I, J, qd) ? 1 : 0;
  }
  return w;
}

// The row splits of a Gram over n rows: nsplit_req > 0 equal splits; 0 (auto) a guided schedule.
// Waves take items dynamically, split by split, so the run ends on the last split's items: each
// split holds about half the remaining work per wave slot (rows = W1 R / (2 slots) of the R rows
// left, W1 live quadrants per split), at most half of R, at least ~1 % of a slot's whole share
// (and 256 rows), so the first splits keep every wave busy and the last ones are short.  C3's S
// (W1 = 2,016 on 2,048 wave slots): 8 splits of 49 %, 26 %, 13 % ... of the rows; C3's X'X alone
// (W1 = 528): ~28 splits of 13 % of the remaining rows each; C5 (W1 ~ 14,000): 4.  Partials: 32 KB
// per live quadrant and split, kept under 4 GB (<= 64 splits).  bounds: nsplit + 1 row boundaries.
int ppls_gram_plan(int p, int xreal, int xcols, int yreal, int64_t n, int wave_slots, int nsplit_req, int64_t* bounds) {
  const PplsGramCols gc{p, xreal, xcols, xcols + yreal};
  const double w1 = (double)ppls_gram_live_quads(gc);
  if (nsplit_req > 0) {
    if (bounds)
      for (int s = 0; s <= nsplit_req; ++s) bounds[s] = n * s / nsplit_req;
    return nsplit_req;
  }
  const double slots = wave_slots > 0 ? (double)wave_slots : 1.0;
  int maxs = (int)(4.0e9 / (w1 * PPLS_GQ * PPLS_GQ * 8.0));
  maxs = maxs < 1 ? 1 : (maxs > 64 ? 64 : maxs);
  int64_t smin = (int64_t)(0.01 * w1 * (double)n / slots);
  if (smin < 256) smin = 256;
  int ns = 0;
  int64_t done = 0;
  if (bounds) bounds[0] = 0;
  while (done < n) {
    const int64_t R = n - done;
    int64_t sz = (int64_t)(w1 * (double)R / (2.0 * slots));
    if (sz > R / 2) sz = R / 2;
    if (sz < smin) sz = smin;
    if (R - sz < smin || ns + 1 >= maxs) sz = R;   // no sliver, and the last split allowed takes the rest
    done += sz;
    ++ns;
    if (bounds) bounds[ns] = done;
  }
  return ns < 1 ? 1 : ns;
}

int64_t ppls_gram_part_doubles(int p, int nsplit) {
  return (int64_t)nsplit * ppls_gram_tiles(p) * 4 * PPLS_GQ * PPLS_GQ;
}

int64_t ppls_gram_queue_ints(int p, int nsplit) { return 18 + 2 * (int64_t)(nsplit + 1) + (int64_t)ppls_gram_tiles(p) * 4 * nsplit; }

// The queues (device ints, ppls_gram_queue_ints): group g (blockIdx mod 8) gets the live quadrants
// of the tiles [g T / 8, (g + 1) T / 8) in every split, split by split (the large splits first, the
// run ends on the small ones); the row bounds ride along.  Synchronous (host staging); the launch
// resets the counters, so one prepared queue serves any number of launches of that shape.
hipError_t ppls_gram_queue_prepare(int* queue, int p, int xreal, int xcols, int yreal, int64_t n, int wave_slots,
                                   int nsplit_req, hipStream_t st) {
  const PplsGramCols gc{p, xreal, xcols, xcols + yreal};
  const int nsplit = ppls_gram_plan(p, xreal, xcols, yreal, n, wave_slots, nsplit_req, nullptr);
  const int ntiles = ppls_gram_tiles(p);
  std::vector<int> h((size_t)ppls_gram_queue_ints(p, nsplit), 0);
  ppls_gram_plan(p, xreal, xcols, yreal, n, wave_slots, nsplit_req, (int64_t*)(h.data() + 18));
  int* items = h.data() + 18 + 2 * (nsplit + 1);
  int w = 0;
  for (int g = 0; g < 8; ++g) {
    h[(size_t)g] = w;
    const int t0 = ntiles * g / 8, t1 = ntiles * (g + 1) / 8;
    for (int s = 0; s < nsplit; ++s)
      for (int t = t0; t < t1; ++t) {
        int I, J;
        ppls_gram_tile_of(t, &I, &J);
        for (int qd = 0; qd < 4; ++qd)
          if (ppls_gram_quad_live(gc, I, J, qd)) items[w++] = ((s * ntiles + t) << 2) | qd;
      }
  }
  h[8] = w;
  hipError_t e = hipMemcpyAsync(queue, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}

hipError_t ppls_launch_gram_joint(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int ycols,
                                  int yreal, int f32, int64_t n, int p, int nsplit, double* part, int* queue,
                                  hipStream_t st) {
  if (n <= 0 || p <= 0 || nsplit < 1 || !queue || xcols + ycols < 1 || xreal > xcols || yreal > ycols)
    return hipErrorInvalidValue;
  const int ev = f32 ? 4 : 2;
  if (xcols % ev || ycols % ev) return hipErrorInvalidValue;
  const int ntiles = ppls_gram_tiles(p);
  if ((int64_t)ntiles * 4 * nsplit > 0x7fffffff) return hipErrorInvalidValue;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = (cus * ppls_gram_occupancy(f32) + 7) / 8 * 8;
  hipError_t e = hipMemsetAsync(queue + 9, 0, 8 * sizeof(int), st);   // the queue counters
  if (e != hipSuccess) return e;
  if (f32)
    hipLaunchKernelGGL(ppls_gram_mfma_kernel<float>, dim3((unsigned)grid), dim3(256), 0, st, (const float*)X, ldx, xcols,
                       (const float*)Y, ldy, ycols, p, ntiles, nsplit, queue, part);
  else
    hipLaunchKernelGGL(ppls_gram_mfma_kernel<double>, dim3((unsigned)grid), dim3(256), 0, st, (const double*)X, ldx, xcols,
                       (const double*)Y, ldy, ycols, p, ntiles, nsplit, queue, part);
  return hipGetLastError();
}

hipError_t ppls_launch_gram(const void* X, int f32, int64_t n, int ld, int p, int nsplit, double* part, int* queue,
                            hipStream_t st) {
  return ppls_launch_gram_joint(X, ld, ld, p, nullptr, 0, 0, 0, f32, n, p, nsplit, part, queue, st);
}

hipError_t ppls_launch_gram_finish(const double* part, int nsplit, int p, int xreal, int xcols, int yreal, double* G,
                                   hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  const PplsGramCols gc{p, xreal, xcols, xcols + yreal};
  hipLaunchKernelGGL(ppls_gram_finish_kernel, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, part, nsplit,
                     ppls_gram_tiles(p), gc, G);
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
