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

// X'X on MFMA.  Work item L (blockIdx remapped so that each XCD -- blockIdx mod 8 -- gets a
// contiguous range of items, i.e. tiles that share column panels share an L2) = split s x
// lower tile t = (I, J), J <= I.  A wave owns a 64 x 64 sub-tile = 4 x 4 MFMA blocks (64 fp64
// accumulators per lane); per 4-row k-step it reads 4 A and 4 B operands from LDS (lane l: row
// l >> 4 of the step, column l & 15 of its block) -- both straight from the row-major panels, no
// transpose, since A[i][k] = X[k][i] and B[k][j] = X[k][j].  The next stage's global loads are in
// flight during the MFMAs; one barrier per 16-row stage.  Output: part[s][i p + j] for the tile's
// (i, j), i in block I >= block J (row-major of the lower blocks; coalesced over j).
//
// The column space is that of the joint matrix [X | Y] (ppls_xprod.hip's cross-product form of the
// EM iteration): column c is X[:, c] for c < xcols and Y[:, c - xcols] for c - xcols < ycols (zero
// beyond); xcols and ycols are multiples of the 16-B vector, so no load straddles the seam.  The
// Gram of X alone is xcols = ld, ycols = 0, p the output edge.
template <typename T>
__global__ __launch_bounds__(256, 2) void ppls_gram_mfma_kernel(const T* __restrict__ X, int ldx, int xcols,
                                                                 const T* __restrict__ Y, int ldy, int ycols,
                                                                 int64_t n, int p, int ntiles, int nsplit,
                                                                 int64_t work, double* __restrict__ part,
                                                                 int64_t part_stride) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int EV = 16 / sizeof(T);              // elements per 16-B load
  constexpr int VPR = PPLS_GT / EV;               // 16-B vectors per panel row
  constexpr int NV = PPLS_GK * VPR / 256;         // per thread per panel (fp64: 4, fp32: 2)
  __shared__ __attribute__((aligned(16))) double sm[2][2][PPLS_GK][PPLS_GLD];
  const int64_t per = gridDim.x >> 3;
  const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= work) return;
  const int s = (int)(L / ntiles), t = (int)(L - (int64_t)s * ntiles);
  int I = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  const int64_t r0 = n * s / nsplit, r1 = n * (s + 1) / nsplit;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int colA = I * PPLS_GT, colB = J * PPLS_GT;

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
        for (int q = 0; q < 4; ++q) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[q], acc[m][q], 0, 0, 0);
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
  hipError_t e = f32 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<float>, 256, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, ppls_gram_mfma_kernel<double>, 256, 0);
  return e == hipSuccess && occ > 0 ? occ : 1;
}

hipError_t ppls_launch_gram_joint(const void* X, int ldx, int xcols, const void* Y, int ldy, int ycols, int f32,
                                  int64_t n, int p, int nsplit, double* part, int64_t part_stride, hipStream_t st) {
  if (n <= 0 || p <= 0 || nsplit < 1 || xcols + ycols < 1) return hipErrorInvalidValue;
  const int ev = f32 ? 4 : 2;
  if (xcols % ev || ycols % ev) return hipErrorInvalidValue;
  const int ntiles = ppls_gram_tiles(p);
  const int64_t work = (int64_t)ntiles * nsplit;
  const int64_t grid = (work + 7) / 8 * 8;   // a multiple of 8: the XCD remap needs whole rounds
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  if (f32)
    hipLaunchKernelGGL(ppls_gram_mfma_kernel<float>, dim3((unsigned)grid), dim3(256), 0, st, (const float*)X, ldx,
                       xcols, (const float*)Y, ldy, ycols, n, p, ntiles, nsplit, work, part, part_stride);
  else
    hipLaunchKernelGGL(ppls_gram_mfma_kernel<double>, dim3((unsigned)grid), dim3(256), 0, st, (const double*)X, ldx,
                       xcols, (const double*)Y, ldy, ycols, n, p, ntiles, nsplit, work, part, part_stride);
  return hipGetLastError();
}

hipError_t ppls_launch_gram(const void* X, int f32, int64_t n, int ld, int p, int nsplit, double* part,
                            int64_t part_stride, hipStream_t st) {
  return ppls_launch_gram_joint(X, ld, ld, nullptr, 0, 0, f32, n, p, nsplit, part, part_stride, st);
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
