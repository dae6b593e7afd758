// ppls_kernels.hip -- MI355X (gfx950 / CDNA4) kernels for the PPLS_simult EM inner loop.
//
// One EM iteration = ONE pass over X and Y (the "sweep") + a deterministic reduction of the
// per-workgroup partials + a tiny on-device finalize (E-step moments, log-likelihood, M-step).
// Reference path replaced (paths relative to /root/reference):
//   Expect_M closed form  Package/PPLS/R/EM_W_multi.R:668-716   -> sweep + finalize
//   Maximiz_M             Package/PPLS/R/EM_W_multi.R:729-742   -> sweep (X'mu) + finalize (polar)
//   logl_W / loglC_fast   EM_W_multi.R:297-323, src/loglC.cpp:318-338 -> Gram of the next sweep
// Layout in HBM: X is n x ldx row-major fp64, Y is n x ldy row-major fp64 (ld even, pad = 0);
// W, C are kept padded column-major (ldx x r, ldy x r).  See DESIGN.md.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <tuple>
#include <type_traits>

#include "ppls_kernels.h"
#include "ppls_math.h"


// ============================================================================ Philox4x32-10
struct PplsU4 { uint32_t x, y, z, w; };

__host__ __device__ inline PplsU4 ppls_philox(PplsU4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    PplsU4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__global__ void ppls_philox_kernel(const PplsU4* __restrict__ ctr, int64_t count, uint64_t key,
                                   PplsU4* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) out[i] = ppls_philox(ctr[i], (uint32_t)key, (uint32_t)(key >> 32));
}

hipError_t ppls_launch_philox(const uint32_t* ctr, int64_t count, uint64_t key, uint32_t* out, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(ppls_philox_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st,
                     (const PplsU4*)ctr, count, key, (PplsU4*)out);
  return hipGetLastError();
}

// Two standard normals for (seed, stream m, pair index) -- Box-Muller on 53-bit uniforms.
__device__ inline void ppls_normal2(uint64_t seed, uint32_t m, uint64_t pair, double* z0, double* z1) {
  PplsU4 c = {(uint32_t)pair, (uint32_t)(pair >> 32), m, 0u};
  const PplsU4 r = ppls_philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint64_t a = (((uint64_t)r.y << 32) | r.x) >> 11;
  const uint64_t b = (((uint64_t)r.w << 32) | r.z) >> 11;
  const double u1 = ((double)a + 0.5) * 0x1p-53;
  const double u2 = ((double)b + 0.5) * 0x1p-53;
  const double rad = sqrt(-2.0 * log(u1));
  const double ang = 6.283185307179586 * u2;
  *z0 = rad * cos(ang);
  *z1 = rad * sin(ang);
}

__device__ inline double ppls_normal(uint64_t seed, uint32_t m, uint64_t e) {
  double z0, z1;
  ppls_normal2(seed, m, e >> 1, &z0, &z1);
  return (e & 1) ? z1 : z0;
}

// Latent scores of the simulC model (src/loglC.cpp:280-313, generalised to r > 1):
// T = N(0,1) diag(t), U = T diag(b) + sigH N(0,1).   TU: n_local x 2r row-major [T | U].
__global__ void ppls_gen_latent_kernel(int64_t n_local, int64_t row0, int r, PplsScalars truth,
                                       uint64_t seed, double* __restrict__ TU) {
  const int64_t e_loc = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e_loc >= n_local * r) return;
  const int64_t i = e_loc / r;
  const int k = (int)(e_loc - i * r);
  const uint64_t e = (uint64_t)(row0 + i) * (uint64_t)r + (uint64_t)k;
  const double T = truth.t[k] * ppls_normal(seed, 2u, e);
  const double U = T * truth.b[k] + truth.sigH * ppls_normal(seed, 3u, e);
  TU[i * 2 * r + k] = T;
  TU[i * 2 * r + r + k] = U;
}

// X = T W' + sigE E (stream 0) or Y = U C' + sigF F (stream 1).  One thread per output pair.
__global__ void ppls_gen_obs_kernel(int64_t n_local, int64_t row0, int p, int ld, int r,
                                    const double* __restrict__ L, int Loff, const double* __restrict__ Wt,
                                    double sig, uint64_t seed, uint32_t stream, double* __restrict__ out) {
  const int64_t npairs = ld >> 1;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= n_local * npairs) return;
  const int64_t i = gid / npairs;
  const int j = (int)(gid - i * npairs) * 2;
  const double* Li = L + i * 2 * r + Loff;
  double v[2] = {0.0, 0.0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int jj = j + h;
    if (jj < p) {
      double s = 0.0;
      for (int k = 0; k < r; ++k) s = fma(Li[k], Wt[(int64_t)k * p + jj], s);
      const uint64_t e = (uint64_t)(row0 + i) * (uint64_t)p + (uint64_t)jj;
      v[h] = s + sig * ppls_normal(seed, stream, e);
    }
  }
  *(double2*)(out + i * ld + j) = make_double2(v[0], v[1]);
}

// Column-major (n x p, ld n) -> padded row-major (n x ld).  32 x 32 LDS tiles.
__global__ void ppls_colmajor_to_rowmajor_kernel(const double* __restrict__ src, int64_t n, int p,
                                                 int ld, double* __restrict__ dst) {
  __shared__ double tile[32][33];
  const int64_t i0 = (int64_t)blockIdx.x * 32;
  const int j0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
  for (int jj = ty; jj < 32; jj += 8) {
    const int64_t i = i0 + tx;
    const int j = j0 + jj;
    tile[jj][tx] = (i < n && j < p) ? src[(int64_t)j * n + i] : 0.0;
  }
  __syncthreads();
  for (int ii = ty; ii < 32; ii += 8) {
    const int64_t i = i0 + ii;
    const int j = j0 + tx;
    if (i < n && j < ld) dst[i * ld + j] = (j < p) ? tile[tx][ii] : 0.0;
  }
}

// Padded row-major -> column-major (for returning data / mu to the caller).
__global__ void ppls_rowmajor_to_colmajor_kernel(const double* __restrict__ src, int64_t n, int p,
                                                 int ld, double* __restrict__ dst) {
  __shared__ double tile[32][33];
  const int64_t i0 = (int64_t)blockIdx.x * 32;
  const int j0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int ii = ty; ii < 32; ii += 8) {
    const int64_t i = i0 + ii;
    const int j = j0 + tx;
    tile[ii][tx] = (i < n && j < p) ? src[i * ld + j] : 0.0;
  }
  __syncthreads();
  for (int jj = ty; jj < 32; jj += 8) {
    const int64_t i = i0 + tx;
    const int j = j0 + jj;
    if (i < n && j < p) dst[(int64_t)j * n + i] = tile[tx][jj];
  }
}

// ============================================================================ reductions
__device__ inline double ppls_wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ||X P_0 .. P_{m-1}||^2 row by row, P_j = I - w_j w_j' (w_j: columns of Wd, p x m, ld p): the
// residual x P is formed before squaring, so there is no cancellation when X is nearly
// spanned by the w_j (sequential initialiser's rank-collapse test).  One wave per row; m <= 16.
template <typename T>
__global__ __launch_bounds__(256) void ppls_deflated_ssq_kernel(const T* __restrict__ X, int64_t n,
                                                                int ld, int p, const double* __restrict__ Wd,
                                                                int m, double* __restrict__ part) {
  __shared__ double sh[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc = 0.0;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave; row < n; row += (int64_t)gridDim.x * 4) {
    const T* x = X + row * ld;
    double d[16];
    for (int j = 0; j < m; ++j) {   // x P_0 .. P_{m-1}: apply P_0 first
      double s = 0.0;
      for (int i = lane; i < p; i += 64) {
        double v = x[i];
        for (int l = 0; l < j; ++l) v -= d[l] * Wd[(int64_t)l * p + i];
        s = fma(v, Wd[(int64_t)j * p + i], s);
      }
      d[j] = ppls_wave_sum(s);
    }
    double s = 0.0;
    for (int i = lane; i < p; i += 64) {
      double v = x[i];
      for (int l = 0; l < m; ++l) v -= d[l] * Wd[(int64_t)l * p + i];
      s = fma(v, v, s);
    }
    acc += ppls_wave_sum(s);
  }
  if (lane == 0) sh[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// Sum of squares of a contiguous buffer; per-block partials (deterministic two-stage).
__global__ void ppls_sumsq_partial_kernel(const double* __restrict__ a, int64_t len,
                                          double* __restrict__ part) {
  __shared__ double sh[16];
  double s = 0.0;
  const int64_t n2 = len >> 1;
  const double2* a2 = (const double2*)a;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double2 v = a2[i];
    s = fma(v.x, v.x, s);
    s = fma(v.y, v.y, s);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (len & 1)) s = fma(a[len - 1], a[len - 1], s);
  s = ppls_wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sh[w];
    part[blockIdx.x] = t;
  }
}

// fp32-storage helpers: sum of squares in fp64, and element conversions.
__global__ void ppls_sumsq_f32_kernel(const float* __restrict__ a, int64_t len, double* __restrict__ part) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = a[i];
    s = fma(v, v, s);
  }
  s = ppls_wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sh[w];
    part[blockIdx.x] = t;
  }
}

template <typename TI, typename TO>
__global__ void ppls_convert_kernel(const TI* __restrict__ src, TO* __restrict__ dst, int64_t len) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (TO)src[i];
}


// out[j] (+)= sum_g part[g*ld + j], fixed order -> deterministic.
__global__ void ppls_reduce_partials_kernel(const double* __restrict__ part, int ngroups, int64_t ld,
                                            int64_t len, double* __restrict__ out, int accumulate,
    const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= len) return;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int g = 0;
  for (; g + 8 <= ngroups; g += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(int64_t)(g + u) * ld + j];
  }
  for (int u = 0; g < ngroups; ++g, ++u) s[u] += part[(int64_t)g * ld + j];
  const double t = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  out[j] = accumulate ? out[j] + t : t;
}

// One-launch fixed-order reduction: out[j] (+)= sum_g part[g*ld + j].  A 256-thread block owns 64
// consecutive j (a wave reads 512 contiguous bytes per group) and splits the groups over 4 slices
// (slice s: g = s, s+4, ...), each with 8 accumulators so 8 loads per thread are in flight; the
// slices are added in slice order through LDS -> deterministic for a given ngroups.
__global__ __launch_bounds__(256) void ppls_reduce_fused_kernel(const double* __restrict__ part, int ngroups,
                                                                int64_t ld, int64_t len, double* __restrict__ out,
                                                                int accumulate, const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  __shared__ double sh[4][64];
  const int c = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int64_t j = (int64_t)blockIdx.x * 64 + c;
  double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (j < len) {
    int g = sl;
    for (; g + 28 < ngroups; g += 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] += part[(int64_t)(g + 4 * u) * ld + j];
    }
    for (int u = 0; g < ngroups; g += 4, ++u) a[u] += part[(int64_t)g * ld + j];
  }
  sh[sl][c] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (sl == 0 && j < len) {
    const double t = (sh[0][c] + sh[1][c]) + (sh[2][c] + sh[3][c]);
    out[j] = accumulate ? out[j] + t : t;
  }
}

#include "ppls_device.h"

// ============================================================================ split sweep
// One workgroup (NT threads, occupancy-sized grid) owns a contiguous block of rows.  Column
// ownership is split by matrix: threads [0, NT/2) own NSH column pairs of X, threads [NT/2, NT)
// own NSH pairs of Y, for the whole sweep, and keep W (or C) and the X'mu_T (or Y'mu_U)
// accumulators for them in VGPRs.  Rows stream HBM -> LDS through a ring of SLOTS row slots filled
// by LDS-DMA (global_load_lds_dwordx4; the first ceil(nch/CPW) waves copy CPW 1-KiB chunks of
// every row, so the steady-state vmcnt is a compile-time immediate).  The loop handles RP rows
// per step, software-pipelined, ONE workgroup barrier per step.  A wave's partial dots are then
// Xw only or Yc only, so the per-row wave reduce-scatter handles R*RP values (not 2R*RP) and each
// wave broadcasts only the mu it uses (mu_T for X waves, mu_U for Y waves).
//   PIPE = true : step g computes group g+1's dots before group g's update (x of both in VGPRs)
//   PIPE = false: step g applies group g's update, then computes group g+1's dots (one x set)
template <int R, int NSH, int NT, int RP, bool PIPE, int SLOTS, int CPW>
__global__ __launch_bounds__(NT, 2 * NT / 512) void ppls_sweep_split_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, const PplsScalars* __restrict__ sc,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu, int nt_loads,
    const int* __restrict__ stop, long long* __restrict__ trace, const int64_t* __restrict__ row_bounds,
    const int* __restrict__ wg_seg) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  static_assert(SLOTS >= 2 * RP, "ring must hold the group being read and the group in flight");
  // diagnostics (set_option "strace"): per workgroup wall-clock stamps at entry, after the ring
  // prologue, after the row loop and after the partial write-out
  long long* tr = (trace && threadIdx.x == 0) ? trace + 4 * blockIdx.x : nullptr;
  if (tr) tr[0] = (long long)wall_clock64();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int V = R * RP;                           // partial dots per thread per step
  constexpr int VP = V + (V & 1);                     // reduce-scatter scratch
  constexpr int NWAVES = NT / 64;
  constexpr int HT = NT / 2;                          // threads per matrix
  constexpr int AHEAD = SLOTS / RP - 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool isx = wave < NWAVES / 2;                 // wave-uniform
  const int th = tid - (isx ? 0 : HT);
  const int nchx = (ldx * 8 + 1023) >> 10, nchy = (ldy * 8 + 1023) >> 10;
  const int nch = nchx + nchy;
  const int slot_bytes = nch << 10;
  const bool dma_wave = wave * CPW < nch;
  double* red = (double*)(smem + (size_t)SLOTS * slot_bytes);          // [2][NWAVES][V]
  double* bc = red + 2 * NWAVES * V + wave * (2 * V);                 // per wave: [Xw Yc] rows
  double* cf = red + 2 * NWAVES * V + NWAVES * 2 * V;                 // alpha | beta | gamma | delta
  const int64_t g = blockIdx.x, G = gridDim.x;
  // contiguous row block: the even split, or the calibrated per-XCD-weighted one (ppls_capi.cpp)
  const int64_t rb = row_bounds ? row_bounds[g] : n_local * g / G;
  const int64_t re = row_bounds ? row_bounds[g + 1] : n_local * (g + 1) / G;
  const int nrows = (int)(re - rb);
  const int ngroups = (nrows + RP - 1) / RP;
  const int np = isx ? (ldx >> 1) : (ldy >> 1);
  const int ld = isx ? ldx : ldy;
  const double* Wm = isx ? Wp : Cp;
  const int xoff = isx ? 0 : nchx * 1024;             // byte offset of this matrix in a slot

  bool vs[NSH];
  double2 w[NSH][R], acc[NSH][R];
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    const int pp = th + s * HT;
    vs[s] = pp < np;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      w[s][k] = vs[s] ? *(const double2*)(Wm + (int64_t)k * ld + 2 * pp) : make_double2(0.0, 0.0);
      acc[s][k] = make_double2(0.0, 0.0);
    }
  }
  const int mj = lane / R, mk = lane - (lane / R) * R;
  if (tid < R) {
    // segmented sweeps (meta_PPLSi's populations): workgroup g's rows lie in one population and use
    // that population's scalars sc[wg_seg[g]]
    const PplsScalars* scg = wg_seg ? sc + wg_seg[g] : sc;
    cf[tid] = scg->alpha[tid];
    cf[R + tid] = scg->beta[tid];
    cf[2 * R + tid] = scg->gamma[tid];
    cf[3 * R + tid] = scg->delta[tid];
  }
  const int ge = wave * 64 + lane;
  int gi = 0, gj = 0;
  const bool has_g = ge < R * (2 * R + 1);
  if (has_g) {
    int e = ge, j = 0;
    while (e >= j + 1) { e -= j + 1; ++j; }
    gi = e;
    gj = j;
  }
  double gacc = 0.0;
  // no wait here: the W / C loads (issued first) complete before the ring prologue's first group,
  // which the prologue waits for, so their latency overlaps the first rows' DMA
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // chunk j of this wave: matrix (wave-uniform) and the lane's clamped byte offset in the row, fixed
  // for the sweep, so a row's copies need only its scalar base address (saddr-form DMA)
  uint32_t coff[CPW];
  bool cinx[CPW];
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int ch = min(wave * CPW + j, nch - 1);
    cinx[j] = ch < nchx;
    coff[j] = cinx[j] ? (uint32_t)min(ch * 1024 + lane * 16, ldx * 8 - 16)
                      : (uint32_t)min((ch - nchx) * 1024 + lane * 16, ldy * 8 - 16);
  }
  // nt: the non-temporal load policy (nt_loads), a compile-time choice per copy of the loop
  auto issue_row = [&](int i, auto nt) {
    if (!dma_wave) return;
    const int64_t row = rb + i;
    const char* xr = (const char*)(X + row * (int64_t)ldx);
    const char* yr = (const char*)(Y + row * (int64_t)ldy);
    const uint32_t sb = lds_base + (uint32_t)((i % SLOTS) * slot_bytes);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int ch = min(wave * CPW + j, nch - 1);
      const char* base = cinx[j] ? xr : yr;
      if constexpr (decltype(nt)::value) ppls_dma16s_nt(base, coff[j], sb + (uint32_t)(ch * 1024));
      else ppls_dma16s(base, coff[j], sb + (uint32_t)(ch * 1024));
    }
  };
  auto issue_group = [&](int grp, auto nt) {
    for (int j = 0; j < RP; ++j)
      if (grp * RP + j < nrows) issue_row(grp * RP + j, nt);
  };
  // FULL: this thread's NSH column pairs all lie inside the matrix's 1-KiB-aligned part of a slot,
  // which the DMA fills completely (lanes past the row's end copy its last 16 B), so the reads need
  // no guard: a pair past the row reads finite data and meets zero weights (w = 0 there)
  auto load_x = [&](int grp, double2 (&xv)[RP][NSH], auto full) {
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const int row = min(grp * RP + j, nrows - 1);
      const char* sb = smem + (size_t)(row % SLOTS) * slot_bytes + xoff;
#pragma unroll
      for (int s = 0; s < NSH; ++s) {
        if constexpr (decltype(full)::value) xv[j][s] = *(const double2*)(sb + (th + s * HT) * 16);
        else xv[j][s] = vs[s] ? *(const double2*)(sb + (th + s * HT) * 16) : make_double2(0.0, 0.0);
      }
    }
  };
  // partial dots of group grp (x already loaded) -> reduce-scatter -> red[grp & 1]
  auto dots = [&](int grp, const double2 (&xv)[RP][NSH]) {
    double v[VP];
#pragma unroll
    for (int j = 0; j < RP; ++j)
#pragma unroll
      for (int k = 0; k < R; ++k) {
        double sx = 0.0;
#pragma unroll
        for (int s = 0; s < NSH; ++s) {
          sx = fma(xv[j][s].x, w[s][k].x, sx);
          sx = fma(xv[j][s].y, w[s][k].y, sx);
        }
        v[j * R + k] = sx;
      }
    if constexpr (VP > V) v[V] = 0.0;
    int idx = 0;
    bool canon = true;
    ppls_rs<V, 0, VP>(v, lane, idx, canon);
    if (canon && idx < V) red[((grp & 1) * NWAVES + wave) * V + idx] = v[0];
  };
  // cross-wave sums of group gg: lane m < R*RP -> (a, b, mu_T, mu_U) of row m/R, comp m%R
  auto zsum = [&](int gg, double& mta, double& mua) {
    if (lane < R * RP) {
      const double* rr = red + (gg & 1) * NWAVES * V;
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int ww = 0; ww < NWAVES / 2; ++ww) {
        a += rr[ww * V + lane];
        b += rr[(ww + NWAVES / 2) * V + lane];
      }
      bc[mj * 2 * R + mk] = a;
      bc[mj * 2 * R + R + mk] = b;
      mta = cf[mk] * a + cf[R + mk] * b;               // mu_T (EM_W_multi.R:691-692)
      mua = cf[2 * R + mk] * a + cf[3 * R + mk] * b;   // mu_U (EM_W_multi.R:693-694)
    }
  };
  auto update = [&](int gg, double mta, double mua, const double2 (&xv)[RP][NSH]) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's bc writes are visible
    const double msel = isx ? mta : mua;                   // wave-uniform choice
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      if (gg * RP + j >= nrows) break;
      if (has_g) gacc = fma(bc[j * 2 * R + gi], bc[j * 2 * R + gj], gacc);
      double m[R];
#pragma unroll
      for (int k = 0; k < R; ++k)
        m[k] = __hiloint2double(__builtin_amdgcn_readlane((int)__double2hiint(msel), j * R + k),
                                __builtin_amdgcn_readlane((int)__double2loint(msel), j * R + k));
      if (write_mu && (wave == 0 || wave == NWAVES / 2) && lane < R) {
        const int64_t row = rb + gg * RP + j;
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k)
          if (lane == k) a = m[k];
        mu[(int64_t)((isx ? 0 : R) + lane) * n_local + row] = a;
      }
#pragma unroll
      for (int s = 0; s < NSH; ++s)
#pragma unroll
        for (int k = 0; k < R; ++k) {
          acc[s][k].x = fma(xv[j][s].x, m[k], acc[s][k].x);
          acc[s][k].y = fma(xv[j][s].y, m[k], acc[s][k].y);
        }
    }
  };

  auto run = [&](auto full, auto nt) {
    if (ngroups > 0) {
      const int npro = min(SLOTS, nrows);
      for (int i = 0; i < npro; ++i) issue_row(i, nt);
      if (write_mu) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else ppls_wait_vmcnt((npro - min(RP, nrows)) * CPW);
      ppls_lds_barrier();
      if (tr) tr[1] = (long long)wall_clock64();
      double2 xc[RP][NSH] = {};
      load_x(0, xc, full);
      dots(0, xc);
      for (int gg = 0; gg < ngroups; ++gg) {
        if (write_mu) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else if ((gg + 2 + AHEAD) * RP <= nrows && gg >= 1) {
          if constexpr (AHEAD * RP * CPW == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          else ppls_wait_vmcnt(AHEAD * RP * CPW);
        } else {
          const int last_issued = min(gg >= 1 ? (gg - 1) * RP + SLOTS + RP - 1 : SLOTS - 1, nrows - 1);
          ppls_wait_vmcnt(max(0, last_issued - ((gg + 2) * RP - 1)) * CPW);
        }
        ppls_lds_barrier();   // red[gg&1] complete, group gg+1 landed, slots of group gg free
        if (gg * RP + SLOTS < nrows) issue_group(gg + SLOTS / RP, nt);
        double mta = 0.0, mua = 0.0;
        zsum(gg, mta, mua);
        if constexpr (PIPE) {
          double2 xn[RP][NSH] = {};
          if (gg + 1 < ngroups) {
            load_x(gg + 1, xn, full);
            dots(gg + 1, xn);
          }
          update(gg, mta, mua, xc);
  #pragma unroll
          for (int j = 0; j < RP; ++j)
  #pragma unroll
            for (int s = 0; s < NSH; ++s) xc[j][s] = xn[j][s];
        } else {
          update(gg, mta, mua, xc);
          if (gg + 1 < ngroups) {
            load_x(gg + 1, xc, full);
            dots(gg + 1, xc);
          }
        }
      }
    }
  };
  const bool full = NSH * HT * 16 <= nchx * 1024 && NSH * HT * 16 <= nchy * 1024;
  if (nt_loads) {
    if (full) run(std::true_type{}, std::true_type{});
    else run(std::false_type{}, std::true_type{});
  } else {
    if (full) run(std::true_type{}, std::false_type{});
    else run(std::false_type{}, std::false_type{});
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tr) tr[2] = (long long)wall_clock64();
  double* pg = part + g * part_ld;
  double* po = pg + (isx ? 0 : (int64_t)R * ldx);
#pragma unroll
  for (int s = 0; s < NSH; ++s) {
    const int pp = th + s * HT;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (vs[s]) *(double2*)(po + (int64_t)k * ld + 2 * pp) = acc[s][k];
  }
  if (has_g) {
    double* G2 = pg + (int64_t)R * ldx + (int64_t)R * ldy;
    G2[gj * 2 * R + gi] = gacc;
    G2[gi * 2 * R + gj] = gacc;
  }
  if (trace) {
    __syncthreads();   // every thread's stores issued
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tr) tr[3] = (long long)wall_clock64();
  }
}

// ============================================================================ Maximiz_M on given moments
// X'mu_T / Y'mu_U partials over a chunk of rows from caller-supplied moments Z = [mu_T | mu_U]
// (ppls_mstep: Maximiz_M, EM_W_multi.R:732-733), one thread per column pair; the Gram partial of
// the chunk is computed by the block with blockIdx.x == 0.
__global__ __launch_bounds__(256) void ppls_acc_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Z, int r, const PplsScalars* __restrict__ sc, int64_t rows_per_chunk,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu,
    const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  const int chunk = blockIdx.y;
  const int64_t r0 = (int64_t)chunk * rows_per_chunk;
  const int64_t r1 = min(n_local, r0 + rows_per_chunk);
  const int npx = ldx >> 1, npy = ldy >> 1;
  const int pidx = blockIdx.x * blockDim.x + threadIdx.x;   // pair index over [X pairs | Y pairs]
  double* pg = part + (int64_t)chunk * part_ld;
  const int V = 2 * r;
  if (pidx < npx + npy) {
    const bool isx = pidx < npx;
    const int pp = isx ? pidx : pidx - npx;
    double2 acc[PPLS_RMAX];
    for (int k = 0; k < r; ++k) acc[k] = make_double2(0.0, 0.0);
    const double* base = isx ? X : Y;
    const int ld = isx ? ldx : ldy;
    for (int64_t row = r0; row < r1; ++row) {
      const double2 x = *(const double2*)(base + row * ld + 2 * pp);
      const double* zr = Z + row * V;
      for (int k = 0; k < r; ++k) {
        const double m = isx ? (sc->alpha[k] * zr[k] + sc->beta[k] * zr[r + k])
                             : (sc->gamma[k] * zr[k] + sc->delta[k] * zr[r + k]);
        acc[k].x = fma(x.x, m, acc[k].x);
        acc[k].y = fma(x.y, m, acc[k].y);
      }
    }
    for (int k = 0; k < r; ++k) {
      if (isx) *(double2*)(pg + (int64_t)k * ldx + 2 * pp) = acc[k];
      else *(double2*)(pg + (int64_t)r * ldx + (int64_t)k * ldy + 2 * pp) = acc[k];
    }
  }
  if (blockIdx.x == 0) {
    double* G2 = pg + (int64_t)r * ldx + (int64_t)r * ldy;
    for (int e = threadIdx.x; e < V * V; e += blockDim.x) {
      const int i = e % V, j = e / V;
      double s = 0.0;
      for (int64_t row = r0; row < r1; ++row) s = fma(Z[row * V + i], Z[row * V + j], s);
      G2[e] = s;
    }
    if (write_mu) {
      for (int64_t row = r0 + threadIdx.x; row < r1; row += blockDim.x) {
        const double* zr = Z + row * V;
        for (int k = 0; k < r; ++k) {
          mu[(int64_t)k * n_local + row] = sc->alpha[k] * zr[k] + sc->beta[k] * zr[r + k];
          mu[(int64_t)(r + k) * n_local + row] = sc->gamma[k] * zr[k] + sc->delta[k] * zr[r + k];
        }
      }
    }
  }
}

// ============================================================================ panel sweep (wide p)
// When p r is too large for per-thread column ownership (C5: p = 1e4, r = 10 -> 1e5 accumulators
// per matrix), the sweep is two GEMM-shaped passes over X and Y:
//   dots: Z_i = [x_i W | y_i C | mu_T,i | mu_U,i] (n x 4R fp64) -- 64-row tiles per workgroup,
//         W staged transposed in LDS, 16-B coalesced loads of X, fp64 FMA, 16-lane DPP sums;
//   acc : [X' mu_T | Y' mu_U] partials per row chunk -- each thread owns one 16-B column vector
//         with R fp64 accumulators per element and streams the chunk's rows; mu_T / mu_U are
//         wave-uniform (scalar loads); the first column tile also accumulates the 2R x 2R Gram
//         of [Xw Yc].
// T is the storage type of X, Y (double or float); arithmetic is fp64.  Algorithmic bytes:
// 2 sizeof(T) n (p + q) (two HBM passes) + 64 R n (Z written and read twice).
__device__ __forceinline__ double ppls_group16_sum(double v) {
  v += ppls_dpp_partner<5>(v);   // quad xor 1
  v += ppls_dpp_partner<4>(v);   // quad xor 2
  v += ppls_dpp_partner<3>(v);   // half-row mirror: lane l <-> 7 - l
  v += ppls_dpp_partner<2>(v);   // row mirror: lane l <-> 15 - l
  return v;
}

template <typename T>
struct PplsVec16 {   // one 16-B load of T
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

template <typename T, bool NT = false>
__device__ __forceinline__ PplsVec16<T> ppls_load16(const T* p) {
  PplsVec16<T> r;
  if constexpr (sizeof(T) == 8) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v d = NT ? __builtin_nontemporal_load((const d2v*)p) : *(const d2v*)p;
    r.v[0] = d.x;
    r.v[1] = d.y;
  } else {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v f = NT ? __builtin_nontemporal_load((const f4v*)p) : *(const f4v*)p;
    r.v[0] = f.x;
    r.v[1] = f.y;
    r.v[2] = f.z;
    r.v[3] = f.w;
  }
  return r;
}

#define PPLS_PANEL_ROWS 64

// MFMA dots (default panel dots): Z_tile = X_tile (16 rows x K) . W (K x 16, R columns used) on
// v_mfma_f64_16x16x4_f64.  Each wave owns 32 rows (two 16-row blocks sharing the B operand) and
// walks the columns in 128-B tiles: a tile (32 rows x 128 B) is loaded with 16-B coalesced loads,
// transposed through padded per-wave LDS, and each lane reads its A operands for several MFMA
// steps with one ds_read_b128 -- the k order is permuted so that lane group g = lane >> 4 owns the
// contiguous columns [g KT/4, (g+1) KT/4) of the tile, step s using column g KT/4 + s; the B
// operand (lane l: W[that column][l & 15]) is a plain per-lane load of the transposed, zero-padded
// W.  The next tile's global loads are in flight during the MFMAs.  Result lane map (f64 MFMA):
// row (l >> 4) + 4 reg, component l & 15 -- the same for the X and the Y product, so mu_T/mu_U are
// formed in registers.  KS = 2 splits each row tile's columns over a wave pair of the workgroup
// (the second half's dot sums are added to the first's through LDS, in that fixed order): for
// shards with fewer row tiles than resident wave slots (C5's 8-GPU share: 977 tiles of 64 rows for
// 2,048 slots), which would otherwise run one wave per SIMD.
template <typename T, int R, int NB, int KS, bool NT>
__global__ __launch_bounds__(256) void ppls_panel_mfmadots_kernel(
    const T* __restrict__ X, const T* __restrict__ Y, int64_t n, int ldx, int ldy, int px, int py,
    const double* __restrict__ Wt, const double* __restrict__ Ct, const PplsScalars* __restrict__ sc,
    double* __restrict__ Z, double* __restrict__ mu,
    const int* __restrict__ stop, const int64_t* __restrict__ seg_ends, int nseg) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  // Round 3 at the C5 share (compile-time ablations of an experiment build: no MFMAs, no X loads,
  // no B loads -- every variant ran 574-591 us, profiles/r3_dots_ablate_c5s.txt): the per-tile LDS
  // transpose and its waits bound the kernel, not the MFMAs or either load stream; yet loading the
  // MFMA operands straight from global memory (16 rows x 16 B per load instruction, no LDS) was
  // slower still, 616 vs 560 us and 4.53 vs 3.92 ms at C5 (profiles/r3_dots_direct_ab.txt): the
  // 16-row scatter costs more in the vector-memory pipeline than the transpose does in LDS.
  typedef double d4 __attribute__((ext_vector_type(4)));
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int ES = (int)sizeof(T);
  constexpr int KT = 128 / ES;        // columns per tile
  constexpr int KQ = KT / 4;          // MFMA steps per tile (columns per lane group)
  constexpr int RB = 16 * NB;         // rows per wave: NB 16-row blocks sharing the B operand
  constexpr int NL = RB / 8;          // 16-B loads per lane per tile
  constexpr int RS = 144;             // padded LDS row stride (bytes)
  constexpr int V4 = 4 * R;
  static_assert(R <= 16, "one 16-wide MFMA tile of components");
  __shared__ __attribute__((aligned(16))) char lds[4 * 2 * RB * RS];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: scalar branches below
  const int i16 = lane & 15, kq = lane >> 4;
  const int lrow = lane >> 3, lchunk = lane & 7;   // loading: 8 lanes per row, 8 rows per load
  const int comp = i16 < R ? i16 : 0;
  const double al = sc->alpha[comp], be = sc->beta[comp], ga = sc->gamma[comp], de = sc->delta[comp];
  static_assert(KS == 1 || KS == 2, "one wave or a wave pair per row tile");
  static_assert(2 * NB * 4 * 64 * 8 <= 2 * RB * RS, "a wave's dot sums fit its transpose buffers");
  constexpr int TPW = 4 / KS;                          // row tiles per workgroup pass
  const int part = wave % KS;                          // this wave's share of the columns
  const int64_t ntiles = (n + RB - 1) / RB;
  // the trip count is uniform over the workgroup (the pair combine has workgroup barriers)
  for (int64_t tb = (int64_t)blockIdx.x * TPW; tb < ntiles; tb += (int64_t)gridDim.x * TPW) {
    const int64_t t = tb + wave / KS;
    const bool active = t < ntiles;
    const int64_t row0 = t * RB;
    d4 res[2][NB];   // [mat][block]
    if (active) {
#pragma unroll
    for (int mat = 0; mat < 2; ++mat) {
      const T* M = mat ? Y : X;
      const int ld = mat ? ldy : ldx, pc = mat ? py : px;
      const double* Wm = mat ? Ct : Wt;
      d4 acc[NB];
#pragma unroll
      for (int bk = 0; bk < NB; ++bk) acc[bk] = d4{0.0, 0.0, 0.0, 0.0};
      const T* src[NL];
#pragma unroll
      for (int u = 0; u < NL; ++u) {
        int64_t rr = row0 + lrow + 8 * u;
        if (rr >= n) rr = n - 1;
        src[u] = M + rr * ld + lchunk * (16 / ES);
      }
      // the tiles holding the pc data columns (row padding beyond them is zero and skipped, so a
      // padded layout sums the same tiles in the same order as a 16-B-row one), split over the pair
      const int ntc = (pc + KT - 1) / KT;
      const int tc0 = ntc * part / KS, tc1 = ntc * (part + 1) / KS;   // this wave's column tiles
      // Loads are unconditional (no exec-mask branches, so the waitcnts stay precise): a partial
      // last tile reads past the row end into the next row (or the allocation's slack after the
      // last row), which meets the zero rows of Wt beyond ld and adds exactly 0; prefetches past
      // the last tile re-read it.  Issue order per tile: this tile's B operands, then the next
      // tile's X loads, so the MFMAs wait only for B while the next tile streams in.
      f4 xa[NL];
      // NT (the sweep's nt policy: data larger than the MALL): non-temporal X/Y loads -- round 5,
      // steady state at C5: 7.24 vs 7.33-7.36 ms per iteration over 6 interleaved pairs, the 8-GPU
      // share even (profiles/r5_dots_nt_ab.txt; round 2's isolated-launch A/B had them 16 % slower)
      auto ld4 = [&](const T* p) -> f4 {
        if constexpr (NT) return __builtin_nontemporal_load((const f4*)p);
        else return *(const f4*)p;
      };
      auto load_tile = [&](int tc, f4 (&b)[NL]) {
        const int c = tc < tc1 ? tc : tc1 - 1;   // a prefetch past the range re-reads its last tile
#pragma unroll
        for (int u = 0; u < NL; ++u) b[u] = ld4(src[u] + c * KT);
      };
      // B operand of lane l at k-step s: W[tile column kq KQ + s][i16] (Wt: 16 zero-padded columns,
      // k-steps in pairs: one 16-B load per two steps)
      const double* wb0 = Wm + (int64_t)kq * KQ * 16 + 2 * i16;   // pair layout (transpose kernel)
      auto step = [&](int tc, f4 (&b)[NL]) {
        char* wl = lds + (wave * 2 + (tc & 1)) * RB * RS;
#pragma unroll
        for (int u = 0; u < NL; ++u) *(f4*)(wl + (lrow + 8 * u) * RS + lchunk * 16) = b[u];
        asm volatile("" ::: "memory");   // keep the loads below after the stores (buf is reused)
        double bw[KQ];
        const double* wb = wb0 + (int64_t)tc * KT * 16;
#pragma unroll
        for (int s2 = 0; s2 < KQ; s2 += 2) {
          const double2 w2 = *(const double2*)(wb + s2 * 16);
          bw[s2] = w2.x;
          bw[s2 + 1] = w2.y;
        }
        asm volatile("" ::: "memory");   // B before the next tiles' X in the vmcnt order
        load_tile(tc + 1, b);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // A operands: rows 16 bk + i16, columns [kq KQ, kq KQ + KQ) of the tile
#pragma unroll
        for (int bk = 0; bk < NB; ++bk) {
          T a[KQ];
#pragma unroll
          for (int h = 0; h < KQ * ES / 16; ++h) {
            const float4 v = *(const float4*)(wl + (16 * bk + i16) * RS + kq * KQ * ES + h * 16);
            const T* pv = (const T*)&v;
#pragma unroll
            for (int u = 0; u < 16 / ES; ++u) a[h * (16 / ES) + u] = pv[u];
          }
#pragma unroll
          for (int s2 = 0; s2 < KQ; ++s2)
            acc[bk] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)a[s2], bw[s2], acc[bk], 0, 0, 0);
        }
      };
      if (tc0 < tc1) {
        load_tile(tc0, xa);
        for (int tc = tc0; tc < tc1; ++tc) step(tc, xa);
      }
#pragma unroll
      for (int bk = 0; bk < NB; ++bk) res[mat][bk] = acc[bk];
    }
    }   // active
    if constexpr (KS == 2) {
      // the second wave of the pair hands its sums over through its own (now idle) transpose buffer
      double* cb = (double*)(lds + (wave | 1) * 2 * RB * RS);
      if (active && part == 1) {
#pragma unroll
        for (int mat = 0; mat < 2; ++mat)
#pragma unroll
          for (int bk = 0; bk < NB; ++bk)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) cb[((mat * NB + bk) * 4 + reg) * 64 + lane] = res[mat][bk][reg];
      }
      __syncthreads();
      if (active && part == 0) {
#pragma unroll
        for (int mat = 0; mat < 2; ++mat)
#pragma unroll
          for (int bk = 0; bk < NB; ++bk)
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) res[mat][bk][reg] += cb[((mat * NB + bk) * 4 + reg) * 64 + lane];
      }
      __syncthreads();   // the buffer is the partner's again
    }
    if (active && part == 0 && i16 < R) {
      // segmented (meta_PPLSi): each row's population scalars; the lane's rows increase, so its
      // segment index only moves forward from the tile's first row's (a wave-uniform binary search)
      int sj = 0;
      if (seg_ends) {
        int lo = 0, hi = nseg - 1;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (row0 < seg_ends[mid]) hi = mid;
          else lo = mid + 1;
        }
        sj = lo;
      }
#pragma unroll
      for (int blk = 0; blk < NB; ++blk)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int64_t row = row0 + 16 * blk + kq + 4 * reg;
          if (row >= n) continue;
          double cal = al, cbe = be, cga = ga, cde = de;
          if (seg_ends) {
            while (sj + 1 < nseg && row >= seg_ends[sj]) ++sj;
            const PplsScalars* ss = sc + sj;
            cal = ss->alpha[comp];
            cbe = ss->beta[comp];
            cga = ss->gamma[comp];
            cde = ss->delta[comp];
          }
          const double a = res[0][blk][reg], bb = res[1][blk][reg];
          const double mt = cal * a + cbe * bb, mu_u = cga * a + cde * bb;
          double* zr = Z + row * V4;
          zr[i16] = a;
          zr[R + i16] = bb;
          zr[2 * R + i16] = mt;
          zr[3 * R + i16] = mu_u;
          if (mu) {
            mu[(int64_t)i16 * n + row] = mt;
            mu[(int64_t)(R + i16) * n + row] = mu_u;
          }
        }
    }
  }
}

// W (ldx x r, column-major) -> Wt (ldxp x rs: rows >= ldx and columns >= r zero, pair layout below); C alike.
__global__ void ppls_transpose_wc_kernel(const double* __restrict__ W, const double* __restrict__ C,
                                         int ldx, int ldy, int ldxp, int ldyp, int r, int rs, double* __restrict__ Wt,
                                         double* __restrict__ Ct,
    const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nx = (int64_t)ldxp * rs;
  // pair layout: rows 2m, 2m + 1 interleaved per component, element (i, k) at
  // (i >> 1) * 2 rs + 2 k + (i & 1), so one 16-B load gives a lane two consecutive k-steps
  if (e < nx) {
    const int i = (int)(e / rs), k = (int)(e % rs);
    Wt[(int64_t)(i >> 1) * 2 * rs + 2 * k + (i & 1)] = (i < ldx && k < r) ? W[(int64_t)k * ldx + i] : 0.0;
  } else if (e < nx + (int64_t)ldyp * rs) {
    const int64_t f = e - nx;
    const int i = (int)(f / rs), k = (int)(f % rs);
    Ct[(int64_t)(i >> 1) * 2 * rs + 2 * k + (i & 1)] = (i < ldy && k < r) ? C[(int64_t)k * ldy + i] : 0.0;
  }
}

// Row chunks of the accumulation grid: chunks [0, nbig) hold `big` rows each, the rest `small`
// rows (a guided static schedule: workgroups are dispatched in chunk order, so the large chunks run
// first and the small ones fill the tail; fewer partials to write and reduce than equal chunks with
// the same tail).  Fixed by (n, chunk count), so results stay deterministic.
// bnd (meta_PPLSi on the panel sweep): explicit boundaries instead, each chunk inside one population.
struct PplsChunks {
  int64_t big, small;
  int nbig;
  const int64_t* bnd;
  __host__ __device__ void range(int c, int64_t n, int64_t& r0, int64_t& r1) const {
    if (bnd) {
      r0 = bnd[c];
      r1 = bnd[c + 1];
      return;
    }
    r0 = c < nbig ? (int64_t)c * big : (int64_t)nbig * big + (int64_t)(c - nbig) * small;
    const int64_t len = c < nbig ? big : small;
    if (r0 > n) r0 = n;
    r1 = r0 + len < n ? r0 + len : n;
  }
};

template <typename T, int R, bool NT>
__global__ __launch_bounds__(256) void ppls_panel_acc_kernel(
    const T* __restrict__ X, const T* __restrict__ Y, int64_t n, int ldx, int ldy,
    const double* __restrict__ Z, PplsChunks ck, double* __restrict__ part, int64_t part_ld,
    const int* __restrict__ stop) {
  if (stop && *stop) return;   // em_run converged earlier (device stop flag)
  constexpr int VEC = PplsVec16<T>::N;
  constexpr int V4 = 4 * R;
  const int tid = threadIdx.x;
  const int ntx = (ldx + 256 * VEC - 1) / (256 * VEC);
  const bool isx = (int)blockIdx.x < ntx;
  const int col = (isx ? blockIdx.x : blockIdx.x - ntx) * 256 * VEC + tid * VEC;
  const int ld = isx ? ldx : ldy;
  const T* M = isx ? X : Y;
  const int off = isx ? 2 * R : 3 * R;
  int64_t r0, r1;
  ck.range(blockIdx.y, n, r0, r1);
  double* pg = part + (int64_t)blockIdx.y * part_ld;
  // mu (mu_T for X tiles, mu_U for Y tiles) of BR rows at a time in LDS (every lane reads the same
  // address: broadcast).  Software-pipelined: the next batch's mu is loaded into registers while the
  // current batch is computed (LDS double-buffered, one barrier per batch), and the X rows stream in
  // groups of 8 with the next group's loads in flight during the current group's FMAs.  (Round 5:
  // each row's mu read a row ahead into registers, so its LDS reads overlap the previous row's FMAs:
  // 4 % faster in isolated launches at C5, 0.2 % in back-to-back iterations -- the clock, not the LDS
  // latency, bounds the FMAs -- and 1 % slower at C5's 8-GPU share; not kept.  DESIGN.md 4.2)
  constexpr int BR = 128;
  constexpr int MPT = (BR * R + 255) / 256;
  __shared__ double smu[2][BR * R];
  double acc[VEC][R];
#pragma unroll
  for (int v = 0; v < VEC; ++v)
#pragma unroll
    for (int k = 0; k < R; ++k) acc[v][k] = 0.0;
  const bool act = col < ld;
  const bool wact = col - (tid & 63) * VEC < ld;   // some lane of this wave has columns (wave-uniform)
  const T* base = M + (act ? col : 0);
  double mreg[MPT];
  auto load_mu = [&](int64_t b0) {
#pragma unroll
    for (int u = 0; u < MPT; ++u) {
      const int e = tid + 256 * u;
      const int rr = e / R, k = e - rr * R;
      mreg[u] = (e < BR * R && b0 + rr < r1) ? Z[(b0 + rr) * V4 + off + k] : 0.0;
    }
  };
  auto store_mu = [&](int buf) {
#pragma unroll
    for (int u = 0; u < MPT; ++u) {
      const int e = tid + 256 * u;
      if (e < BR * R) smu[buf][e] = mreg[u];
    }
  };
  const int64_t nbatch = (r1 - r0 + BR - 1) / BR;
  if (nbatch > 0) {
    load_mu(r0);
    store_mu(0);
  }
  __syncthreads();
  for (int64_t bt = 0; bt < nbatch; ++bt) {
    const int64_t b0 = r0 + bt * BR;
    const int nb = (int)(r1 - b0 < BR ? r1 - b0 : BR);
    if (bt + 1 < nbatch) load_mu(b0 + BR);
    const double* sm = smu[bt & 1];
    if (wact) {
      constexpr int G = 8;   // rows per load group (4: 168 VGPRs, 3 waves/SIMD, no faster at C5)
      PplsVec16<T> xa[G], xb[G];
      auto load8 = [&](int rr, PplsVec16<T> (&xv)[G]) {
#pragma unroll
        for (int u = 0; u < G; ++u) xv[u] = ppls_load16<T, NT>(base + (b0 + min(rr + u, nb - 1)) * ld);
      };
      auto fma8 = [&](int rr, const PplsVec16<T> (&xv)[G]) {
#pragma unroll
        for (int u = 0; u < G; ++u) {
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const double m = sm[(rr + u) * R + k];
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[v][k] = fma((double)xv[u].v[v], m, acc[v][k]);
          }
        }
      };
      // Branch-free: every load is issued (rows clamped to the batch's last row; lanes beyond ld
      // read column 0), and rows past nb (last batch only, up to the next multiple of 2G <= BR)
      // meet mu = 0 in LDS and add exactly 0.  So the compiler's vmcnt waits count the prefetched
      // group as in flight; the earlier conditional form waited vmcnt(0) on it before each pair
      // (a load behind a branch is not counted): C5 acc 4.0 -> 3.97 ms.
      const int ng = (nb + 2 * G - 1) / (2 * G);
      load8(0, xa);
      for (int gp = 0; gp + 1 < ng; ++gp) {
        const int rr = 2 * G * gp;
        load8(rr + G, xb);
        fma8(rr, xa);
        load8(rr + 2 * G, xa);
        fma8(rr + G, xb);
      }
      const int rr = 2 * G * (ng - 1);
      load8(rr + G, xb);
      fma8(rr, xa);
      fma8(rr + G, xb);
    }
    if (bt + 1 < nbatch) store_mu((bt + 1) & 1);
    __syncthreads();
  }
  if (act) {
    double* dst = isx ? pg : pg + (int64_t)R * ldx;
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int v = 0; v < VEC; ++v)   // streaming stores: the partials are read once, by the reduce
        __builtin_nontemporal_store(acc[v][k], dst + (int64_t)k * ld + col + v);
  }
  if (blockIdx.x == 0) {   // Gram of [Xw Yc] over the chunk (2R x 2R, column-major)
    constexpr int V2 = 2 * R, NP = V2 * (V2 + 1) / 2, BR = 64;
    __shared__ double sz[BR * V2];
    double* G2 = pg + (int64_t)R * ldx + (int64_t)R * ldy;
    double gs[(NP + 255) / 256];
    int pi[(NP + 255) / 256], pj[(NP + 255) / 256];
#pragma unroll
    for (int u = 0; u < (NP + 255) / 256; ++u) {
      gs[u] = 0.0;
      int e = tid + 256 * u, i = 0;   // packed upper triangle: e -> (i <= j)
      while (e >= V2 - i && i < V2) { e -= V2 - i; ++i; }
      pi[u] = i;
      pj[u] = i + e;
    }
    for (int64_t b0 = r0; b0 < r1; b0 += BR) {   // stage BR rows of [a | b], then sum from LDS
      __syncthreads();
      for (int e = tid; e < BR * V2; e += 256) {
        const int rr = e / V2, f = e - rr * V2;
        sz[e] = (b0 + rr < r1) ? Z[(b0 + rr) * V4 + f] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int u = 0; u < (NP + 255) / 256; ++u)
        if (tid + 256 * u < NP)
          for (int rr = 0; rr < BR; ++rr) gs[u] = fma(sz[rr * V2 + pi[u]], sz[rr * V2 + pj[u]], gs[u]);
    }
#pragma unroll
    for (int u = 0; u < (NP + 255) / 256; ++u)
      if (tid + 256 * u < NP) {
        G2[pj[u] * V2 + pi[u]] = gs[u];
        G2[pi[u] * V2 + pj[u]] = gs[u];
      }
  }
}

// ============================================================================ finalize
// Block-wide sum of nv values per thread (blockDim.x <= 1024); result broadcast to all threads.
__device__ void ppls_block_sum(double* vals, int nv, double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
  for (int k = 0; k < nv; ++k) {
    const double s = ppls_wave_sum(vals[k]);
    if (lane == 0) sh[wave * PPLS_RMAX + k] = s;
  }
  __syncthreads();
  for (int k = 0; k < nv; ++k) {
    double t = 0.0;
    for (int w = 0; w < nwaves; ++w) t += sh[w * PPLS_RMAX + k];
    vals[k] = t;
  }
  __syncthreads();
}

// Polar factor of the p x r matrix S (ld lds): Householder QR S = QR, Jacobi R = U S V',
// out = Q U V'.  A, E: p x r scratch (ld p).  Returns status through *status.
__device__ __noinline__ void ppls_block_polar(const double* S, int64_t lds, int p, int r, double* out,
                                 int64_t ldo, int ldo_rows, double* A, double* E, int* status, int qr) {
  __shared__ double sh[16 * PPLS_RMAX];
  __shared__ double Rm[PPLS_RMAX * PPLS_RMAX];
  __shared__ double P[PPLS_RMAX * PPLS_RMAX];
  __shared__ double jw[2 * PPLS_RMAX * PPLS_RMAX];   // Jacobi workspace
  __shared__ double vtv_s[PPLS_RMAX];
  const int tid = threadIdx.x, nt = blockDim.x;
  for (int k = 0; k < r; ++k)
    for (int i = tid; i < p; i += nt) A[(int64_t)k * p + i] = S[(int64_t)k * lds + i];
  __syncthreads();
  double vals[PPLS_RMAX];
  for (int k = 0; k < r; ++k) {
    vals[0] = 0.0;
    for (int i = k + tid; i < p; i += nt) vals[0] = fma(A[(int64_t)k * p + i], A[(int64_t)k * p + i], vals[0]);
    ppls_block_sum(vals, 1, sh);
    const double sig = sqrt(vals[0]);
    const double akk = A[(int64_t)k * p + k];
    const double alpha = (akk >= 0.0) ? -sig : sig;
    const double vtv = 2.0 * sig * (sig + fabs(akk));
    __syncthreads();
    if (tid == 0) {
      A[(int64_t)k * p + k] = akk - alpha;
      Rm[k * r + k] = alpha;
      vtv_s[k] = vtv;
      if (!(sig > 0.0)) *status = -3;
    }
    __syncthreads();
    const int nj = r - k - 1;
    for (int j = 0; j < nj; ++j) vals[j] = 0.0;
    for (int i = k + tid; i < p; i += nt) {
      const double vi = A[(int64_t)k * p + i];
      for (int j = 0; j < nj; ++j) vals[j] = fma(vi, A[(int64_t)(k + 1 + j) * p + i], vals[j]);
    }
    ppls_block_sum(vals, nj, sh);
    for (int i = k + tid; i < p; i += nt) {
      const double vi = A[(int64_t)k * p + i];
      for (int j = 0; j < nj; ++j) {
        const double f = (vtv > 0.0) ? 2.0 * vals[j] / vtv : 0.0;
        A[(int64_t)(k + 1 + j) * p + i] -= f * vi;
      }
    }
    __syncthreads();
    if (tid == 0)
      for (int j = 0; j < nj; ++j) Rm[(k + 1 + j) * r + k] = A[(int64_t)(k + 1 + j) * p + k];
    __syncthreads();
  }
  if (tid == 0)
    for (int j = 0; j < r; ++j)
      for (int i = j + 1; i < r; ++i) Rm[j * r + i] = 0.0;
  // E = H_0 ... H_{r-1} [I; 0]
  for (int j = 0; j < r; ++j)
    for (int i = tid; i < p; i += nt) E[(int64_t)j * p + i] = (i == j) ? 1.0 : 0.0;
  __syncthreads();
  for (int k = r - 1; k >= 0; --k) {
    for (int j = 0; j < r; ++j) vals[j] = 0.0;
    for (int i = k + tid; i < p; i += nt) {
      const double vi = A[(int64_t)k * p + i];
      for (int j = 0; j < r; ++j) vals[j] = fma(vi, E[(int64_t)j * p + i], vals[j]);
    }
    ppls_block_sum(vals, r, sh);
    const double vtv = vtv_s[k];
    for (int i = k + tid; i < p; i += nt) {
      const double vi = A[(int64_t)k * p + i];
      for (int j = 0; j < r; ++j) {
        const double f = (vtv > 0.0) ? 2.0 * vals[j] / vtv : 0.0;
        E[(int64_t)j * p + i] -= f * vi;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    if (qr) {   // orth(type = "QR") = sign_e * qr.Q(qr(S)), sign_e = sign(<e_1, S_1>) = sign(R_11)
      const double sg = Rm[0] < 0.0 ? -1.0 : 1.0;   // (Package/functions.R:257-259)
      for (int j = 0; j < r; ++j)
        for (int i = 0; i < r; ++i) P[j * r + i] = (i == j) ? sg : 0.0;
    } else if (ppls_small_polar_ws<PPLS_RMAX>(Rm, r, P, jw, jw + r * r) != 0) {
      *status = -3;
    }
  }
  __syncthreads();
  for (int j = 0; j < r; ++j)
    for (int i = tid; i < ldo_rows; i += nt) {
      double s = 0.0;
      if (i < p)
        for (int k = 0; k < r; ++k) s = fma(E[(int64_t)k * p + i], P[j * r + k], s);
      out[(int64_t)j * ldo + i] = s;
    }
}

// Block-wide sum of NV <= 64 values per thread (every thread gets the sums): a wave
// reduce-scatter (ppls_rs: permlane/DPP, no LDS round trips) leaves each wave sum on one lane,
// which writes it to LDS; the cross-wave sums are read back by every thread.
template <int NV, int NW = 0>
__device__ __forceinline__ void ppls_block_sum_t(double (&vals)[NV], double* sh) {
  static_assert(NV >= 1 && NV <= 64, "block sum of at most 64 values");
  constexpr int NB = NV + (NV & 1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nwaves = NW > 0 ? NW : (int)(blockDim.x >> 6);
  double a[NB];
#pragma unroll
  for (int k = 0; k < NV; ++k) a[k] = vals[k];
  int idx = 0;
  bool canon = true;
  ppls_rs<NV, 0, NB>(a, lane, idx, canon);
  if (canon && idx < NV) sh[wave * NV + idx] = a[0];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < (NW > 0 ? NW : 16); ++w)
      if (NW > 0 || w < nwaves) t += sh[w * NV + k];
    vals[k] = t;
  }
  __syncthreads();
}

// Diagnostics stamp (finalize phases; tr == nullptr in production).
__device__ __forceinline__ void ppls_stamp(long long* tr, int slot) {
  if (tr && threadIdx.x == 0) tr[slot] = (long long)wall_clock64();
}

// ---- r x r algebra in registers (compile-time R, fully unrolled; run by one thread) -----------
// Matrices are T[row][col].

// 1/x and 1/sqrt(x) from the hardware estimates plus two Newton steps (~1 ulp; x normal, > 0
// for rsq).  The serial r x r code is latency-bound on one wave, and these are 5-7 dependent
// instructions against ~12-15 for the IEEE-exact expansions.
__device__ __forceinline__ double ppls_rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}
__device__ __forceinline__ double ppls_rsq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double r = fma(-x * y, y, 1.0);
  y = fma(0.5 * y, r, y);
  r = fma(-x * y, y, 1.0);
  return fma(0.5 * y, r, y);
}

// Block Gram of rows x (R values per thread) accumulated into the packed upper triangle.
template <int R>
__device__ __forceinline__ void ppls_gram_acc(const double (&x)[R], double (&vals)[R * (R + 1) / 2]) {
  int e = 0;
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int a = 0; a <= b; ++a) { vals[e] = fma(x[a], x[b], vals[e]); ++e; }
}

template <int R>
__device__ __forceinline__ void ppls_gram_unpack(const double (&vals)[R * (R + 1) / 2], double (&G)[R][R]) {
  int e = 0;
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int a = 0; a <= b; ++a) { G[a][b] = vals[e]; G[b][a] = vals[e]; ++e; }
}

// Packed upper triangles (element (a, b), a <= b, at b (b + 1) / 2 + a: the Gram sums' order) --
// the register forms below then hold R(R+1)/2 values instead of R^2, so one thread keeps R = 10 in
// registers.
__host__ __device__ constexpr int ppls_pk(int a, int b) { return b * (b + 1) / 2 + a; }

// In place: P = the packed Gram on entry, its upper Cholesky factor U (G = U'U) on exit.
template <int R>
__device__ __forceinline__ bool ppls_chol_pk(double (&P)[R * (R + 1) / 2], double (&dinv)[R]) {
  bool ok = true;
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int i = 0; i <= j; ++i) {
      double s = P[ppls_pk(i, j)];
#pragma unroll
      for (int k = 0; k < i; ++k) s = fma(-P[ppls_pk(k, i)], P[ppls_pk(k, j)], s);
      if (i == j) {
        ok = ok && (s > 0.0);
        P[ppls_pk(j, j)] = sqrt(s > 0.0 ? s : 1.0);
        dinv[j] = 1.0 / P[ppls_pk(j, j)];
      } else {
        P[ppls_pk(i, j)] = s * dinv[i];
      }
    }
  return ok;
}

// In place: P = U on entry, inv(U) on exit.  Columns last to first: column j of the inverse needs
// U's columns <= j only, and within the column the rows bottom-up.
template <int R>
__device__ __forceinline__ void ppls_inv_upper_pk(double (&P)[R * (R + 1) / 2], const double (&dinv)[R]) {
#pragma unroll
  for (int jj = 0; jj < R; ++jj) {
    const int j = R - 1 - jj;
#pragma unroll
    for (int ii = 0; ii < R; ++ii) {
      const int i = R - 1 - ii;
      if (i > j) continue;
      double s = (i == j) ? 1.0 : 0.0;
#pragma unroll
      for (int k = i + 1; k <= j; ++k) s = fma(-P[ppls_pk(i, k)], P[ppls_pk(k, j)], s);
      P[ppls_pk(i, j)] = s * dinv[i];
    }
  }
}

// Sum over an aligned group of 8 lanes (DPP quad xor1, quad xor2, half-row mirror); every lane of
// the group gets the bitwise-same total.  All 64 lanes must be active.
__device__ __forceinline__ double ppls_group8_sum(double v) {
  v += ppls_dpp_partner<5>(v);
  v += ppls_dpp_partner<4>(v);
  v += ppls_dpp_partner<3>(v);
  return v;
}

__device__ __forceinline__ void ppls_wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Pair k of round m of the circle-method (round-robin) schedule of the R(R-1)/2 column pairs:
// N-1 rounds of N/2 disjoint pairs, N = R rounded up to even, pairs with the dummy column R
// dropped by the caller; i < j.
template <int R>
__device__ __forceinline__ void ppls_rr_pair(int m, int k, int& i, int& j) {
  constexpr int N = R + (R & 1);
  const int pa = k == 0 ? 0 : ((k - 1 + m) % (N - 1)) + 1;
  const int pb = ((N - 2 - k + m) % (N - 1)) + 1;
  i = pa < pb ? pa : pb;
  j = pa < pb ? pb : pa;
}

// Small dense algebra on one wave with R x R matrices in LDS as G x G column blocks
// (element (row t, col c) at [c * G + t], G = 8 for R <= 8 else 16, rows >= R zero).  All 64
// lanes of the wave must call (DPP sums); results are wave-uniform.
template <int R>
struct PplsWaveBlk {
  static constexpr int G = R <= 8 ? 8 : 16;
  static constexpr int SZ = G * G;
};

template <int G>
__device__ __forceinline__ double ppls_groupG_sum(double v) {
  if constexpr (G == 8) return ppls_group8_sum(v);
  else return ppls_group16_sum(v);
}

// Upper Cholesky G = U'U (right-looking, lane-parallel updates); ok = false if a pivot <= 0.
// sW: G x G scratch (destroyed); sU receives U (zero below the diagonal).
template <int R>
__device__ bool ppls_chol_wave(double* sW, double* sU) {
  constexpr int G = PplsWaveBlk<R>::G;
  const int lane = threadIdx.x & 63;
  bool ok = true;
  for (int e = lane; e < G * G; e += 64) sU[e] = 0.0;
  ppls_wave_lds_fence();
  for (int j = 0; j < R; ++j) {
    const double piv = sW[j * G + j];
    ok = ok && (piv > 0.0);
    const double d = sqrt(piv > 0.0 ? piv : 1.0);
    const double di = 1.0 / d;
    if (lane == 0) sU[j * G + j] = d;
    if (lane > j && lane < R) sU[lane * G + j] = sW[lane * G + j] * di;   // U[j][lane]
    ppls_wave_lds_fence();
    for (int e = lane; e < G * G; e += 64) {   // W[a][b] -= U[j][a] U[j][b], j < a, b < R
      const int a = e % G, b = e / G;
      if (a > j && b > j && a < R && b < R) sW[b * G + a] -= sU[a * G + j] * sU[b * G + j];
    }
    ppls_wave_lds_fence();
  }
  return ok;
}

// sUi = inv(U), U upper triangular: lane c < R back-substitutes column c.
template <int R>
__device__ void ppls_inv_upper_wave(const double* sU, double* sUi) {
  constexpr int G = PplsWaveBlk<R>::G;
  const int lane = threadIdx.x & 63;
  for (int e = lane; e < G * G; e += 64) sUi[e] = 0.0;
  ppls_wave_lds_fence();
  if (lane < R) {
    const int c = lane;
    double col[R];
#pragma unroll
    for (int ii = 0; ii < R; ++ii) {
      const int i = R - 1 - ii;
      double s = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int kk = i + 1; kk < R; ++kk) s = fma(-sU[kk * G + i], col[kk], s);
      col[i] = (i <= c) ? s / sU[i * G + i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < R; ++i) sUi[c * G + i] = col[i];
  }
  ppls_wave_lds_fence();
}

// sC = op(A) sB with A transposed if TA; entries (a, b) on lanes.
template <int R, bool TA>
__device__ void ppls_matmul_wave(const double* sA, const double* sB, double* sC) {
  constexpr int G = PplsWaveBlk<R>::G;
  const int lane = threadIdx.x & 63;
  for (int e = lane; e < G * G; e += 64) {
    const int a = e % G, b = e / G;
    double s = 0.0;
    if (a < R && b < R)
#pragma unroll
      for (int kk = 0; kk < R; ++kk) s = fma(TA ? sA[a * G + kk] : sA[kk * G + a], sB[b * G + kk], s);
    sC[e] = s;
  }
  ppls_wave_lds_fence();
}

// One-sided Jacobi on one wave: A V = U Sigma with A, V in LDS (G x G blocks).  Round m of a
// sweep rotates the N/2 (<= 8) disjoint pairs of the circle-method schedule at once: lane group
// g = lane / 8 owns pair g, lane t = lane % 8 owns rows t and t + 8 (R > 8) of its two columns,
// the column dots are 8-lane DPP sums.  Same rotation and stopping rule as ppls_small_polar_n
// (ppls_math.h).  Wave-uniform.
template <int R>
__device__ __forceinline__ int ppls_jacobi_wave(double* sA, double* sV) {
  constexpr int N = R + (R & 1);
  constexpr int G = PplsWaveBlk<R>::G;
  constexpr int RPL = (R + 7) / 8;                  // rows per lane (G = 16 layout for R > 8)
  static_assert(N / 2 <= 8, "one pass of 8-lane groups per round");
  const int lane = threadIdx.x & 63, t = lane & 7;
  int sweeps = 0;
  for (int sweep = 0; sweep < 60; ++sweep) {
    ++sweeps;
    bool rot_any = false;
    double cmax = 0.0;   // largest cos^2 between rotated column pairs this sweep (g^2 / (a b))
#pragma unroll
    for (int m = 0; m < N - 1; ++m) {
      const int k = lane >> 3;
      const bool grp = k < N / 2;
      int i, j;
      ppls_rr_pair<R>(m, grp ? k : 0, i, j);
      const bool act = grp && j < R;
      const int ci = (act ? i : 0) * G + t, cj = (act ? j : 1) * G + t;
      double x[RPL], y[RPL], vx[RPL], vy[RPL];
      double aa = 0.0, bb = 0.0, gg = 0.0;
#pragma unroll
      for (int u = 0; u < RPL; ++u) {
        x[u] = sA[ci + 8 * u];
        y[u] = sA[cj + 8 * u];
        vx[u] = sV[ci + 8 * u];
        vy[u] = sV[cj + 8 * u];
        aa = fma(x[u], x[u], aa);
        bb = fma(y[u], y[u], bb);
        gg = fma(x[u], y[u], gg);
      }
      const double a = ppls_group8_sum(aa), b = ppls_group8_sum(bb), g = ppls_group8_sum(gg);
      const bool rot = act && (g * g >= 1e-30 * (a * b)) && g != 0.0;
      if (rot) cmax = fmax(cmax, g * g / (a * b));
      const double z = (b - a) * ppls_rcp(rot ? 2.0 * g : 1.0);
      const double z2 = fma(z, z, 1.0);
      const double uu = fabs(z) + z2 * ppls_rsq(z2);
      const double w = ppls_rsq(fma(uu, uu, 1.0));
      const double c = uu * w, sn = z >= 0.0 ? w : -w;
      if (rot) {
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
          sA[ci + 8 * u] = fma(c, x[u], -sn * y[u]);
          sA[cj + 8 * u] = fma(sn, x[u], c * y[u]);
          sV[ci + 8 * u] = fma(c, vx[u], -sn * vy[u]);
          sV[cj + 8 * u] = fma(sn, vx[u], c * vy[u]);
        }
      }
      rot_any = rot_any || rot;
      ppls_wave_lds_fence();
    }
    if (!__any(rot_any)) break;
    // Jacobi converges quadratically: after a sweep whose largest cosine was <= 1e-8 the remaining
    // ones are ~1e-16, so the sweep that would only confirm it is skipped
    if (!__any(cmax > 1e-16)) break;
  }
  return sweeps;
}

// A team of K workgroups computing one polar factor together (wide p): each owns rows
// [p rank / K, p (rank + 1) / K); the R x R Grams of passes 1-2 are exchanged through `part` (one
// 64-double slot per rank and phase, summed in rank order by every member, so all members hold
// bitwise-identical values and run the identical small algebra) at a counter barrier; the Gram
// of the result is summed by the last member to finish.  K = 1 is the single-block form (no
// exchange).  Barrier waits are bounded: a member that waits longer than ~100 ms sets status -7
// and carries on, so a missing member can never hang the GPU.
struct PplsTeam {
  int rank, K;
  unsigned* bar;    // [0] barrier arrivals, [1] members done, [2] result-Gram arrivals (per matrix)
  double* part;     // 3 phases x K x 64 doubles
  int* status;
  long long* tr;    // diagnostics (member 0): stamps inside the first barrier
};

// Members publish with plain stores and one agent-scope release fence, wait with relaxed polling of
// the arrival counter and one acquire fence (measured: memory-side atomic swaps for the values
// instead cost more, profiles/r2_finalize_team.txt).
__device__ void ppls_team_barrier(const PplsTeam& tm, unsigned target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();   // release this member's partials
    atomicAdd(&tm.bar[0], 1u);
    if (tm.tr && target == (unsigned)tm.K) tm.tr[9] = (long long)wall_clock64();
    long spins = 0;
    // relaxed polling (no cache invalidation per poll); one acquire fence after the wait
    while (__hip_atomic_load(&tm.bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (++spins > (1L << 21)) {
        atomicExch(tm.status, -7);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (tm.tr && target == (unsigned)tm.K) tm.tr[10] = (long long)wall_clock64();
    __threadfence();   // acquire the others' partials
  }
  __syncthreads();
}

// After a member's last barrier: the last member to leave resets the counters for the next launch.
__device__ void ppls_team_leave(const PplsTeam& tm) {
  if (tm.K <= 1 || threadIdx.x != 0) return;
  if (atomicAdd(&tm.bar[1], 1u) == (unsigned)tm.K - 1) {
    atomicExch(&tm.bar[0], 0u);
    atomicExch(&tm.bar[1], 0u);
  }
}

// vals (NG per thread, identical in every thread of the block) -> the team's sum over members.
template <int NG>
__device__ void ppls_team_sum(const PplsTeam& tm, int phase, double (&vals)[NG], double* sh) {
  if (tm.K <= 1) return;
  double* slot = tm.part + ((int64_t)phase * tm.K) * 64;
  if (threadIdx.x < NG) {
#pragma unroll
    for (int e = 0; e < NG; ++e)
      if ((int)threadIdx.x == e) slot[(int64_t)tm.rank * 64 + e] = vals[e];
  }
  ppls_team_barrier(tm, (unsigned)(phase + 1) * tm.K);
  if (threadIdx.x < NG) {
    double t = 0.0;
    for (int k = 0; k < tm.K; ++k) t += __builtin_nontemporal_load(slot + (int64_t)k * 64 + threadIdx.x);
    sh[threadIdx.x] = t;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = sh[e];
  __syncthreads();
}

// Polar factor U V' of the p x R matrix S (column-major, ld lds) by Cholesky-QR2 (S = Q1 R1,
// Q1 = Q R2) and one-sided Jacobi on T = R2 R1 = U_T Sigma V': U V' = Q1 R2^-1 U_T V'.  Three
// block passes: the first stages S into LDS (Sl, p*R doubles; nullptr = re-read from global); the
// second forms Q1 = S R1^-1 (kept in Sl, else in out) and its Gram; the last
// writes out = Q1 P, P = R2^-1 U_T V', and, if gram_out != nullptr, the Gram out'out the next
// iteration's scalar update needs.  All R x R algebra runs on wave 0 in LDS; the Jacobi is
// warm-started from vstate (the previous iteration's V; nullptr = identity).  sm: >= 2 R^2
// doubles of LDS.  Returns false when S is numerically rank deficient (a Cholesky pivot fails or
// sigma_min < 1e-14 sigma_max); the caller then falls back to Householder (which reports it).
// The staged rows live in LDS: accessed through this type the compiler emits ds_read/ds_write
// (a plain double* to LDS compiles to flat loads and stores, which take the vector-memory path).
typedef __attribute__((address_space(3))) double ppls_lds_double;

#ifndef PPLS_REG_RMAX
#define PPLS_REG_RMAX 10   // the polar's Cholesky factors and inverses by one thread in registers up to this R
#endif
template <int R, int NT>
__device__ bool ppls_block_polar_fast(const double* __restrict__ S, int64_t lds, int p,
                                      double* __restrict__ out, int64_t ldo, int ldo_rows, double* Sl,
                                      double* sh, double* sm, double* __restrict__ gram_out,
                                      double* __restrict__ vstate, long long* tr, const PplsTeam& tm,
                                      bool polar1, double kbound, bool reorth) {
  constexpr int NG = R * (R + 1) / 2;
  constexpr int NW = NT / 64;
  constexpr int G = PplsWaveBlk<R>::G, GG = G * G;
  static_assert(R <= 16 && NG <= 64, "block sums of at most 64 values");
  const int tid = threadIdx.x, lane = tid & 63;
  const int i0 = (int)((int64_t)p * tm.rank / tm.K), i1 = (int)((int64_t)p * (tm.rank + 1) / tm.K);
  const int nr = i1 - i0;                                     // this member's rows
  const int o1 = tm.rank == tm.K - 1 ? ldo_rows : i1;        // output rows (the last takes the padding)
  double* sF = sm;            // R x R (column-major, ld R): R1^-1 for pass 2, then F for pass 3
  __shared__ double sA[GG], sV[GG], sT[GG], sU[GG], ssv[16];
  __shared__ int ok;
  // the carried V (wave 0), fetched now so its latency hides under pass 1
  double vprev[(GG + 63) / 64];
#pragma unroll
  for (int u = 0; u < (GG + 63) / 64; ++u) {
    const int e = lane + 64 * u, cb = e / G, rt = e % G;
    vprev[u] = (cb == rt && cb < R) ? 1.0 : 0.0;
    if (vstate && tid < 64 && cb < R && rt < R) vprev[u] = vstate[cb * R + rt];
  }
  double vals[NG];
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = 0.0;
  // pass 1: G1 = S'S, staging S into LDS; chunks of PU rows per thread with every load of a
  // chunk issued before the first use
  constexpr int PU = R >= 6 ? 4 : 8;
  for (int c0 = i0; c0 < i1; c0 += PU * NT) {
    double x[PU][R];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int i = c0 + u * NT + tid;
#pragma unroll
      for (int k = 0; k < R; ++k) x[u][k] = (i < i1) ? S[(int64_t)k * lds + i] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int i = c0 + u * NT + tid;
      if (Sl && i < i1) {
        ppls_lds_double* L = (ppls_lds_double*)Sl;
#pragma unroll
        for (int k = 0; k < R; ++k) L[k * nr + (i - i0)] = x[u][k];
      }
      ppls_gram_acc<R>(x[u], vals);
    }
  }
  ppls_stamp(tr, 13);
  ppls_block_sum_t<NG, NW>(vals, sh);
  ppls_stamp(tr, 14);
  ppls_team_sum<NG>(tm, 0, vals, sh);
  ppls_stamp(tr, 1);
  if constexpr (R <= PPLS_REG_RMAX) {   // one thread in registers is faster than the wave form
    if (tid < 64) {
      for (int e = lane; e < GG; e += 64) sT[e] = 0.0;   // (in order before lane 0's stores)
      if (lane == 0) {
        double P[NG], dinv[R];
#pragma unroll
        for (int e = 0; e < NG; ++e) P[e] = vals[e];
        ok = ppls_chol_pk<R>(P, dinv);
#pragma unroll
        for (int b = 0; b < R; ++b)
#pragma unroll
          for (int a = 0; a <= b; ++a) sT[b * G + a] = P[ppls_pk(a, b)];
        ppls_inv_upper_pk<R>(P, dinv);
#pragma unroll
        for (int b = 0; b < R; ++b)
#pragma unroll
          for (int a = 0; a < R; ++a) sF[b * R + a] = a <= b ? P[ppls_pk(a, b)] : 0.0;
      }
    }
  } else if (tid < 64) {   // R1 = chol(G1) -> sT, R1^-1 -> sF (ld R)
    for (int e = lane; e < GG; e += 64) {
      const int a = e % G, b = e / G;
      double v = 0.0;
      if (a < R && b < R) {
        const int lo = a < b ? a : b, hi = a < b ? b : a;
        v = vals[hi * (hi + 1) / 2 + lo];
      }
      sA[e] = v;
    }
    ppls_wave_lds_fence();
    const bool good = ppls_chol_wave<R>(sA, sT);
    ppls_inv_upper_wave<R>(sT, sU);
    for (int e = lane; e < R * R; e += 64) sF[e] = sU[(e / R) * G + e % R];
    if (lane == 0) ok = good;
  }
  __syncthreads();
  ppls_stamp(tr, 2);
  if (!ok) {   // identical verdict in every member
    ppls_team_leave(tm);
    return false;
  }
  // row i of S / Q1 at Sr[k * ldr + i - sro]: own rows staged in LDS, else S in global memory
  const double* Sr = Sl ? Sl : S;
  const int64_t ldr = Sl ? nr : lds;
  const int sro = Sl ? i0 : 0;
  // the carried V in sV, re-orthonormalised (modified Gram-Schmidt, rows on lanes; wave 0) when
  // reorth: every 8th iteration by default (context option "vorth", mode bits 16-23) -- between, the
  // Jacobi's rotations keep it orthonormal to a few eps per iteration (1.6 us of the C3
  // cross-product finalize's critical path saved 7 times in 8; tests/test_gpu_nonfinite.py runs
  // 400 iterations at cadence 8 against cadence 1)
  auto load_vprev = [&]() {
    for (int e = lane; e < GG; e += 64) {
#pragma unroll
      for (int u = 0; u < (GG + 63) / 64; ++u)
        if (e == lane + 64 * u) sV[e] = vprev[u];
    }
    ppls_wave_lds_fence();
    if (vstate && reorth) {
      const int rt = lane % G;
      for (int j = 0; j < R; ++j) {
        double vj = sV[j * G + rt];
        for (int i = 0; i < j; ++i) {
          const double vi = sV[i * G + rt];
          vj = fma(-ppls_groupG_sum<G>(vi * vj), vi, vj);
        }
        vj *= ppls_rsq(ppls_groupG_sum<G>(vj * vj));
        if (lane < G) sV[j * G + rt] = vj;
        ppls_wave_lds_fence();
      }
    }
  };
  // Cholesky-QR1 fast path (polar1): when kappa(S) = kappa(R1) is small, Q1 = S R1^-1 is already
  // orthonormal to O(eps kappa^2) (~1e-14), so pass 2, its team barrier and chol(G2) are skipped:
  // T = R1 = U_T Sigma V' by the Jacobi, out = S F, F = R1^-1 U_T V'.  The test is the bound
  // kappa_2(R1) <= ||R1||_F ||R1^-1||_F <= kbound (option polar1_kappa; default min(8 R, 40): the
  // loss of orthogonality ~ eps kappa^2 stays <= 1e-13; no Jacobi is spent on a matrix
  // that then takes the Cholesky-QR2 path).  Every member decides on the bitwise-identical G1, so
  // a team takes one path.
  __shared__ int fast;
  if (tid < 64) {
    bool fst = false;
    if (polar1) {
      double fr = 0.0, fi = 0.0;
      for (int e = lane; e < R * R; e += 64) {
        const double t = sT[(e / R) * G + e % R], u = sF[e];
        fr = fma(t, t, fr);
        fi = fma(u, u, fi);
      }
      fr = ppls_wave_sum(fr);
      fi = ppls_wave_sum(fi);
      const double kb = kbound > 0.0 ? kbound : PPLS_POLAR1_KAPPA * R;
      fst = __shfl(fr * fi <= kb * kb ? 1 : 0, 0, 64) != 0;
    }
    if (fst) {
      load_vprev();
      ppls_stamp(tr, 6);
      ppls_matmul_wave<R, false>(sT, sV, sA);                // sA = R1 V (sT keeps R1)
      ppls_stamp(tr, 7);
      ppls_jacobi_wave<R>(sA, sV);
      ppls_stamp(tr, 8);
      if (lane < R) {
        double nrm = 0.0;
#pragma unroll
        for (int t = 0; t < R; ++t) nrm = fma(sA[lane * G + t], sA[lane * G + t], nrm);
        ssv[lane] = sqrt(nrm);
      }
      ppls_wave_lds_fence();
      {
        for (int e = lane; e < GG; e += 64) {                  // sU = U_T V'
          const int a = e % G, b = e / G;
          double s = 0.0;
          if (a < R && b < R)
#pragma unroll
            for (int kk = 0; kk < R; ++kk) s = fma(sA[kk * G + a] * (1.0 / ssv[kk]), sV[kk * G + b], s);
          sU[e] = s;
        }
        ppls_wave_lds_fence();
        for (int e = lane; e < R * R; e += 64) {               // F = R1^-1 U_T V' -> sm + R^2 (ld R)
          const int a = e % R, b = e / R;
          double s = 0.0;
#pragma unroll
          for (int kk = 0; kk < R; ++kk) s = fma(sF[kk * R + a], sU[b * G + kk], s);
          sF[R * R + b * R + a] = s;
          if (vstate && tm.rank == 0) vstate[b * R + a] = sV[b * G + a];   // every member's V is identical
        }
      }
    }
    if (lane == 0) fast = fst;
  }
  __syncthreads();
  const bool use1 = fast != 0;
  // the rows pass 3 multiplies: S itself (fast path), else Q1, kept where pass 3 reads it back
  // (each thread its own rows): over S in LDS, else in out
  const double* Qs = use1 ? Sr : (Sl ? Sl : out);
  const int64_t ldq = use1 ? ldr : (Sl ? nr : ldo);
  const int qo = use1 ? sro : (Sl ? i0 : 0);
  if (use1) {
    ppls_team_leave(tm);   // no further barrier on this path
    ppls_stamp(tr, 4);
  } else {
  double* Qw = Sl ? Sl : out;
  // pass 2: G2 = Q1'Q1, Q1 = S R1^-1
  {
    double M[R][R];
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
      for (int b = 0; b < R; ++b) M[a][b] = sF[b * R + a];
#pragma unroll
    for (int e = 0; e < NG; ++e) vals[e] = 0.0;
    auto pass2 = [&](auto SrP, auto QwP) {
#pragma unroll 2
      for (int i = i0 + tid; i < i1; i += NT) {
        double xq[R], qv[R];
#pragma unroll
        for (int k = 0; k < R; ++k) xq[k] = SrP[(int64_t)k * ldr + i - sro];
#pragma unroll
        for (int j = 0; j < R; ++j) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k <= j; ++k) s = fma(xq[k], M[k][j], s);
          qv[j] = s;
        }
        ppls_gram_acc<R>(qv, vals);
#pragma unroll
        for (int j = 0; j < R; ++j) QwP[(int64_t)j * ldq + i - qo] = qv[j];
      }
    };
    if (Sl) pass2((const ppls_lds_double*)Sl, (ppls_lds_double*)Sl);
    else pass2(Sr, Qw);
  }
  ppls_stamp(tr, 15);
  ppls_block_sum_t<NG, NW>(vals, sh);
  ppls_team_sum<NG>(tm, 1, vals, sh);
  ppls_team_leave(tm);   // the last barrier of this member
  ppls_stamp(tr, 3);
  if (tid < 64) {   // wave 0: R2 = chol(G2), T = R2 R1, warm start, Jacobi, F
    if constexpr (R > PPLS_REG_RMAX) {
      for (int e = lane; e < GG; e += 64) {
        const int a = e % G, b = e / G;
        double v = 0.0;
        if (a < R && b < R) {
          const int lo = a < b ? a : b, hi = a < b ? b : a;
          v = vals[hi * (hi + 1) / 2 + lo];
        }
        sA[e] = v;
      }
    }
    ppls_wave_lds_fence();
    bool good = true;
    if constexpr (R <= PPLS_REG_RMAX) {
      for (int e = lane; e < GG; e += 64) { sA[e] = 0.0; sU[e] = 0.0; }   // (before lane 0's stores)
      if (lane == 0) {
        double P[NG], R1[NG], dinv[R];
#pragma unroll
        for (int e = 0; e < NG; ++e) P[e] = vals[e];
#pragma unroll
        for (int b = 0; b < R; ++b)
#pragma unroll
          for (int a = 0; a <= b; ++a) R1[ppls_pk(a, b)] = sT[b * G + a];
        good = ppls_chol_pk<R>(P, dinv);            // P = R2
#pragma unroll
        for (int b = 0; b < R; ++b)                 // T = R2 R1 (upper); sU = R2
#pragma unroll
          for (int a = 0; a <= b; ++a) {
            double sacc = 0.0;
#pragma unroll
            for (int kk = a; kk <= b; ++kk) sacc = fma(P[ppls_pk(a, kk)], R1[ppls_pk(kk, b)], sacc);
            sA[b * G + a] = sacc;
            sU[b * G + a] = P[ppls_pk(a, b)];
          }
      }
      ppls_wave_lds_fence();
    } else {
      good = ppls_chol_wave<R>(sA, sU);                     // sU = R2
      ppls_matmul_wave<R, false>(sU, sT, sA);               // sA = R2 R1 = T
    }
    ppls_stamp(tr, 6);
    load_vprev();                                          // sV = the carried V, re-orthonormalised
    ppls_matmul_wave<R, false>(sA, sV, sT);                // sT = T V (A of the Jacobi)
    ppls_stamp(tr, 7);
    const int sweeps = ppls_jacobi_wave<R>(sT, sV);
    ppls_stamp(tr, 8);
    if (tr && lane == 0 && tm.K <= 1) tr[10] = sweeps;
    if (lane < R) {
      double nrm = 0.0;
#pragma unroll
      for (int t = 0; t < R; ++t) nrm = fma(sT[lane * G + t], sT[lane * G + t], nrm);
      ssv[lane] = sqrt(nrm);
    }
    ppls_wave_lds_fence();
    double smax = 0.0;
#pragma unroll
    for (int i = 0; i < R; ++i) smax = fmax(smax, ssv[i]);
#pragma unroll
    for (int i = 0; i < R; ++i) good = good && (ssv[i] > smax * 1e-14);
    // P = R2^-1 U_T V' with U_T = (T V) Sigma^-1 (the Jacobi's columns, sT): then the polar factor
    // is Q1 P.  Q1 is the computed factor whose Gram R2 was taken from and R2^-1, U_T V' are well
    // conditioned, so out = Q1 P is orthonormal to O(eps) for any kappa(S) CholQR2 accepts (the
    // one-step form S V Sigma^-1 V' would lose O(eps kappa(S)) of orthogonality).
    ppls_inv_upper_wave<R>(sU, sA);                        // sA = R2^-1
    for (int e = lane; e < GG; e += 64) {                  // sU = U_T V'
      const int a = e % G, b = e / G;
      double s = 0.0;
      if (a < R && b < R)
#pragma unroll
        for (int kk = 0; kk < R; ++kk) s = fma(sT[kk * G + a] * (1.0 / ssv[kk]), sV[kk * G + b], s);
      sU[e] = s;
    }
    ppls_wave_lds_fence();
    for (int e = lane; e < R * R; e += 64) {               // P -> sm + R^2 (ld R)
      const int a = e % R, b = e / R;
      double s = 0.0;
#pragma unroll
      for (int kk = 0; kk < R; ++kk) s = fma(sA[kk * G + a], sU[b * G + kk], s);
      sF[R * R + b * R + a] = s;
      if (vstate && tm.rank == 0) vstate[b * R + a] = sV[b * G + a];   // every member's V is identical
    }
    good = __shfl(good ? 1 : 0, 0, 64) != 0 && good;   // lane 0 holds the chol2 verdict for small R
    // Cholesky-QR2 yields an orthonormal factor only while Q1 = S R1^-1 is nearly orthonormal
    // (||Q1'Q1 - I|| ~ eps kappa(S)^2 small, kappa(S) <~ 1e7): otherwise the Householder fallback
    {
      bool orth_ok = true;
#pragma unroll
      for (int b = 0; b < R; ++b)
#pragma unroll
        for (int a2 = 0; a2 <= b; ++a2)
          orth_ok = orth_ok && fabs(vals[b * (b + 1) / 2 + a2] - (a2 == b ? 1.0 : 0.0)) <= 0.1;
      good = good && orth_ok;
    }
    if (lane == 0) ok = ok && good;
  }
  __syncthreads();
  ppls_stamp(tr, 4);
  if (!ok) return false;
  }   // CholQR2 path
  // pass 3: out = Q1 P, or S F on the fast path (+ Gram of out)
  double F[R][R];
#pragma unroll
  for (int a = 0; a < R; ++a)
#pragma unroll
    for (int b = 0; b < R; ++b) F[a][b] = sF[R * R + b * R + a];
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = 0.0;
  auto pass3 = [&](auto QsP) {
#pragma unroll 2
    for (int i = i0 + tid; i < o1; i += NT) {
      double xq[R], o[R];
#pragma unroll
      for (int k = 0; k < R; ++k) xq[k] = (i < p) ? QsP[(int64_t)k * ldq + i - qo] : 0.0;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < R; ++k) s = fma(xq[k], F[k][j], s);
        o[j] = s;
        out[(int64_t)j * ldo + i] = s;
      }
      ppls_gram_acc<R>(o, vals);
    }
  };
  if (Sl) pass3((const ppls_lds_double*)Sl);   // Qs is the staged S (fast path) or Q1 in LDS
  else pass3(Qs);
  if (use1) ppls_stamp(tr, 3);   // (fast path) pass-3 rows done
  if (gram_out) {
    ppls_block_sum_t<NG, NW>(vals, sh);
    if (use1) ppls_stamp(tr, 15);
    if (tm.K > 1) {   // the last member to finish sums the members' Grams in rank order
      __shared__ int last;
      double* slot = tm.part + ((int64_t)2 * tm.K) * 64;
      if (tid < NG) {
#pragma unroll
        for (int e = 0; e < NG; ++e)
          if (tid == e) slot[(int64_t)tm.rank * 64 + e] = vals[e];
      }
      __syncthreads();
      if (tid == 0) {
        __threadfence();
        last = atomicAdd(&tm.bar[2], 1u) == (unsigned)tm.K - 1;
        if (last) {
          __threadfence();
          atomicExch(&tm.bar[2], 0u);
        }
      }
      __syncthreads();
      if (!last) return true;
      if (tid < NG) {
        double t = 0.0;
        for (int k = 0; k < tm.K; ++k) t += __builtin_nontemporal_load(slot + (int64_t)k * 64 + tid);
        sh[tid] = t;
      }
      __syncthreads();
#pragma unroll
      for (int e = 0; e < NG; ++e) vals[e] = sh[e];
    }
    if (tid == 0) {
      double Gm[R][R];
      ppls_gram_unpack<R>(vals, Gm);
#pragma unroll
      for (int a = 0; a < R; ++a)
#pragma unroll
        for (int b = 0; b < R; ++b) gram_out[b * R + a] = Gm[a][b];
    }
  }
  return true;
}

// Gram out'out of a p x R column-major matrix written earlier by this block (fallback path).
template <int R, int NT>
__device__ void ppls_block_gram_of(const double* __restrict__ M, int64_t ld, int p, double* sh,
                                   double* __restrict__ gram_out) {
  constexpr int NG = R * (R + 1) / 2;
  double vals[NG];
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = 0.0;
  for (int i = threadIdx.x; i < p; i += NT) {
    double x[R];
#pragma unroll
    for (int k = 0; k < R; ++k) x[k] = M[(int64_t)k * ld + i];
    ppls_gram_acc<R>(x, vals);
  }
  ppls_block_sum_t<NG>(vals, sh);
  if (threadIdx.x == 0) {
    double G[R][R];
    ppls_gram_unpack<R>(vals, G);
#pragma unroll
    for (int a = 0; a < R; ++a)
#pragma unroll
      for (int b = 0; b < R; ++b) gram_out[b * R + a] = G[a][b];
  }
}

// Sum over the 64 lanes of a wave; every lane gets the bitwise-same total.
__device__ __forceinline__ double ppls_wave_allsum(double v) {
  double a[2] = {v, 0.0};
  int idx = 0;
  bool canon = true;
  ppls_rs<1, 0, 2>(a, threadIdx.x & 63, idx, canon);
  return a[0];
}

// The finalize's scalar part on one wave: lane k < R evaluates component k (coefficients, diagonal
// moments, log-likelihood terms, M-step, next mu coefficients), lane k + R l < R^2 the pair
// (k, l) terms; the O(1) combinations use wave sums.  Same formulas as the serial host form
// (ppls_estep_moments, ppls_loglik_from_gram, ppls_mstep_scalars in ppls_math.h); only the
// summation order differs.  sG, sWtW, sCtC, sc, m, nx live in LDS; nx must hold a copy of *sc.
template <int R>
__device__ void ppls_scalars_wave(const double* sG, const double* sWtW, const double* sCtC, double ssqX,
                                  double ssqY, double N, int p, int q, const PplsScalars* sc,
                                  PplsMoments* m, PplsScalars* nx, double* loglik_out) {
  const int lane = threadIdx.x & 63;
  const bool kact = lane < R;
  const int k = kact ? lane : 0;
  double c1, c2, c3;
  ppls_coef_estep(sc->t[k], sc->b[k], sc->sigE, sc->sigF, sc->sigH, &c1, &c2, &c3, nullptr);
  double Ctt, Cuu, Cut, xk, yk;
  ppls_moment_diag(sG, R, k, sc, c1, c2, c3, N, &Ctt, &Cuu, &Cut, &xk, &yk);
  double zsum = 0.0, wsum = 0.0, hsum = 0.0;
#pragma unroll
  for (int u = 0; u < (R * R + 63) / 64; ++u) {   // component pairs (k, l) on lanes
    const int e = lane + 64 * u;
    const bool pact = e < R * R;
    const int pk = pact ? e % R : 0, pl = pact ? e / R : 0;
    const double c1k = __shfl(c1, pk, 64), c2k = __shfl(c2, pk, 64), c3k = __shfl(c3, pk, 64);
    const double c1l = __shfl(c1, pl, 64), c2l = __shfl(c2, pl, 64), c3l = __shfl(c3, pl, 64);
    double z, w, chh;
    ppls_moment_pair(sG, R, pk, pl, c1k, c2k, c3k, c1l, c2l, c3l, sWtW[pl * R + pk], sCtC[pl * R + pk],
                     sc, N, &z, &w, &chh);
    if (pact) {
      zsum += z;
      wsum += w;
      if (pk == pl) hsum += chh;
      m->Chh[pl * R + pk] = chh;
    }
  }
  const double xz = ppls_wave_allsum(kact ? xk : 0.0), yz = ppls_wave_allsum(kact ? yk : 0.0);
  const double sc1 = ppls_wave_allsum(kact ? c1 : 0.0), sc3 = ppls_wave_allsum(kact ? c3 : 0.0);
  const double zz = ppls_wave_allsum(zsum), ww = ppls_wave_allsum(wsum);
  const double trChh = ppls_wave_allsum(hsum);
  double Cee, Cff;
  ppls_moment_noise(ssqX, ssqY, N, p, q, sc, xz, yz, zz, ww, sc1, sc3, &Cee, &Cff);
  if (loglik_out) {
    double lg, tk;
    ppls_logl_k(sG, R, k, sc, &lg, &tk);
    const double LG = ppls_wave_allsum(kact ? lg : 0.0), TK = ppls_wave_allsum(kact ? tk : 0.0);
    if (lane == 0) *loglik_out = ppls_logl_total(LG, TK, ssqX, ssqY, N, p, q, R, sc);
  }
  if (kact) { m->Ctt[k] = Ctt; m->Cuu[k] = Cuu; m->Cut[k] = Cut; }
  // Maximiz_M scalars (EM_W_multi.R:734-738) and the next mu coefficients (:691-694)
  const double sE = sqrt(Cee / 1.0), sF = sqrt(Cff / 1.0), sH = sqrt(trChh / (double)R);
  const double bn = Cut * (1.0 / Ctt), tn = sqrt(Ctt);
  double al, be, ga, de;
  ppls_mu_coef_k(tn, bn, sE, sF, sH, &al, &be, &ga, &de);
  if (kact) {
    nx->b[k] = bn; nx->t[k] = tn;
    nx->alpha[k] = al; nx->beta[k] = be; nx->gamma[k] = ga; nx->delta[k] = de;
  }
  if (lane == 0) {
    m->Cee = Cee; m->Cff = Cff;
    nx->sigE = sE; nx->sigF = sF; nx->sigH = sH;
  }
}

// The PPLS_simult stop rule on the device (EM_W_multi.R:792: logl[i] - logl[i-1] < atol, i > 1),
// evaluated by one thread right after it wrote loglik[idx]: sets the stop flag (every later kernel
// of the run then exits at once) and its host-mapped mirror the host polls.  A NaN increment is
// R's `if (NA < atol)`, which stops PPLS_simult with an error: the run stops there too and
// stop[1] = 1 tells the host to report it (every rank computes the same all-reduced increment).
__device__ __forceinline__ void ppls_stop_test(const double* loglik, int idx, int* stop, int* stop_mirror,
                                               int stop_check, int stop_step, double atol) {
  if (!stop_check || !stop || idx < 1) return;
  const double d = loglik[idx] - loglik[idx - 1];
  const bool nan = d != d;
  if (nan || d < atol) {
    if (nan) stop[1] = 1;
    *stop = stop_step;
    if (stop_mirror) __hip_atomic_store(stop_mirror, stop_step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The cross-product form's Gram B'M (B = blockdiag(W, C), M = S B) on the finalize's scalar block,
// in the slack of the polar blocks: entries (a, b) of the X rows with a < r, b in [a, 2r)
// (W'X'XW upper triangle, then W'X'YC) and of the Y rows with a <= b < r (C'Y'YC upper triangle),
// 2r^2 + r sums, in passes of 64 entries (one pass up to r = 5; 3 at r = 8, which re-read the rows
// from L2 but keep 64 accumulators per thread instead of 192 -- all of them spilled to scratch):
// per thread a stride of rows, then ppls_block_sum_t.  Written mirrored to sG (LDS, what the
// moments read) and G (stats' Gram slot).  r <= 8.
template <int R, int NT>
__device__ void ppls_xp_gram_block(const double* __restrict__ M, const double* __restrict__ Wc,
                                   const double* __restrict__ Cc, int ldx, int ldy, double* sG, double* G,
                                   long long* tr) {
  constexpr int R2 = 2 * R, NX = R * (R + 1) / 2 + R * R, NE = NX + R * (R + 1) / 2;
  constexpr int NPASS = (NE + 63) / 64;
  // U rows per thread per batch, all their loads issued before the FMAs: M was just written by the
  // tile kernel on other XCDs, so every load is a far (MALL) round trip, and one batch of U rows
  // costs one round trip instead of U.  Rows past the end load the last row with weight 0 (adds
  // +-0: the sums equal the row-by-row loop's bitwise).
  constexpr int U = R <= 5 ? 4 : (R == 6 ? 2 : 1);   // larger batches spill beyond r = 5
  __shared__ double sh[(NT / 64) * 64];
  const int P = ldx + ldy, tid = threadIdx.x;
#pragma unroll
  for (int ps = 0; ps < NPASS; ++ps) {
    const int lo = ps * 64;
    double acc[64];
#pragma unroll
    for (int e = 0; e < 64; ++e) acc[e] = 0.0;
    if (lo < NX) {
      for (int i0 = tid; i0 < ldx; i0 += U * NT) {
        double w[U][R], m[U][R2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = min(i0 + u * NT, ldx - 1);
#pragma unroll
          for (int a = 0; a < R; ++a) w[u][a] = Wc[(int64_t)a * ldx + i];
#pragma unroll
          for (int b = 0; b < R2; ++b) m[u][b] = M[(int64_t)b * P + i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = i0 + u * NT < ldx;
          int e = 0;
#pragma unroll
          for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = a; b < R2; ++b, ++e)
              if (e >= lo && e < lo + 64) acc[e - lo] = fma(ok ? w[u][a] : 0.0, m[u][b], acc[e - lo]);
        }
      }
    }
    if (ps == 0) ppls_stamp(tr, 5);   // X rows of the first pass
    if (lo + 64 > NX) {
      for (int i0 = tid; i0 < ldy; i0 += U * NT) {
        double cv[U][R], m[U][R];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = min(i0 + u * NT, ldy - 1);
#pragma unroll
          for (int a = 0; a < R; ++a) cv[u][a] = Cc[(int64_t)a * ldy + i];
#pragma unroll
          for (int b = 0; b < R; ++b) m[u][b] = M[(int64_t)(R + b) * P + ldx + i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = i0 + u * NT < ldy;
          int e = NX;
#pragma unroll
          for (int a = 0; a < R; ++a)
#pragma unroll
            for (int b = a; b < R; ++b, ++e)
              if (e >= lo && e < lo + 64) acc[e - lo] = fma(ok ? cv[u][a] : 0.0, m[u][b], acc[e - lo]);
        }
      }
    }
    if (ps == 0) ppls_stamp(tr, 6);   // rows of the first pass summed per thread
    // block sums as ppls_block_sum_t forms them (wave reduce-scatter, then the waves' partials in
    // wave order), but each entry summed and placed by its own thread
    {
      constexpr int NW = NT / 64;
      const int lane = tid & 63, wave = tid >> 6;
      int idx = 0;
      bool canon = true;
      ppls_rs<64, 0, 64>(acc, lane, idx, canon);
      if (canon && idx < 64) sh[wave * 64 + idx] = acc[0];
      __syncthreads();
      const int e = lo + tid;
      if (tid < 64 && e < NE) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += sh[w * 64 + tid];
        int a = 0, b, f = e;   // entry e -> (a, b): X rows' (a <= b < 2R), then Y rows' (a <= b < R)
        const bool yp = f >= NX;
        if (yp) f -= NX;
        const int span = yp ? R : R2;
        while (f >= span - a) {
          f -= span - a;
          ++a;
        }
        b = a + f;
        const int o = yp ? R : 0;
        sG[(o + b) * R2 + o + a] = t;
        sG[(o + a) * R2 + o + b] = t;
        G[(o + b) * R2 + o + a] = t;
        G[(o + a) * R2 + o + b] = t;
      }
      __syncthreads();
    }
    if (ps == 0) ppls_stamp(tr, 7);
  }
}

#define PPLS_FIN_THREADS 256   // 1 wave per SIMD: the r x r code may use all 512 VGPR+AGPRs

// Block 0: W_next = orth(S_X); block 1: C_next = orth(S_Y); block 2: scalars (moments, loglik,
// M-step).  stats = [SX ldx*R][SY ldy*R][G 4R^2];  ssq = {||X||^2, ||Y||^2}.
// gram_cur = [W'W | C'C] of the parameters the sweep used (written by the previous finalize or
// by the host upload); the polar blocks write gram_nxt for the parameters they produce, so the
// scalar block needs no pass over W and C.  Dynamic LDS (if any) stages S for the polar blocks.
template <int R>
__global__ __launch_bounds__(PPLS_FIN_THREADS) void ppls_finalize_kernel(
    const double* __restrict__ stats, const double* __restrict__ ssq, double N, int p, int q, int ldx,
    int ldy, const double* __restrict__ Wc, const double* __restrict__ Cc,
    const PplsScalars* __restrict__ sc_cur, double* __restrict__ Wn, double* __restrict__ Cn,
    PplsScalars* __restrict__ sc_nxt, PplsMoments* __restrict__ mom, double* __restrict__ loglik,
    int logl_index, double* __restrict__ work, int* __restrict__ status, int qr, int mode,
    const double* __restrict__ gram_cur, double* __restrict__ gram_nxt, double* __restrict__ vstate,
    int stage_lds, long long* __restrict__ trace,
    int* __restrict__ stop, int* __restrict__ stop_mirror, int stop_check, int stop_step, double atol,
    int KX, int KY, unsigned* __restrict__ team_bar, double* __restrict__ team_part, const double* __restrict__ xpM) {
  // em_run converged at an EARLIER iteration: exit.  The flag this launch's own scalar block may
  // set (== stop_step) must not stop a polar-team member that starts late, or its teammates would
  // wait at the team barrier for a member that never comes.
  if (stop && *stop && *stop != stop_step) return;
  constexpr int NT = PPLS_FIN_THREADS;
  constexpr int NG = R * (R + 1) / 2;
  extern __shared__ double dyn_lds[];
  __shared__ double sh[(NT / 64) * 2 * NG];
  __shared__ double sm[2 * R * R];
  __shared__ PplsScalars s_cur, s_nx;
  __shared__ PplsMoments s_m;
  __shared__ double s_G[4 * R * R], s_WtW[R * R], s_CtC[R * R];
  const double* SX = stats;
  const double* SY = stats + (int64_t)R * ldx;
  const double* G = SY + (int64_t)R * ldy;
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  // blocks [0, KX): the team computing W_next; [KX, KX + KY): C_next; the last block: scalars
  const int slot = b < KX ? 0 : b < KX + KY ? 1 : 2;
  const bool lead = b == 0 || b == KX || b == KX + KY;   // member 0 of its team / the scalar block
  long long* tr = (trace && lead) ? trace + 16 * slot : nullptr;
  ppls_stamp(tr, 0);
  if (tr && tid == 0) tr[11] = (long long)clock64();
  if (slot < 2) {
    if (!(mode & 1)) return;
    const bool isx = slot == 0;
    const double* S = isx ? SX : SY;
    const int ld = isx ? ldx : ldy, rows = isx ? p : q;
    double* out = isx ? Wn : Cn;
    double* gout = gram_nxt ? gram_nxt + (isx ? 0 : R * R) : nullptr;
    // W'W of the new loadings (the next scalar update's Gram), computed exactly (mode bit 16, the
    // default) or taken as I (they are orthonormal to O(eps kappa^2) <= 1e-13, and a team's pass 3
    // then needs no last-member exchange; but Cee = (||X||^2 - 2 s tr + s^2 tr(Z'Z G)) / (N p)
    // cancels at small sigma_E and amplifies the difference: option exact_gram).
    const bool exact_gram = (mode & 16) != 0;
    double* gacc = exact_gram ? gout : nullptr;
    double* w2 = work + (isx ? 0 : 2 * (int64_t)p * R);
    double* vs = vstate ? vstate + (isx ? 0 : R * R) : nullptr;
    PplsTeam tm;
    tm.K = isx ? KX : KY;
    tm.rank = isx ? b : b - KX;
    tm.bar = team_bar + (isx ? 0 : 4);
    tm.part = team_part + (isx ? 0 : (int64_t)3 * PPLS_TEAM_MAX * 64);
    tm.status = status;
    tm.tr = tr;
    if (qr || !ppls_block_polar_fast<R, NT>(S, ld, rows, out, ld, ld, stage_lds ? dyn_lds : nullptr, sh,
                                            sm, gacc, vs, tr, tm, (mode & 4) != 0,
                                            (double)((mode >> 8) & 255),
                                            logl_index < 0 || ((mode >> 16) & 255) <= 1 ||
                                                logl_index % ((mode >> 16) & 255) == 0)) {
      if (tm.rank != 0) return;   // the Householder fallback runs on one block
      ppls_block_polar(S, ld, rows, R, out, ld, ld, w2, w2 + (int64_t)rows * R, status, qr);
      if (gacc) {
        __syncthreads();
        ppls_block_gram_of<R, NT>(out, ld, rows, sh, gacc);
      }
    }
    if (gout && !exact_gram && tm.rank == 0)
      for (int e = tid; e < R * R; e += NT) gout[e] = (e % (R + 1) == 0) ? 1.0 : 0.0;
    ppls_stamp(tr, 5);
    if (tr && tid == 0) tr[12] = (long long)clock64();
    return;
  }
  if (!(mode & 2)) return;
  // stage theta's scalars, the Gram and W'W, C'C in LDS (all threads) -- first, so that these loads
  // are not one more far round trip after the cross-product Gram's
  {
    const double* src = (const double*)sc_cur;
    double* dst = (double*)&s_cur;
    for (int i = tid; i < (int)(sizeof(PplsScalars) / 8); i += NT) dst[i] = src[i];
    if (!xpM || R > 8)
      for (int i = tid; i < 4 * R * R; i += NT) s_G[i] = G[i];
    if (gram_cur)
      for (int i = tid; i < R * R; i += NT) { s_WtW[i] = gram_cur[i]; s_CtC[i] = gram_cur[R * R + i]; }
  }
  // cross-product form: the Gram of [XW YC] = B'M from M = S B (the polar blocks run meanwhile)
  if constexpr (R <= 8)
    if (xpM) ppls_xp_gram_block<R, NT>(xpM, Wc, Cc, ldx, ldy, s_G, const_cast<double*>(G), tr);
  ppls_stamp(tr, 8);
  if (!gram_cur) {   // W'W and C'C by a pass over W, then one over C
    for (int mat = 0; mat < 2; ++mat) {
      const double* M = mat ? Cc : Wc;
      const int ld = mat ? ldy : ldx, rows = mat ? q : p;
      double* dst = mat ? s_CtC : s_WtW;
      double vals[NG];
#pragma unroll
      for (int e = 0; e < NG; ++e) vals[e] = 0.0;
      for (int i = tid; i < rows; i += NT) {
        double wv[R];
#pragma unroll
        for (int k = 0; k < R; ++k) wv[k] = M[(int64_t)k * ld + i];
        ppls_gram_acc<R>(wv, vals);
      }
      ppls_block_sum_t<NG, NT / 64>(vals, sh);
      if (tid == 0) {
        int e = 0;
        for (int b = 0; b < R; ++b)
          for (int a = 0; a <= b; ++a) {
            dst[b * R + a] = dst[a * R + b] = vals[e];
            ++e;
          }
      }
    }
  }
  __syncthreads();
  {
    const double* a = (const double*)&s_cur;
    double* b = (double*)&s_nx;
    for (int i = tid; i < (int)(sizeof(PplsScalars) / 8); i += NT) b[i] = a[i];
  }
  __syncthreads();
  ppls_stamp(tr, 1);
  if (tid < 64)
    ppls_scalars_wave<R>(s_G, s_WtW, s_CtC, ssq[0], ssq[1], N, p, q, &s_cur, &s_m, &s_nx,
                         logl_index >= 0 ? loglik + logl_index : nullptr);
  __syncthreads();
  if (tid == 0) ppls_stop_test(loglik, logl_index, stop, stop_mirror, stop_check, stop_step, atol);
  ppls_stamp(tr, 2);
  {
    const double* a = (const double*)&s_m;
    double* b = (double*)mom;
    for (int i = tid; i < (int)(sizeof(PplsMoments) / 8); i += NT) b[i] = a[i];
    const double* c = (const double*)&s_nx;
    double* d = (double*)sc_nxt;
    for (int i = tid; i < (int)(sizeof(PplsScalars) / 8); i += NT) d[i] = c[i];
  }
}

// Generic finalize for r > 8 (runtime r; Householder polar).  Block 0: W_next = orth(S_X);
// block 1: C_next = orth(S_Y); block 2: scalars.
// stats = [SX ldx*r][SY ldy*r][G 4r^2];  ssq = {||X||^2, ||Y||^2}.
__global__ __launch_bounds__(256) void ppls_finalize_generic_kernel(
    const double* __restrict__ stats, const double* __restrict__ ssq, double N, int p, int q, int r,
    int ldx, int ldy, const double* __restrict__ Wc, const double* __restrict__ Cc,
    const PplsScalars* __restrict__ sc_cur, double* __restrict__ Wn, double* __restrict__ Cn,
    PplsScalars* __restrict__ sc_nxt, PplsMoments* __restrict__ mom, double* __restrict__ loglik,
    int logl_index, double* __restrict__ work, int* __restrict__ status, int qr, int mode,
    int* __restrict__ stop, int* __restrict__ stop_mirror, int stop_check, int stop_step, double atol) {
  if (stop && *stop && *stop != stop_step) return;   // converged at an earlier iteration
  const double* SX = stats;
  const double* SY = stats + (int64_t)r * ldx;
  const double* G = SY + (int64_t)r * ldy;
  if (blockIdx.x == 0) {
    if (mode & 1) ppls_block_polar(SX, ldx, p, r, Wn, ldx, ldx, work, work + (int64_t)p * r, status, qr);
    return;
  }
  if (blockIdx.x == 1) {
    double* w2 = work + 2 * (int64_t)p * r;
    if (mode & 1) ppls_block_polar(SY, ldy, q, r, Cn, ldy, ldy, w2, w2 + (int64_t)q * r, status, qr);
    return;
  }
  if (!(mode & 2)) return;
  __shared__ double sh[16 * PPLS_RMAX];
  __shared__ double WtW[PPLS_RMAX * PPLS_RMAX], CtC[PPLS_RMAX * PPLS_RMAX];
  double vals[PPLS_RMAX];
  for (int a = 0; a < r; ++a) {
    for (int b = 0; b < r; ++b) vals[b] = 0.0;
    for (int i = threadIdx.x; i < p; i += blockDim.x) {
      const double wa = Wc[(int64_t)a * ldx + i];
      for (int b = 0; b < r; ++b) vals[b] = fma(wa, Wc[(int64_t)b * ldx + i], vals[b]);
    }
    ppls_block_sum(vals, r, sh);
    if (threadIdx.x == 0)
      for (int b = 0; b < r; ++b) WtW[b * r + a] = vals[b];
    for (int b = 0; b < r; ++b) vals[b] = 0.0;
    for (int i = threadIdx.x; i < q; i += blockDim.x) {
      const double ca = Cc[(int64_t)a * ldy + i];
      for (int b = 0; b < r; ++b) vals[b] = fma(ca, Cc[(int64_t)b * ldy + i], vals[b]);
    }
    ppls_block_sum(vals, r, sh);
    if (threadIdx.x == 0)
      for (int b = 0; b < r; ++b) CtC[b * r + a] = vals[b];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    PplsScalars cur = *sc_cur;
    if (logl_index >= 0) loglik[logl_index] = ppls_loglik_from_gram(G, ssq[0], ssq[1], N, p, q, r, &cur);
    ppls_stop_test(loglik, logl_index, stop, stop_mirror, stop_check, stop_step, atol);
    PplsMoments m;
    ppls_estep_moments(G, WtW, CtC, ssq[0], ssq[1], N, p, q, r, &cur, &m);
    *mom = m;
    PplsScalars nx = cur;
    ppls_mstep_scalars(&m, r, &nx);
    *sc_nxt = nx;
  }
}

// ============================================================================ initialiser step
// Loading update of one rank-1 EM step (EMstepC_fast, src/loglC.cpp:357, :385): t = S (the sweep's
// X'mu_T over the undeflated data), deflated t = P_{m-1}..P_0 t (= Xc'mu_T), t /= N, normalised --
// or the fixed loading of an fconstraint -- then the next sweep's weight dst = P_0..P_{m-1} t
// (so the sweep over X computes Xc t).  Every thread keeps its own indices i = tid + k * nt, so
// only the block sums synchronise.
__device__ void ppls_rank1_loading(const double* __restrict__ S, int n, double* __restrict__ t,
                                   const double* __restrict__ Wp, int m, double N, const double* __restrict__ fixed,
                                   double* __restrict__ dst, int ld, double* sh) {
  const int tid = threadIdx.x, nt = blockDim.x;
  double v[1];
  if (fixed) {
    for (int i = tid; i < n; i += nt) t[i] = fixed[i];
  } else {
    for (int i = tid; i < n; i += nt) t[i] = S[i];
    for (int j = 0; j < m; ++j) {
      const double* w = Wp + (int64_t)j * n;
      v[0] = 0.0;
      for (int i = tid; i < n; i += nt) v[0] = fma(w[i], t[i], v[0]);
      ppls_block_sum(v, 1, sh);
      const double d = v[0];
      for (int i = tid; i < n; i += nt) t[i] -= d * w[i];
    }
    v[0] = 0.0;
    for (int i = tid; i < n; i += nt) {
      t[i] /= N;
      v[0] = fma(t[i], t[i], v[0]);
    }
    ppls_block_sum(v, 1, sh);
    const double nrm = sqrt(v[0]);
    for (int i = tid; i < n; i += nt) t[i] /= nrm;
  }
  for (int i = tid; i < ld; i += nt) dst[i] = i < n ? t[i] : 0.0;
  for (int jj = 0; jj < m; ++jj) {
    const double* w = Wp + (int64_t)(m - 1 - jj) * n;
    v[0] = 0.0;
    for (int i = tid; i < n; i += nt) v[0] = fma(w[i], dst[i], v[0]);
    ppls_block_sum(v, 1, sh);
    const double d = v[0];
    for (int i = tid; i < n; i += nt) dst[i] -= d * w[i];
  }
}

// One EM step of PPLSi (EM_W_multi.R:151-173) on the device, after the sweep of the current
// component t: logvalue[step] = logl_W(t) from the sweep's Gram (:149, :172); the stop rule
// critfunc(logvalue[i] - logvalue[i-1]) < atol (:173); the sigma < 100 eps guard (:152-154); then
// EMstepC_fast's update (scalars ppls_rank1_scalars, loadings above), the constraints (:165-169)
// and the next sweep's weights and scalars.  Once the fit has ended, every later sweep and step
// kernel of it exits at once (the stop flag).
__global__ __launch_bounds__(1024) void ppls_rank1_step_kernel(PplsRank1StepArgs a) {
  __shared__ double sh[16 * PPLS_RMAX];
  __shared__ int s_exit;
  __shared__ PplsRank1 s_new;
  const int tid = threadIdx.x;
  if (a.stop[0] || a.stop[1]) return;
  if (tid == 0) {
    const double* Gs = a.stats + a.ldx + a.ldy;
    const double G[4] = {Gs[0], Gs[1], Gs[2], Gs[3]};
    const PplsRank1 t = *a.st;
    const double l = ppls_rank1_loglik(&t, G, a.ssqX, a.ssqY, a.N, a.p, a.q);
    a.lv[a.step] = l;
    for (int e = 0; e < 4; ++e) a.Gkeep[e] = G[e];
    int ex = 0;
    if (a.step >= 1) {
      const double incr = l - a.lv[a.step - 1];
      if ((a.crit_abs ? fabs(incr) : incr) < a.atol) {
        a.stop[0] = a.step;
        ex = 1;
      } else if (incr != incr) {   // `if (critfunc(NA) < atol)` stops PPLSi with an error (:173)
        a.stop[0] = a.step;
        a.stop[1] = 2;
        ex = 1;
      }
    }
    if (!ex && a.step >= a.max_steps) ex = 1;
    const double tiny = 100.0 * 2.220446049250313e-16;   // 100 * .Machine$double.eps
    if (!ex && (t.sigE < tiny || t.sigF < tiny)) {
      a.stop[1] = 1;
      a.stop[0] = -(a.step + 1);   // nonzero: the fit's remaining sweeps exit at entry too
      ex = 1;
    }
    // mirror = the step the fit ended at + 1, so every rank can break at the same host iteration
    if (ex && a.stop_mirror)
      __hip_atomic_store(a.stop_mirror, a.step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!ex) {
      PplsRank1 n;
      ppls_rank1_scalars(&t, G, a.ssqX, a.ssqY, a.N, a.p, a.q, &n);
      if (a.cons_mask & 1) n.B = a.cons_val.B;
      if (a.cons_mask & 2) n.sigE = a.cons_val.sigE;
      if (a.cons_mask & 4) n.sigF = a.cons_val.sigF;
      if (a.cons_mask & 8) n.sigH = a.cons_val.sigH;
      if (a.cons_mask & 16) n.sigT = a.cons_val.sigT;
      s_new = n;
    }
    s_exit = ex;
  }
  __syncthreads();
  if (s_exit) return;
  ppls_rank1_loading(a.stats, a.p, a.tw, a.Wp, a.m, a.N, a.consW, a.Wdst, a.ldx, sh);
  ppls_rank1_loading(a.stats + a.ldx, a.q, a.tc, a.Cp, a.m, a.N, a.consC, a.Cdst, a.ldy, sh);
  if (tid == 0) {
    *a.st = s_new;
    ppls_rank1_sweep_scalars(&s_new, a.scdst);
  }
}

// One EM step of meta_PPLSi (EM_W_multi.R:551-578) on the device, after the segmented sweep of the
// current parameters theta_i over every population (its per-population statistics stats[j] =
// [X_j'mu_T | Y_j'mu_U | Gram]):
//   step >= 1: logvalue[i+1, j] = logl_W of population j from its Gram (:571-573), the stop rule on
//              critfunc(sum(logvalue[i+1, ]) - sum(logvalue[i, ])) < atol (:575) -- a NaN increment
//              is R's `if (NA < atol)` error (stop[1] = 2) -- and the end of EMsteps;
//   then, unless the fit ended: meta_EMstep's M-step (:453-484): meta_Mstep per population
//              (ppls_rank1_scalars, the EMstepC_fast formulas with N_j, ssq(X_j), ssq(Y_j)), and the
//              shared W. = orth(sum_j sign(<Cxt_1, Cxt_j>) Cxt_j), C. likewise (Cxt_j = X_j'mu_T / N_j,
//              orth of one column = v / ||v||), written as the next sweep's loadings and scalars.
// One 1024-thread block: population j's scalars on thread j, the p- and q-long sums block-wide.
__global__ __launch_bounds__(1024) void ppls_meta_step_kernel(PplsMetaStepArgs a) {
  __shared__ double sh[16 * PPLS_RMAX];
  __shared__ int s_end;
  __shared__ double s_sg[PPLS_META_KMAX];
  const int tid = threadIdx.x, K = a.K;
  if (a.stop[0]) return;   // the fit ended at an earlier step
  const double* Gs = a.stats + a.ldx + a.ldy;   // population j's Gram at Gs + j part_ld
  if (a.step == 0 && tid == 0) {   // logvalue[1, ] = rep(logl_W(X, Y, theta0), K) (:544)
    double G[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < K; ++j)
      for (int e = 0; e < 4; ++e) G[e] += Gs[(int64_t)j * a.part_ld + e];
    const double l0 = ppls_rank1_loglik(&a.st[0], G, a.ssqX, a.ssqY, a.Ntot, a.p, a.q);
    for (int j = 0; j < K; ++j) a.log[(int64_t)j * a.log_ld] = l0;
  }
  if (a.step >= 1) {
    double l = 0.0;
    if (tid < K) {
      const double* G = Gs + (int64_t)tid * a.part_ld;
      const double Gj[4] = {G[0], G[1], G[2], G[3]};
      l = ppls_rank1_loglik(&a.st[tid], Gj, a.ssq[2 * tid], a.ssq[2 * tid + 1], a.N[tid], a.p, a.q);
      a.log[(int64_t)tid * a.log_ld + a.step] = l;
    }
    __syncthreads();
    if (tid == 0) {
      double s_new = 0.0, s_old = 0.0;   // population order, like the host's sums
      for (int j = 0; j < K; ++j) {
        s_new += a.log[(int64_t)j * a.log_ld + a.step];
        s_old += a.log[(int64_t)j * a.log_ld + a.step - 1];
      }
      const double incr = s_new - s_old;
      int end = 0;
      if (incr != incr) {
        a.stop[1] = 2;
        end = 1;
      } else if ((a.crit_abs ? fabs(incr) : incr) < a.atol || a.step >= a.max_steps) {
        end = 1;
      }
      if (end) {
        a.stop[0] = a.step;
        if (a.stop_mirror) __hip_atomic_store(a.stop_mirror, a.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      s_end = end;
    }
    __syncthreads();
    if (s_end) return;
  }
  // M-step: signs of <SX_1 / N_1, SX_j / N_j>, then the shared loadings
  const double N1 = a.N[0];
  for (int j0 = 0; j0 < K; j0 += PPLS_RMAX) {
    const int nj = K - j0 < PPLS_RMAX ? K - j0 : PPLS_RMAX;
    double v[PPLS_RMAX];
    for (int u = 0; u < nj; ++u) v[u] = 0.0;
    for (int i = tid; i < a.p; i += blockDim.x) {
      const double x1 = a.stats[i] / N1;
      for (int u = 0; u < nj; ++u) v[u] = fma(x1, a.stats[(int64_t)(j0 + u) * a.part_ld + i] / a.N[j0 + u], v[u]);
    }
    ppls_block_sum(v, nj, sh);
    if (tid == 0)
      for (int u = 0; u < nj; ++u) s_sg[j0 + u] = v[u] > 0 ? 1.0 : (v[u] < 0 ? -1.0 : 0.0);   // R's sign()
  }
  __syncthreads();
  double nrm[2] = {0.0, 0.0};
  for (int i = tid; i < a.ldx; i += blockDim.x) {
    double w = 0.0;
    if (i < a.p)
      for (int j = 0; j < K; ++j) w += s_sg[j] * (a.stats[(int64_t)j * a.part_ld + i] / a.N[j]);
    a.W[i] = w;
    nrm[0] = fma(w, w, nrm[0]);
  }
  for (int i = tid; i < a.ldy; i += blockDim.x) {
    double cv = 0.0;
    if (i < a.q)
      for (int j = 0; j < K; ++j) cv += s_sg[j] * (a.stats[(int64_t)j * a.part_ld + a.ldx + i] / a.N[j]);
    a.C[i] = cv;
    nrm[1] = fma(cv, cv, nrm[1]);
  }
  ppls_block_sum(nrm, 2, sh);
  const double nw = sqrt(nrm[0]), nc = sqrt(nrm[1]);
  for (int i = tid; i < a.ldx; i += blockDim.x) a.W[i] /= nw;
  for (int i = tid; i < a.ldy; i += blockDim.x) a.C[i] /= nc;
  if (tid < K) {   // meta_Mstep of population tid, then its next sweep's mu coefficients
    const double* G = Gs + (int64_t)tid * a.part_ld;
    const double Gj[4] = {G[0], G[1], G[2], G[3]};
    PplsRank1 nt;
    ppls_rank1_scalars(&a.st[tid], Gj, a.ssq[2 * tid], a.ssq[2 * tid + 1], a.N[tid], a.p, a.q, &nt);
    a.st[tid] = nt;
    ppls_rank1_sweep_scalars(&nt, &a.sc[tid]);
  }
}

hipError_t ppls_launch_meta_step(const PplsMetaStepArgs* a, hipStream_t st) {
  if (a->K < 1 || a->K > PPLS_META_KMAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(ppls_meta_step_kernel, dim3(1), dim3(1024), 0, st, *a);
  return hipGetLastError();
}

// loglC_fast from explicit coefficients (the drop-in of src/loglC.cpp:318-338).
__global__ void ppls_loglc_kernel(const double* __restrict__ G, const double* __restrict__ ssq, double N,
                                  int p, int q, int r, double sigX, double sigY,
                                  const double* __restrict__ coefs, double* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const double* sig2T = coefs;
    *out = ppls_loglc_fast_from_gram(G, ssq[0], ssq[1], N, p, q, r, sigX, sigY, sig2T, coefs + r,
                                     coefs + 2 * r, coefs + 3 * r, coefs + 4 * r);
  }
}

// ============================================================================ launchers
namespace {
#define PPLS_FIN_STAGE_MAX (136 * 1024)   // dynamic LDS for staging S (static use is < 8 KB)

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device, size): contexts on
// different devices or host threads each get the attribute set on their own current device.
hipError_t set_dyn_lds(const void* kern, int bytes) {
  static std::mutex mu;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_tuple(kern, dev, bytes);
  if (done.count(key)) return hipSuccess;
  e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e == hipSuccess) done.insert(key);
  return e;
}

template <int R>
hipError_t launch_finalize_t(const PplsFinalizeArgs* f, hipStream_t st) {
  auto kern = ppls_finalize_kernel<R>;
  // dynamic LDS left next to the kernel's static LDS (160 KB per WG); thread-safe static init
  static const size_t dyn_max = []() -> size_t {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, (const void*)ppls_finalize_kernel<R>) != hipSuccess) return 0;
    const size_t budget = 160 * 1024 - fa.sharedSizeBytes - 1024;
    return budget < PPLS_FIN_STAGE_MAX ? budget : PPLS_FIN_STAGE_MAX;
  }();
  if (dyn_max == 0) return hipErrorInvalidDeviceFunction;
  {
    const hipError_t e = set_dyn_lds((const void*)kern, (int)dyn_max);
    if (e != hipSuccess) return e;
  }
  // teams for wide p: one member per PPLS_TEAM_ROWS rows (QR: one block, Householder)
  auto team = [&](int rows) {
    if (f->qr || !f->team_bar) return 1;
    const int tr = f->team_rows > 0 ? f->team_rows : PPLS_TEAM_ROWS;
    const int k = (rows + tr - 1) / tr;
    return k < 1 ? 1 : k > PPLS_TEAM_MAX ? PPLS_TEAM_MAX : k;
  };
  const int KX = team(f->p), KY = team(f->q);
  const int mrows = (f->p + KX - 1) / KX > (f->q + KY - 1) / KY ? (f->p + KX - 1) / KX : (f->q + KY - 1) / KY;
  const size_t stage = (size_t)R * mrows * sizeof(double);   // a member stages its own rows
  const int use = stage <= dyn_max && !f->qr;
  hipLaunchKernelGGL(kern, dim3(KX + KY + 1), dim3(PPLS_FIN_THREADS), use ? stage : 0, st, f->stats, f->ssq,
                     f->N, f->p, f->q, f->ldx, f->ldy, f->Wc, f->Cc, f->sc_cur, f->Wn, f->Cn, f->sc_nxt, f->mom,
                     f->loglik, f->logl_index, f->work, f->status, f->qr, f->mode, f->gram_cur,
                     f->gram_nxt, f->vstate, use, f->trace, f->stop, f->stop_mirror, f->stop_check,
                     f->stop_step, f->atol, KX, KY, f->team_bar, f->team_part, f->xpM);
  return hipGetLastError();
}


size_t split_lds(int r, int ldx, int ldy, int threads, int rp) {
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  const int v = r * rp, nw = threads / 64;
  return (size_t)PPLS_SWEEP_SLOTS * (nch << 10) + (size_t)(2 * nw * v + nw * 2 * v + 4 * r) * 8;
}

template <int R, int NSH, int RP, bool PIPE, int CPW>
hipError_t launch_split_t(const PplsSweepArgs& a, hipStream_t st) {
  auto kern = ppls_sweep_split_kernel<R, NSH, 512, RP, PIPE, PPLS_SWEEP_SLOTS, CPW>;
  {
    const hipError_t e = set_dyn_lds((const void*)kern, 160 * 1024);
    if (e != hipSuccess) return e;
  }
  if (a.occ_out) {   // query: resident workgroups per CU for this instantiation and shape
    int nb = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (const void*)kern, 512,
                                                                split_lds(R, a.ldx, a.ldy, 512, RP));
    *a.occ_out = nb;
    return e;
  }
  hipLaunchKernelGGL(kern, dim3(a.grid), dim3(512), split_lds(R, a.ldx, a.ldy, 512, RP), st, a.X, a.Y,
                     a.n_local, a.ldx, a.ldy, a.Wp, a.Cp, a.sc, a.part, a.part_ld, a.mu, a.write_mu,
                     a.nt, a.stop, a.trace, a.row_bounds, a.wg_seg);
  return hipGetLastError();
}

template <int R, int NSH, int RP, bool PIPE>
hipError_t launch_split_cpw(const PplsSweepArgs& a, hipStream_t st) {
  const int nch = ((a.ldx * 8 + 1023) >> 10) + ((a.ldy * 8 + 1023) >> 10);
  const int need = (nch + 7) / 8;
  if (need <= 2) return launch_split_t<R, NSH, RP, PIPE, 2>(a, st);
  if (need <= 4) return launch_split_t<R, NSH, RP, PIPE, 4>(a, st);
  return hipErrorInvalidValue;
}

// split-ownership variants (512 threads): NSH pairs per thread in {1, 2, 4}; RP/PIPE from a.rp,
// a.pipe.  Instantiated only where they fit in registers (see ppls_split_supported).
template <int R>
hipError_t launch_split_r(const PplsSweepArgs& a, hipStream_t st) {
  if (a.ns <= 1) {
    if (a.rp != 1) return launch_split_cpw<R, 1, 2, true>(a, st);
    return launch_split_cpw<R, 1, 1, true>(a, st);
  }
  if (a.ns == 2) {
    if constexpr (R <= 6) {
      if (a.rp != 1) return launch_split_cpw<R, 2, 2, true>(a, st);
    }
    return launch_split_cpw<R, 2, 1, true>(a, st);
  }
  if constexpr (R <= 5) {
    if (a.ns <= 4) {
      if (a.rp != 1) return launch_split_cpw<R, 4, 2, false>(a, st);
      if (a.pipe) return launch_split_cpw<R, 4, 1, true>(a, st);
      return launch_split_cpw<R, 4, 1, false>(a, st);
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

int ppls_split_supported(int r, int ldx, int ldy) {
  const int npmax = (ldx > ldy ? ldx : ldy) / 2;
  const int nsh = (npmax + 255) / 256;
  if (r < 1 || r > PPLS_FUSED_RMAX) return 0;
  int ns = nsh <= 1 ? 1 : nsh <= 2 ? 2 : nsh <= 4 ? 4 : 0;
  if (ns == 0 || (ns == 4 && r > 5)) return 0;
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  if (nch > 32) return 0;
  return split_lds(r, ldx, ldy, 512, 2) <= 160 * 1024 ? ns : 0;
}

// The split instantiation ppls_launch_sweep_split picks for *a (mirrors launch_split_r and
// launch_split_cpw): "split<R,NSH,NT,RP,PIPE,SLOTS,CPW>".  Returns 0, or -1 if none fits.
int ppls_split_describe(const PplsSweepArgs* a, char* buf, int len) {
  const int R = a->r;
  int nsh = 0, rp = 1, pipe = 1;
  if (a->ns <= 1) { nsh = 1; rp = a->rp != 1 ? 2 : 1; }
  else if (a->ns == 2) { nsh = 2; rp = (R <= 6 && a->rp != 1) ? 2 : 1; }
  else if (a->ns <= 4 && R <= 5) { nsh = 4; rp = a->rp != 1 ? 2 : 1; pipe = a->rp != 1 ? 0 : (a->pipe ? 1 : 0); }
  const int nch = ((a->ldx * 8 + 1023) >> 10) + ((a->ldy * 8 + 1023) >> 10);
  const int need = (nch + 7) / 8, cpw = need <= 2 ? 2 : need <= 4 ? 4 : 0;
  if (!nsh || !cpw || R < 1 || R > PPLS_FUSED_RMAX) return -1;
  snprintf(buf, (size_t)len, "split<%d,%d,512,%d,%s,%d,%d>", R, nsh, rp, pipe ? "true" : "false", PPLS_SWEEP_SLOTS, cpw);
  return 0;
}

hipError_t ppls_launch_sweep_split(const PplsSweepArgs* a, hipStream_t st) {
  switch (a->r) {
    case 1: return launch_split_r<1>(*a, st);
    case 2: return launch_split_r<2>(*a, st);
    case 3: return launch_split_r<3>(*a, st);
    case 4: return launch_split_r<4>(*a, st);
    case 5: return launch_split_r<5>(*a, st);
    case 6: return launch_split_r<6>(*a, st);
    case 7: return launch_split_r<7>(*a, st);
    case 8: return launch_split_r<8>(*a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t ppls_launch_accumulate(const PplsSweepArgs* a, const double* Z, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  const int np = (a->ldx >> 1) + (a->ldy >> 1);
  const int64_t rpc = (a->n_local + a->grid - 1) / a->grid;
  const int chunks = (int)((a->n_local + rpc - 1) / rpc);
  hipLaunchKernelGGL(ppls_acc_kernel, dim3((np + 255) / 256, chunks), dim3(256), 0, st, a->X, a->Y,
                     a->n_local, a->ldx, a->ldy, Z, a->r, a->sc, rpc, a->part, a->part_ld, a->mu, 0, a->stop);
  return hipGetLastError();
}

// ---- panel sweep launchers
}  // extern "C"
namespace {

template <typename T, int R>
hipError_t launch_panel_t(const PplsSweepArgs* a, const T* X, const T* Y, double* Z, int chunks, hipStream_t st) {
  // transposed W, C behind Z (see ppls_panel_z_len), rows padded to whole 32-column tiles
  const int ldxp = (a->ldx + 31) & ~31, ldyp = (a->ldy + 31) & ~31;
  const int rs = 16;   // the MFMA's B operand: 16 component columns, zero beyond R
  double* Wt = Z + a->n_local * 4 * R;
  double* Ct = Wt + (int64_t)ldxp * rs;
  const int64_t ne = (int64_t)(ldxp + ldyp) * rs;
  hipLaunchKernelGGL(ppls_transpose_wc_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, st, a->Wp,
                     a->Cp, a->ldx, a->ldy, ldxp, ldyp, R, rs, Wt, Ct, a->stop);
  {   // MFMA dots (profiles/r1_c5_*_dots_variants.txt: faster than the VALU and LDS-DMA forms)
    // rows per wave: 64 (four 16-row blocks per B load: half the B traffic of 32 rows; 246 VGPRs,
    // 2 waves/SIMD) from 32768 rows per shard, else 32 (146 VGPRs, 3 waves/SIMD).  C5 fp32: 8.28 ->
    // 7.80 ms per sweep; C5's 8-GPU share (62,500 rows): 1.125 -> 1.09 ms (profiles/r2_c5_dots_rows.txt).
    // Option dots_rows (32 or 64) forces one.
    const int rb = a->dots_rows == 32 || a->dots_rows == 64 ? a->dots_rows : a->n_local >= 32768 ? 64 : 32;
    const int64_t wtiles = (a->n_local + rb - 1) / rb;
    // column split over wave pairs when one wave per row tile would leave resident wave slots
    // (2 waves/SIMD at 64 rows, 3 at 32) empty; option dots_pair (0 or 1) forces one form
    const int64_t slots = (int64_t)(a->num_cus > 0 ? a->num_cus : 256) * 4 * (rb == 64 ? 2 : 3);
    const int ks = a->dots_pair >= 0 ? (a->dots_pair ? 2 : 1) : wtiles < slots ? 2 : 1;
    const int64_t wgs = (wtiles + 4 / ks - 1) / (4 / ks);
    // the grid option (dots_grid) forces a smaller grid: tests of the grid-stride loop
    const int mblocks = (int)(a->dots_grid > 0 && a->dots_grid < wgs ? a->dots_grid : wgs < 16384 ? wgs : 16384);
    double* mu_out = a->write_mu ? a->mu : nullptr;
    // (also measured: the B operands prefetched a tile ahead, 256 VGPRs -- no faster, 7.70-7.88 vs
    // 7.69-7.78 ms; profiles/r2_c5_dots_rows.txt.  Round 5: X tiles by LDS-DMA, two in flight per
    // wave, 1.5 % faster at C5 -- removed: its uncounted inline-asm B loads were copied by the register
    // allocator before they landed in some instantiations)
#define PPLS_LAUNCH_DOTS(NBV, KSV, NTV)                                                              \
  hipLaunchKernelGGL((ppls_panel_mfmadots_kernel<T, R, NBV, KSV, NTV>), dim3(mblocks), dim3(256), 0, st, X, Y, \
                     a->n_local, a->ldx, a->ldy, a->p, a->q, Wt, Ct, a->sc, Z, mu_out, a->stop, a->seg_ends, \
                     a->nseg)
    if (a->nt) {
      if (rb == 64 && ks == 2) PPLS_LAUNCH_DOTS(4, 2, true);
      else if (rb == 64) PPLS_LAUNCH_DOTS(4, 1, true);
      else if (ks == 2) PPLS_LAUNCH_DOTS(2, 2, true);
      else PPLS_LAUNCH_DOTS(2, 1, true);
    } else {
      if (rb == 64 && ks == 2) PPLS_LAUNCH_DOTS(4, 2, false);
      else if (rb == 64) PPLS_LAUNCH_DOTS(4, 1, false);
      else if (ks == 2) PPLS_LAUNCH_DOTS(2, 2, false);
      else PPLS_LAUNCH_DOTS(2, 1, false);
    }
#undef PPLS_LAUNCH_DOTS
  }
  constexpr int VEC = PplsVec16<T>::N;
  if (a->dots_only) return hipGetLastError();   // scores: Z and mu only
  PplsChunks ck;   // half the chunks at 4x the rows of the other half (equal chunks: profiles/r2_c5_dots_rows.txt)
  ck.bnd = a->chunk_bounds;
  ck.nbig = chunks / 2;
  const int nsmall = chunks - ck.nbig;
  ck.big = (4 * a->n_local + 4 * ck.nbig + nsmall - 1) / (4 * ck.nbig + nsmall);
  ck.small = (ck.big + 3) / 4;
  if (ck.small < 1) ck.small = 1;
  // VALU accumulation: at C5 an MFMA form measured no faster in fp64 storage (7.7 vs 7.5 ms) and
  // slower in fp32 (6.0 vs 4.5 ms; profiles/r1_c5_*_acc_variants.txt) -- the pass is load-bound
  const int ntx = (a->ldx + 256 * VEC - 1) / (256 * VEC), nty = (a->ldy + 256 * VEC - 1) / (256 * VEC);
  // the accumulation pass's once-read stream: non-temporal loads where X, Y exceed the MALL (the
  // sweep's nt policy): C5 fp32 4.05 -> 3.89 ms (profiles/r2_c5_nt_policy.txt)
  if (a->nt)
    hipLaunchKernelGGL((ppls_panel_acc_kernel<T, R, true>), dim3(ntx + nty, chunks), dim3(256), 0, st, X, Y,
                       a->n_local, a->ldx, a->ldy, Z, ck, a->part, a->part_ld, a->stop);
  else
    hipLaunchKernelGGL((ppls_panel_acc_kernel<T, R, false>), dim3(ntx + nty, chunks), dim3(256), 0, st, X, Y,
                       a->n_local, a->ldx, a->ldy, Z, ck, a->part, a->part_ld, a->stop);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_panel_dt(const PplsSweepArgs* a, const T* X, const T* Y, double* Z, int chunks, hipStream_t st) {
  switch (a->r) {
    case 1: return launch_panel_t<T, 1>(a, X, Y, Z, chunks, st);
    case 2: return launch_panel_t<T, 2>(a, X, Y, Z, chunks, st);
    case 3: return launch_panel_t<T, 3>(a, X, Y, Z, chunks, st);
    case 4: return launch_panel_t<T, 4>(a, X, Y, Z, chunks, st);
    case 5: return launch_panel_t<T, 5>(a, X, Y, Z, chunks, st);
    case 6: return launch_panel_t<T, 6>(a, X, Y, Z, chunks, st);
    case 7: return launch_panel_t<T, 7>(a, X, Y, Z, chunks, st);
    case 8: return launch_panel_t<T, 8>(a, X, Y, Z, chunks, st);
    case 9: return launch_panel_t<T, 9>(a, X, Y, Z, chunks, st);
    case 10: return launch_panel_t<T, 10>(a, X, Y, Z, chunks, st);
    case 11: return launch_panel_t<T, 11>(a, X, Y, Z, chunks, st);
    case 12: return launch_panel_t<T, 12>(a, X, Y, Z, chunks, st);
    case 13: return launch_panel_t<T, 13>(a, X, Y, Z, chunks, st);
    case 14: return launch_panel_t<T, 14>(a, X, Y, Z, chunks, st);
    case 15: return launch_panel_t<T, 15>(a, X, Y, Z, chunks, st);
    case 16: return launch_panel_t<T, 16>(a, X, Y, Z, chunks, st);
    default: return hipErrorInvalidValue;
  }
}

template <typename T, int R>
hipError_t acc_occ_t(int* occ) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, (const void*)ppls_panel_acc_kernel<T, R, false>, 256, 0);
}

template <typename T>
hipError_t acc_occ_dt(int r, int* occ) {
  switch (r) {
    case 1: return acc_occ_t<T, 1>(occ);
    case 2: return acc_occ_t<T, 2>(occ);
    case 3: return acc_occ_t<T, 3>(occ);
    case 4: return acc_occ_t<T, 4>(occ);
    case 5: return acc_occ_t<T, 5>(occ);
    case 6: return acc_occ_t<T, 6>(occ);
    case 7: return acc_occ_t<T, 7>(occ);
    case 8: return acc_occ_t<T, 8>(occ);
    case 9: return acc_occ_t<T, 9>(occ);
    case 10: return acc_occ_t<T, 10>(occ);
    case 11: return acc_occ_t<T, 11>(occ);
    case 12: return acc_occ_t<T, 12>(occ);
    case 13: return acc_occ_t<T, 13>(occ);
    case 14: return acc_occ_t<T, 14>(occ);
    case 15: return acc_occ_t<T, 15>(occ);
    case 16: return acc_occ_t<T, 16>(occ);
    default: return hipErrorInvalidValue;
  }
}

hipError_t panel_acc_occupancy(int dtype_f32, int r, int* occ) {
  return dtype_f32 ? acc_occ_dt<float>(r, occ) : acc_occ_dt<double>(r, occ);
}
}  // namespace
extern "C" {

int64_t ppls_panel_z_len(int64_t n_local, int ldx, int ldy, int r) {
  return (n_local > 0 ? n_local : 1) * 4 * r + (int64_t)(((ldx + 31) & ~31) + ((ldy + 31) & ~31)) * 16;
}

int ppls_panel_chunks(int64_t n_local, int ldx, int ldy, int num_cus, int dtype_f32, int r) {
  // The accumulation grid is column tiles x row chunks, sized in rounds of the resident slots (CUs x
  // workgroups per CU at the kernel's register use).
  const int vec = dtype_f32 ? 4 : 2;
  const int tiles = (ldx + 256 * vec - 1) / (256 * vec) + (ldy + 256 * vec - 1) / (256 * vec);
  int occ = 0;
  if (panel_acc_occupancy(dtype_f32, r, &occ) != hipSuccess || occ < 1) occ = 1;
  const int64_t slots = (int64_t)num_cus * occ;
  const int64_t maxch = (n_local + 255) / 256;   // at least 256 rows per chunk
  // Equal chunks needed about 8 rounds (round 1, C5 fp32: 93 chunks 9.08 ms, 196 8.70, 450 8.57):
  // more rounds shorten the tail, while the partials written and reduced grow with the chunk count
  // (profiles/r2_row_alignment_probe.txt: the write-out is the kernel's largest overhead).  Now 4
  // rounds, half of them large chunks (PplsChunks): half the partials, about the same tail.
  int64_t ch = 4 * slots / tiles;
  // Round 5: where those chunks would be short (< 1200 rows on average), 2 rounds: the partials'
  // write-out and reduction outweigh the longer tail.  C5's 8-GPU share (62,500 rows, 336 rows per
  // chunk at 4 rounds): 1.04-1.05 -> 1.008 ms per iteration; 1.25e5 / 1.875e5 rows: 1 % / 0.2 %
  // faster; 2.5e5 and the full 5e5: 4 rounds stay 0.3-0.4 % faster (profiles/r5_acc_chunks_ab.txt).
  if (n_local < 1200 * ch) ch = 2 * slots / tiles;
  if (ch > maxch) ch = maxch;
  if (ch > 1024) ch = 1024;
  if (ch < 1) ch = 1;
  return (int)ch;
}

hipError_t ppls_launch_panel_dots(const PplsSweepArgs* a, int dtype_f32, double* Z, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  PplsSweepArgs b = *a;
  b.dots_only = 1;
  if (dtype_f32) return launch_panel_dt<float>(&b, (const float*)a->X, (const float*)a->Y, Z, 0, st);
  return launch_panel_dt<double>(&b, a->X, a->Y, Z, 0, st);
}

hipError_t ppls_launch_sweep_panel(const PplsSweepArgs* a, int dtype_f32, double* Z, int chunks, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  if (dtype_f32)
    return launch_panel_dt<float>(a, (const float*)a->X, (const float*)a->Y, Z, chunks, st);
  return launch_panel_dt<double>(a, a->X, a->Y, Z, chunks, st);
}

int ppls_acc_groups(int64_t n_local, int grid) {
  const int64_t rpc = (n_local + grid - 1) / grid;
  return (int)((n_local + rpc - 1) / rpc);
}

// Scratch the statistics reduction needs behind the partials: none (one-launch fixed-order
// reduction, ppls_reduce_fused_kernel; measured against the former two-stage form in
// profiles/r2_reduce_fused_ab.txt).
int64_t ppls_reduce_tmp_len(int ngroups, int64_t len) {
  (void)ngroups;
  (void)len;
  return 0;
}

hipError_t ppls_launch_reduce2(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                               double* tmp, const int* stop, hipStream_t st) {
  (void)tmp;   // one launch (ppls_reduce_fused_kernel); the two-stage form it replaced needed scratch
  hipLaunchKernelGGL(ppls_reduce_fused_kernel, dim3((unsigned)((len + 63) / 64)), dim3(256), 0,
                     st, part, ngroups, ld, len, out, 0, stop);
  return hipGetLastError();
}

hipError_t ppls_launch_reduce(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                              int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0,
                     st, part, ngroups, ld, len, out, accumulate, nullptr);
  return hipGetLastError();
}

hipError_t ppls_launch_finalize(const PplsFinalizeArgs* f, hipStream_t st) {
  switch (f->r) {
    case 1: return launch_finalize_t<1>(f, st);
    case 2: return launch_finalize_t<2>(f, st);
    case 3: return launch_finalize_t<3>(f, st);
    case 4: return launch_finalize_t<4>(f, st);
    case 5: return launch_finalize_t<5>(f, st);
    case 6: return launch_finalize_t<6>(f, st);
    case 7: return launch_finalize_t<7>(f, st);
    case 8: return launch_finalize_t<8>(f, st);
    case 9: return launch_finalize_t<9>(f, st);
    case 10: return launch_finalize_t<10>(f, st);
    default:   // r = 11..16: runtime-r finalize (R(R+1)/2 > 64 block-sum values)
      hipLaunchKernelGGL(ppls_finalize_generic_kernel, dim3(3), dim3(256), 0, st, f->stats, f->ssq, f->N,
                         f->p, f->q, f->r, f->ldx, f->ldy, f->Wc, f->Cc, f->sc_cur, f->Wn, f->Cn,
                         f->sc_nxt, f->mom, f->loglik, f->logl_index, f->work, f->status, f->qr, f->mode,
                         f->stop, f->stop_mirror, f->stop_check, f->stop_step, f->atol);
      return hipGetLastError();
  }
}

hipError_t ppls_launch_rank1_step(const PplsRank1StepArgs* a, hipStream_t st) {
  hipLaunchKernelGGL(ppls_rank1_step_kernel, dim3(1), dim3(1024), 0, st, *a);
  return hipGetLastError();
}

hipError_t ppls_launch_loglc(const double* G, const double* ssq, double N, int p, int q, int r,
                             double sigX, double sigY, const double* coefs, double* out,
                             hipStream_t st) {
  hipLaunchKernelGGL(ppls_loglc_kernel, dim3(1), dim3(64), 0, st, G, ssq, N, p, q, r, sigX, sigY,
                     coefs, out);
  return hipGetLastError();
}

hipError_t ppls_launch_sumsq_f32(const float* a, int64_t len, double* part, int nblocks, double* out,
                                 hipStream_t st) {
  hipLaunchKernelGGL(ppls_sumsq_f32_kernel, dim3(nblocks), dim3(256), 0, st, a, len, part);
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3(1), dim3(64), 0, st, part, nblocks, 1, 1, out, 0, nullptr);
  return hipGetLastError();
}

hipError_t ppls_launch_convert(const void* src, int src_f32, void* dst, int dst_f32, int64_t len, hipStream_t st) {
  if (len <= 0) return hipSuccess;
  const int blocks = (int)((len + 255) / 256 < 16384 ? (len + 255) / 256 : 16384);
  if (!src_f32 && dst_f32)
    hipLaunchKernelGGL((ppls_convert_kernel<double, float>), dim3(blocks), dim3(256), 0, st, (const double*)src,
                       (float*)dst, len);
  else if (src_f32 && !dst_f32)
    hipLaunchKernelGGL((ppls_convert_kernel<float, double>), dim3(blocks), dim3(256), 0, st, (const float*)src,
                       (double*)dst, len);
  else
    return hipMemcpyAsync(dst, src, (size_t)len * (src_f32 ? 4 : 8), hipMemcpyDeviceToDevice, st);
  return hipGetLastError();
}

hipError_t ppls_launch_sumsq(const double* a, int64_t len, double* part, int nblocks, double* out,
                             int out_accumulate, hipStream_t st) {
  hipLaunchKernelGGL(ppls_sumsq_partial_kernel, dim3(nblocks), dim3(256), 0, st, a, len, part);
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3(1), dim3(64), 0, st, part, nblocks, 1, 1, out,
                     out_accumulate, nullptr);
  return hipGetLastError();
}

hipError_t ppls_launch_deflated_ssq(const void* X, int f32, int64_t n, int ld, int p, const double* Wd, int m,
                                    double* part, int nblocks, double* out, hipStream_t st) {
  if (m < 0 || m > 16) return hipErrorInvalidValue;
  if (f32)
    hipLaunchKernelGGL(ppls_deflated_ssq_kernel<float>, dim3(nblocks), dim3(256), 0, st, (const float*)X, n, ld,
                       p, Wd, m, part);
  else
    hipLaunchKernelGGL(ppls_deflated_ssq_kernel<double>, dim3(nblocks), dim3(256), 0, st, (const double*)X, n,
                       ld, p, Wd, m, part);
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3(1), dim3(64), 0, st, part, nblocks, 1, 1, out, 0, nullptr);
  return hipGetLastError();
}

hipError_t ppls_launch_generate(int64_t n_local, int64_t row0, int p, int q, int ldx, int ldy, int r,
                                const PplsScalars* truth, const double* Wt, const double* Ct,
                                uint64_t seed, double* TU, double* X, double* Y, hipStream_t st) {
  if (n_local <= 0) return hipSuccess;
  const int64_t nl = n_local * r;
  hipLaunchKernelGGL(ppls_gen_latent_kernel, dim3((unsigned)((nl + 255) / 256)), dim3(256), 0, st,
                     n_local, row0, r, *truth, seed, TU);
  const int64_t nx = n_local * (ldx >> 1), ny = n_local * (ldy >> 1);
  hipLaunchKernelGGL(ppls_gen_obs_kernel, dim3((unsigned)((nx + 255) / 256)), dim3(256), 0, st,
                     n_local, row0, p, ldx, r, TU, 0, Wt, truth->sigE, seed, 0u, X);
  hipLaunchKernelGGL(ppls_gen_obs_kernel, dim3((unsigned)((ny + 255) / 256)), dim3(256), 0, st,
                     n_local, row0, q, ldy, r, TU, r, Ct, truth->sigF, seed, 1u, Y);
  return hipGetLastError();
}

hipError_t ppls_launch_to_rowmajor(const double* src, int64_t n, int p, int ld, double* dst,
                                   hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ppls_colmajor_to_rowmajor_kernel, dim3((unsigned)((n + 31) / 32), (ld + 31) / 32),
                     dim3(256), 0, st, src, n, p, ld, dst);
  return hipGetLastError();
}

hipError_t ppls_launch_to_colmajor(const double* src, int64_t n, int p, int ld, double* dst,
                                   hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(ppls_rowmajor_to_colmajor_kernel, dim3((unsigned)((n + 31) / 32), (p + 31) / 32),
                     dim3(256), 0, st, src, n, p, ld, dst);
  return hipGetLastError();
}

}  // extern "C"
