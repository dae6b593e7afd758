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

// out[j] (+)= sum_g part[g*ld + j], fixed order -> deterministic.
__global__ void ppls_reduce_partials_kernel(const double* __restrict__ part, int ngroups, int64_t ld,
                                            int64_t len, double* __restrict__ out, int accumulate) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= len) return;
  double s = 0.0;
  for (int g = 0; g < ngroups; ++g) s += part[(int64_t)g * ld + j];
  out[j] = accumulate ? out[j] + s : s;
}

// ============================================================================ wave reduce-scatter
// V values per lane -> after 6 butterfly levels lane holds the full wave sum of value `idx`.
// Levels: 0 permlane32_swap (bit5), 1 permlane16_swap (bit4), 2 row_mirror (bit3),
// 3 row_half_mirror (bit2), 4 quad_perm xor2 (bit1), 5 quad_perm xor1 (bit0).
template <int L>
__device__ __forceinline__ double ppls_dpp_partner(double v) {
  constexpr int ctrl = (L == 2) ? 0x140 : (L == 3) ? 0x141 : (L == 4) ? 0x4E : 0xB1;
  const int lo = __builtin_amdgcn_mov_dpp((int)__double2loint(v), ctrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)__double2hiint(v), ctrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

template <int L>
__device__ __forceinline__ void ppls_swap_pair(double& A, double& B) {
  unsigned alo = __double2loint(A), ahi = __double2hiint(A);
  unsigned blo = __double2loint(B), bhi = __double2hiint(B);
  if constexpr (L == 0) {
    auto s = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
    auto t = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
    A = __hiloint2double(t[0], s[0]);
    B = __hiloint2double(t[1], s[1]);
  } else {
    auto s = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
    auto t = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
    A = __hiloint2double(t[0], s[0]);
    B = __hiloint2double(t[1], s[1]);
  }
}

template <int M, int L, int N>
__device__ __forceinline__ void ppls_rs(double (&a)[N], int lane, int& idx, bool& canon) {
  if constexpr (L < 6) {
    const int beta = (lane >> (5 - L)) & 1;
    if constexpr (M == 1) {
      if constexpr (L <= 1) {
        double A = a[0], B = a[0];
        ppls_swap_pair<L>(A, B);
        a[0] = A + B;
      } else {
        a[0] += ppls_dpp_partner<L>(a[0]);
      }
      canon = canon && (beta == 0);
      ppls_rs<1, L + 1, N>(a, lane, idx, canon);
    } else {
      constexpr int H = (M + 1) / 2;
      static_assert(2 * H <= N, "reduce-scatter buffer too small");
      if constexpr (M & 1) a[M] = 0.0;
#pragma unroll
      for (int j = 0; j < H; ++j) {
        if constexpr (L <= 1) {
          double A = a[j], B = a[j + H];
          ppls_swap_pair<L>(A, B);
          a[j] = A + B;
        } else {
          const double send = beta ? a[j] : a[j + H];
          const double keep = beta ? a[j + H] : a[j];
          a[j] = keep + ppls_dpp_partner<L>(send);
        }
      }
      idx += beta * H;
      ppls_rs<H, L + 1, N>(a, lane, idx, canon);
    }
  }
}

// ============================================================================ LDS-DMA helpers
__device__ __forceinline__ void ppls_wait_vmcnt(int n) {
#define PPLS_VMC(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    PPLS_VMC(1) PPLS_VMC(2) PPLS_VMC(3) PPLS_VMC(4) PPLS_VMC(5) PPLS_VMC(6) PPLS_VMC(7)
    PPLS_VMC(8) PPLS_VMC(9) PPLS_VMC(10) PPLS_VMC(11) PPLS_VMC(12) PPLS_VMC(13) PPLS_VMC(14)
    PPLS_VMC(15) PPLS_VMC(16) PPLS_VMC(17) PPLS_VMC(18) PPLS_VMC(19) PPLS_VMC(20) PPLS_VMC(21)
    PPLS_VMC(22) PPLS_VMC(23) PPLS_VMC(24) PPLS_VMC(25) PPLS_VMC(26) PPLS_VMC(27) PPLS_VMC(28)
    PPLS_VMC(29) PPLS_VMC(30) PPLS_VMC(31)
    default:
      if (n >= 32) asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      break;
  }
#undef PPLS_VMC
}

// HBM -> LDS copy of 16 B per lane (global_load_lds_dwordx4): LDS destination = m0 + 16 * lane.
// Issued through inline asm on purpose: the compiler then does not track the DMA, so it does not
// put vmcnt(0) in front of every ds_read of the ring (it cannot prove the slots do not alias);
// the ring's completion is waited for explicitly with ppls_wait_vmcnt.  Invisible VMEM ops can
// only make the compiler's own vmcnt waits stricter, never unsafe.
__device__ __forceinline__ void ppls_dma16(const void* gptr, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               :: "s"(lds_addr), "v"(gptr) : "memory", "m0");
}

__device__ __forceinline__ void ppls_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ============================================================================ fused sweep
// One workgroup (512 threads, one per CU) owns a contiguous block of rows. Each thread owns NS
// column pairs of X and NS of Y for the whole sweep: it keeps W/C for those columns and the
// X'mu_T / Y'mu_U accumulators in registers.  Rows stream HBM -> LDS through a SLOTS-deep ring
// of LDS-DMA (global_load_lds_dwordx4) copies; per row: partial dots -> wave reduce-scatter ->
// cross-wave sum in LDS -> mu_T/mu_U (registers) -> rank-1 update of the accumulators, plus the
// 2r x 2r Gram of [Xw Yc].  X and Y are read from HBM exactly once.
template <int R, int NS, int SLOTS>
__global__ __launch_bounds__(PPLS_SWEEP_THREADS, 2) void ppls_sweep_fused_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, const PplsScalars* __restrict__ sc,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int V = 2 * R;
  constexpr int VP = (V < 2) ? 2 : V + (V & 1) + 2;   // reduce-scatter scratch (pads)
  constexpr int NWAVES = PPLS_SWEEP_THREADS / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchx = (ldx * 8 + 1023) >> 10, nchy = (ldy * 8 + 1023) >> 10;
  const int nch = nchx + nchy;
  const int slot_bytes = nch << 10;
  const int ndma = (nch + NWAVES - 1) / NWAVES;
  double* red = (double*)(smem + (size_t)SLOTS * slot_bytes);
  const int64_t g = blockIdx.x, G = gridDim.x;
  const int64_t rb = n_local * g / G, re = n_local * (g + 1) / G;
  const int nrows = (int)(re - rb);
  const int npx = ldx >> 1, npy = ldy >> 1;

  bool vx[NS], vy[NS];
  double2 w[NS][R], c[NS][R], ax[NS][R], ay[NS][R];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int px = tid + s * PPLS_SWEEP_THREADS;
    vx[s] = px < npx;
    vy[s] = px < npy;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      w[s][k] = vx[s] ? *(const double2*)(Wp + (int64_t)k * ldx + 2 * px) : make_double2(0.0, 0.0);
      c[s][k] = vy[s] ? *(const double2*)(Cp + (int64_t)k * ldy + 2 * px) : make_double2(0.0, 0.0);
      ax[s][k] = make_double2(0.0, 0.0);
      ay[s][k] = make_double2(0.0, 0.0);
    }
  }
  double al[R], be[R], ga[R], de[R];
#pragma unroll
  for (int k = 0; k < R; ++k) {
    al[k] = sc->alpha[k];
    be[k] = sc->beta[k];
    ga[k] = sc->gamma[k];
    de[k] = sc->delta[k];
  }
  // Gram entry owned by this thread (upper triangle of the 2R x 2R Gram, one entry per thread)
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto issue_row = [&](int i, int slot) {
    const int64_t row = rb + i;
    const char* xr = (const char*)(X + row * (int64_t)ldx);
    const char* yr = (const char*)(Y + row * (int64_t)ldy);
    const uint32_t sb = lds_base + (uint32_t)(slot * slot_bytes);
    for (int j = 0; j < ndma; ++j) {
      int ch = wave + j * NWAVES;
      while (ch >= nch) ch -= nch;   // surplus issues duplicate a real chunk (identical bytes)
      const char* src;
      if (ch < nchx) {
        const int off = ch * 1024 + lane * 16;
        src = xr + min(off, ldx * 8 - 16);
      } else {
        const int off = (ch - nchx) * 1024 + lane * 16;
        src = yr + min(off, ldy * 8 - 16);
      }
      ppls_dma16(src, sb + (uint32_t)(ch * 1024));
    }
  };

  for (int i = 0; i < SLOTS - 1 && i < nrows; ++i) issue_row(i, i);

  for (int i = 0; i < nrows; ++i) {
    const int ahead = min(SLOTS - 2, nrows - 1 - i);
    ppls_wait_vmcnt(write_mu ? 0 : ahead * ndma);
    ppls_lds_barrier();
    if (i + SLOTS - 1 < nrows) issue_row(i + SLOTS - 1, (i + SLOTS - 1) % SLOTS);
    const char* sb = smem + (size_t)(i % SLOTS) * slot_bytes;
    double2 xv[NS], yv[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int px = tid + s * PPLS_SWEEP_THREADS;
      xv[s] = vx[s] ? *(const double2*)(sb + px * 16) : make_double2(0.0, 0.0);
      yv[s] = vy[s] ? *(const double2*)(sb + nchx * 1024 + px * 16) : make_double2(0.0, 0.0);
    }
    double v[VP];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      double sx = 0.0, sy = 0.0;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        sx = fma(xv[s].x, w[s][k].x, sx);
        sx = fma(xv[s].y, w[s][k].y, sx);
        sy = fma(yv[s].x, c[s][k].x, sy);
        sy = fma(yv[s].y, c[s][k].y, sy);
      }
      v[k] = sx;
      v[R + k] = sy;
    }
#pragma unroll
    for (int k = V; k < VP; ++k) v[k] = 0.0;
    int idx = 0;
    bool canon = true;
    ppls_rs<V, 0, VP>(v, lane, idx, canon);
    if (canon && idx < V) red[wave * V + idx] = v[0];
    ppls_lds_barrier();
    double z = 0.0;
    if (lane < V) {
#pragma unroll
      for (int ww = 0; ww < NWAVES; ++ww) z += red[ww * V + lane];
    }
    double za[R], zb[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      za[k] = __hiloint2double(__builtin_amdgcn_readlane((int)__double2hiint(z), k),
                               __builtin_amdgcn_readlane((int)__double2loint(z), k));
      zb[k] = __hiloint2double(__builtin_amdgcn_readlane((int)__double2hiint(z), R + k),
                               __builtin_amdgcn_readlane((int)__double2loint(z), R + k));
    }
    {
      const double zi = __shfl(z, gi, 64), zj = __shfl(z, gj, 64);
      if (has_g) gacc = fma(zi, zj, gacc);
    }
    double mt[R], mu_u[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      mt[k] = al[k] * za[k] + be[k] * zb[k];
      mu_u[k] = ga[k] * za[k] + de[k] * zb[k];
    }
    if (write_mu && wave == 0 && lane < R) {
      double a = 0.0, b = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k)
        if (lane == k) { a = mt[k]; b = mu_u[k]; }
      mu[(int64_t)lane * n_local + rb + i] = a;
      mu[(int64_t)(R + lane) * n_local + rb + i] = b;
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int k = 0; k < R; ++k) {
        ax[s][k].x = fma(xv[s].x, mt[k], ax[s][k].x);
        ax[s][k].y = fma(xv[s].y, mt[k], ax[s][k].y);
        ay[s][k].x = fma(yv[s].x, mu_u[k], ay[s][k].x);
        ay[s][k].y = fma(yv[s].y, mu_u[k], ay[s][k].y);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // partials: [SX ldx*R][SY ldy*R][G 4R^2]
  double* pg = part + g * part_ld;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int px = tid + s * PPLS_SWEEP_THREADS;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (vx[s]) *(double2*)(pg + (int64_t)k * ldx + 2 * px) = ax[s][k];
      if (vy[s]) *(double2*)(pg + (int64_t)R * ldx + (int64_t)k * ldy + 2 * px) = ay[s][k];
    }
  }
  if (has_g) {
    double* G2 = pg + (int64_t)R * ldx + (int64_t)R * ldy;
    G2[gj * V + gi] = gacc;
    G2[gi * V + gj] = gacc;
  }
}

// ============================================================================ generic two-pass
// Pass 1: Z = [X W | Y C] (n_local x 2R row-major), one wave per row.
__global__ __launch_bounds__(256) void ppls_dots_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, int r, double* __restrict__ Z) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int npx = ldx >> 1, npy = ldy >> 1;
  for (int64_t row = wid; row < n_local; row += nw) {
    double acc[2 * PPLS_RMAX];
    for (int k = 0; k < 2 * r; ++k) acc[k] = 0.0;
    const double2* xr = (const double2*)(X + row * ldx);
    const double2* yr = (const double2*)(Y + row * ldy);
    for (int pp = lane; pp < npx; pp += 64) {
      const double2 x = xr[pp];
      for (int k = 0; k < r; ++k) {
        const double2 wv = *(const double2*)(Wp + (int64_t)k * ldx + 2 * pp);
        acc[k] = fma(x.x, wv.x, fma(x.y, wv.y, acc[k]));
      }
    }
    for (int pp = lane; pp < npy; pp += 64) {
      const double2 y = yr[pp];
      for (int k = 0; k < r; ++k) {
        const double2 cv = *(const double2*)(Cp + (int64_t)k * ldy + 2 * pp);
        acc[r + k] = fma(y.x, cv.x, fma(y.y, cv.y, acc[r + k]));
      }
    }
    for (int k = 0; k < 2 * r; ++k) {
      const double s = ppls_wave_sum(acc[k]);
      if (lane == 0) Z[row * 2 * r + k] = s;
    }
  }
}

// Pass 2: S_X / S_Y partials over a chunk of rows, one thread per column pair; the Gram partial
// of the chunk is computed by the block with blockIdx.x == 0.
__global__ __launch_bounds__(256) void ppls_acc_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Z, int r, const PplsScalars* __restrict__ sc, int64_t rows_per_chunk,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu) {
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
__device__ void ppls_block_polar(const double* S, int64_t lds, int p, int r, double* out,
                                 int64_t ldo, int ldo_rows, double* A, double* E, int* status, int qr) {
  __shared__ double sh[16 * PPLS_RMAX];
  __shared__ double Rm[PPLS_RMAX * PPLS_RMAX];
  __shared__ double P[PPLS_RMAX * PPLS_RMAX];
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
    if (qr) {
      for (int j = 0; j < r; ++j)
        for (int i = 0; i < r; ++i) P[j * r + i] = (i == j) ? 1.0 : 0.0;
    } else if (ppls_small_polar(Rm, r, P) != 0) {
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

// Block 0: W_next = polar(S_X); block 1: C_next = polar(S_Y); block 2: scalars.
// stats = [SX ldx*r][SY ldy*r][G 4r^2];  ssq = {||X||^2, ||Y||^2}.
__global__ __launch_bounds__(256) void ppls_finalize_kernel(
    const double* __restrict__ stats, const double* __restrict__ ssq, double N, int p, int q, int r,
    int ldx, int ldy, const double* __restrict__ Wc, const double* __restrict__ Cc,
    const PplsScalars* __restrict__ sc_cur, double* __restrict__ Wn, double* __restrict__ Cn,
    PplsScalars* __restrict__ sc_nxt, PplsMoments* __restrict__ mom, double* __restrict__ loglik,
    int logl_index, double* __restrict__ work, int* __restrict__ status, int qr, int mode) {
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
    PplsMoments m;
    ppls_estep_moments(G, WtW, CtC, ssq[0], ssq[1], N, p, q, r, &cur, &m);
    *mom = m;
    PplsScalars nx = cur;
    ppls_mstep_scalars(&m, r, &nx);
    *sc_nxt = nx;
  }
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
template <int R, int NS, int SLOTS>
hipError_t launch_fused_t(const PplsSweepArgs& a, hipStream_t st) {
  auto kern = ppls_sweep_fused_kernel<R, NS, SLOTS>;
  static bool attr_set = false;
  const int nch = ((a.ldx * 8 + 1023) >> 10) + ((a.ldy * 8 + 1023) >> 10);
  const size_t lds = (size_t)SLOTS * (nch << 10) + (size_t)(PPLS_SWEEP_THREADS / 64) * 2 * R * 8;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.grid), dim3(PPLS_SWEEP_THREADS), lds, st, a.X, a.Y, a.n_local,
                     a.ldx, a.ldy, a.Wp, a.Cp, a.sc, a.part, a.part_ld, a.mu, a.write_mu);
  return hipGetLastError();
}

template <int R>
hipError_t launch_fused_r(const PplsSweepArgs& a, hipStream_t st) {
  switch (a.ns) {
    case 1: return launch_fused_t<R, 1, PPLS_SWEEP_SLOTS>(a, st);
    case 2: return launch_fused_t<R, 2, PPLS_SWEEP_SLOTS>(a, st);
    default: return hipErrorInvalidValue;
  }
}
}  // namespace

extern "C" {

int ppls_fused_supported(int r, int ldx, int ldy) {
  const int npmax = (ldx > ldy ? ldx : ldy) / 2;
  const int ns = (npmax + PPLS_SWEEP_THREADS - 1) / PPLS_SWEEP_THREADS;
  if (ns < 1 || ns > 2 || r < 1 || r > PPLS_FUSED_RMAX) return 0;
  if (ns * r > 10) return 0;   // register budget (W, C and accumulators stay in VGPRs)
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  const size_t lds = (size_t)PPLS_SWEEP_SLOTS * (nch << 10) + 8 * 2 * r * 8;
  return lds <= 160 * 1024 ? ns : 0;
}

size_t ppls_fused_lds_bytes(int r, int ldx, int ldy) {
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  return (size_t)PPLS_SWEEP_SLOTS * (nch << 10) + 8 * 2 * r * 8;
}

hipError_t ppls_launch_sweep_fused(const PplsSweepArgs* a, hipStream_t st) {
  switch (a->r) {
    case 1: return launch_fused_r<1>(*a, st);
    case 2: return launch_fused_r<2>(*a, st);
    case 3: return launch_fused_r<3>(*a, st);
    case 4: return launch_fused_r<4>(*a, st);
    case 5: return launch_fused_r<5>(*a, st);
    case 6: return launch_fused_r<6>(*a, st);
    case 7: return launch_fused_r<7>(*a, st);
    case 8: return launch_fused_r<8>(*a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t ppls_launch_sweep_twopass(const PplsSweepArgs* a, double* Z, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  const int64_t nw = a->n_local;
  int blocks = (int)((nw * 64 + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ppls_dots_kernel, dim3(blocks), dim3(256), 0, st, a->X, a->Y, a->n_local,
                     a->ldx, a->ldy, a->Wp, a->Cp, a->r, Z);
  const int np = (a->ldx >> 1) + (a->ldy >> 1);
  const int64_t rpc = (a->n_local + a->grid - 1) / a->grid;
  const int chunks = (int)((a->n_local + rpc - 1) / rpc);
  hipLaunchKernelGGL(ppls_acc_kernel, dim3((np + 255) / 256, chunks), dim3(256), 0, st, a->X, a->Y,
                     a->n_local, a->ldx, a->ldy, Z, a->r, a->sc, rpc, a->part, a->part_ld, a->mu,
                     a->write_mu);
  return hipGetLastError();
}

hipError_t ppls_launch_accumulate(const PplsSweepArgs* a, const double* Z, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  const int np = (a->ldx >> 1) + (a->ldy >> 1);
  const int64_t rpc = (a->n_local + a->grid - 1) / a->grid;
  const int chunks = (int)((a->n_local + rpc - 1) / rpc);
  hipLaunchKernelGGL(ppls_acc_kernel, dim3((np + 255) / 256, chunks), dim3(256), 0, st, a->X, a->Y,
                     a->n_local, a->ldx, a->ldy, Z, a->r, a->sc, rpc, a->part, a->part_ld, a->mu, 0);
  return hipGetLastError();
}

int ppls_twopass_groups(int64_t n_local, int grid) {
  const int64_t rpc = (n_local + grid - 1) / grid;
  return (int)((n_local + rpc - 1) / rpc);
}

hipError_t ppls_launch_reduce(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                              int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0,
                     st, part, ngroups, ld, len, out, accumulate);
  return hipGetLastError();
}

hipError_t ppls_launch_finalize(const PplsFinalizeArgs* f, hipStream_t st) {
  hipLaunchKernelGGL(ppls_finalize_kernel, dim3(3), dim3(256), 0, st, f->stats, f->ssq, f->N, f->p,
                     f->q, f->r, f->ldx, f->ldy, f->Wc, f->Cc, f->sc_cur, f->Wn, f->Cn, f->sc_nxt,
                     f->mom, f->loglik, f->logl_index, f->work, f->status, f->qr, f->mode);
  return hipGetLastError();
}

hipError_t ppls_launch_loglc(const double* G, const double* ssq, double N, int p, int q, int r,
                             double sigX, double sigY, const double* coefs, double* out,
                             hipStream_t st) {
  hipLaunchKernelGGL(ppls_loglc_kernel, dim3(1), dim3(64), 0, st, G, ssq, N, p, q, r, sigX, sigY,
                     coefs, out);
  return hipGetLastError();
}

hipError_t ppls_launch_sumsq(const double* a, int64_t len, double* part, int nblocks, double* out,
                             int out_accumulate, hipStream_t st) {
  hipLaunchKernelGGL(ppls_sumsq_partial_kernel, dim3(nblocks), dim3(256), 0, st, a, len, part);
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3(1), dim3(64), 0, st, part, nblocks, 1, 1, out,
                     out_accumulate);
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
