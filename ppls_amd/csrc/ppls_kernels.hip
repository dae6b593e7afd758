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

// Stage 1 of the two-stage reduction: tmp[chunk][j] = sum of groups [chunk*32, chunk*32+32).
__global__ void ppls_reduce_chunks_kernel(const double* __restrict__ part, int ngroups, int64_t ld,
                                          int64_t len, double* __restrict__ tmp) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= len) return;
  const int g0 = blockIdx.y * 32, g1 = min(ngroups, g0 + 32);
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int g = g0;
  for (; g + 8 <= g1; g += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += part[(int64_t)(g + u) * ld + j];
  }
  for (int u = 0; g < g1; ++g, ++u) s[u] += part[(int64_t)g * ld + j];
  tmp[(int64_t)blockIdx.y * len + j] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
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
// One workgroup (NT threads, one per CU) owns a contiguous block of rows.  Each thread owns NS
// column pairs of X and NS of Y for the whole sweep: it keeps W/C for those columns and the
// X'mu_T / Y'mu_U accumulators in registers.  Rows stream HBM -> LDS through a ring of SLOTS row
// slots filled by LDS-DMA (global_load_lds_dwordx4; the first ceil(nch/CPW) waves copy CPW 1-KiB
// chunks of every row, so the steady-state vmcnt is a compile-time immediate).  The loop handles
// RP rows per step, software-pipelined: step g sums group g's dots (cross-wave, LDS), computes
// group g+1's dots + wave reduce-scatter, then applies group g's rank-RP update -- ONE workgroup
// barrier per step (reduction scratch double-buffered).  mu_T / mu_U and [Xw Yc] rows are
// broadcast through a per-wave LDS scratch (no readlane / SGPR traffic).  X, Y are read once.
template <int R, int NS, int NT, int RP, int SLOTS, int CPW>
__global__ __launch_bounds__(NT, 2 * NT / 512) void ppls_sweep_fused_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, const PplsScalars* __restrict__ sc,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu, int ablate) {
  // ablate (timing experiments only; results are garbage): bit0 skips the per-row compute,
  // bit1 skips the HBM->LDS copies.
  static_assert(SLOTS >= 2 * RP, "ring must hold the group being read and the group in flight");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int V = 2 * R * RP;                       // partial dots per thread per step
  constexpr int VP = V;                               // reduce-scatter scratch (V is even)
  constexpr int NWAVES = NT / 64;
  constexpr int AHEAD = SLOTS / RP - 2;               // groups in flight beyond the next one
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchx = (ldx * 8 + 1023) >> 10, nchy = (ldy * 8 + 1023) >> 10;
  const int nch = nchx + nchy;
  const int slot_bytes = nch << 10;
  const bool dma_wave = wave * CPW < nch;
  double* red = (double*)(smem + (size_t)SLOTS * slot_bytes);          // [2][NWAVES][V]
  double* bc = red + 2 * NWAVES * V + wave * V;                       // per wave: [Xw Yc] rows
  double* cf = red + 3 * NWAVES * V;                                  // alpha | beta | gamma | delta
  const int64_t g = blockIdx.x, G = gridDim.x;
  const int64_t rb = n_local * g / G, re = n_local * (g + 1) / G;
  const int nrows = (int)(re - rb);
  const int ngroups = (nrows + RP - 1) / RP;
  const int npx = ldx >> 1, npy = ldy >> 1;

  bool vx[NS], vy[NS];
  double2 w[NS][R], c[NS][R], ax[NS][R], ay[NS][R];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int px = tid + s * NT;
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
  // lane m < R*RP of every wave turns (a, b) = (Xw, Yc) of row m/R, component m%R into mu_T, mu_U;
  // the coefficients live in LDS (no registers, no VMEM inside the DMA-counted loop)
  const int mj = lane / R, mk = lane - (lane / R) * R;
  if (tid < R) {
    cf[tid] = sc->alpha[tid];
    cf[R + tid] = sc->beta[tid];
    cf[2 * R + tid] = sc->gamma[tid];
    cf[3 * R + tid] = sc->delta[tid];
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
  auto issue_row = [&](int i) {
    if ((ablate & 2) || !dma_wave) return;
    const int64_t row = rb + i;
    const char* xr = (const char*)(X + row * (int64_t)ldx);
    const char* yr = (const char*)(Y + row * (int64_t)ldy);
    const uint32_t sb = lds_base + (uint32_t)((i % SLOTS) * slot_bytes);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int ch = min(wave * CPW + j, nch - 1);   // surplus issues repeat the last chunk
      const char* src;
      if (ch < nchx) src = xr + min(ch * 1024 + lane * 16, ldx * 8 - 16);
      else src = yr + min((ch - nchx) * 1024 + lane * 16, ldy * 8 - 16);
      ppls_dma16(src, sb + (uint32_t)(ch * 1024));
    }
  };
  auto issue_group = [&](int grp) {
    for (int j = 0; j < RP; ++j)
      if (grp * RP + j < nrows) issue_row(grp * RP + j);
  };
  // group grp's partial dots -> wave reduce-scatter -> red[grp & 1]; keeps the rows' x/y pairs
  auto dots_group = [&](int grp, double2 (&xv)[RP][NS], double2 (&yv)[RP][NS]) {
    if (ablate & 1) return;
    double v[VP];
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const int row = min(grp * RP + j, nrows - 1);   // a partial last group repeats its last row
      const char* sb = smem + (size_t)(row % SLOTS) * slot_bytes;
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int px = tid + s * NT;
        xv[j][s] = vx[s] ? *(const double2*)(sb + px * 16) : make_double2(0.0, 0.0);
        yv[j][s] = vy[s] ? *(const double2*)(sb + nchx * 1024 + px * 16) : make_double2(0.0, 0.0);
      }
#pragma unroll
      for (int k = 0; k < R; ++k) {
        double sx = 0.0, sy = 0.0;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          sx = fma(xv[j][s].x, w[s][k].x, sx);
          sx = fma(xv[j][s].y, w[s][k].y, sx);
          sy = fma(yv[j][s].x, c[s][k].x, sy);
          sy = fma(yv[j][s].y, c[s][k].y, sy);
        }
        v[j * 2 * R + k] = sx;
        v[j * 2 * R + R + k] = sy;
      }
    }
#pragma unroll
    for (int k = V; k < VP; ++k) v[k] = 0.0;
    int idx = 0;
    bool canon = true;
    ppls_rs<V, 0, VP>(v, lane, idx, canon);
    if (canon && idx < V) red[((grp & 1) * NWAVES + wave) * V + idx] = v[0];
  };

  if (ngroups > 0) {
    const int npro = min(SLOTS, nrows);
    for (int i = 0; i < npro; ++i) issue_row(i);
    if (write_mu) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else ppls_wait_vmcnt((npro - min(RP, nrows)) * CPW);
    ppls_lds_barrier();
    double2 xc[RP][NS] = {}, yc[RP][NS] = {};
    dots_group(0, xc, yc);
    for (int gg = 0; gg < ngroups; ++gg) {
      // rows issued after group gg+1: steady state AHEAD groups (compile-time wait)
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
      if (gg * RP + SLOTS < nrows) issue_group(gg + SLOTS / RP);
      if (ablate & 1) continue;
      // cross-wave sums of group gg: lane m < R*RP holds (a, b) = (Xw, Yc)[row m/R][comp m%R]
      // and its mu_T / mu_U; [Xw Yc] rows go to the per-wave LDS scratch for the Gram
      double mta = 0.0, mua = 0.0;
      if (lane < R * RP) {
        const double* rr = red + (gg & 1) * NWAVES * V;
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int ww = 0; ww < NWAVES; ++ww) {
          a += rr[ww * V + mj * 2 * R + mk];
          b += rr[ww * V + mj * 2 * R + R + mk];
        }
        bc[mj * 2 * R + mk] = a;
        bc[mj * 2 * R + R + mk] = b;
        mta = cf[mk] * a + cf[R + mk] * b;           // mu_T (EM_W_multi.R:691-692)
        mua = cf[2 * R + mk] * a + cf[3 * R + mk] * b;   // mu_U (EM_W_multi.R:693-694)
      }
      double2 xn[RP][NS] = {}, yn[RP][NS] = {};
      if (gg + 1 < ngroups) dots_group(gg + 1, xn, yn);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's bc writes are visible
#pragma unroll
      for (int j = 0; j < RP; ++j) {
        if (gg * RP + j >= nrows) break;
        if (has_g) gacc = fma(bc[j * 2 * R + gi], bc[j * 2 * R + gj], gacc);
        double mt[R], mu_u[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
          mt[k] = __hiloint2double(__builtin_amdgcn_readlane((int)__double2hiint(mta), j * R + k),
                                   __builtin_amdgcn_readlane((int)__double2loint(mta), j * R + k));
          mu_u[k] = __hiloint2double(__builtin_amdgcn_readlane((int)__double2hiint(mua), j * R + k),
                                     __builtin_amdgcn_readlane((int)__double2loint(mua), j * R + k));
        }
        if (write_mu && wave == 0 && lane < R) {
          const int64_t row = rb + gg * RP + j;
          double a = 0.0, b = 0.0;
#pragma unroll
          for (int k = 0; k < R; ++k)
            if (lane == k) { a = mt[k]; b = mu_u[k]; }
          mu[(int64_t)lane * n_local + row] = a;
          mu[(int64_t)(R + lane) * n_local + row] = b;
        }
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
          for (int k = 0; k < R; ++k) {
            ax[s][k].x = fma(xc[j][s].x, mt[k], ax[s][k].x);
            ax[s][k].y = fma(xc[j][s].y, mt[k], ax[s][k].y);
            ay[s][k].x = fma(yc[j][s].x, mu_u[k], ay[s][k].x);
            ay[s][k].y = fma(yc[j][s].y, mu_u[k], ay[s][k].y);
          }
      }
#pragma unroll
      for (int j = 0; j < RP; ++j)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          xc[j][s] = xn[j][s];
          yc[j][s] = yn[j][s];
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // partials: [SX ldx*R][SY ldy*R][G 4R^2]
  double* pg = part + g * part_ld;
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const int px = tid + s * NT;
#pragma unroll
    for (int k = 0; k < R; ++k) {
      if (vx[s]) *(double2*)(pg + (int64_t)k * ldx + 2 * px) = ax[s][k];
      if (vy[s]) *(double2*)(pg + (int64_t)R * ldx + (int64_t)k * ldy + 2 * px) = ay[s][k];
    }
  }
  if (has_g) {
    double* G2 = pg + (int64_t)R * ldx + (int64_t)R * ldy;
    G2[gj * 2 * R + gi] = gacc;
    G2[gi * 2 * R + gj] = gacc;
  }
}

// ============================================================================ fused sweep v3
// Same ring and pipeline as above, but column ownership is split by matrix: threads [0, NT/2) own
// NSH column pairs of X, threads [NT/2, NT) own NSH pairs of Y.  A wave's partial dots are then
// Xw only or Yc only, so the per-row wave reduce-scatter handles R*RP values (not 2R*RP) and each
// wave broadcasts only the mu it uses (mu_T for X waves, mu_U for Y waves).
//   PIPE = true : step g computes group g+1's dots before group g's update (x of both in VGPRs)
//   PIPE = false: step g applies group g's update, then computes group g+1's dots (one x set)
template <int R, int NSH, int NT, int RP, bool PIPE, int SLOTS, int CPW>
__global__ __launch_bounds__(NT, 2 * NT / 512) void ppls_sweep_split_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int64_t n_local, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, const PplsScalars* __restrict__ sc,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu, int ablate) {
  static_assert(SLOTS >= 2 * RP, "ring must hold the group being read and the group in flight");
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
  const int64_t rb = n_local * g / G, re = n_local * (g + 1) / G;
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
    cf[tid] = sc->alpha[tid];
    cf[R + tid] = sc->beta[tid];
    cf[2 * R + tid] = sc->gamma[tid];
    cf[3 * R + tid] = sc->delta[tid];
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto issue_row = [&](int i) {
    if ((ablate & 2) || !dma_wave) return;
    const int64_t row = rb + i;
    const char* xr = (const char*)(X + row * (int64_t)ldx);
    const char* yr = (const char*)(Y + row * (int64_t)ldy);
    const uint32_t sb = lds_base + (uint32_t)((i % SLOTS) * slot_bytes);
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int ch = min(wave * CPW + j, nch - 1);
      const char* src;
      if (ch < nchx) src = xr + min(ch * 1024 + lane * 16, ldx * 8 - 16);
      else src = yr + min((ch - nchx) * 1024 + lane * 16, ldy * 8 - 16);
      ppls_dma16(src, sb + (uint32_t)(ch * 1024));
    }
  };
  auto issue_group = [&](int grp) {
    for (int j = 0; j < RP; ++j)
      if (grp * RP + j < nrows) issue_row(grp * RP + j);
  };
  auto load_x = [&](int grp, double2 (&xv)[RP][NSH]) {
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      const int row = min(grp * RP + j, nrows - 1);
      const char* sb = smem + (size_t)(row % SLOTS) * slot_bytes + xoff;
#pragma unroll
      for (int s = 0; s < NSH; ++s)
        xv[j][s] = vs[s] ? *(const double2*)(sb + (th + s * HT) * 16) : make_double2(0.0, 0.0);
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

  if (ngroups > 0) {
    const int npro = min(SLOTS, nrows);
    for (int i = 0; i < npro; ++i) issue_row(i);
    if (write_mu) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else ppls_wait_vmcnt((npro - min(RP, nrows)) * CPW);
    ppls_lds_barrier();
    double2 xc[RP][NSH] = {};
    load_x(0, xc);
    if (!(ablate & 1)) dots(0, xc);
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
      if (gg * RP + SLOTS < nrows) issue_group(gg + SLOTS / RP);
      if (ablate & 1) continue;
      double mta = 0.0, mua = 0.0;
      zsum(gg, mta, mua);
      if constexpr (PIPE) {
        double2 xn[RP][NSH] = {};
        if (gg + 1 < ngroups) {
          load_x(gg + 1, xn);
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
          load_x(gg + 1, xc);
          dots(gg + 1, xc);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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
    if (qr) {
      for (int j = 0; j < r; ++j)
        for (int i = 0; i < r; ++i) P[j * r + i] = (i == j) ? 1.0 : 0.0;
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

// Block-wide sum of NV values per thread with a compile-time count (registers, no scratch).
template <int NV>
__device__ __forceinline__ void ppls_block_sum_t(double (&vals)[NV], double* sh) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwaves = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const double s = ppls_wave_sum(vals[k]);
    if (lane == 0) sh[wave * NV + k] = s;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    double t = 0.0;
    for (int w = 0; w < nwaves; ++w) t += sh[w * NV + k];
    vals[k] = t;
  }
  __syncthreads();
}

// Upper Cholesky G = R'R of an r x r SPD matrix (column-major); false if not numerically SPD.
template <int R>
__device__ bool ppls_chol_upper(const double* G, double* Rm) {
  for (int j = 0; j < R; ++j) {
    for (int i = 0; i <= j; ++i) {
      double s = G[j * R + i];
      for (int k = 0; k < i; ++k) s -= Rm[i * R + k] * Rm[j * R + k];
      if (i == j) {
        if (!(s > 0.0)) return false;
        Rm[j * R + j] = sqrt(s);
      } else {
        Rm[j * R + i] = s / Rm[i * R + i];
      }
    }
    for (int i = j + 1; i < R; ++i) Rm[j * R + i] = 0.0;
  }
  return true;
}

// inv(U) for upper-triangular U (column-major), into Ui.
template <int R>
__device__ void ppls_inv_upper(const double* U, double* Ui) {
  for (int j = 0; j < R; ++j)
    for (int i = R - 1; i >= 0; --i) {
      double s = (i == j) ? 1.0 : 0.0;
      for (int k = i + 1; k < R; ++k) s -= U[k * R + i] * Ui[j * R + k];
      Ui[j * R + i] = (i <= j) ? s / U[i * R + i] : 0.0;
    }
}

// Polar factor U V' of the p x r matrix S (column-major, ld lds) by Cholesky-QR2:
//   G1 = S'S = R1'R1, Q1 = S R1^-1, G2 = Q1'Q1 = R2'R2, R = R2 R1 (orthogonality O(eps kappa)),
//   R = U_R Sigma V_R' (one-sided Jacobi), polar(S) = S R^-1 U_R V_R'.
// Two block reductions instead of the 3r of Householder.  The r x r algebra runs on one thread
// with every operand in LDS (sm: >= 10 R^2 doubles).  Returns false when a Cholesky pivot fails
// (kappa(S) ~> 1e8); the caller then falls back to Householder.
template <int R>
__device__ bool ppls_block_polar_cholqr2(const double* S, int64_t lds, int p, double* out, int64_t ldo,
                                        int ldo_rows, double* sh, double* sm) {
  constexpr int NG = R * (R + 1) / 2;
  constexpr int RR = R * R;
  const int tid = threadIdx.x, nt = blockDim.x;
  double* R1 = sm;               // R1, later the final r x r multiplier
  double* M = sm + RR;           // R1^-1
  double* Gm = sm + 2 * RR;
  double* R2 = sm + 3 * RR;
  double* Rr = sm + 4 * RR;
  double* R2i = sm + 5 * RR;
  double* P = sm + 6 * RR;
  double* T = sm + 7 * RR;
  double* A = sm + 8 * RR;       // Jacobi workspace (2 RR)
  __shared__ int ok;
  double vals[NG];
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = 0.0;
  for (int i = tid; i < p; i += nt) {
    double x[R];
#pragma unroll
    for (int k = 0; k < R; ++k) x[k] = S[(int64_t)k * lds + i];
    int e = 0;
#pragma unroll
    for (int b = 0; b < R; ++b)
#pragma unroll
      for (int a = 0; a <= b; ++a) { vals[e] = fma(x[a], x[b], vals[e]); ++e; }
  }
  ppls_block_sum_t<NG>(vals, sh);
  if (tid == 0) {
    int e = 0;
    for (int b = 0; b < R; ++b)
      for (int a = 0; a <= b; ++a) { Gm[b * R + a] = vals[e]; Gm[a * R + b] = vals[e]; ++e; }
    ok = ppls_chol_upper<R>(Gm, R1);
    if (ok) ppls_inv_upper<R>(R1, M);
  }
  __syncthreads();
  if (!ok) return false;
#pragma unroll
  for (int e = 0; e < NG; ++e) vals[e] = 0.0;
  for (int i = tid; i < p; i += nt) {
    double x[R], qv[R];
#pragma unroll
    for (int k = 0; k < R; ++k) x[k] = S[(int64_t)k * lds + i];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k <= j; ++k) s = fma(x[k], M[j * R + k], s);
      qv[j] = s;
    }
    int e = 0;
#pragma unroll
    for (int b = 0; b < R; ++b)
#pragma unroll
      for (int a = 0; a <= b; ++a) { vals[e] = fma(qv[a], qv[b], vals[e]); ++e; }
  }
  ppls_block_sum_t<NG>(vals, sh);
  if (tid == 0) {
    int e = 0;
    for (int b = 0; b < R; ++b)
      for (int a = 0; a <= b; ++a) { Gm[b * R + a] = vals[e]; Gm[a * R + b] = vals[e]; ++e; }
    ok = ppls_chol_upper<R>(Gm, R2);
    if (ok) {
      for (int j = 0; j < R; ++j)            // R = R2 R1
        for (int i = 0; i < R; ++i) {
          double s = 0.0;
          for (int k = 0; k < R; ++k) s += R2[k * R + i] * R1[j * R + k];
          Rr[j * R + i] = s;
        }
      ok = ppls_small_polar_ws<R>(Rr, R, P, A, A + RR) == 0;
      ppls_inv_upper<R>(R2, R2i);
      for (int j = 0; j < R; ++j)            // T = R2^-1 P
        for (int i = 0; i < R; ++i) {
          double s = 0.0;
          for (int k = 0; k < R; ++k) s += R2i[k * R + i] * P[j * R + k];
          T[j * R + i] = s;
        }
      for (int j = 0; j < R; ++j)            // R1 <- R1^-1 R2^-1 P
        for (int i = 0; i < R; ++i) {
          double s = 0.0;
          for (int k = 0; k < R; ++k) s += M[k * R + i] * T[j * R + k];
          R1[j * R + i] = s;
        }
    }
  }
  __syncthreads();
  if (!ok) return false;
  for (int i = tid; i < ldo_rows; i += nt) {
    double x[R];
#pragma unroll
    for (int k = 0; k < R; ++k) x[k] = (i < p) ? S[(int64_t)k * lds + i] : 0.0;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < R; ++k) s = fma(x[k], R1[j * R + k], s);
      out[(int64_t)j * ldo + i] = s;
    }
  }
  return true;
}

// Block 0: W_next = orth(S_X); block 1: C_next = orth(S_Y); block 2: scalars (moments, loglik,
// M-step).  stats = [SX ldx*R][SY ldy*R][G 4R^2];  ssq = {||X||^2, ||Y||^2}.  Every sequential
// working set lives in LDS (no private-memory scratch).
template <int R>
__global__ __launch_bounds__(256) void ppls_finalize_kernel(
    const double* __restrict__ stats, const double* __restrict__ ssq, double N, int p, int q, int ldx,
    int ldy, const double* __restrict__ Wc, const double* __restrict__ Cc,
    const PplsScalars* __restrict__ sc_cur, double* __restrict__ Wn, double* __restrict__ Cn,
    PplsScalars* __restrict__ sc_nxt, PplsMoments* __restrict__ mom, double* __restrict__ loglik,
    int logl_index, double* __restrict__ work, int* __restrict__ status, int qr, int mode) {
  constexpr int NG = R * (R + 1) / 2;
  __shared__ double sh[4 * 2 * NG];
  __shared__ double sm[10 * R * R];
  __shared__ PplsScalars s_cur, s_nx;
  __shared__ PplsMoments s_m;
  __shared__ double s_G[4 * R * R], s_WtW[R * R], s_CtC[R * R];
  const double* SX = stats;
  const double* SY = stats + (int64_t)R * ldx;
  const double* G = SY + (int64_t)R * ldy;
  const int tid = threadIdx.x;
  if (blockIdx.x < 2) {
    if (!(mode & 1)) return;
    const bool isx = blockIdx.x == 0;
    const double* S = isx ? SX : SY;
    const int ld = isx ? ldx : ldy, rows = isx ? p : q;
    double* out = isx ? Wn : Cn;
    double* w2 = work + (isx ? 0 : 2 * (int64_t)p * R);
    if (qr || !ppls_block_polar_cholqr2<R>(S, ld, rows, out, ld, ld, sh, sm))
      ppls_block_polar(S, ld, rows, R, out, ld, ld, w2, w2 + (int64_t)rows * R, status, qr);
    return;
  }
  if (!(mode & 2)) return;
  // stage theta's scalars and the Gram in LDS (all threads)
  {
    const double* src = (const double*)sc_cur;
    double* dst = (double*)&s_cur;
    for (int i = tid; i < (int)(sizeof(PplsScalars) / 8); i += blockDim.x) dst[i] = src[i];
    for (int i = tid; i < 4 * R * R; i += blockDim.x) s_G[i] = G[i];
  }
  // W'W and C'C of the parameters the sweep used (one batched reduction)
  double vals[2 * NG];
#pragma unroll
  for (int e = 0; e < 2 * NG; ++e) vals[e] = 0.0;
  for (int i = tid; i < (p > q ? p : q); i += blockDim.x) {
    double wv[R], cv[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      wv[k] = (i < p) ? Wc[(int64_t)k * ldx + i] : 0.0;
      cv[k] = (i < q) ? Cc[(int64_t)k * ldy + i] : 0.0;
    }
    int e = 0;
#pragma unroll
    for (int b = 0; b < R; ++b)
#pragma unroll
      for (int a = 0; a <= b; ++a) {
        vals[e] = fma(wv[a], wv[b], vals[e]);
        vals[NG + e] = fma(cv[a], cv[b], vals[NG + e]);
        ++e;
      }
  }
  ppls_block_sum_t<2 * NG>(vals, sh);
  if (tid == 0) {
    int e = 0;
    for (int b = 0; b < R; ++b)
      for (int a = 0; a <= b; ++a) {
        s_WtW[b * R + a] = s_WtW[a * R + b] = vals[e];
        s_CtC[b * R + a] = s_CtC[a * R + b] = vals[NG + e];
        ++e;
      }
    const double s0 = ssq[0], s1 = ssq[1];
    if (logl_index >= 0) loglik[logl_index] = ppls_loglik_from_gram(s_G, s0, s1, N, p, q, R, &s_cur);
    ppls_estep_moments(s_G, s_WtW, s_CtC, s0, s1, N, p, q, R, &s_cur, &s_m);
    s_nx = s_cur;
    ppls_mstep_scalars(&s_m, R, &s_nx);
  }
  __syncthreads();
  {
    const double* a = (const double*)&s_m;
    double* b = (double*)mom;
    for (int i = tid; i < (int)(sizeof(PplsMoments) / 8); i += blockDim.x) b[i] = a[i];
    const double* c = (const double*)&s_nx;
    double* d = (double*)sc_nxt;
    for (int i = tid; i < (int)(sizeof(PplsScalars) / 8); i += blockDim.x) d[i] = c[i];
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
template <int R>
hipError_t launch_finalize_t(const PplsFinalizeArgs* f, hipStream_t st) {
  hipLaunchKernelGGL(ppls_finalize_kernel<R>, dim3(3), dim3(256), 0, st, f->stats, f->ssq, f->N, f->p,
                     f->q, f->ldx, f->ldy, f->Wc, f->Cc, f->sc_cur, f->Wn, f->Cn, f->sc_nxt, f->mom,
                     f->loglik, f->logl_index, f->work, f->status, f->qr, f->mode);
  return hipGetLastError();
}


size_t fused_lds(int r, int ldx, int ldy, int threads, int rp) {
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  const int v = 2 * r * rp, nw = threads / 64;
  return (size_t)PPLS_SWEEP_SLOTS * (nch << 10) + (size_t)(3 * nw * v + 4 * r) * 8;
}

template <int R, int NS, int NT, int RP, int CPW>
hipError_t launch_fused_t(const PplsSweepArgs& a, hipStream_t st) {
  auto kern = ppls_sweep_fused_kernel<R, NS, NT, RP, PPLS_SWEEP_SLOTS, CPW>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.grid), dim3(NT), fused_lds(R, a.ldx, a.ldy, NT, RP), st, a.X, a.Y,
                     a.n_local, a.ldx, a.ldy, a.Wp, a.Cp, a.sc, a.part, a.part_ld, a.mu, a.write_mu,
                     a.ablate);
  return hipGetLastError();
}

template <int R, int NS, int NT, int RP>
hipError_t launch_fused_cpw(const PplsSweepArgs& a, hipStream_t st) {
  const int nch = ((a.ldx * 8 + 1023) >> 10) + ((a.ldy * 8 + 1023) >> 10);
  const int need = (nch + NT / 64 - 1) / (NT / 64);   // chunks per wave with every wave copying
  if (need <= 2) return launch_fused_t<R, NS, NT, RP, 2>(a, st);
  if (need <= 4) return launch_fused_t<R, NS, NT, RP, 4>(a, st);
  return hipErrorInvalidValue;   // cannot happen: nch <= 16 * NS (ppls_fused_supported)
}

// Only the (R, NS, NT, RP) combinations ppls_fused_supported admits are instantiated (the others
// would not fit in 256 VGPRs).
size_t split_lds(int r, int ldx, int ldy, int threads, int rp) {
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  const int v = r * rp, nw = threads / 64;
  return (size_t)PPLS_SWEEP_SLOTS * (nch << 10) + (size_t)(2 * nw * v + nw * 2 * v + 4 * r) * 8;
}

template <int R, int NSH, int RP, bool PIPE, int CPW>
hipError_t launch_split_t(const PplsSweepArgs& a, hipStream_t st) {
  auto kern = ppls_sweep_split_kernel<R, NSH, 512, RP, PIPE, PPLS_SWEEP_SLOTS, CPW>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
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
                     a.ablate);
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

template <int R>
hipError_t launch_fused_r(const PplsSweepArgs& a, hipStream_t st) {
  if (a.threads == 1024) {
    if constexpr (R <= 3) {
      if (a.ns == 1) return launch_fused_cpw<R, 1, 1024, 1>(a, st);
    }
    return hipErrorInvalidValue;
  }
  if constexpr (R <= 4) {
    if (a.rp == 2 && a.ns == 1) return launch_fused_cpw<R, 1, 512, 2>(a, st);
  }
  if (a.ns == 1) return launch_fused_cpw<R, 1, 512, 1>(a, st);
  if constexpr (2 * R <= 10) {
    if (a.ns == 2) return launch_fused_cpw<R, 2, 512, 1>(a, st);
  }
  return hipErrorInvalidValue;
}
}  // namespace

extern "C" {

int ppls_fused_supported(int r, int ldx, int ldy, int threads) {
  const int npmax = (ldx > ldy ? ldx : ldy) / 2;
  const int ns = (npmax + threads - 1) / threads;
  if (r < 1 || r > PPLS_FUSED_RMAX) return 0;
  if (threads == 1024) {
    if (ns != 1 || r > 3) return 0;   // 4 waves/SIMD: W, C, accumulators in <= 128 VGPRs
  } else if (threads == 512) {
    if (ns < 1 || ns > 2 || ns * r > 10) return 0;   // W, C and accumulators stay in VGPRs
  } else {
    return 0;
  }
  const int nch = ((ldx * 8 + 1023) >> 10) + ((ldy * 8 + 1023) >> 10);
  if (nch > 4 * (threads / 64)) return 0;   // at most 4 DMA chunks per wave per row
  return ppls_fused_lds_bytes(r, ldx, ldy, threads) <= 160 * 1024 ? ns : 0;
}

size_t ppls_fused_lds_bytes(int r, int ldx, int ldy, int threads) {
  return fused_lds(r, ldx, ldy, threads, 2);
}

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

// Fixed-order two-stage reduction: stage 1 sums chunks of RCHUNK groups (many blocks busy), stage 2
// sums the chunk results.  tmp: ceil(ngroups / RCHUNK) * len doubles (taken from the tail of part
// when the caller passes tmp == nullptr is not allowed; see ppls_reduce_tmp_len).
#define PPLS_RCHUNK 32
int64_t ppls_reduce_tmp_len(int ngroups, int64_t len) {
  return ngroups > PPLS_RCHUNK ? (int64_t)((ngroups + PPLS_RCHUNK - 1) / PPLS_RCHUNK) * len : 0;
}

hipError_t ppls_launch_reduce2(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                               double* tmp, hipStream_t st) {
  if (ngroups <= PPLS_RCHUNK || tmp == nullptr) {
    hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0,
                       st, part, ngroups, ld, len, out, 0);
    return hipGetLastError();
  }
  const int nch = (ngroups + PPLS_RCHUNK - 1) / PPLS_RCHUNK;
  hipLaunchKernelGGL(ppls_reduce_chunks_kernel, dim3((unsigned)((len + 255) / 256), nch), dim3(256), 0,
                     st, part, ngroups, ld, len, tmp);
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0,
                     st, tmp, nch, len, len, out, 0);
  return hipGetLastError();
}

hipError_t ppls_launch_reduce(const double* part, int ngroups, int64_t ld, int64_t len, double* out,
                              int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(ppls_reduce_partials_kernel, dim3((unsigned)((len + 255) / 256)), dim3(256), 0,
                     st, part, ngroups, ld, len, out, accumulate);
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
    default:   // r = 7..16: runtime-r finalize (the unrolled batched reductions would spill)
      hipLaunchKernelGGL(ppls_finalize_generic_kernel, dim3(3), dim3(256), 0, st, f->stats, f->ssq, f->N,
                         f->p, f->q, f->r, f->ldx, f->ldy, f->Wc, f->Cc, f->sc_cur, f->Wn, f->Cn,
                         f->sc_nxt, f->mom, f->loglik, f->logl_index, f->work, f->status, f->qr, f->mode);
      return hipGetLastError();
  }
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
