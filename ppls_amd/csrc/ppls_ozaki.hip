// ppls_ozaki.hip -- the cross-product Gram S = D'D (D = [X | Y], ppls_xprod.hip's S) on INT8 MFMA
// by the Chinese-remainder ("Ozaki scheme II") form (round 6).  S is 92 % of a
// default PPLS_simult call and the fp64 MFMA Gram runs at 0.90 of the fp64 peak; gfx950's
// v_mfma_i32_32x32x32_i8 issues 64x the fp64 MFMA's multiply-adds per clock.
//
//   1. column scaling (host, from ppls_oz_colstats_kernel; gram_run_oz in ppls_capi.cpp): per live
//      column j, e_j with max_k |D_kj| < 2^e_j and L_j bits from the column's spread
//      c_j = 2^e_j sqrt(n) / sqrt(S_jj); every element becomes the integer x'_kj = rint(D_kj 2^s_j),
//      s_j = L_j - e_j, |x'| < 2^L_j, exact in fp64 (a power-of-2 scale, then a rounding to an
//      integer).  The rounding error of S_ij is then at most
//      2^-(s_i+1) sum|D_kj| + 2^-(s_j+1) sum|D_ki| <= 2^-55 sqrt(S_ii S_jj).
//   2. residues (ppls_oz_residue_kernel): x' mod m_l for NMOD pairwise coprime moduli m_l <= 256,
//      symmetric (|r| <= 128, int8), written as NMOD planes [n / 64][Pp][64] (a stage's 64 rows of
//      one column contiguous: 16 KB per 256-column panel stage).
//   3. SYRK per modulus (ppls_oz_syrk_kernel): the lower 256 x 256 tiles of R_l' R_l on
//      v_mfma_i32_32x32x32_i8, exact in int32 (reduced mod m_l every 65,536 rows), -> uint8 residues.
//   4. CRT (ppls_oz_finish_kernel): Garner's mixed-radix digits of the NMOD residues, the exact
//      integer sum_k x'_ki x'_kj in 192 bits (|.| < M / 2, M = prod m_l > 2 max_ij |sum|), ONE
//      rounding to fp64, times 2^-(s_i + s_j) -> S, mirrored.
// Integer sums are exact, so S depends on the data only (not on the schedule): bitwise repeatable.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ppls_device.h"
#include "ppls_kernels.h"

namespace {

constexpr int OZ_TT = 256;                 // output tile edge
constexpr int OZ_KS = PPLS_OZ_KS;          // rows per stage (one column's stage: 64 B)
constexpr int OZ_PANEL = OZ_TT * OZ_KS;    // bytes of one 256-column panel stage (16 KB)
constexpr int OZ_SPLIT_STAGES = 1024;      // stages per SYRK item: 65,536 rows, |sum| <= 2^30 in int32

// pairwise coprime moduli, largest first: 2^8, 3*5*17, 11*23, 251, 13*19, then primes and 7*31.  A
// switch, so an unrolled loop over l sees compile-time moduli (multiply-high forms of % m).
__host__ __device__ constexpr int oz_mod(int l) {
  switch (l) {
    case 0: return 256;  case 1: return 255;  case 2: return 253;  case 3: return 251;  case 4: return 247;
    case 5: return 241;  case 6: return 239;  case 7: return 233;  case 8: return 229;  case 9: return 227;
    case 10: return 223; case 11: return 217; case 12: return 211; case 13: return 199; case 14: return 197;
    case 15: return 193; case 16: return 191; case 17: return 181; case 18: return 179; case 19: return 173;
    default: return 1;
  }
}

constexpr int oz_inv(int a, int m) {   // a^-1 mod m (gcd 1), extended Euclid
  int t = 0, nt = 1, r = m, nr = ((a % m) + m) % m;
  while (nr) {
    const int q = r / nr;
    const int tt = t - q * nt;
    t = nt;
    nt = tt;
    const int rr = r - q * nr;
    r = nr;
    nr = rr;
  }
  return t < 0 ? t + m : t;
}

// Garner's inverses inv[l][k] = m_k^-1 mod m_l (k < l) and, per modulus count N, M_N = prod_{l<N} m_l
// and floor(M_N / 2) in 6 little-endian 32-bit limbs.
struct OzTab {
  int inv[PPLS_OZ_MAXMOD][PPLS_OZ_MAXMOD];
  uint32_t M[PPLS_OZ_MAXMOD + 1][6], halfM[PPLS_OZ_MAXMOD + 1][6];
};
constexpr OzTab oz_make_tab() {
  OzTab t{};
  for (int l = 0; l < PPLS_OZ_MAXMOD; ++l)
    for (int k = 0; k < l; ++k) t.inv[l][k] = oz_inv(oz_mod(k), oz_mod(l));
  uint64_t w[6] = {1, 0, 0, 0, 0, 0};
  for (int n = 0; n <= PPLS_OZ_MAXMOD; ++n) {
    for (int q = 0; q < 6; ++q) t.M[n][q] = (uint32_t)w[q];
    uint32_t c = 0;
    for (int q = 5; q >= 0; --q) {
      t.halfM[n][q] = (t.M[n][q] >> 1) | (c << 31);
      c = t.M[n][q] & 1u;
    }
    if (n < PPLS_OZ_MAXMOD) {
      uint64_t carry = 0;
      for (int q = 0; q < 6; ++q) {
        const uint64_t v = w[q] * (uint64_t)oz_mod(n) + carry;
        w[q] = v & 0xffffffffull;
        carry = v >> 32;
      }
    }
  }
  return t;
}
__constant__ OzTab oz_tab = oz_make_tab();

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// s_waitcnt immediate (gfx9 encoding) that waits for vmcnt <= N only: expcnt 7, lgkmcnt 15 (no wait)
#define OZ_VMCNT(N) (((N) & 15) | (7 << 4) | (15 << 8) | (((N) >> 4) << 14))

__host__ __device__ inline void oz_tile_of(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

// a joint column c of [X | Y] (X's xcols stored columns, then Y's): its row base and whether live
struct OzCols {
  int xreal, xcols, yreal;
};
__device__ __forceinline__ bool oz_live(const OzCols& g, int c) {
  return c < g.xreal || (c >= g.xcols && c - g.xcols < g.yreal);
}

template <typename T>
__device__ __forceinline__ double oz_ld(const T* X, int ldx, const T* Y, int ldy, const OzCols& g, int64_t row, int c) {
  if (c < g.xreal) return (double)X[row * ldx + c];
  if (c >= g.xcols && c - g.xcols < g.yreal) return (double)Y[row * ldy + (c - g.xcols)];
  return 0.0;
}

}  // namespace

// ---------------------------------------------------------------------------- 1. column statistics
// part[chunk][2][Pp]: per column the max |D| and sum D^2 over the chunk's rows (one thread per
// column, rows strided by the grid's y dimension).
template <typename T>
__global__ __launch_bounds__(256) void ppls_oz_colstats_kernel(const T* __restrict__ X, int ldx, const T* __restrict__ Y,
                                                               int ldy, OzCols g, int Pp, int64_t n, int64_t rpc,
                                                               double* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= Pp) return;
  const int64_t r0 = (int64_t)blockIdx.y * rpc, r1 = r0 + rpc < n ? r0 + rpc : n;
  double mx = 0.0, ss = 0.0;
  if (oz_live(g, c))
    for (int64_t r = r0; r < r1; ++r) {
      const double v = oz_ld(X, ldx, Y, ldy, g, r, c);
      mx = fmax(mx, fabs(v));
      ss = fma(v, v, ss);
    }
  double* o = part + (int64_t)blockIdx.y * 2 * Pp;
  o[c] = mx;
  o[Pp + c] = ss;
}

__global__ void ppls_oz_colstats_finish_kernel(const double* __restrict__ part, int chunks, int Pp, double* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= Pp) return;
  double mx = 0.0, ss = 0.0;
  for (int k = 0; k < chunks; ++k) {   // fixed order
    mx = fmax(mx, part[(int64_t)k * 2 * Pp + c]);
    ss += part[(int64_t)k * 2 * Pp + Pp + c];
  }
  out[c] = mx;
  out[Pp + c] = ss;
}

// ---------------------------------------------------------------------------- 2. residue planes
// Block: one 64-row stage kb x 64 columns.  Thread: column c0 + (tid >> 2), rows 16 (tid & 3) .. + 15
// of the stage.  x' = rint(D 2^shift_c) (exact), u = x' + 2^62 in [0, 2^63) as three 21-bit limbs
// u = a 2^42 + b 2^21 + c; per modulus  u mod m = (a (2^42 mod m) + b (2^21 mod m) + c) mod m  -- two
// 24-bit multiply-adds (operands < 2^24) and ONE 32-bit reduction of a value < 2^31 -- then minus
// 2^62 mod m (folded into the sum as m - (2^62 mod m)), symmetric.  (The residue arithmetic, not the
// 106 GB of C3 traffic, bounded the first form's three 32-bit reductions per residue: 41 ms.)
// biash = m - (2^62 mod m) + floor(m / 2): then (t mod m) - floor(m / 2) is the symmetric residue
// (in [-(m-1)/2, (m-1)/2] for odd m, [-128, 127] for 256) without a compare and select.
__host__ __device__ __forceinline__ int oz_residue21(uint32_t a, uint32_t b, uint32_t c, uint32_t m, uint32_t k42,
                                                     uint32_t k21, uint32_t biash) {
  const uint32_t t = a * k42 + b * k21 + c + biash;   // < 2^21 255 2 + 2^21 + 384 < 2^31
  return (int)(t % m) - (int)(m / 2);
}

template <typename T, int NMOD>
__global__ __launch_bounds__(256) void ppls_oz_residue_kernel(const T* __restrict__ X, int ldx, const T* __restrict__ Y,
                                                              int ldy, OzCols g, int Pp, int64_t n,
                                                              const int* __restrict__ shift, int8_t* __restrict__ planes,
                                                              int64_t pstride) {
  const int tid = threadIdx.x;
  // 4 lanes per column (row groups fastest): a wave stores 16 columns x 64 B = 1 KB contiguous per
  // plane (lanes 64 B apart, the first form, left every store a 16-B scatter) and loads 4 rows x 128 B
  const int c = blockIdx.x * 64 + (tid >> 2), grp = tid & 3;
  const int64_t kb = blockIdx.y;
  const int64_t row0 = kb * OZ_KS + 16 * grp;
  uint32_t la[16], lb[16], lc[16];
  const bool live = c < Pp && oz_live(g, c);
  const int sh = live ? shift[c] : 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t row = row0 + k;
    const double x = (live && row < n) ? oz_ld(X, ldx, Y, ldy, g, row, c) : 0.0;
    const double xs = rint(ldexp(x, sh));                        // |xs| < 2^L <= 2^62, an exact integer
    const uint64_t u = (uint64_t)((int64_t)xs + (int64_t)(1ull << 62));
    la[k] = (uint32_t)(u >> 42);
    lb[k] = (uint32_t)(u >> 21) & 0x1FFFFFu;
    lc[k] = (uint32_t)u & 0x1FFFFFu;
  }
  if (c >= Pp) return;
  int8_t* dst = planes + (kb * Pp + c) * OZ_KS + 16 * grp;
#pragma unroll
  for (int l = 0; l < NMOD; ++l) {
    const uint32_t m = (uint32_t)oz_mod(l);
    const uint32_t k42 = (uint32_t)((1ull << 42) % m), k21 = (uint32_t)((1ull << 21) % m);
    const uint32_t bias = m - (uint32_t)((1ull << 62) % m) + m / 2;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k)
      w[k >> 2] |= ((uint32_t)oz_residue21(la[k], lb[k], lc[k], m, k42, k21, bias) & 255u) << (8 * (k & 3));
    *(v4i*)(dst + (int64_t)l * pstride) = v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
  }
}

// ---------------------------------------------------------------------------- 3. int8 SYRK per modulus
// One workgroup per (modulus, 65,536-row split, lower 256 x 256 tile); 4 waves of 128 x 128 (4 x 4
// blocks of v_mfma_i32_32x32x32_i8, 256 int32 accumulators per lane).  The two panels of a 64-row
// stage (16 KB each; a diagonal tile's B panel is its A panel, copied twice: one code path, 8 % faster
// on the C3 grid than a diagonal specialised to one panel) go HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging) into a ring of 4 buffers, three stages in flight; one
// barrier per stage, before which every wave waits for its own copies of that stage: vmcnt <= the
// 2 x 8 copies it issued for the two later stages.  The copies go through the product's inline-asm
// helper (ppls_dma16s), which the compiler does not track: with the compiler's own builtin it put
// vmcnt(0) -- the whole prefetch -- in front of the first fragment read of three stages in four (it
// cannot tell the ring's buffers apart across the loop's joins), and DMA and MFMA time added up
// (10.3 ms per C3 plane against 6.1 compute-only and 6.4 copies-only; 7.8 ms untracked;
// profiles/r6_int8_syrk_ab.txt, tools/oz_lab.hip).  Hand-counted waits as in the split sweep, checked
// on the built code object by tools/isa_check.py (tests/test_isa_dma_ring.py).  The stage is
// branch-free: the tail copies the last stage again into the buffer no one reads, so every wait is the
// same count.  The copies of stage s + 3 go out one per MFMA group during stage s's first k-step, and
// the second k-step's fragments are read during the first's MFMAs.  The 16-B chunks are XOR-swizzled
// on the source side (LDS chunk q of column c holds global chunk q ^ ((c >> 2) & 3)), so the fragment
// reads (ds_read_b128) are conflict-free.  Both MFMA operands are read from the same layout, so
// whatever order the instruction gives the 32 k values of a step, each k meets itself.
// |r| <= 128: a split's 65,536 rows sum to at most 2^30 -- exact in int32, no reduction in the loop
// (one there made the compiler spill the accumulators).  Output: the split's tile sums mod m, uint8,
// column-major [col][row].
//   A (lab ablations, tools/oz_lab.hip only; 0 in the product): A & 1 no copies (compute on whatever
//   the ring holds), A & 2 no fragment reads or MFMAs (the copies alone), A & 4 eight waves of
//   128 x 64 (two per SIMD: one can issue MFMAs while the other stalls on a copy) -- 7.30-7.40 vs
//   7.36 ms per C3 plane, no gain (profiles/r6_int8_syrk_ab.txt).
__device__ __forceinline__ int oz_lds_off(int c, int q) { return c * OZ_KS + ((q ^ ((c >> 2) & 3)) << 4); }

typedef __attribute__((address_space(3))) void* oz_lptr;

template <int A>
__global__ __launch_bounds__((A & 4) ? 512 : 256, 1) void ppls_oz_syrk_kernel(
    const int8_t* __restrict__ planes, int64_t pstride, int Pp, int64_t nkb, int nmod, int nsplit, int ntiles,
    uint8_t* __restrict__ out) {
  constexpr int NWV = (A & 4) ? 8 : 4;   // (lab: A & 4, 8 waves of 128 x 64, two per SIMD)
  constexpr int CT = 256 / (NWV / 2);    // output columns per wave
  constexpr int NJ = CT / 32;            // 32-column MFMA blocks per wave
  constexpr int NU = 16 / NWV;           // LDS-DMA instructions per wave per panel stage (16 KB / 1 KB)
  constexpr int NC = 2 * NU;             // per wave per stage: both panels
  __shared__ __attribute__((aligned(16))) int8_t ring[4 * 2 * OZ_PANEL];   // 4 x [A panel | B panel]
  const int b = blockIdx.x, nb = gridDim.x;
  const int it = (b & 7) * (nb >> 3) + (b >> 3);   // XCD x (b mod 8) takes a contiguous item range
  if (it >= nmod * nsplit * ntiles) return;
  // item = (modulus, split, tile), tile fastest: concurrent items share the split's row stages
  const int l = it / (nsplit * ntiles), rem = it - l * nsplit * ntiles;
  const int sp = rem / ntiles, t = rem - sp * ntiles;
  const int64_t s0 = (int64_t)sp * OZ_SPLIT_STAGES;
  const int64_t s1 = s0 + OZ_SPLIT_STAGES < nkb ? s0 + OZ_SPLIT_STAGES : nkb;
  const int m = oz_mod(l);
  int I, J;
  oz_tile_of(t, &I, &J);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave / (NWV / 2), wj = wave % (NWV / 2);
  const bool idle = I == J && wi == 0 && wj * CT >= 128;   // the diagonal tile's upper-right quadrant
  const int8_t* pl = planes + (int64_t)l * pstride;
  const int8_t* pa = pl + (int64_t)I * OZ_PANEL;
  const int8_t* pb = pl + (int64_t)J * OZ_PANEL;
  const int64_t sstride = (int64_t)Pp * OZ_KS;
  v16i acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v16i{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  // this lane's source offset in a panel stage: wave instruction g = NU wave + u fills LDS bytes
  // [1024 g, + 1024); lane l the 16 B at 16 l: column 16 g + l / 4, chunk l % 4 (swizzled)
  int soff[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int c = 16 * (NU * wave + u) + (lane >> 2), pos = lane & 3;
    soff[u] = c * OZ_KS + ((pos ^ ((c >> 2) & 3)) << 4);
  }
  const uint32_t lring = (uint32_t)(uintptr_t)(oz_lptr)ring;
  auto last = [&](int64_t s) { return s < s1 ? s : s1 - 1; };
  // copy g of this wave's NC for stage s into ring buffer bq
  auto dma = [&](int bq, int64_t s, int g) __attribute__((always_inline)) {
    if constexpr ((A & 1) != 0) return;
    const int8_t* src = (g < NU ? pa : pb) + s * sstride;
    const int u = g < NU ? g : g - NU;
    const uint32_t dst = lring + (uint32_t)(bq * 2 * OZ_PANEL + (g < NU ? 0 : OZ_PANEL) + 1024 * (NU * wave + u));
    ppls_dma16s(src, (uint32_t)soff[u], (uint32_t)__builtin_amdgcn_readfirstlane((int)dst));   // wave-uniform
  };
  const int ca0 = 128 * wi + (lane & 31), cb0 = CT * wj + (lane & 31), h = lane >> 5;
  // stage s from ring buffer bq; meanwhile the copies of stage s + 3 into buffer (bq + 3) % 4
  auto stage = [&](int bq, int64_t s) __attribute__((always_inline)) {
    ppls_wait_vmcnt(2 * NC);   // own copies of stage s landed (s + 1, s + 2 in flight)
    ppls_lds_barrier();        // everyone's; the buffer of stage s - 1 is free
    const int64_t sn = last(s + 3);
    const int nq = (bq + 3) & 3;
    if constexpr ((A & 2) != 0) {
#pragma unroll
      for (int g = 0; g < NC; ++g) dma(nq, sn, g);
      return;
    }
    const int8_t* ca = ring + bq * 2 * OZ_PANEL;
    const int8_t* cbp = ca + OZ_PANEL;
    v4i a0[4], b0[NJ], a1[4], b1[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) a0[i] = *(const v4i*)(ca + oz_lds_off(ca0 + 32 * i, h));
#pragma unroll
    for (int j = 0; j < NJ; ++j) b0[j] = *(const v4i*)(cbp + oz_lds_off(cb0 + 32 * j, h));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0[i], b0[j], acc[i][j], 0, 0, 0);
      if (i < NC) dma(nq, sn, i);
      // the second k-step's fragments, spread over the groups
      a1[i] = *(const v4i*)(ca + oz_lds_off(ca0 + 32 * i, 2 + h));
      if (i < NJ) b1[i] = *(const v4i*)(cbp + oz_lds_off(cb0 + 32 * i, 2 + h));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1[i], b1[j], acc[i][j], 0, 0, 0);
      if (4 + i < NC) dma(nq, sn, 4 + i);
    }
  };
  // prologue: stages s0 .. s0 + 2 (clamped) into buffers 0 .. 2
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int g = 0; g < NC; ++g) dma(k, last(s0 + k), g);
  for (int64_t s = s0; s < s1; s += 4) {
    stage(0, s);
    if (s + 1 < s1) stage(1, s + 1);
    if (s + 2 < s1) stage(2, s + 2);
    if (s + 3 < s1) stage(3, s + 3);
  }
  ppls_wait_vmcnt(0);   // no copy may land after the workgroup's LDS is gone
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int v = acc[i][j][r] % m;
        acc[i][j][r] = v < 0 ? v + m : v;
      }
  if (idle) return;
  uint8_t* o = out + (int64_t)it * OZ_TT * OZ_TT;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = CT * wj + 32 * j + (lane & 31);
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {   // 32 x 32 D map: rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
        const int row = 128 * wi + 32 * i + 8 * gq + 4 * h;
        const uint32_t v = (uint32_t)acc[i][j][4 * gq] | ((uint32_t)acc[i][j][4 * gq + 1] << 8) |
                           ((uint32_t)acc[i][j][4 * gq + 2] << 16) | ((uint32_t)acc[i][j][4 * gq + 3] << 24);
        *(uint32_t*)(o + (int64_t)col * OZ_TT + row) = v;
      }
    }
}

// ---------------------------------------------------------------------------- 4. CRT and scaling
namespace {

// The signed integer with residues r[l] (0 <= r < m_l, |value| < M / 2) as a double (one rounding).
template <int NMOD>
__host__ __device__ __forceinline__ double oz_crt(const int (&r)[NMOD], const OzTab& tab) {
  int d[NMOD];
#pragma unroll
  for (int l = 0; l < NMOD; ++l) {
    const int m = oz_mod(l);
    int t = r[l];
#pragma unroll
    for (int k = 0; k < l; ++k) {
      t = t - d[k] + 2 * m;                    // >= 0: d[k] < 256 <= 2 m
      t = (t * tab.inv[l][k]) % m;             // < 3 m 256: int
    }
    d[l] = t;
  }
  // v = d0 + m0 (d1 + m1 (d2 + ...)): Horner from the top digit in 6 x 32-bit limbs
  uint32_t v[6] = {(uint32_t)d[NMOD - 1], 0, 0, 0, 0, 0};
#pragma unroll
  for (int l = NMOD - 2; l >= 0; --l) {
    uint64_t carry = (uint64_t)d[l];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint64_t x = (uint64_t)v[q] * (uint64_t)oz_mod(l) + carry;
      v[q] = (uint32_t)x;
      carry = x >> 32;
    }
  }
  // v > M / 2 -> negative: |value| = M - v
  bool gt = false, eq = true;
#pragma unroll
  for (int q = 5; q >= 0; --q) {
    if (eq && v[q] != tab.halfM[NMOD][q]) {
      gt = v[q] > tab.halfM[NMOD][q];
      eq = false;
    }
  }
  const bool neg = gt;
  if (neg) {
    uint64_t borrow = 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const uint64_t x = (uint64_t)tab.M[NMOD][q] - (uint64_t)v[q] - borrow;
      v[q] = (uint32_t)x;
      borrow = (x >> 32) & 1u;
    }
  }
  // top 64 bits + sticky -> double (correctly rounded), times 2^(32 k)
  int top = 5;
  while (top > 0 && v[top] == 0) --top;
  if (top == 0) return neg ? -(double)v[0] : (double)v[0];
  uint64_t hi = ((uint64_t)v[top] << 32) | v[top - 1];
  int e = 32 * (top - 1);
  uint32_t sticky = 0;
  for (int q = 0; q < top - 1; ++q) sticky |= v[q];
  const int lz = __builtin_clzll(hi);   // hi >= 2^32: lz <= 31
  if (lz > 0 && top >= 2) {   // pull the next limb's bits under the leading zeros
    hi = (hi << lz) | ((uint64_t)v[top - 2] >> (32 - lz));
    e -= lz;
    sticky = (v[top - 2] & ((1u << (32 - lz)) - 1u)) != 0u ? 1u : 0u;   // the bits not pulled up
    for (int q = 0; q < top - 2; ++q) sticky |= v[q];
  } else if (lz > 0) {
    hi <<= lz;
    e -= lz;
  }
  const double dv = ldexp((double)(hi | (sticky ? 1ull : 0ull)), e);
  return neg ? -dv : dv;
}

}  // namespace

// One workgroup per lower 256 x 256 tile and 16-column strip: thread i computes rows i of the
// strip's 16 columns (element (I 256 + i, J 256 + j)), writes it column-major into G, and the
// mirror element through an LDS transpose.  Columns / rows not live are 0.
template <int NMOD>
__global__ __launch_bounds__(256) void ppls_oz_finish_kernel(const uint8_t* __restrict__ part, int nsplit, int ntiles,
                                                             OzCols g, int P, const int* __restrict__ shift,
                                                             double* __restrict__ G) {
  __shared__ double tr[16][OZ_TT + 1];
  const int t = blockIdx.x, strip = blockIdx.y;
  int I, J;
  oz_tile_of(t, &I, &J);
  const int i = threadIdx.x;
  const int a = I * OZ_TT + i;
#pragma unroll 1
  for (int jj = 0; jj < 16; ++jj) {
    const int j = strip * 16 + jj;
    const int bcol = J * OZ_TT + j;
    double v = 0.0;
    const bool lower = !(I == J && j > i);
    if (a < P && bcol < P && lower && oz_live(g, a) && oz_live(g, bcol)) {
      int r[NMOD];
#pragma unroll
      for (int l = 0; l < NMOD; ++l) {   // the splits' residues, summed mod m_l
        int acc = 0;
        for (int sp = 0; sp < nsplit; ++sp)
          acc += part[(((int64_t)l * nsplit + sp) * ntiles + t) * OZ_TT * OZ_TT + (int64_t)j * OZ_TT + i];
        r[l] = acc % oz_mod(l);
      }
      v = ldexp(oz_crt<NMOD>(r, oz_tab), -(shift[a] + shift[bcol]));
    }
    tr[jj][i] = v;
    if (a < P && bcol < P && lower) G[(int64_t)bcol * P + a] = v;   // (a, b) of the lower triangle
  }
  __syncthreads();
  // mirror: element (b, a) = G[a * P + b]; lanes along b (16 columns) x 16 rows a per pass
  const int jj = threadIdx.x & 15;
  for (int ib = threadIdx.x >> 4; ib < OZ_TT; ib += 16) {
    const int aa = I * OZ_TT + ib, bb = J * OZ_TT + strip * 16 + jj;
    if (aa < P && bb < P && !(I == J && strip * 16 + jj >= ib)) G[(int64_t)aa * P + bb] = tr[jj][ib];
  }
}

extern "C" {

int ppls_oz_modulus(int l) { return l >= 0 && l < PPLS_OZ_MAXMOD ? oz_mod(l) : 0; }

// Host copies of the device arithmetic, for unit tests without a GPU (tests/test_ozaki_host.py).
int ppls_oz_residue_host(double x, int shift, int l, int* r) {
  if (l < 0 || l >= PPLS_OZ_MAXMOD || !r) return -1;
  const double xs = rint(ldexp(x, shift));
  if (!(fabs(xs) < 4611686018427387904.0)) return -1;   // |x'| < 2^62
  const uint64_t u = (uint64_t)((int64_t)xs + (int64_t)(1ull << 62));
  const uint32_t m = (uint32_t)oz_mod(l);
  *r = oz_residue21((uint32_t)(u >> 42), (uint32_t)(u >> 21) & 0x1FFFFFu, (uint32_t)u & 0x1FFFFFu, m,
                    (uint32_t)((1ull << 42) % m), (uint32_t)((1ull << 21) % m), m - (uint32_t)((1ull << 62) % m) + m / 2);
  return 0;
}

int ppls_oz_crt_host(const int* r, int nmod, double* out) {
  static constexpr OzTab tab = oz_make_tab();
  if (!r || !out) return -1;
#define OZ_CRT_H(N)                                         \
  case N: {                                                 \
    int rr[N];                                              \
    for (int l = 0; l < N; ++l) rr[l] = r[l];               \
    *out = oz_crt<N>(rr, tab);                              \
    return 0;                                               \
  }
  switch (nmod) {
    OZ_CRT_H(12) OZ_CRT_H(13) OZ_CRT_H(14) OZ_CRT_H(15) OZ_CRT_H(16) OZ_CRT_H(17) OZ_CRT_H(18) OZ_CRT_H(19)
    OZ_CRT_H(20)
    default: return -1;
  }
#undef OZ_CRT_H
}

hipError_t ppls_launch_oz_colstats(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int yreal,
                                   int f32, int Pp, int64_t n, int chunks, double* part, double* out, hipStream_t st) {
  const OzCols g{xreal, xcols, yreal};
  const int64_t rpc = (n + chunks - 1) / chunks;
  const dim3 grid((unsigned)((Pp + 255) / 256), (unsigned)chunks);
  if (f32)
    hipLaunchKernelGGL(ppls_oz_colstats_kernel<float>, grid, dim3(256), 0, st, (const float*)X, ldx, (const float*)Y,
                       ldy, g, Pp, n, rpc, part);
  else
    hipLaunchKernelGGL(ppls_oz_colstats_kernel<double>, grid, dim3(256), 0, st, (const double*)X, ldx,
                       (const double*)Y, ldy, g, Pp, n, rpc, part);
  hipLaunchKernelGGL(ppls_oz_colstats_finish_kernel, dim3((unsigned)((Pp + 255) / 256)), dim3(256), 0, st, part, chunks,
                     Pp, out);
  return hipGetLastError();
}

#define OZ_NMOD_CASES(X) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20)

hipError_t ppls_launch_oz_residues(const void* X, int ldx, int xcols, int xreal, const void* Y, int ldy, int yreal,
                                   int f32, int Pp, int64_t n, int64_t nkb, const int* shift, int nmod, int8_t* planes,
                                   int64_t pstride, hipStream_t st) {
  const OzCols g{xreal, xcols, yreal};
  const dim3 grid((unsigned)((Pp + 63) / 64), (unsigned)nkb);
#define OZ_RES(N)                                                                                               \
  case N:                                                                                                       \
    if (f32)                                                                                                    \
      hipLaunchKernelGGL((ppls_oz_residue_kernel<float, N>), grid, dim3(256), 0, st, (const float*)X, ldx,      \
                         (const float*)Y, ldy, g, Pp, n, shift, planes, pstride);                               \
    else                                                                                                        \
      hipLaunchKernelGGL((ppls_oz_residue_kernel<double, N>), grid, dim3(256), 0, st, (const double*)X, ldx,    \
                         (const double*)Y, ldy, g, Pp, n, shift, planes, pstride);                              \
    break;
  switch (nmod) {
    OZ_NMOD_CASES(OZ_RES)
    default: return hipErrorInvalidValue;
  }
#undef OZ_RES
  return hipGetLastError();
}

int ppls_oz_splits(int64_t nkb) { return (int)((nkb + OZ_SPLIT_STAGES - 1) / OZ_SPLIT_STAGES); }

hipError_t ppls_launch_oz_syrk_v(int variant, const int8_t* planes, int64_t pstride, int Pp, int64_t nkb, int nmod,
                                 uint8_t* part, hipStream_t st) {
  const int T = Pp / OZ_TT, ntiles = T * (T + 1) / 2, nsplit = ppls_oz_splits(nkb);
  const int64_t items = (int64_t)nmod * nsplit * ntiles;
  const int64_t grid = (items + 7) / 8 * 8;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
#define OZ_SYRK(AV)                                                                                             \
  case AV:                                                                                                      \
    hipLaunchKernelGGL(ppls_oz_syrk_kernel<AV>, dim3((unsigned)grid), dim3(((AV) & 4) ? 512 : 256), 0, st, planes, \
                       pstride, Pp, nkb, nmod, nsplit, ntiles, part);                                           \
    break;
  switch (variant) {
    OZ_SYRK(0)
#ifdef OZ_LAB
    OZ_SYRK(1) OZ_SYRK(2) OZ_SYRK(4) OZ_SYRK(5) OZ_SYRK(6)
#endif
    default: return hipErrorInvalidValue;
  }
#undef OZ_SYRK
  return hipGetLastError();
}

hipError_t ppls_launch_oz_syrk(const int8_t* planes, int64_t pstride, int Pp, int64_t nkb, int nmod, uint8_t* part,
                               hipStream_t st) {
  return ppls_launch_oz_syrk_v(0, planes, pstride, Pp, nkb, nmod, part, st);
}

hipError_t ppls_launch_oz_finish(const uint8_t* part, int nmod, int nsplit, int Pp, int xcols, int xreal, int yreal,
                                 int P, const int* shift, double* G, hipStream_t st) {
  const OzCols g{xreal, xcols, yreal};
  const int T = Pp / OZ_TT, ntiles = T * (T + 1) / 2;
  const dim3 grid((unsigned)ntiles, (unsigned)(OZ_TT / 16));
#define OZ_FIN(N)                                                                                               \
  case N:                                                                                                       \
    hipLaunchKernelGGL((ppls_oz_finish_kernel<N>), grid, dim3(256), 0, st, part, nsplit, ntiles, g, P, shift, G); \
    break;
  switch (nmod) {
    OZ_NMOD_CASES(OZ_FIN)
    default: return hipErrorInvalidValue;
  }
#undef OZ_FIN
  return hipGetLastError();
}

}  // extern "C"
