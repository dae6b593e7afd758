// ppls_device.h -- device helpers shared by the sweep kernels (ppls_kernels.hip):
// the wave reduce-scatter (permlane / DPP butterflies) and the LDS-DMA ring primitives.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

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

// real: how many of the lane's current M values are real; an odd M is padded with one zero at its
// end, and a lane whose kept half holds that pad below the top level would otherwise claim the
// global index of a real value of the other half (both lanes "canonical": a write race).
template <int M, int L, int N>
__device__ __forceinline__ void ppls_rs_r(double (&a)[N], int lane, int& idx, bool& canon, int& real) {
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
      ppls_rs_r<1, L + 1, N>(a, lane, idx, canon, real);
    } else {
      constexpr int H = (M + 1) / 2;
      static_assert(2 * H <= N, "reduce-scatter buffer too small");
      real = beta ? (real > H ? real - H : 0) : (real < H ? real : H);
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
      ppls_rs_r<H, L + 1, N>(a, lane, idx, canon, real);
    }
  }
}

// V values per lane -> lane holds the wave sum of value idx (of the first LEFT <= 1 values for
// M <= 64); canon = this lane is the one lane to publish it (pad slots and duplicates are not).
template <int M, int L, int N>
__device__ __forceinline__ void ppls_rs(double (&a)[N], int lane, int& idx, bool& canon) {
  int real = M;
  ppls_rs_r<M, L, N>(a, lane, idx, canon, real);
  canon = canon && real > 0;
}
// The same; for M > 64 (several values per lane) nreal = how many of the lane's values
// idx, idx + 1, ... are real -- only those may be published (the rest are pad slots whose indices
// belong to real values of other lanes).
template <int M, int L, int N>
__device__ __forceinline__ void ppls_rs(double (&a)[N], int lane, int& idx, bool& canon, int& nreal) {
  int real = M;
  ppls_rs_r<M, L, N>(a, lane, idx, canon, real);
  canon = canon && real > 0;
  nreal = real;
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

// HBM -> LDS copy of 16 B per lane (global_load_lds_dwordx4): LDS destination = m0 + 16 * lane;
// source = a wave-uniform 64-bit base in SGPRs + a per-lane 32-bit byte offset (saddr form: no
// per-row 64-bit VALU address arithmetic; measured 1-3 % faster sweeps, profiles/r2_split_saddr_unguarded_ab.txt).
// Issued through inline asm on purpose: the compiler then does not track the DMA, so it does not
// put vmcnt(0) in front of every ds_read of the ring (it cannot prove the slots do not alias);
// the ring's completion is waited for explicitly with ppls_wait_vmcnt.  Invisible VMEM ops can
// only make the compiler's own vmcnt waits stricter, never unsafe.
__device__ __forceinline__ void ppls_dma16s_nt(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt"
               :: "s"(lds_addr), "v"(voff), "s"(sbase) : "memory", "m0");
}
__device__ __forceinline__ void ppls_dma16s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2"
               :: "s"(lds_addr), "v"(voff), "s"(sbase) : "memory", "m0");
}

__device__ __forceinline__ void ppls_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

