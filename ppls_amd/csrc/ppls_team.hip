// ppls_team.hip -- single-pass sweep for wide data (C5: p = 1e4, r = 10), where one workgroup
// cannot hold X'mu for all columns (the split sweep keeps W and the accumulators of ALL columns in
// one workgroup's registers; at p r = 1e5 that is 800 KB).
//
// A TEAM of S workgroups (one per CU, on one XCD) shares a block of rows; each of its data waves
// owns 64 16-B column vectors of [X | Y] (lane = one vector: W and the X'mu accumulators of those
// columns live in its registers for the whole sweep), so the team holds every column once.
// Per group of RP rows:
//   data waves  LDS-DMA their own 16 B of each row into a ring (PF groups ahead), partial dots
//               x . W of their columns, wave reduce-scatter, per-wave sums to LDS;
//   comm wave   (wave 0: issues no DMA, so its vmcnt waits never drain the ring) sums the waves,
//               publishes the workgroup's partial [Xw | Yc] of the group to the team exchange
//               buffer, gathers the team's partials of the group L steps back (prefetched one step
//               ahead), forms mu_T, mu_U of those rows (EM_W_multi.R:691-694), the Gram of
//               [Xw Yc] (member 0) and the optional mu write-out;
//   data waves  rank-RP update X'mu_T / Y'mu_U of their columns with the rows of group L+1 steps
//               back (still in the LDS ring) while the comm wave works on the next mu.
// X and Y are read from HBM once per EM iteration (the panel sweep reads them twice).
//
// Exchange protocol (no fences, no flags): every published double travels with a 64-bit check
// word = tag ^ mix(bits(value)), tag = (epoch << 32) | (group + 1), stored together in one 16-B
// store; a reader accepts a value only when its check word matches the tag it expects -- a stale
// or torn entry fails the check and is polled again.  Stores and loads are L2-scope (sc0): the
// members of a team share one XCD's L2 (blockIdx mod 8 = XCD, checked against HW_REG_XCC_ID).
// Slots are reused every DEPTH = 2L + 2 groups, which the lag structure makes safe (a member cannot publish group h + DEPTH before every member consumed group h).  Every wait
// is bounded: a timeout sets *status and the whole team leaves the loop (no hang).  The kernel is
// launched cooperatively (all workgroups co-resident, or the launch fails and the host falls back
// to the panel sweep).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ppls_device.h"
#include "ppls_kernels.h"

#define PPLS_TEAM_RP 2     // rows per group
#define PPLS_TEAM_PF 4     // groups of DMA in flight ahead of the dots
#define PPLS_TEAM_L 2      // exchange lag (steps) between publishing and gathering
#define PPLS_TEAM_RING (PPLS_TEAM_PF + PPLS_TEAM_L + 3)
#define PPLS_TEAM_DEPTH (2 * PPLS_TEAM_L + 2)
#define PPLS_TEAM_MAXWAVES 8   // 1 comm + up to 7 data waves
#define PPLS_TEAM_SMAX 16      // workgroups per team

namespace {

__device__ __forceinline__ uint64_t ppls_mix(uint64_t x) { return x * 0x9E3779B97F4A7C15ull; }

// One exchange entry: 16 B {value, tag ^ mix(bits(value))} in one store.  L2 scope (sc0: past the
// CU's L1, into its XCD's L2) -- team members share an XCD, which the kernel verifies.
__device__ __forceinline__ void ppls_xstore(uint64_t* p, double v, uint64_t tag) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const uint64_t b = (uint64_t)__double_as_longlong(v), c = tag ^ ppls_mix(b);
  u4 w;
  w.x = (unsigned)b;
  w.y = (unsigned)(b >> 32);
  w.z = (unsigned)c;
  w.w = (unsigned)(c >> 32);
  asm volatile("global_store_dwordx4 %0, %1, off" :: "v"(p), "v"(w) : "memory");
}

template <typename T>
struct TeamVec;
template <>
struct TeamVec<float> {
  static constexpr int EV = 4;
  __device__ static __forceinline__ void get(const char* p, double (&x)[4]) {
    const float4 v = *(const float4*)p;
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
};
template <>
struct TeamVec<double> {
  static constexpr int EV = 2;
  __device__ static __forceinline__ void get(const char* p, double (&x)[2]) {
    const double2 v = *(const double2*)p;
    x[0] = v.x; x[1] = v.y;
  }
};

}  // namespace

// grid: gridDim.x workgroups (a multiple of 8: blockIdx mod 8 is the XCD under round-robin
// dispatch; correctness does not depend on it), 1 + wpw waves each.  part: nteams rows of
// part_ld = R ldx + R ldy + 4 R^2 doubles, written completely.
template <typename T, int R>
__global__ __launch_bounds__(64 * PPLS_TEAM_MAXWAVES, 1) void ppls_sweep_team_kernel(
    const T* __restrict__ X, const T* __restrict__ Y, int64_t n, int ldx, int ldy,
    const double* __restrict__ Wp, const double* __restrict__ Cp, const PplsScalars* __restrict__ sc,
    double* __restrict__ part, int64_t part_ld, double* __restrict__ mu, int write_mu,
    uint64_t* __restrict__ xch, int S, int wpw, int nwx, int nwy, uint32_t epoch, int nt_loads,
    int* __restrict__ status, int ablate) {
  // ablate (timing experiments only; results are garbage while set): 32 = no team exchange,
  // 64 = data waves skip the dots / update arithmetic, 128 = data waves skip the HBM -> LDS copies
  const bool no_xch = ablate & 32, no_math = ablate & 64, no_dma = ablate & 128;
  constexpr int EV = TeamVec<T>::EV;
  constexpr int RP = PPLS_TEAM_RP, PF = PPLS_TEAM_PF, L = PPLS_TEAM_L;
  constexpr int RING = PPLS_TEAM_RING, DEPTH = PPLS_TEAM_DEPTH;
  constexpr int V = R * RP;                 // partial dots per group per wave (one matrix)
  constexpr int VP = V + (V & 1);
  constexpr int E2 = 2 * V;                 // exchanged values per member per group: [Xw | Yc]
  constexpr int NPAIR = R * (2 * R + 1);    // Gram pairs (2R x 2R, upper triangle)
  constexpr int GPL = (NPAIR + 63) / 64;    // Gram pairs per comm lane
  static_assert(V <= 64, "one comm lane per exchanged value");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int per_xcd = gridDim.x >> 3;
  const int teams_per_xcd = per_xcd / S;
  const int xcd = blockIdx.x & 7, slot_in_xcd = blockIdx.x >> 3;
  const int tix = slot_in_xcd / S, m = slot_in_xcd - tix * S;
  if (tix >= teams_per_xcd) return;                  // spare workgroups of this XCD
  const int nteams = 8 * teams_per_xcd;
  const int team = xcd * teams_per_xcd + tix;
  const int64_t rb = n * team / nteams, re = n * (team + 1) / nteams;
  const int nrows = (int)(re - rb);
  const int ngroups = (nrows + RP - 1) / RP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row_bytes = wpw * 1024;                  // one row's share of this workgroup in the ring
  char* ring = smem;
  double* red = (double*)(smem + (size_t)RING * RP * row_bytes);   // [2][MAXWAVES][V]
  double* mush = red + 2 * PPLS_TEAM_MAXWAVES * V;                 // [2][RP][2R]: mu_T | mu_U
  double* zsh = mush + 2 * RP * 2 * R;                             // [2][RP][2R]: Xw | Yc (Gram)
  uint64_t* pf = (uint64_t*)(zsh + 2 * RP * 2 * R);               // [S x 2V entries][2 words]
  int* abort_sh = (int*)(pf + (size_t)((S * E2 + 63) / 64) * 64 * 2);
  const uint32_t pf_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)pf;
  uint64_t* xt = xch + (size_t)team * DEPTH * S * E2 * 2;          // this team's slots
  // the exchange uses L2-scope memory operations, so every member of a team must sit on the XCD
  // the blockIdx -> XCD round-robin assigns; verified here (a mismatch aborts the sweep: status -8)
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  const bool xcd_mismatch = (int)(xcc & 0xf) != xcd;
  if (tid == 0) {
    *abort_sh = xcd_mismatch ? 1 : 0;
    if (xcd_mismatch) {
      int expected = 0;
      __hip_atomic_compare_exchange_strong(status, &expected, -8, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();

  if (wave == 0) {
    // ============================================================ comm wave
    const int comp = lane < V ? lane % R : 0;
    const double al = sc->alpha[comp], be = sc->beta[comp], ga = sc->gamma[comp], de = sc->delta[comp];
    int gi[GPL], gj[GPL];
    double gacc[GPL];
#pragma unroll
    for (int u = 0; u < GPL; ++u) {
      int e = lane + 64 * u, j = 0;
      gacc[u] = 0.0;
      gi[u] = -1;
      gj[u] = 0;
      if (e < NPAIR) {
        while (e >= j + 1) { e -= j + 1; ++j; }
        gi[u] = e;
        gj[u] = j;
      }
    }
    // the team's published partials of one group, (value, check) words of all members, land in
    // LDS by DMA (a contiguous copy of the group's slot: S x 2V entries of 16 B) with L2-scope
    // loads (sc0), so the members' stores in the shared L2 are seen
    const int nent = S * E2;
    auto prefetch = [&](int h) {
      const uint64_t* s0 = xt + (size_t)(h % DEPTH) * S * E2 * 2;
      for (int i = 0; i * 64 < nent; ++i) {
        const int f = i * 64 + lane;
        ppls_dma16_l2(s0 + (size_t)(f < nent ? f : nent - 1) * 2, pf_base + (uint32_t)(i * 1024));
      }
    };
    // lane idx < V: a = sum over members of Xw[idx], b = of Yc[idx], in member order; checks ok?
    auto gather = [&](uint64_t tag, double& a, double& b) {
      bool ok = true;
      a = 0.0;
      b = 0.0;
      if (lane < V) {
        for (int mm = 0; mm < S; ++mm) {
          const uint64_t* ea = pf + ((size_t)mm * E2 + lane) * 2;
          const uint64_t* eb = pf + ((size_t)mm * E2 + V + lane) * 2;
          const uint64_t va = ea[0], wa = ea[1], vb = eb[0], wb = eb[1];
          ok = ok && ((wa ^ ppls_mix(va)) == tag) && ((wb ^ ppls_mix(vb)) == tag);
          a += __longlong_as_double((long long)va);
          b += __longlong_as_double((long long)vb);
        }
      }
      return ok;
    };
    bool aborted = xcd_mismatch;
    int nst = 0;                                    // exchange stores issued after the last prefetch
    // Step g (between the barriers closing steps g-1 and g): publish group gp = g - 1 (its red is
    // complete), gather group hm = g - 1 - L and form its mu for the data waves' update in step g + 1.
    for (int g = 0; g <= ngroups + L + 1; ++g) {
      const int gp = g - 1, hm = g - 1 - L;
      // 1. gather group hm (prefetched during the previous step; re-polled if not yet published).
      //    VMEM completes in issue order: waiting until only the later stores are outstanding
      //    means the prefetch has landed, without waiting for those stores.
      double a = 0.0, b = 0.0;
      if (hm >= 0 && hm < ngroups && !aborted && !no_xch) {
        const uint64_t tag = ((uint64_t)epoch << 32) | (uint32_t)(hm + 1);
        if (hm == 0) {
          prefetch(0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          ppls_wait_vmcnt(nst);
        }
        bool ok = gather(tag, a, b);
        int spins = 0;
        bool timed_out = false;
        while (!__all(ok)) {                        // some member's partials are not there yet
          if (++spins > (1 << 22)) {
            timed_out = true;
            aborted = true;
            break;
          }
          if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
            aborted = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // LDS reads done before the re-copy
          prefetch(hm);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          ok = gather(tag, a, b);
        }
        if (timed_out && !ok && lane < 4) {   // diagnostics: which member's entry never showed up
          for (int mm = 0; mm < S; ++mm)
            for (int ab = 0; ab < 2; ++ab) {
              const uint64_t* e = pf + ((size_t)mm * E2 + ab * V + lane) * 2;
              const uint64_t seen = e[1] ^ ppls_mix(e[0]);
              if (seen != tag)
                printf("ppls team sweep timeout: team %d member %d group %d of %d: lane %d member %d %s "
                       "tag seen %016llx expected %016llx\n", team, m, hm, ngroups, lane, mm, ab ? "Yc" : "Xw",
                       (unsigned long long)seen, (unsigned long long)tag);
            }
        }
        if (aborted && lane == 0) {
          int expected = 0;
          __hip_atomic_compare_exchange_strong(status, &expected, -7, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
          *abort_sh = 1;
        }
      }
      // 2. mu of group hm -> LDS (parity hm & 1), Gram, write-out
      if (hm >= 0 && hm < ngroups && !aborted) {
        const int j = lane < V ? lane / R : 0;
        const bool valid = lane < V && (hm * RP + j) < nrows;
        const double xa = valid ? a : 0.0, yb = valid ? b : 0.0;
        double* mh = mush + (hm & 1) * RP * 2 * R;
        double* zh = zsh + (hm & 1) * RP * 2 * R;
        if (lane < V) {
          mh[j * 2 * R + comp] = al * xa + be * yb;         // mu_T (EM_W_multi.R:691-692)
          mh[j * 2 * R + R + comp] = ga * xa + de * yb;     // mu_U (EM_W_multi.R:693-694)
          zh[j * 2 * R + comp] = xa;
          zh[j * 2 * R + R + comp] = yb;
          if (write_mu && m == 0 && valid) {
            const int64_t row = rb + (int64_t)hm * RP + j;
            mu[(int64_t)comp * n + row] = al * xa + be * yb;
            mu[(int64_t)(R + comp) * n + row] = ga * xa + de * yb;
          }
        }
        if (m == 0) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int u = 0; u < GPL; ++u)
            if (gi[u] >= 0)
#pragma unroll
              for (int jj = 0; jj < RP; ++jj)
                gacc[u] = fma(zh[jj * 2 * R + gi[u]], zh[jj * 2 * R + gj[u]], gacc[u]);
        }
      }
      // 3. prefetch the partials of group hm + 1 (after this step's LDS reads of the buffer)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (!aborted && !no_xch && hm + 1 >= 1 && hm + 1 < ngroups) prefetch(hm + 1);
      // 4. publish this workgroup's partials of group gp (two stores, after the prefetch)
      nst = 0;
      if (gp >= 0 && gp < ngroups && !aborted && !no_xch) {
        if (lane < V) {
          const double* rg = red + (gp & 1) * PPLS_TEAM_MAXWAVES * V;
          double sa = 0.0, sb = 0.0;
          for (int w = 0; w < wpw; ++w) {
            const double v = rg[w * V + lane];
            if (m * wpw + w < nwx) sa += v;
            else sb += v;
          }
          const uint64_t tag = ((uint64_t)epoch << 32) | (uint32_t)(gp + 1);
          uint64_t* s0 = xt + ((size_t)(gp % DEPTH) * S * E2 + (size_t)m * E2) * 2;
          ppls_xstore(s0 + (size_t)lane * 2, sa, tag);
          ppls_xstore(s0 + (size_t)(V + lane) * 2, sb, tag);
        }
        nst = 2;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                 // end of step g: mu of hm, red of g visible
      asm volatile("" ::: "memory");
      if (*abort_sh) break;
    }
    if (m == 0 && !aborted) {
      double* G2 = part + (int64_t)team * part_ld + (int64_t)R * ldx + (int64_t)R * ldy;
#pragma unroll
      for (int u = 0; u < GPL; ++u)
        if (gi[u] >= 0) {
          G2[gj[u] * 2 * R + gi[u]] = gacc[u];
          G2[gi[u] * 2 * R + gj[u]] = gacc[u];
        }
    }
    return;
  }

  // ============================================================ data waves
  const int dw = wave - 1;                            // 0 .. wpw-1
  const int gw = m * wpw + dw;                        // team-global data wave
  const bool isx = gw < nwx;                          // wave-uniform
  const bool owns = gw < nwx + nwy;
  const int vi = (isx ? gw : gw - nwx) * 64 + lane;   // 16-B column vector of this lane
  const int ld = isx ? ldx : ldy;
  const int nv = ld / EV;
  const bool act = owns && vi < nv;
  const T* M = isx ? X : Y;
  const double* Wm = isx ? Wp : Cp;
  double w[EV][R], acc[EV][R];
#pragma unroll
  for (int e = 0; e < EV; ++e)
#pragma unroll
    for (int k = 0; k < R; ++k) {
      w[e][k] = act ? Wm[(int64_t)k * ld + (int64_t)vi * EV + e] : 0.0;
      acc[e][k] = 0.0;
    }
  const int vcl = act ? vi : 0;                        // clamped vector for the DMA address
  const uint32_t lds_base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  auto issue = [&](int grp) {
    if (grp >= ngroups || no_dma) return;
#pragma unroll
    for (int j = 0; j < RP; ++j) {
      int r = grp * RP + j;
      if (r >= nrows) r = nrows - 1;
      const T* src = M + (rb + r) * (int64_t)ld + (int64_t)vcl * EV;
      const uint32_t dst = lds_base + (uint32_t)(((grp % RING) * RP + j) * row_bytes + dw * 1024);
      if (nt_loads) ppls_dma16_nt(src, dst);
      else ppls_dma16(src, dst);
    }
  };
  auto xrow = [&](int grp, int j, double (&x)[EV]) {
    TeamVec<T>::get(ring + ((grp % RING) * RP + j) * row_bytes + dw * 1024 + lane * 16, x);
    if (grp * RP + j >= nrows || !act)
#pragma unroll
      for (int e = 0; e < EV; ++e) x[e] = 0.0;
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // W loads done: only DMA is outstanding below
  for (int grp = 0; grp < PF; ++grp) issue(grp);
  // Step g: dots of group g (-> red parity g & 1), update with group g - L - 2 (mu from step g - 1);
  // one workgroup barrier per step.
  for (int g = 0; g <= ngroups + L + 1; ++g) {
    if (g < ngroups) {
      issue(g + PF);
      // own DMA of group g landed: at most (groups issued after g) * RP outstanding
      const int after = no_dma ? 0 : (g + PF < ngroups ? g + PF : ngroups - 1) - g;
      ppls_wait_vmcnt(after * RP);
    }
    if (g < ngroups && !no_math) {
      double v[VP];
#pragma unroll
      for (int j = 0; j < RP; ++j) {
        double x[EV];
        xrow(g, j, x);
#pragma unroll
        for (int k = 0; k < R; ++k) {
          double s = 0.0;
#pragma unroll
          for (int e = 0; e < EV; ++e) s = fma(x[e], w[e][k], s);
          v[j * R + k] = s;
        }
      }
      if constexpr (VP > V) v[V] = 0.0;
      int idx = 0;
      bool canon = true;
      ppls_rs<V, 0, VP>(v, lane, idx, canon);
      if (canon && idx < V) red[(g & 1) * PPLS_TEAM_MAXWAVES * V + dw * V + idx] = v[0];
    }
    const int hu = g - L - 2;                         // update group (mu from step g - 1)
    if (hu >= 0 && hu < ngroups && !no_math) {
      const double* mh = mush + (hu & 1) * RP * 2 * R + (isx ? 0 : R);
#pragma unroll
      for (int j = 0; j < RP; ++j) {
        double x[EV];
        xrow(hu, j, x);
#pragma unroll
        for (int k = 0; k < R; ++k) {
          const double mk = mh[j * 2 * R + k];
#pragma unroll
          for (int e = 0; e < EV; ++e) acc[e][k] = fma(x[e], mk, acc[e][k]);
        }
      }
    }
    ppls_lds_barrier();                               // end of step g
    if (*abort_sh) break;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (act && !*abort_sh) {
    double* dst = part + (int64_t)team * part_ld + (isx ? 0 : (int64_t)R * ldx);
#pragma unroll
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int e = 0; e < EV; ++e) dst[(int64_t)k * ld + (int64_t)vi * EV + e] = acc[e][k];
  }
}

namespace {

template <typename T, int R>
hipError_t launch_team_t(const PplsTeamPlan& tp, const PplsSweepArgs& a, uint64_t* xch, uint32_t epoch,
                         int nt_loads, int* status, hipStream_t st) {
  auto kern = ppls_sweep_team_kernel<T, R>;
  const size_t lds = ppls_team_lds_bytes(R, tp.wpw, tp.S);
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const T* Xa = (const T*)a.X;
  const T* Ya = (const T*)a.Y;
  int64_t n = a.n_local;
  int ldx = a.ldx, ldy = a.ldy;
  const double* Wp = a.Wp;
  const double* Cp = a.Cp;
  const PplsScalars* sc = a.sc;
  double* part = a.part;
  int64_t part_ld = a.part_ld;
  double* mu = a.mu;
  int write_mu = a.write_mu;
  int S = tp.S, wpw = tp.wpw, nwx = tp.nwx, nwy = tp.nwy;
  int ablate = a.ablate & (32 | 64 | 128);
  void* args[] = {&Xa, &Ya, &n, &ldx, &ldy, &Wp, &Cp, &sc, &part, &part_ld, &mu, &write_mu,
                  &xch, &S, &wpw, &nwx, &nwy, &epoch, &nt_loads, &status, &ablate};
  return hipLaunchCooperativeKernel((const void*)kern, dim3(tp.grid), dim3(64 * (1 + tp.wpw)), args,
                                    (unsigned)lds, st);
}

template <typename T>
hipError_t launch_team_dt(const PplsTeamPlan& tp, const PplsSweepArgs& a, uint64_t* xch, uint32_t epoch,
                          int nt_loads, int* status, hipStream_t st) {
  switch (a.r) {
#define PPLS_TEAM_CASE(k) \
  case k: return launch_team_t<T, k>(tp, a, xch, epoch, nt_loads, status, st);
    PPLS_TEAM_CASE(1) PPLS_TEAM_CASE(2) PPLS_TEAM_CASE(3) PPLS_TEAM_CASE(4) PPLS_TEAM_CASE(5)
    PPLS_TEAM_CASE(6) PPLS_TEAM_CASE(7) PPLS_TEAM_CASE(8) PPLS_TEAM_CASE(9) PPLS_TEAM_CASE(10)
#undef PPLS_TEAM_CASE
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

extern "C" {

size_t ppls_team_lds_bytes(int r, int wpw, int S) {
  const size_t nent = (size_t)S * 2 * r * PPLS_TEAM_RP;
  return (size_t)PPLS_TEAM_RING * PPLS_TEAM_RP * wpw * 1024 +
         sizeof(double) * ((size_t)2 * PPLS_TEAM_MAXWAVES * r * PPLS_TEAM_RP + 2 * PPLS_TEAM_RP * 2 * r +
                           2 * PPLS_TEAM_RP * 2 * r) +
         (nent + 63) / 64 * 1024 + 16;
}

// Team shape for this problem: S workgroups of wpw data waves (+ 1 comm wave) per team, teams
// inside one XCD (num_cus / 8 CUs, one workgroup each).  Picks the (S, wpw) that keeps the most
// lanes busy: lane utilisation (column vectors / team lanes) x CU utilisation (team CUs / CUs).
int ppls_team_plan(int r, int ldx, int ldy, int f32, int num_cus, int64_t n, PplsTeamPlan* tp) {
  if (r < 1 || r > 10 || num_cus < 8 || (num_cus & 7)) return 0;
  const int ev = f32 ? 4 : 2;
  const int nwx = (ldx / ev + 63) / 64, nwy = (ldy / ev + 63) / 64;
  const int totw = nwx + nwy;
  const int per_xcd = num_cus / 8;
  double best = 0.0;
  int bs = 0, bw = 0;
  for (int S = 1; S <= per_xcd && S <= PPLS_TEAM_SMAX; ++S) {
    const int wpw = (totw + S - 1) / S;
    if (wpw < 1 || wpw > PPLS_TEAM_MAXWAVES - 1) continue;
    if (ppls_team_lds_bytes(r, wpw, S) > 160 * 1024) continue;
    const int tpx = per_xcd / S;
    const double eff = (double)totw / (double)(S * wpw) * (double)(tpx * S) / (double)per_xcd;
    if (eff > best + 1e-9) { best = eff; bs = S; bw = wpw; }
  }
  if (bs == 0) return 0;
  const int nteams = 8 * (per_xcd / bs);
  if (n < (int64_t)nteams * PPLS_TEAM_RP * 8) return 0;   // too few rows to be worth a team
  tp->S = bs;
  tp->wpw = bw;
  tp->nwx = nwx;
  tp->nwy = nwy;
  tp->grid = num_cus;
  tp->nteams = nteams;
  tp->eff = best;
  tp->xch_words = (int64_t)nteams * PPLS_TEAM_DEPTH * bs * 2 * (2 * r * PPLS_TEAM_RP);
  return 1;
}

hipError_t ppls_launch_sweep_team(const PplsTeamPlan* tp, const PplsSweepArgs* a, int f32, uint64_t* xch,
                                  uint32_t epoch, int nt_loads, int* status, hipStream_t st) {
  if (a->n_local <= 0) return hipSuccess;
  if (f32) return launch_team_dt<float>(*tp, *a, xch, epoch, nt_loads, status, st);
  return launch_team_dt<double>(*tp, *a, xch, epoch, nt_loads, status, st);
}

}  // extern "C"
