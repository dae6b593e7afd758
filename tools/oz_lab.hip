// oz_lab.hip -- feasibility lab for an int8-MFMA SYRK of residue planes (the Ozaki-II form of the
// Gram S = D'D): times the residue SYRK alone and checks sampled entries against
// exact int64 sums on the host.  Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/oz_lab tools/oz_lab.hip
//   tools/oz_lab <n> <P> <planes> [check]
//
// Plane layout: [n / 128][Pp][128] int8 -- stage kb's 128 rows of column c contiguous (128 B), so a
// 256-column panel of one stage is 32 KB contiguous.  One workgroup per lower 256 x 256 output tile,
// 4 waves of 128 x 128 (4 x 4 blocks of v_mfma_i32_32x32x32_i8, 256 int32 accumulators per lane),
// panels staged in LDS (double-buffered, XOR-swizzled 16-B chunks: conflict-free ds_read_b128 and
// ds_write_b128), one barrier per 128-row stage.  Output: the tile's sums mod m, uint8, column-major.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <random>
#include <vector>

#define CHK(x)                                                                              \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int TT = 256;   // output tile edge
constexpr int KS = 128;   // rows per stage
constexpr int PANEL = TT * KS;   // bytes of one panel stage (32 KB)

__host__ __device__ inline void tile_of(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

// LDS byte offset of 16-B chunk q (k rows 16 q .. 16 q + 15) of panel column c
__device__ __forceinline__ int lds_off(int c, int q) { return c * KS + ((q ^ ((c >> 1) & 7)) << 4); }

__device__ __forceinline__ int modp(int v, int m) {
  int r = v % m;
  return r < 0 ? r + m : r;
}

__global__ __launch_bounds__(256, 1) void oz_syrk(const int8_t* __restrict__ plane, int Pp, int64_t nkb, int m,
                                                  int ntiles, uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2][2][PANEL];   // [buffer][A | B]
  const int b = blockIdx.x, nb = gridDim.x;
  const int t = (b & 7) * (nb >> 3) + (b >> 3);   // XCD x takes a contiguous tile range
  if (t >= ntiles) return;
  int I, J;
  tile_of(t, &I, &J);
  const bool diag = I == J;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const bool idle = diag && wi == 0 && wj == 1;   // the diagonal tile's upper-right quadrant
  const int8_t* pa = plane + (int64_t)I * PANEL;
  const int8_t* pb = plane + (int64_t)J * PANEL;
  const int64_t sstride = (int64_t)Pp * KS;   // bytes per stage of the plane
  v16i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v16i{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  v4i ga[8], gb[8];
  auto gload = [&](int64_t s) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u;   // 16-B piece: column e / 8, chunk e % 8
      ga[u] = *(const v4i*)(pa + s * sstride + (int64_t)e * 16);
      if (!diag) gb[u] = *(const v4i*)(pb + s * sstride + (int64_t)e * 16);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = tid + 256 * u;
      const int c = e >> 3, q = e & 7;
      *(v4i*)(&lds[buf][0][lds_off(c, q)]) = ga[u];
      if (!diag) *(v4i*)(&lds[buf][1][lds_off(c, q)]) = gb[u];
    }
  };
  const int ca0 = 128 * wi + (lane & 31), cb0 = 128 * wj + (lane & 31), h = lane >> 5;
  auto compute = [&](int buf) {
    const int8_t* la = lds[buf][0];
    const int8_t* lb = diag ? lds[buf][0] : lds[buf][1];
#pragma unroll
    for (int kb = 0; kb < KS / 32; ++kb) {
      v4i a[4], bb[4];
      const int q = 2 * kb + h;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = *(const v4i*)(la + lds_off(ca0 + 32 * i, q));
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = *(const v4i*)(lb + lds_off(cb0 + 32 * j, q));
      if (!idle) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[i], bb[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  auto reduce = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = modp(acc[i][j][r], m);
  };
  gload(0);
  lstore(0);
  __syncthreads();
  for (int64_t s = 0; s < nkb; ++s) {
    if (s + 1 < nkb) gload(s + 1);
    compute((int)(s & 1));
    if (((s + 1) & 511) == 0) reduce();   // every 65,536 rows: |sum| < 2^30 + m
    if (s + 1 < nkb) lstore((int)((s + 1) & 1));
    __syncthreads();
  }
  reduce();
  if (idle) return;
  uint8_t* o = out + (int64_t)t * TT * TT;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = 128 * wj + 32 * j + (lane & 31);
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // rows (r & 3) + 8 (r >> 2) + 4 (lane >> 5), r = 4 g .. 4 g + 3
        const int row = 128 * wi + 32 * i + 8 * g + 4 * h;
        const uint32_t v = (uint32_t)acc[i][j][4 * g] | ((uint32_t)acc[i][j][4 * g + 1] << 8) |
                           ((uint32_t)acc[i][j][4 * g + 2] << 16) | ((uint32_t)acc[i][j][4 * g + 3] << 24);
        *(uint32_t*)(o + (int64_t)col * TT + row) = v;
      }
    }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int P = argc > 2 ? atoi(argv[2]) : 4000;
  const int planes = argc > 3 ? atoi(argv[3]) : 4;
  const int check = argc > 4 ? atoi(argv[4]) : 1;
  const int Pp = (P + TT - 1) / TT * TT;
  const int64_t nkb = (n + KS - 1) / KS, np = nkb * KS;
  const int T = Pp / TT, ntiles = T * (T + 1) / 2;
  const int m = 251;
  const size_t pbytes = (size_t)np * Pp;
  printf("n %lld P %d (Pp %d) tiles %d planes %d: %.2f GB per plane\n", (long long)n, P, Pp, ntiles, planes,
         pbytes / 1e9);
  std::vector<int8_t> h(pbytes);
  std::mt19937_64 rng(7);
  for (size_t i = 0; i < pbytes; i += 8) {
    uint64_t v = rng();
    for (int k = 0; k < 8 && i + k < pbytes; ++k) h[i + k] = (int8_t)((int)((v >> (8 * k)) & 255) % 255 - 127);
  }
  // zero padding rows / columns as the product will
  for (int64_t kb = 0; kb < nkb; ++kb)
    for (int c = 0; c < Pp; ++c)
      for (int k = 0; k < KS; ++k)
        if (c >= P || kb * KS + k >= n) h[((size_t)kb * Pp + c) * KS + k] = 0;
  std::vector<int8_t*> dp(planes);
  for (int i = 0; i < planes; ++i) {
    CHK(hipMalloc(&dp[i], pbytes));
    CHK(hipMemcpy(dp[i], h.data(), pbytes, hipMemcpyHostToDevice));
  }
  uint8_t* dout;
  const size_t obytes = (size_t)ntiles * TT * TT;
  CHK(hipMalloc(&dout, obytes * planes));
  const int grid = (ntiles + 7) / 8 * 8;
  for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(oz_syrk, dim3(grid), dim3(256), 0, 0, dp[0], Pp, nkb, m, ntiles, dout);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  CHK(hipEventRecord(e0));
  for (int i = 0; i < planes; ++i)
    hipLaunchKernelGGL(oz_syrk, dim3(grid), dim3(256), 0, 0, dp[i], Pp, nkb, m, ntiles, dout + obytes * i);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  const double useful = (double)n * P * (P + 1.0) * planes;   // lower triangle incl. diagonal, 2 ops per MAC
  const double exec = (double)np * TT * TT * 2.0 * ntiles * planes;
  printf("%d planes: %.3f ms (%.3f ms per plane); useful %.1f TOPS, executed %.1f TOPS (%.3f of 5000)\n", planes, ms,
         ms / planes, useful / (ms * 1e-3) / 1e12, exec / (ms * 1e-3) / 1e12, exec / (ms * 1e-3) / 5e15);
  if (check) {
    std::vector<uint8_t> ho(obytes);
    CHK(hipMemcpy(ho.data(), dout, obytes, hipMemcpyDeviceToHost));
    std::mt19937 r2(3);
    int bad = 0, tested = 0;
    for (int s = 0; s < 400; ++s) {
      const int t = s < 3 ? (s == 0 ? 0 : s == 1 ? ntiles - 1 : ntiles / 2) : (int)(r2() % ntiles);
      int I, J;
      tile_of(t, &I, &J);
      const int i = r2() % TT, j = r2() % TT;
      if (I == J && j > i) continue;
      const int ci = I * TT + i, cj = J * TT + j;
      int64_t sum = 0;
      for (int64_t kb = 0; kb < nkb; ++kb) {
        const int8_t* a = &h[((size_t)kb * Pp + ci) * KS];
        const int8_t* bq = &h[((size_t)kb * Pp + cj) * KS];
        for (int k = 0; k < KS; ++k) sum += (int64_t)a[k] * bq[k];
      }
      const int want = (int)(((sum % m) + m) % m);
      const int got = ho[(size_t)t * TT * TT + (size_t)j * TT + i];
      ++tested;
      if (want != got && bad++ < 10) printf("  tile %d (%d,%d) entry (%d,%d): got %d want %d\n", t, I, J, i, j, got, want);
    }
    printf("check: %d of %d sampled entries wrong\n", bad, tested);
    if (bad) return 2;
  }
  return 0;
}
