// Read pattern of the panel dots pass without arithmetic or LDS: one wave per row tile of RB rows
// walks the columns in tiles of CW bytes per row (the product: RB = 64, CW = 128: 8 rows x 128 B per
// 16-B load instruction), the next tile's loads in flight while the current one is summed.  C5's X:
// 5e5 rows x 40,960 B.  Asks: is the 128-B-per-row tile shape itself slower to stream than longer
// row segments?
//   hipcc --offload-arch=gfx950 -O3 -o tools/dots_pattern_probe tools/dots_pattern_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int RB, int CW, bool NT, int KS>
__global__ __launch_bounds__(256) void probe(const char* __restrict__ X, long n, long ldb, double* out) {
  constexpr int LPR = CW / 16;          // lanes per row in one load instruction
  constexpr int RPI = 64 / LPR;         // rows per load instruction
  constexpr int NL = RB / RPI;          // load instructions per tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long t = ((long)blockIdx.x * 4 + wave) / KS;   // KS waves share a row tile's columns
  const int part = wave % KS;
  const long ntiles = (n + RB - 1) / RB;
  if (t >= ntiles) return;
  const long row0 = t * RB;
  const int ntcall = (int)(ldb / CW);
  const int tb = ntcall * part / KS, ntc = ntcall * (part + 1) / KS - tb;
  const char* src[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {
    long rr = row0 + lane / LPR + RPI * u;
    if (rr >= n) rr = n - 1;
    src[u] = X + rr * ldb + (lane % LPR) * 16 + (long)tb * CW;
  }
  auto ld = [](const char* p) -> f4 { return NT ? __builtin_nontemporal_load((const f4*)p) : *(const f4*)p; };
  f4 a[NL], b[NL];
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < NL; ++u) a[u] = ld(src[u]);
  for (int tc = 0; tc < ntc; tc += 2) {
    const int c1 = tc + 1 < ntc ? tc + 1 : tc;
#pragma unroll
    for (int u = 0; u < NL; ++u) b[u] = ld(src[u] + (long)c1 * CW);
#pragma unroll
    for (int u = 0; u < NL; ++u) s += (double)a[u].x + (double)a[u].w;
    const int c2 = tc + 2 < ntc ? tc + 2 : c1;
#pragma unroll
    for (int u = 0; u < NL; ++u) a[u] = ld(src[u] + (long)c2 * CW);
#pragma unroll
    for (int u = 0; u < NL; ++u) s += (double)b[u].x + (double)b[u].w;
  }
  if (s == 12345.678) out[0] = s;
}

template <int RB, int CW, bool NT = false, int KS = 1>
void run(const char* X, long n, long ldb, double* out, hipEvent_t e0, hipEvent_t e1) {
  const long ntiles = (n + RB - 1) / RB;
  const int grid = (int)((ntiles * KS + 3) / 4);
  float best = 1e30f;
  for (int rep = 0; rep < 6; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((probe<RB, CW, NT, KS>), dim3(grid), dim3(256), 0, 0, X, n, ldb, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  printf("rows/wave %3d, bytes/row/tile %5d, nt %d, waves/tile %d: %.3f ms  %.2f TB/s\n", RB, CW, (int)NT, KS, best, n * ldb / (best * 1e-3) / 1e12);
}

int main() {
  const long n = 500000, ldb = 40960;
  char* X;
  double* out;
  if (hipMalloc(&X, n * ldb) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
  hipMemset(X, 0, n * ldb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pass = 0; pass < 2; ++pass) {
    run<64, 128>(X, n, ldb, out, e0, e1);
    run<64, 128, true>(X, n, ldb, out, e0, e1);
    run<64, 128, false, 2>(X, n, ldb, out, e0, e1);
    run<64, 128, false, 4>(X, n, ldb, out, e0, e1);
    run<64, 128, true, 2>(X, n, ldb, out, e0, e1);
    run<8, 1024, true>(X, n, ldb, out, e0, e1);
    run<16, 128>(X, n, ldb, out, e0, e1);
  }
  return 0;
}
