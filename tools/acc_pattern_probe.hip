// Read pattern of the panel accumulation pass (C5: 5e5 rows x 40 KB fp32) without arithmetic:
// workgroup (tile, chunk) reads a 4 KB column segment of its rows, 8 rows in flight per lane.
//   mode 0: chunk = a contiguous row range (the kernel's layout)
//   mode 1: chunk = rows chunk, chunk + nchunks, ... (concurrent workgroups read a contiguous band)
// hipcc --offload-arch=gfx950 -O3 -o tools/acc_pattern_probe tools/acc_pattern_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void probe(const char* __restrict__ X, long n, long ldb, long rpc, int nch,
                                             double* out) {
  extern __shared__ char pad_lds[];   // dynamic LDS only to cap the workgroups per CU
  if (out == nullptr) pad_lds[threadIdx.x] = 0;
  const int tile = blockIdx.x, chunk = blockIdx.y;
  const char* base = X + (long)tile * 4096 + threadIdx.x * 16;
  double s = 0.0;
  long r0, r1, step;
  if (MODE != 1) { r0 = (long)chunk * rpc; r1 = r0 + rpc < n ? r0 + rpc : n; step = 1; }
  else { r0 = chunk; r1 = n; step = nch; }
  for (long r = r0; r < r1; r += 8 * step) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      long rr = r + u * step;
      if (rr >= r1) rr = r0;
      v[u] = __builtin_nontemporal_load((const f4*)(base + rr * ldb));
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u].x + (double)v[u].w;
    if (MODE == 2 && ((r - r0) & 127) == 120) __syncthreads();   // a barrier per 128 rows (mu batches)
  }
  if (s == 12345.678) out[0] = s;
}

int main(int argc, char** argv) {
  const long n = 500000, ldb = argc > 1 ? atol(argv[1]) : 40960, bytes = n * ldb;   // row bytes (C5: 40000)
  char* X; double* out;
  if (hipMalloc(&X, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  (void)hipMalloc(&out, 64);
  (void)hipMemset(X, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  printf("row stride %ld B\n", ldb);
  for (int lds : {0, 72 * 1024}) {   // 8+, 2 workgroups per CU
  for (int nch : {372}) {
    const long rpc = (n + nch - 1) / nch;
    for (int mode = 0; mode < 3; mode += 2) {
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        (void)hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(10, nch), dim3(256), lds, 0, X, n, ldb, rpc, nch, out);
        else hipLaunchKernelGGL(probe<2>, dim3(10, nch), dim3(256), lds, 0, X, n, ldb, rpc, nch, out);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
      }
      printf("lds %6d B/WG chunks %4d mode %d (%s): %.3f ms  %.0f GB/s\n", lds, nch, mode,
             mode ? "row ranges, barrier per 128 rows" : "row ranges", best, bytes / 1e6 / best);
    }
  }
  }
  return 0;
}
