// Does a second touch of the panel sweep's rows come for free when it follows the first touch by
// one or two Infinity-Cache-sized row chunks?  (a MALL-resident second pass.)
// Loads only, no arithmetic; the data is one GPU's C5 share by default (62,500 rows x 40,960 B).
//
//   stream   : one pass, every row read once (the HBM floor of a single-pass sweep)
//   two-pass : the same pass twice, back to back (today's dots + accumulation read traffic)
//   pipeline : ONE launch, two roles.  "first" workgroups read chunk c (S rows; HBM); "second"
//              workgroups read chunk c again in the accumulation pass's pattern (4 KB column
//              segment x a row sub-range per workgroup) once every first workgroup has finished
//              it; the first role may run at most L chunks ahead of the second (so the re-read
//              bytes should still be in the 256 MiB MALL).  Ordering by device-scope counters,
//              every wait bounded (an overrun sets err and the workgroup carries on), the grid is
//              far below the resident capacity (8 workgroups per CU at this register use).
//
// hipcc --offload-arch=gfx950 -O3 -o tools/mall_pipeline_probe tools/mall_pipeline_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void sink(double s, double* out) {
  if (s == 12345.678) out[0] = s;
}

// first-touch read of rows [r0, r1): the workgroup streams them as one contiguous byte range
__device__ double read_rows(const char* X, long ldb, long r0, long r1, bool nt) {
  const long b0 = r0 * ldb, b1 = r1 * ldb;
  double s = 0.0;
  for (long b = b0 + threadIdx.x * 16; b < b1; b += 256 * 16 * 8) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      long bb = b + (long)u * 256 * 16;
      if (bb >= b1) bb = b0 + threadIdx.x * 16;
      v[u] = nt ? __builtin_nontemporal_load((const f4*)(X + bb)) : *(const f4*)(X + bb);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u].x + (double)v[u].w;
  }
  return s;
}

// second-touch read (accumulation pattern): a 4 KB column segment (tile) of rows [r0, r1)
__device__ double read_tile(const char* X, long ldb, int tile, long r0, long r1) {
  const char* base = X + (long)tile * 4096 + threadIdx.x * 16;
  double s = 0.0;
  for (long r = r0; r < r1; r += 8) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      long rr = r + u;
      if (rr >= r1) rr = r0;
      v[u] = *(const f4*)(base + rr * ldb);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) s += (double)v[u].x + (double)v[u].w;
  }
  return s;
}

__global__ __launch_bounds__(256) void stream_kernel(const char* X, long n, long ldb, double* out, int nt) {
  const long per = (n + gridDim.x - 1) / gridDim.x;
  const long r0 = blockIdx.x * per, r1 = r0 + per < n ? r0 + per : n;
  sink(r0 < r1 ? read_rows(X, ldb, r0, r1, nt != 0) : 0.0, out);
}

__global__ __launch_bounds__(256) void tile_kernel(const char* X, long n, long ldb, double* out) {
  const long per = (n + gridDim.y - 1) / gridDim.y;
  const long r0 = blockIdx.y * per, r1 = r0 + per < n ? r0 + per : n;
  sink(r0 < r1 ? read_tile(X, ldb, blockIdx.x, r0, r1) : 0.0, out);
}

__device__ bool wait_ge(unsigned* ctr, unsigned target, int* err) {
  long spins = 0;
  while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (++spins > (1L << 22)) { atomicExch(err, 1); return false; }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// blocks [0, NA): first touch; [NA, NA + 10 * J): second touch (tile = b % 10, sub-range b / 10)
__global__ __launch_bounds__(256) void pipeline_kernel(const char* X, long n, long ldb, long S, int K, int NA,
                                                       int J, int L, unsigned* doneA, unsigned* doneB, int* err,
                                                       double* out) {
  __shared__ int s_ok;
  double s = 0.0;
  const int ntile = (int)(ldb / 4096);
  const int NB = ntile * J;
  if ((int)blockIdx.x < NA) {
    const int a = blockIdx.x;
    for (int c = 0; c < K; ++c) {
      if (c >= L) {   // throttle: the second role has finished chunk c - L
        if (threadIdx.x == 0) s_ok = wait_ge(&doneB[c - L], (unsigned)NB, err);
        __syncthreads();
      }
      const long c0 = (long)c * S, c1 = c0 + S < n ? c0 + S : n;
      const long per = (c1 - c0 + NA - 1) / NA;
      const long r0 = c0 + a * per, r1 = r0 + per < c1 ? r0 + per : c1;
      if (r0 < r1) s += read_rows(X, ldb, r0, r1, false);
      __syncthreads();
      if (threadIdx.x == 0) { __threadfence(); atomicAdd(&doneA[c], 1u); }
    }
  } else {
    const int b = blockIdx.x - NA, tile = b % ntile, j = b / ntile;
    for (int c = 0; c < K; ++c) {
      if (threadIdx.x == 0) s_ok = wait_ge(&doneA[c], (unsigned)NA, err);
      __syncthreads();
      const long c0 = (long)c * S, c1 = c0 + S < n ? c0 + S : n;
      const long per = (c1 - c0 + J - 1) / J;
      const long r0 = c0 + j * per, r1 = r0 + per < c1 ? r0 + per : c1;
      if (r0 < r1) s += read_tile(X, ldb, tile, r0, r1);
      __syncthreads();
      if (threadIdx.x == 0) atomicAdd(&doneB[c], 1u);
    }
  }
  sink(s, out);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 62500, ldb = 40960, bytes = n * ldb;
  char* X; double* out; unsigned* ctr; int* err;
  if (hipMalloc(&X, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  (void)hipMalloc(&out, 64);
  (void)hipMemset(X, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  // a 512 MiB buffer written between timed runs evicts the data from the Infinity Cache
  char* flush; (void)hipMalloc(&flush, 512L << 20);
  auto time_it = [&](auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      (void)hipMemsetAsync(flush, rep, 512L << 20);
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep > 0 && ms < best) best = ms;
    }
    return best;
  };
  printf("rows %ld x %ld B = %.3f GB (one GPU's C5 share by default)\n", n, ldb, bytes * 1e-9);
  for (int nt = 0; nt < 2; ++nt) {
    const float t1 = time_it([&] { hipLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, 0, X, n, ldb, out, nt); });
    const float t2 = time_it([&] {
      hipLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, 0, X, n, ldb, out, nt);
      hipLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, 0, X, n, ldb, out, nt);
    });
    printf("stream %s: one pass %.3f ms (%.0f GB/s); two passes %.3f ms\n", nt ? "nt" : "default", t1,
           bytes / (t1 * 1e-3) * 1e-9, t2);
  }
  // chunk-level A/B with separate launches: per chunk of S rows, read it (first touch) and read it
  // again right away (second touch), each launch timed by its own events
  {
    std::vector<hipEvent_t> ev(3);
    for (auto& e : ev) (void)hipEventCreate(&e);
    for (long S : {1536L, 3072L, 6144L}) {
      for (int pat = 0; pat < 2; ++pat) {
        const int K = (int)((n + S - 1) / S);
        (void)hipMemset(flush, 1, 512L << 20);
        (void)hipDeviceSynchronize();
        double t_first = 0, t_second = 0;
        hipEvent_t a0, a1;
        (void)hipEventCreate(&a0); (void)hipEventCreate(&a1);
        (void)hipEventRecord(a0);
        for (int c = 0; c < K; ++c) {
          const long r0 = (long)c * S, rows = r0 + S < n ? S : n - r0;
          const char* Xc = X + r0 * ldb;
          (void)hipEventRecord(ev[0]);
          hipLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, 0, Xc, rows, ldb, out, 0);
          (void)hipEventRecord(ev[1]);
          if (pat == 0)
            hipLaunchKernelGGL(stream_kernel, dim3(1024), dim3(256), 0, 0, Xc, rows, ldb, out, 0);
          else   // the accumulation pattern: 10 tiles x 96 row sub-ranges
            hipLaunchKernelGGL(tile_kernel, dim3(10, 96), dim3(256), 0, 0, Xc, rows, ldb, out);
          (void)hipEventRecord(ev[2]);
          (void)hipEventSynchronize(ev[2]);
          float m1, m2;
          (void)hipEventElapsedTime(&m1, ev[0], ev[1]);
          (void)hipEventElapsedTime(&m2, ev[1], ev[2]);
          if (c > 0) { t_first += m1; t_second += m2; }
        }
        (void)hipEventRecord(a1);
        (void)hipEventSynchronize(a1);
        const double b = (double)(K - 1) * S * ldb;
        printf("chunked launches S=%5ld rows (%.0f MB), second touch %s: first %.0f GB/s, second %.0f GB/s "
               "(sum over chunks 2..K, per-launch events)\n", S, S * ldb * 1e-6,
               pat ? "accumulation pattern" : "same stream pattern", b / (t_first * 1e-3) * 1e-9,
               b / (t_second * 1e-3) * 1e-9);
      }
    }
  }
  const int K_MAX = 4096;
  (void)hipMalloc(&ctr, 2 * K_MAX * sizeof(unsigned));
  (void)hipMalloc(&err, sizeof(int));
  for (long S : {3072L}) {
    const int K = (int)((n + S - 1) / S);
    if (K > K_MAX) continue;
    for (int L : {1, 2, 3}) {
      for (int NA : {256}) {
        const int J = 48;   // second-touch workgroups: 10 tiles x 48 sub-ranges
        const int NB = (int)(ldb / 4096) * J;
        const float t = time_it([&] {
          (void)hipMemsetAsync(ctr, 0, 2 * K_MAX * sizeof(unsigned));
          (void)hipMemsetAsync(err, 0, sizeof(int));
          hipLaunchKernelGGL(pipeline_kernel, dim3(NA + NB), dim3(256), 0, 0, X, n, ldb, S, K, NA, J, L, ctr,
                             ctr + K_MAX, err, out);
        });
        int e = 0;
        (void)hipMemcpy(&e, err, sizeof e, hipMemcpyDeviceToHost);
        printf("pipeline S=%5ld rows (%.0f MB) K=%3d L=%d NA=%3d NB=%d: %.3f ms (%.0f GB/s of first touches, "
               "%.0f GB/s of both)%s\n", S, S * ldb * 1e-6, K, L, NA, NB, t, bytes / (t * 1e-3) * 1e-9,
               2 * bytes / (t * 1e-3) * 1e-9, e ? "  [WAIT OVERRUN]" : "");
        if (e) return 2;
      }
    }
  }
  return 0;
}
