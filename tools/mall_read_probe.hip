// Read rate of a buffer re-read every launch (the cross-product form's S, ppls_xprod.hip): is a
// 128 MB S served from the 256 MiB Infinity Cache, and what does the row-tile access pattern
// (each wave walks its own row of S in 1-KB steps) reach against a flat grid-stride sweep?
//   hipcc -O3 --offload-arch=gfx950 tools/mall_read_probe.hip -o tools/mall_read_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d2v __attribute__((ext_vector_type(2)));

// flat: grid-stride 16-B loads, U in flight per lane
template <int U>
__global__ __launch_bounds__(256) void flat(const d2v* __restrict__ a, size_t n2, double* out) {
  double s = 0.0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n2; i += U * stride) {
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u].x + v[u].y;
  }
  if (s == 12345.678) out[0] = s;
}

// rows: P x P doubles; wave w of workgroup b reads rows RW (4 b + w) .. + RW - 1, 128 columns per
// step, U steps in flight (the row-tile kernel's pattern without its arithmetic)
template <int RW, int U>
__global__ __launch_bounds__(256) void rows(const double* __restrict__ S, int P, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long i0 = ((long)blockIdx.x * 4 + wave) * RW;
  double s = 0.0;
  for (int j = 2 * lane; j < P; j += 128 * U) {
    d2v v[U][RW];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r)
        v[u][r] = (j + 128 * u < P && i0 + r < P) ? *(const d2v*)(S + (i0 + r) * P + j + 128 * u) : d2v{0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < RW; ++r) s += v[u][r].x + v[u][r].y;
  }
  if (s == 12345.678) out[0] = s;
}

template <typename F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  f();
  hipEventRecord(a);
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  double* out;
  hipMalloc(&out, 8);
  for (int P : {2000, 4000, 6000, 8000, 10752}) {
    const size_t bytes = (size_t)P * P * 8;
    double* S;
    if (hipMalloc(&S, bytes) != hipSuccess) return 1;
    hipMemset(S, 0, bytes);
    const size_t n2 = bytes / 16;
    auto rep = [&](const char* name, float ms) {
      printf("P=%5d (%6.1f MB)  %-28s %8.2f us  %6.2f TB/s\n", P, bytes / 1e6, name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    };
    rep("flat x8 grid 2048", timeit([&] { hipLaunchKernelGGL(flat<8>, dim3(2048), dim3(256), 0, 0, (const d2v*)S, n2, out); }, 20));
    rep("flat x8 grid 8192", timeit([&] { hipLaunchKernelGGL(flat<8>, dim3(8192), dim3(256), 0, 0, (const d2v*)S, n2, out); }, 20));
    rep("flat x4 grid 4096", timeit([&] { hipLaunchKernelGGL(flat<4>, dim3(4096), dim3(256), 0, 0, (const d2v*)S, n2, out); }, 20));
    const unsigned b1 = (P + 3) / 4, b2 = (P + 7) / 8;
    rep("rows RW1 U1", timeit([&] { hipLaunchKernelGGL((rows<1, 1>), dim3(b1), dim3(256), 0, 0, S, P, out); }, 20));
    rep("rows RW1 U4", timeit([&] { hipLaunchKernelGGL((rows<1, 4>), dim3(b1), dim3(256), 0, 0, S, P, out); }, 20));
    rep("rows RW2 U2", timeit([&] { hipLaunchKernelGGL((rows<2, 2>), dim3(b2), dim3(256), 0, 0, S, P, out); }, 20));
    rep("rows RW2 U4", timeit([&] { hipLaunchKernelGGL((rows<2, 4>), dim3(b2), dim3(256), 0, 0, S, P, out); }, 20));
    hipFree(S);
  }
  return 0;
}
