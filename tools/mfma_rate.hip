// Issue rate of the gfx950 fp64 MFMA shapes (and fp64 VALU FMA beside them): every wave of a
// full-chip grid runs ITER rounds of 4 independent accumulator chains; reports cycles per
// instruction per SIMD and the chip-wide fp64 rate.  hipcc --offload-arch=gfx950 -O3 -o mfma_rate tools/mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITER = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void rate_kernel(double* out, double seed) {
  const double a = seed + threadIdx.x * 1e-9, b = seed * 0.5;
  double s = 0.0;
  if constexpr (MODE == 0) {   // v_mfma_f64_16x16x4_f64: 2048 flops
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < ITER; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    s = c0[0] + c1[1] + c2[2] + c3[3];
  } else if constexpr (MODE == 1) {   // v_mfma_f64_4x4x4_4b_f64: 4 blocks x 4x4x4 = 512 flops
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    for (int i = 0; i < ITER; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
    }
    s = c0 + c1 + c2 + c3;
  } else if constexpr (MODE == 3) {   // interleaved: 4 MFMA 16x16x4 chains + 16 VALU FMA per round
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = 0.0;
    for (int i = 0; i < ITER; ++i) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = fma(a, b + u, v[u]);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
#pragma unroll
      for (int u = 4; u < 8; ++u) v[u] = fma(a, b + u, v[u]);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
#pragma unroll
      for (int u = 8; u < 12; ++u) v[u] = fma(a, b + u, v[u]);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
#pragma unroll
      for (int u = 12; u < 16; ++u) v[u] = fma(a, b + u, v[u]);
    }
    s = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  } else {   // fp64 VALU FMA, 8 chains: 128 flops per wave instruction
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < ITER; ++i)
#pragma unroll
      for (int u = 0; u < 8; ++u) c[u] = fma(a, b + u, c[u]);
    for (int u = 0; u < 8; ++u) s += c[u];
  }
  if (s == 12345.0) out[0] = s;   // keep the work
}

template <int MODE>
void run(const char* name, double flops_per_inst, int insts_per_iter) {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  double* out;
  (void)hipMalloc(&out, 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int waves_per_simd = 1; waves_per_simd <= 4; waves_per_simd *= 2) {
    const int grid = cus * waves_per_simd;   // 256 threads = 4 waves = 1 per SIMD per block
    hipLaunchKernelGGL(rate_kernel<MODE>, dim3(grid), dim3(256), 0, 0, out, 1.0);
    (void)hipEventRecord(e0);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL(rate_kernel<MODE>, dim3(grid), dim3(256), 0, 0, out, 1.0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double insts = 5.0 * grid * 4.0 * ITER * insts_per_iter;
    const double tf = insts * flops_per_inst / (ms * 1e-3) / 1e12;
    const double per_simd = insts / (cus * 4.0);
    printf("%-26s waves/SIMD %d: %.2f TFLOP/s, %.1f ns per instruction per SIMD\n", name, waves_per_simd, tf,
           ms * 1e6 / per_simd);
  }
  (void)hipFree(out);
}

int main() {
  run<0>("mfma_f64_16x16x4", 2048.0, 4);
  run<1>("mfma_f64_4x4x4_4b", 512.0, 4);
  run<2>("valu fma_f64", 128.0, 8);
  // 4 MFMA (2048 flops) + 16 VALU FMA (128 flops) per round: if the pipes overlap, the time per round
  // is max(4 x MFMA, 16 x FMA) instead of their sum (report: ns per round per SIMD)
  run<3>("mfma 16x16x4 + valu fma", (4 * 2048.0 + 16 * 128.0) / 20.0, 20);
  run<0>("mfma_f64_16x16x4 (again)", 2048.0, 4);
  return 0;
}
