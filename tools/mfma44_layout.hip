// Operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 (determined empirically): A = lane id,
// B = one-hot at lane `target`; prints the lanes with a nonzero result and their values.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* out, int target) {
  const int l = threadIdx.x;
  const double a = 100.0 + l, b = (l == target) ? 1.0 : 0.0;
  out[l] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
}
int main() {
  double* d;
  (void)hipMalloc(&d, 64 * 8);
  double h[64];
  const int targets[] = {0, 1, 2, 3, 4, 8, 12, 16, 17, 20};
  for (int t : targets) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, t);
    (void)hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
    printf("B one-hot at lane %2d ->", t);
    for (int l = 0; l < 64; ++l)
      if (h[l] != 0.0) printf(" D[lane %d]=A[lane %d]", l, (int)h[l] - 100);
    printf("\n");
  }
  return 0;
}
