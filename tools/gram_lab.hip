// Gram lab: the MFMA Gram X'X (X: n x P fp64 row-major, C3's joint width P = 4000) in the product's
// LDS-staged form (ppls_variances.hip, static and persistent scheduling) against an LDS-free form in
// which every wave loads its own MFMA operands straight from global memory into a register ring D
// k-steps deep -- no LDS, no workgroup barrier, waves independent.  Same work items (split x lower
// 128 x 128 tile), same k order per MFMA: the partials must be bitwise equal.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Ippls_amd/csrc -Iinclude tools/gram_lab.hip -o gram_lab
//   ./gram_lab [n=1000000] [P=4000] [reps=3]
#include "../ppls_amd/csrc/ppls_variances.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void lab_fill(double* X, int64_t len, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    X[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

// LDS-free: wave (wi, wj) of the 4 owns the 64 x 64 sub-tile of the item's tile.  Per 4-row k-step a
// lane loads, for rows k0 + (lane >> 4): A = columns colA + wi 64 + {2 i, 2 i + 1, 32 + 2 i, 33 + 2 i}
// (i = lane & 15; two 16-B loads, each 16-lane group reading 256 contiguous bytes) and B likewise --
// block m of the MFMA then covers columns 32 (m >> 1) + 2 i + (m & 1).  D k-steps of operands are in
// flight (16 VGPRs each).
template <int D>
__global__ __launch_bounds__(256, 2) void gram_direct(const double* __restrict__ X, int ld, int64_t n, int p,
                                                      int ntiles, int nsplit, int64_t work, double* __restrict__ part,
                                                      int64_t part_stride) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  const int64_t per = gridDim.x >> 3;
  const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= work) return;
  const int s = (int)(L / ntiles), t = (int)(L - (int64_t)s * ntiles);
  int I, J;
  ppls_gram_tile_of(t, &I, &J);
  const int64_t r0 = n * s / nsplit, r1 = n * (s + 1) / nsplit;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int kr = lane >> 4, i2 = 2 * (lane & 15);
  const int ca = I * PPLS_GT + wi * 64 + i2, cb = J * PPLS_GT + wj * 64 + i2;
  // columns past p (the last block's padding) read column 0: garbage that only ever meets its own
  // output rows / columns, which are never written -- so the steady state needs no masks at all
  const int64_t ldl = ld;
  const double* pa0 = X + r0 * ldl + kr * ldl + (ca < p ? ca : 0);
  const double* pa1 = X + r0 * ldl + kr * ldl + (ca + 32 < p ? ca + 32 : 0);
  const double* pb0 = X + r0 * ldl + kr * ldl + (cb < p ? cb : 0);
  const double* pb1 = X + r0 * ldl + kr * ldl + (cb + 32 < p ? cb + 32 : 0);
  const int64_t step = 4 * ldl;
  const int64_t nfull = (r1 - r0) / 4;   // whole 4-row k-steps
  double2 ra0[D], ra1[D], rb0[D], rb1[D];
  int64_t o = 0;   // element offset of the next step to load
  auto ld_step = [&](int d) {
    ra0[d] = *(const double2*)(pa0 + o);
    ra1[d] = *(const double2*)(pa1 + o);
    rb0[d] = *(const double2*)(pb0 + o);
    rb1[d] = *(const double2*)(pb1 + o);
    o += step;
  };
  d4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = d4{0.0, 0.0, 0.0, 0.0};
  auto mma = [&](const double2& x0, const double2& x1, const double2& y0, const double2& y1) {
    const double a[4] = {x0.x, x0.y, x1.x, x1.y};
    const double b[4] = {y0.x, y0.y, y1.x, y1.y};
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[q], acc[m][q], 0, 0, 0);
  };
  int64_t kk = 0;
  if (nfull >= 2 * D) {
#pragma unroll
    for (int d = 0; d < D; ++d) ld_step(d);
    // steady state: every prefetched step lies inside the split, no branch between the loads
    for (; kk + 2 * D <= nfull; kk += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        mma(ra0[d], ra1[d], rb0[d], rb1[d]);
        ld_step(d);
        // keep the loads in ring order (the oldest step is consumed next: vmcnt(4 (D - 1)) suffices)
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) mma(ra0[d], ra1[d], rb0[d], rb1[d]);
    kk += D;
  }
  for (; kk < nfull; ++kk) {   // the last < D whole steps
    ld_step(0);
    mma(ra0[0], ra1[0], rb0[0], rb1[0]);
  }
  if (r1 - r0 > 4 * nfull) {   // a partial last step: rows past r1 are zeros
    const bool ok = r0 + 4 * nfull + kr < r1;
    const double z = 0.0;
    const double2 zz{z, z};
    double2 x0 = zz, x1 = zz, y0 = zz, y1 = zz;
    if (ok) {
      x0 = *(const double2*)(pa0 + o);
      x1 = *(const double2*)(pa1 + o);
      y0 = *(const double2*)(pb0 + o);
      y1 = *(const double2*)(pb1 + o);
    }
    mma(x0, x1, y0, y1);
  }
  double* out = part + (int64_t)s * part_stride;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = J * PPLS_GT + wj * 64 + 32 * (q >> 1) + 2 * (lane & 15) + (q & 1);
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // D row = (lane >> 4) + 4 g, column = lane & 15
        const int i = I * PPLS_GT + wi * 64 + 32 * (m >> 1) + 2 * ((lane >> 4) + 4 * g) + (m & 1);
        if (i < p && j < p) out[(int64_t)i * p + j] = acc[m][q][g];
      }
    }
}

template <typename F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    (void)hipEventRecord(a, 0);
    f();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 0 || reps == 1) best = ms < best ? ms : best;
  }
  return best;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int P = argc > 2 ? atoi(argv[2]) : 4000;
  const int reps = argc > 3 ? atoi(argv[3]) : 3;
  double *X, *part_ref, *part;
  int* queue;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int slots = cus * ppls_gram_occupancy(0);
  const int nsplit = ppls_gram_splits(P, n, slots, 0);
  const int ntiles = ppls_gram_tiles(P);
  const int64_t work = (int64_t)ntiles * nsplit;
  const size_t pp = (size_t)P * P;
  if (hipMalloc(&X, sizeof(double) * (size_t)n * P) || hipMalloc(&part_ref, sizeof(double) * pp * nsplit) ||
      hipMalloc(&part, sizeof(double) * pp * nsplit) || hipMalloc(&queue, sizeof(int) * ppls_gram_queue_ints(P, nsplit))) {
    printf("alloc failed\n");
    return 1;
  }
  hipLaunchKernelGGL(lab_fill, dim3(4096), dim3(256), 0, 0, X, (int64_t)n * P, 12345ull);
  (void)hipMemset(part_ref, 0, sizeof(double) * pp * nsplit);
  (void)hipDeviceSynchronize();
  const double flops = 2.0 * n * ntiles * 128.0 * 128.0, useful = (double)n * P * (P + 1.0);
  printf("n=%lld P=%d nsplit=%d tiles=%d slots=%d\n", (long long)n, P, nsplit, ntiles, slots);
  auto report = [&](const char* name, float ms, bool check) {
    bool same = true;
    if (check) {
      std::vector<double> a(pp), b(pp);
      for (int sp = 0; sp < nsplit && same; ++sp) {
        (void)hipMemcpy(a.data(), part_ref + pp * sp, sizeof(double) * pp, hipMemcpyDeviceToHost);
        (void)hipMemcpy(b.data(), part + pp * sp, sizeof(double) * pp, hipMemcpyDeviceToHost);
        for (int i = 0; i < P && same; ++i)
          for (int j = 0; j <= i && same; ++j)
            if (memcmp(&a[(size_t)i * P + j], &b[(size_t)i * P + j], 8) != 0) {
              printf("  mismatch split %d (%d, %d): %.17g vs %.17g\n", sp, i, j, a[(size_t)i * P + j], b[(size_t)i * P + j]);
              same = false;
            }
      }
    }
    printf("%-34s %9.2f ms  executed %6.2f TF/s  useful %6.2f TF/s  %s\n", name, ms, flops / ms / 1e9, useful / ms / 1e9,
           check ? (same ? "bitwise = LDS static" : "DIFFERS") : "");
    fflush(stdout);
  };
  (void)ppls_gram_queue_prepare(queue, P, P, P, 0, nsplit, 2, 0);
  float ms = timeit([&] { (void)ppls_launch_gram_joint(X, P, P, P, nullptr, 0, 0, 0, 0, n, P, nsplit, part_ref, (int64_t)pp, queue, 0, 0); }, reps);
  report("LDS static (product variant 0)", ms, false);
  ms = timeit([&] { (void)ppls_launch_gram_joint(X, P, P, P, nullptr, 0, 0, 0, 0, n, P, nsplit, part, (int64_t)pp, queue, 2, 0); }, reps);
  report("LDS persistent (product variant 2)", ms, true);
  const int64_t grid = (work + 7) / 8 * 8;
#define LAB_DIRECT(DD)                                                                                              \
  (void)hipMemset(part, 0, sizeof(double) * pp * nsplit);                                                           \
  ms = timeit([&] { hipLaunchKernelGGL(gram_direct<DD>, dim3((unsigned)grid), dim3(256), 0, 0, X, P, n, P, ntiles, nsplit, \
                                       work, part, (int64_t)pp); }, reps);                                            \
  report("LDS-free direct, ring " #DD, ms, true);
  LAB_DIRECT(2)
  LAB_DIRECT(3)
  LAB_DIRECT(4)

  return 0;
}
