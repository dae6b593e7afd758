// oz_lab.hip -- feasibility lab for an int8-MFMA SYRK of residue planes (the Ozaki-II form of the
// Gram S = D'D): times the residue SYRK alone and checks sampled entries against
// exact int64 sums on the host.  Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ippls_amd/csrc -o tools/oz_lab tools/oz_lab.hip
//   tools/oz_lab <n> <P> <planes> [check] [variant]
//
// Random int8 residues in the product's plane layout [n / 64][Pp][64]; `planes` moduli go through ONE
// launch of the product SYRK (ppls_ozaki.hip: ppls_launch_oz_syrk_v; variant 0 the product, 1 no
// copies, 2 the copies alone), and sampled entries are checked against exact int64 sums mod m on
// the host.  (The round-6 variants of profiles/r6_int8_syrk_ab.txt were built in this lab at
// commits 4a40cc5 .. aac738c and removed from the product source afterwards.)
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

#define OZ_LAB 1
#include "../ppls_amd/csrc/ppls_ozaki.hip"   // the product kernels (ppls_launch_oz_syrk)

constexpr int TT = 256;   // output tile edge
constexpr int KS = 64;    // rows per stage (the product's OZ_KS)

static void tile_of_h(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const int P = argc > 2 ? atoi(argv[2]) : 4000;
  const int planes = argc > 3 ? atoi(argv[3]) : 4;
  const int check = argc > 4 ? atoi(argv[4]) : 1;
  const int Pp = (P + TT - 1) / TT * TT;
  const int64_t nkb = (n + KS - 1) / KS, np = nkb * KS;
  const int T = Pp / TT, ntiles = T * (T + 1) / 2;

  const size_t pbytes = (size_t)np * Pp;
  printf("n %lld P %d (Pp %d) tiles %d splits %d planes %d: %.2f GB per plane\n", (long long)n, P, Pp, ntiles,
         ppls_oz_splits(nkb), planes, pbytes / 1e9);
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
  int8_t* dp;   // `planes` moduli: the same residues in every plane (each plane its own copy)
  CHK(hipMalloc(&dp, pbytes * planes));
  for (int i = 0; i < planes; ++i) CHK(hipMemcpy(dp + pbytes * i, h.data(), pbytes, hipMemcpyHostToDevice));
  const int nsplit = ppls_oz_splits(nkb);
  uint8_t* dout;
  const size_t obytes = (size_t)ntiles * nsplit * TT * TT;   // per modulus
  CHK(hipMalloc(&dout, obytes * planes));
  const int variant = argc > 5 ? atoi(argv[5]) : -1;   // -1: every variant
  for (int v : {0, 4, 5, 6, 0, 4}) {
    if (variant >= 0 && v != variant) continue;
    for (int w = 0; w < 2; ++w) CHK(ppls_launch_oz_syrk_v(v, dp, (int64_t)pbytes, Pp, nkb, planes, dout, 0));
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    CHK(hipEventRecord(e0));
    CHK(ppls_launch_oz_syrk_v(v, dp, (int64_t)pbytes, Pp, nkb, planes, dout, 0));
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double useful = (double)n * P * (P + 1.0) * planes;   // lower triangle incl. diagonal, 2 ops per MAC
    const double exec = (double)np * TT * TT * 2.0 * ntiles * planes;
    printf("variant %d: %d planes in one launch: %.3f ms (%.3f ms per plane); useful %.1f TOPS, executed %.1f TOPS "
           "(%.3f of 5000)\n", v, planes, ms, ms / planes, useful / (ms * 1e-3) / 1e12, exec / (ms * 1e-3) / 1e12,
           exec / (ms * 1e-3) / 5e15);
  }
  if (check) {
    std::vector<uint8_t> ho(obytes * planes);
    CHK(hipMemcpy(ho.data(), dout, ho.size(), hipMemcpyDeviceToHost));
    std::mt19937 r2(3);
    int bad = 0, tested = 0;
    for (int s = 0; s < 300; ++s) {
      const int t = s < 3 ? (s == 0 ? 0 : s == 1 ? ntiles - 1 : ntiles / 2) : (int)(r2() % ntiles);
      const int l = s % planes, m = ppls_oz_modulus(l);
      int I, J;
      tile_of_h(t, &I, &J);
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
      int got = 0;
      for (int sp = 0; sp < nsplit; ++sp)
        got += ho[(((size_t)l * nsplit + sp) * ntiles + t) * TT * TT + (size_t)j * TT + i];
      got %= m;
      ++tested;
      if (want != got && bad++ < 10) printf("  mod %d tile %d (%d,%d) entry (%d,%d): got %d want %d\n", m, t, I, J, i, j, got, want);
    }
    printf("check: %d of %d sampled entries wrong\n", bad, tested);
    if (bad) return 2;
  }
  return 0;
}
