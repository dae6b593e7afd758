// Probe: the residue kernel's planes against the host copy of its arithmetic, element by element.
//   hipcc -O2 -std=c++17 -Iinclude -Ippls_amd/csrc tools/oz_residue_probe.cpp -Lppls_amd -lppls_amd \
//         -Wl,-rpath,$PWD/ppls_amd -o tools/oz_residue_probe && tools/oz_residue_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <cmath>
#include <random>
#include <vector>

#include "ppls_kernels.h"

extern "C" int ppls_oz_residue_host(double x, int shift, int l, int* r);

int main() {
  const int n = 256, P = 64, Pp = 64, nmod = 17;
  const int64_t nkb = n / 64, pstride = nkb * Pp * 64;
  std::mt19937_64 rng(7);
  std::normal_distribution<double> nd;
  std::vector<double> X((size_t)n * P);
  for (auto& v : X) v = nd(rng);
  std::vector<int> sh(Pp);
  for (int c = 0; c < P; ++c) {
    double mx = 0;
    for (int r = 0; r < n; ++r) mx = std::max(mx, std::fabs(X[(size_t)r * P + c]));
    int e;
    std::frexp(mx, &e);
    sh[c] = 55 + (c % 8) - e;   // |x'| < 2^(55 .. 62)
  }
  double* dX;
  int* dS;
  int8_t* dP;
  if (hipMalloc(&dX, X.size() * 8) || hipMalloc(&dS, Pp * 4) || hipMalloc(&dP, nmod * pstride)) return 2;
  (void)hipMemcpy(dX, X.data(), X.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dS, sh.data(), Pp * 4, hipMemcpyHostToDevice);
  if (ppls_launch_oz_residues(dX, P, P, P, dX, P, 0, 0, Pp, n, nkb, dS, nmod, dP, pstride, nullptr) != hipSuccess) return 3;
  std::vector<int8_t> pl((size_t)nmod * pstride);
  if (hipMemcpy(pl.data(), dP, pl.size(), hipMemcpyDeviceToHost) != hipSuccess) return 4;
  long bad = 0, badpar[2] = {0, 0};
  for (int l = 0; l < nmod; ++l) {
    long bl = 0;
    for (int r = 0; r < n; ++r)
      for (int c = 0; c < P; ++c) {
        int want = 0;
        ppls_oz_residue_host(X[(size_t)r * P + c], sh[c], l, &want);
        const int got = pl[(size_t)l * pstride + ((size_t)(r / 64) * Pp + c) * 64 + r % 64];
        if (got != want) {
          if (bl < 3) printf("l=%d row=%d col=%d got %d want %d\n", l, r, c, got, want);
          ++bl;
          ++badpar[r & 1];
        }
      }
    bad += bl;
    if (bl) printf("plane %d: %ld mismatches\n", l, bl);
  }
  printf("mismatches %ld (even rows %ld, odd rows %ld) of %ld\n", bad, badpar[0], badpar[1], (long)nmod * n * P);
  return bad ? 1 : 0;
}
