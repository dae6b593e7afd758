// Probe: cross-CU visibility and round-trip latency of 16-B exchange entries for several cache-
// policy combinations (writer and reader workgroups on the same XCD, or on different XCDs).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned u4 __attribute__((ext_vector_type(4)));

#define STORE(name, bits) \
  __device__ __forceinline__ void st_##name(unsigned* p, unsigned v) { \
    u4 w; w.x = v; w.y = v; w.z = v; w.w = v; \
    asm volatile("global_store_dwordx4 %0, %1, off " bits :: "v"(p), "v"(w) : "memory"); }
STORE(plain, "") STORE(sc0, "sc0") STORE(sc1, "sc1") STORE(sys, "sc0 sc1")
#define DLOAD(name, bits) \
  __device__ __forceinline__ unsigned ld_##name(unsigned* p, unsigned* lds_word) { \
    unsigned a = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned*)lds_word; \
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off " bits "\n\ts_waitcnt vmcnt(0)" \
                 :: "s"(a), "v"(p) : "memory", "m0"); \
    return lds_word[threadIdx.x * 4]; }
DLOAD(sc0, "sc0") DLOAD(sc1, "sc1") DLOAD(sys, "sc0 sc1")
__device__ __forceinline__ unsigned ld_plain(unsigned* p, unsigned*) {
  unsigned v; asm volatile("global_load_dword %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory"); return v; }

template <void (*ST)(unsigned*, unsigned), unsigned (*LD)(unsigned*, unsigned*)>
__global__ void pingpong(unsigned* buf, int iters, int cross, long long* out) {
  __shared__ __attribute__((aligned(16))) unsigned lds[64 * 4];
  const int b = blockIdx.x;            // grid 16: pairs (x, x+8) share XCD x; cross: (x, x+9)
  const int x = b & 7;
  const bool writer = b < 8;
  const int pair = writer ? x : (cross ? ((x + 7) & 7) : x);
  unsigned* A = buf + pair * 64;        // writer -> reader
  unsigned* B = buf + pair * 64 + 32;   // reader -> writer
  if (threadIdx.x >= 1) return;
  long long t0 = clock64();
  int k;
  for (k = 1; k <= iters; ++k) {
    if (writer) {
      ST(A, k);
      int spins = 0;
      while (LD(B, lds) != (unsigned)k) { if (++spins > (1 << 20)) { out[b] = -k; return; } }
    } else {
      int spins = 0;
      while (LD(A, lds) != (unsigned)k) { if (++spins > (1 << 20)) { out[b] = -k; return; } }
      ST(B, k);
    }
  }
  out[b] = clock64() - t0;
}

template <void (*ST)(unsigned*, unsigned), unsigned (*LD)(unsigned*, unsigned*)>
void run(const char* name, unsigned* buf, long long* out, int cross) {
  (void)hipMemset(buf, 0, 4096 * 4);
  (void)hipMemset(out, 0, 16 * 8);
  hipLaunchKernelGGL((pingpong<ST, LD>), dim3(16), dim3(64), 0, 0, buf, 2000, cross, out);
  (void)hipDeviceSynchronize();
  long long h[16];
  (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  int fails = 0; double mean = 0;
  for (int i = 0; i < 16; ++i) { if (h[i] <= 0) ++fails; else mean += h[i]; }
  printf("%-28s %s fails=%2d  round trip = %8.0f clocks\n", name, cross ? "cross-XCD" : "same-XCD ", fails,
         fails == 16 ? 0.0 : mean / (16 - fails) / 2000.0);
}

int main() {
  unsigned* buf; long long* out;
  (void)hipMalloc(&buf, 4096 * 4); (void)hipMalloc(&out, 16 * 8);
  for (int cross = 0; cross < 2; ++cross) {
    run<st_plain, ld_sc1>("store plain / dma sc1", buf, out, cross);
    run<st_sc0, ld_sc1>("store sc0 / dma sc1", buf, out, cross);
    run<st_sc1, ld_sc1>("store sc1 / dma sc1", buf, out, cross);
    run<st_sys, ld_sys>("store sc0sc1 / dma sc0sc1", buf, out, cross);
    run<st_sc1, ld_sys>("store sc1 / dma sc0sc1", buf, out, cross);
    run<st_plain, ld_sc0>("store plain / dma sc0", buf, out, cross);
    run<st_sc1, ld_plain>("store sc1 / load sc1", buf, out, cross);
    run<st_plain, ld_plain>("store plain / load sc1", buf, out, cross);
  }
  return 0;
}
