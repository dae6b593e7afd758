// Gram lab: the product MFMA Gram X'X (ppls_variances.hip: LDS-free waves taking work items from
// per-XCD-group queues, every MFMA operand loaded from global memory into a register ring) against
// the LDS-staged kernel it replaced (copied below: 16-row panels in LDS behind one barrier per stage,
// one item per workgroup).  X: n x P fp64 row-major (C3's joint width P = 4000).  With the
// baseline's equal splits the two give the same sums bit for bit (same items, same k order per MFMA).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Ippls_amd/csrc -Iinclude tools/gram_lab.hip -o tools/gram_lab
//   tools/gram_lab [n=1000000] [P=4000] [reps=3]
#include "../ppls_amd/csrc/ppls_variances.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

// ---- baseline: the round-4/5 LDS-staged Gram kernel (copied here when the product moved to the
// LDS-free form; same work items and k order, so the partials are bitwise equal)
#define PPLS_GK 16
#define PPLS_GLD 144
template <typename T> struct LabVec;
template <> struct LabVec<double> {
  double2 v;
  __device__ __forceinline__ void load(const double* p) { v = *(const double2*)p; }
  __device__ __forceinline__ void zero() { v = make_double2(0.0, 0.0); }
  __device__ __forceinline__ void store(double* d) const { *(double2*)d = v; }
};
template <> struct LabVec<float> {
  float4 v;
  __device__ __forceinline__ void load(const float* p) { v = *(const float4*)p; }
  __device__ __forceinline__ void zero() { v = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ void store(double* d) const {
    *(double2*)d = make_double2((double)v.x, (double)v.y);
    *(double2*)(d + 2) = make_double2((double)v.z, (double)v.w);
  }
};
// The columns of the joint space that can be non-zero: [0, xreal) of X and [xcols, xcols + yreal) of
// Y -- between and after them lie the rows' zero padding (C5: X columns 10,000 .. 10,239).
struct LabCols {
  int p, xreal, xcols, yend;
};

// Whether the 16 columns [a, a + 16) of the joint space hold any that can be non-zero.
__host__ __device__ inline bool lab_lds_gram_live(const LabCols& g, int a) {
  return a < g.p && (a < g.xreal || (a + 16 > g.xcols && a < g.yend));
}

// Active 16 x 16 MFMA blocks of wave (wi, wj) in the lower tile (I, J) of a p x p Gram: bit m * 4 + q
// for the wave's block row m and block column q.  A block is skipped when its rows or columns are
// all zero padding (past p, or between X's real columns and Y's), or -- in a diagonal tile -- when it
// lies wholly above the diagonal (the finish kernel reads only the lower triangle).  C3 (p = 4000 ->
// 32 blocks of 128): the last block row is 3/4 padding and the diagonal tiles 7/16 upper half, 7 %
// of the executed flops; C5 also skips the 240 padding columns of X's 40,960-B rows (4 %).  Skipped
// blocks inside p are written as the zeros they are (their accumulators are never touched).
__host__ __device__ inline unsigned lab_lds_gram_active(int I, int J, int wi, int wj, const LabCols& g) {
  unsigned act = 0;
  for (int m = 0; m < 4; ++m)
    for (int q = 0; q < 4; ++q) {
      const int i0 = I * PPLS_GT + wi * 64 + m * 16, j0 = J * PPLS_GT + wj * 64 + q * 16;
      if (lab_lds_gram_live(g, i0) && lab_lds_gram_live(g, j0) && (I != J || wj * 4 + q <= wi * 4 + m))
        act |= 1u << (m * 4 + q);
    }
  return act;
}

// Whether tile (I, J) has any skipped block (its items take the masked code path).
__host__ __device__ inline bool lab_lds_gram_partial(int I, int J, const LabCols& g) {
  if (I == J) return true;
  for (int a = 0; a < PPLS_GT; a += 16)
    if (!lab_lds_gram_live(g, I * PPLS_GT + a) || !lab_lds_gram_live(g, J * PPLS_GT + a)) return true;
  return false;
}

__host__ __device__ inline void lab_lds_gram_tile_of(int t, int* I, int* J) {
  int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((i + 1) * (i + 2) / 2 <= t) ++i;
  while (i * (i + 1) / 2 > t) --i;
  *I = i;
  *J = t - i * (i + 1) / 2;
}

// The persistent form's next work item: group g's queue first (its workgroups share an XCD, so
// their items -- consecutive tiles of one row split -- share column panels in that L2), then the
// other groups' (stealing: an XCD that runs ahead takes the cheap tail of a slower one).  One
// global atomic per grab (items take milliseconds); -1 when every queue is empty.
__device__ inline int lab_lds_gram_next(unsigned* cnt, const int* qoff, const int* items, int g) {
  for (int k = 0; k < 8; ++k) {
    const int gg = (g + k) & 7;
    const int len = qoff[gg + 1] - qoff[gg];
    const unsigned idx = atomicAdd(&cnt[gg], 1u);
    if ((int)idx < len) return items[qoff[gg] + idx];
  }
  return -1;
}

// X'X on MFMA.  Work item L = split s x lower tile t = (I, J), J <= I.  A wave owns a 64 x 64
// sub-tile = 4 x 4 MFMA blocks (64 fp64 accumulators per lane); per 4-row k-step it reads 4 A and 4
// B operands from LDS (lane l: row l >> 4 of the step, column l & 15 of its block) -- both straight
// from the row-major panels, no transpose, since A[i][k] = X[k][i] and B[k][j] = X[k][j].  The next
// stage's global loads are in flight during the MFMAs; one barrier per 16-row stage.  Output:
// part[s][i p + j] for the tile's (i, j), i in block I >= block J (row-major of the lower blocks;
// coalesced over j).
//
// Scheduling (template DYN): the static form runs one work item per workgroup, blockIdx remapped so
// that each XCD -- blockIdx mod 8 -- gets a contiguous range of items (tiles that share column panels
// share an L2).  Its items all take the same time, so the last round of them leaves the slots that
// have none idle (C3: 6,336 items on 512 slots, the 13th round 3/8 full: ~5 % of the kernel).  The
// persistent form (DYN) launches one workgroup per slot; each takes items from the queue of its group
// (blockIdx mod 8: the same contiguous ranges), costliest first -- tiles with skipped blocks (SKIP)
// are cheaper and come last, so the final items of every queue are short -- and steals from the
// other groups' queues once its own is empty.  Each item's sums depend only on the item, so the
// result is the same bit for bit whichever workgroup runs it.
//
// The column space is that of the joint matrix [X | Y] (ppls_xprod.hip's cross-product form of the
// EM iteration): column c is X[:, c] for c < xcols and Y[:, c - xcols] for c - xcols < ycols (zero
// beyond); xcols and ycols are multiples of the 16-B vector, so no load straddles the seam.  The
// Gram of X alone is xcols = ld, ycols = 0, p the output edge.
template <typename T, bool SKIP, bool MASKED>
__device__ __forceinline__ void lab_lds_gram_item(const T* __restrict__ X, int ldx, int xcols, const T* __restrict__ Y,
                                               int ldy, int ycols, int64_t n, int p, int ntiles, int nsplit,
                                               int64_t L, double* __restrict__ part, int64_t part_stride,
                                               const LabCols gc, double (*sm)[2][PPLS_GK][PPLS_GLD]) {
  typedef double d4 __attribute__((ext_vector_type(4)));
  constexpr int EV = 16 / sizeof(T);              // elements per 16-B load
  constexpr int VPR = PPLS_GT / EV;               // 16-B vectors per panel row
  constexpr int NV = PPLS_GK * VPR / 256;         // per thread per panel (fp64: 4, fp32: 2)
  const int s = (int)(L / ntiles), t = (int)(L - (int64_t)s * ntiles);
  int I, J;
  lab_lds_gram_tile_of(t, &I, &J);
  const int64_t r0 = n * s / nsplit, r1 = n * (s + 1) / nsplit;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wi = wave >> 1, wj = wave & 1;
  const int colA = I * PPLS_GT, colB = J * PPLS_GT;
  // wave-uniform (SGPR) block mask; MASKED code paths test it per MFMA, the full path does not
  const unsigned act = SKIP ? lab_lds_gram_active(I, J, wi, wj, gc) : 0xffffu;

  LabVec<T> ra[NV], rb[NV];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = tid + 256 * v, row = c / VPR, cv = c - row * VPR;
      const int64_t gr = k0 + row;
      const int ca = colA + cv * EV, cb = colB + cv * EV;
      if (gr < r1 && ca < xcols) ra[v].load(X + gr * ldx + ca);
      else if (gr < r1 && ca - xcols < ycols) ra[v].load(Y + gr * ldy + (ca - xcols));
      else ra[v].zero();
      if (gr < r1 && cb < xcols) rb[v].load(X + gr * ldx + cb);
      else if (gr < r1 && cb - xcols < ycols) rb[v].load(Y + gr * ldy + (cb - xcols));
      else rb[v].zero();
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = tid + 256 * v, row = c / VPR, cv = c - row * VPR;
      ra[v].store(&sm[buf][0][row][cv * EV]);
      rb[v].store(&sm[buf][1][row][cv * EV]);
    }
  };

  d4 acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[m][q] = d4{0.0, 0.0, 0.0, 0.0};
  const int64_t nsteps = (r1 - r0 + PPLS_GK - 1) / PPLS_GK;
  if (nsteps > 0) {
    load(r0);
    store(0);
  }
  __syncthreads();
  const int ko = lane >> 4, cl = lane & 15;
  for (int64_t st = 0; st < nsteps; ++st) {
    const int buf = (int)(st & 1);
    if (st + 1 < nsteps) load(r0 + (st + 1) * PPLS_GK);
    if (!MASKED || act) {
#pragma unroll
      for (int kk = 0; kk < PPLS_GK / 4; ++kk) {
        const double* ar = &sm[buf][0][kk * 4 + ko][wi * 64 + cl];
        const double* br = &sm[buf][1][kk * 4 + ko][wj * 64 + cl];
        double a[4], b[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = ar[m * 16];
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = br[q * 16];
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (!MASKED || ((act >> (m * 4 + q)) & 1u))
              acc[m][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[q], acc[m][q], 0, 0, 0);
      }
    }
    if (st + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  double* out = part + (int64_t)s * part_stride;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = colB + wj * 64 + q * 16 + cl;
#pragma unroll
      for (int g = 0; g < 4; ++g) {   // f64 MFMA D map: col = lane & 15, row = (lane >> 4) + 4 g
        const int i = colA + wi * 64 + m * 16 + ko + 4 * g;
        if (i < p && j < p) out[(int64_t)i * p + j] = acc[m][q][g];
      }
    }
}

template <typename T, bool DYN, bool SKIP>
__global__ __launch_bounds__(256, 2) void lab_lds_gram_mfma_kernel(const T* __restrict__ X, int ldx, int xcols,
                                                                 const T* __restrict__ Y, int ldy, int ycols,
                                                                 int64_t n, int p, int ntiles, int nsplit,
                                                                 int64_t work, double* __restrict__ part,
                                                                 int64_t part_stride, int* __restrict__ queue,
                                                                 LabCols gc) {
  __shared__ __attribute__((aligned(16))) double sm[2][2][PPLS_GK][PPLS_GLD];
  if constexpr (!DYN) {
    const int64_t per = gridDim.x >> 3;
    const int64_t L = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (L >= work) return;
    if (SKIP) {
      int I, J;
      lab_lds_gram_tile_of((int)(L % ntiles), &I, &J);
      if (lab_lds_gram_partial(I, J, gc)) {   // a tile with skipped blocks: the masked code path
        lab_lds_gram_item<T, true, true>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
        return;
      }
    }
    lab_lds_gram_item<T, false, false>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
  } else {
    // queue = [qoff (9) | counters (8, zeroed before the launch) | items (work)]
    const int* qoff = queue;
    unsigned* cnt = (unsigned*)(queue + 9);
    const int* items = queue + 17;
    __shared__ int s_next;
    const int g = blockIdx.x & 7;
    for (;;) {
      if (threadIdx.x == 0) s_next = lab_lds_gram_next(cnt, qoff, items, g);
      __syncthreads();
      const int L = s_next;
      __syncthreads();   // every thread has read s_next before thread 0 writes the next one
      if (L < 0) return;
      int I, J;
      lab_lds_gram_tile_of(L % ntiles, &I, &J);
      if (SKIP && lab_lds_gram_partial(I, J, gc))
        lab_lds_gram_item<T, true, true>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
      else
        lab_lds_gram_item<T, false, false>(X, ldx, xcols, Y, ldy, ycols, n, p, ntiles, nsplit, L, part, part_stride, gc, sm);
    }
  }
}


__global__ void lab_fill(double* X, int64_t len, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    X[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

// The baseline's finish: its partials are p x p row-major per split (lower tiles only).
__global__ void lab_lds_finish(const double* __restrict__ part, int nsplit, int64_t part_stride, int p, double* G) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)p * p) return;
  const int b = (int)(e / p), a = (int)(e - (int64_t)b * p);
  const int hi = a > b ? a : b, lo = a > b ? b : a;
  double v = 0.0;
  for (int s = 0; s < nsplit; ++s) v += part[(int64_t)s * part_stride + (int64_t)hi * p + lo];
  G[e] = v;
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
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int occ_lds = 1;
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_lds, lab_lds_gram_mfma_kernel<double, false, false>, 256, 0);
  const int slots = cus * occ_lds;
  const int ntiles = ppls_gram_tiles(P);
  // the baseline's split count (whole rounds of its one-item-per-workgroup grid, as it chose them)
  int nsplit = 1;
  {
    double best = -1.0;
    for (int sp = 1; sp <= 32; ++sp) {
      if (sp > 1 && ((int64_t)sp * 512 > n || (double)sp * P * P * 8.0 > 4.0e9)) break;
      const int64_t w = (int64_t)ntiles * sp;
      const double eff = (double)w / (double)(((w + slots - 1) / slots) * slots);
      if (eff > best + 1e-9) { best = eff; nsplit = sp; }
      if (eff >= 0.95) break;
    }
  }
  const int wave_slots = cus * ppls_gram_occupancy(0) * 4;
  const int nauto = ppls_gram_plan(P, P, P, 0, n, wave_slots, 0, nullptr);
  const int64_t work = (int64_t)ntiles * nsplit;
  const size_t pp = (size_t)P * P;
  const int nmax = nsplit > nauto ? nsplit : nauto;
  double *X, *part_ref, *part, *Gref, *G;
  int* queue;
  if (hipMalloc(&X, sizeof(double) * (size_t)n * P) || hipMalloc(&part_ref, sizeof(double) * pp * nsplit) ||
      hipMalloc(&part, sizeof(double) * ppls_gram_part_doubles(P, nmax)) || hipMalloc(&Gref, sizeof(double) * pp) ||
      hipMalloc(&G, sizeof(double) * pp) || hipMalloc(&queue, sizeof(int) * ppls_gram_queue_ints(P, nmax))) {
    printf("alloc failed\n");
    return 1;
  }
  hipLaunchKernelGGL(lab_fill, dim3(4096), dim3(256), 0, 0, X, (int64_t)n * P, 12345ull);
  (void)hipDeviceSynchronize();
  const double flops = 2.0 * n * ntiles * 128.0 * 128.0, useful = (double)n * P * (P + 1.0);
  printf("n=%lld P=%d baseline nsplit=%d auto nsplit=%d tiles=%d slots=%d wave slots=%d\n", (long long)n, P, nsplit,
         nauto, ntiles, slots, wave_slots);
  auto report = [&](const char* name, float ms, int check) {   // check: 0 none, 1 bitwise, 2 1e-13 relative
    const char* verdict = "";
    if (check) {
      std::vector<double> a(pp), b(pp);
      (void)hipMemcpy(a.data(), Gref, sizeof(double) * pp, hipMemcpyDeviceToHost);
      (void)hipMemcpy(b.data(), G, sizeof(double) * pp, hipMemcpyDeviceToHost);
      double mx = 0.0, dmax = 0.0;
      bool same = true;
      for (size_t e = 0; e < pp; ++e) {
        mx = fmax(mx, fabs(a[e]));
        dmax = fmax(dmax, fabs(a[e] - b[e]));
        same = same && !memcmp(&a[e], &b[e], 8);
      }
      verdict = check == 1 ? (same ? "bitwise = baseline" : "DIFFERS from baseline")
                           : (dmax <= 1e-13 * mx ? "= baseline to 1e-13" : "DIFFERS from baseline");
      printf("  max |diff| / max |G| = %.2e\n", dmax / mx);
    }
    printf("%-44s %9.2f ms  tile flops %6.2f TF/s  useful %6.2f TF/s  %s\n", name, ms, flops / ms / 1e9, useful / ms / 1e9,
           verdict);
    fflush(stdout);
  };
  const int64_t grid = (work + 7) / 8 * 8;
  float ms = timeit([&] {
    hipLaunchKernelGGL((lab_lds_gram_mfma_kernel<double, false, false>), dim3((unsigned)grid), dim3(256), 0, 0, X, P, P,
                       (const double*)nullptr, 0, 0, n, P, ntiles, nsplit, work, part_ref, (int64_t)pp, (int*)nullptr,
                       LabCols{P, P, P, P});
  }, reps);
  hipLaunchKernelGGL(lab_lds_finish, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, 0, part_ref, nsplit, (int64_t)pp, P,
                     Gref);
  (void)hipDeviceSynchronize();
  report("LDS-staged, one item per workgroup (round 4)", ms, 0);
  for (int req : {nsplit, 0}) {
    (void)ppls_gram_queue_prepare(queue, P, P, P, 0, n, wave_slots, req, 0);
    const int ns = ppls_gram_plan(P, P, P, 0, n, wave_slots, req, nullptr);
    ms = timeit([&] { (void)ppls_launch_gram_joint(X, P, P, P, nullptr, 0, 0, 0, 0, n, P, ns, part, queue, 0); }, reps);
    (void)ppls_launch_gram_finish(part, ns, P, P, P, 0, G, 0);
    (void)hipDeviceSynchronize();
    char name[96];
    snprintf(name, sizeof name, "LDS-free waves, queues, %d %s splits", ns, req ? "equal" : "halving");
    report(name, ms, req ? 1 : 2);
  }
  return 0;
}
