// Microbenchmark (tuning aid, not product code): thin_k_kernel durations at
// the C3 shapes (M = 4096, N = 1024, K = 64 / 16) with parts of its epilogue
// switched off, to see where the time goes.  Prints avg us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
__device__ unsigned long long g_st[8192 * 5];
// per-block phase clocks summed over the row walk: g_ph[b][i] += time since
// the previous stamp of block b, for the stamp i that ends the phase
__device__ unsigned long long g_ph[8192 * 8], g_last[8192];
#define TK_STAMP(i)                                                                        \
  if (threadIdx.x == 0) {                                                                  \
    const int b_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);         \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                            \
    if ((i) < 4) g_st[b_ * 5 + (i)] = t_;                                                      \
    if ((i) > 0) g_ph[b_ * 8 + (i)] += t_ - g_last[b_];                                    \
    g_last[b_] = t_;                                                                       \
  }
#include "../distributed_ddpg_amd/csrc/thin_k.h"
#ifdef WITH_OLD
#include "../build_variants/thin_k_old.h"
#endif
#include <vector>
#include <algorithm>

// per-phase block averages and whole-grid span of the LAST launch (core clocks)
// per-phase clocks summed over each block's row walk, averaged over blocks:
// [1] up to the tile barrier (first trip: W panel + X; later: colsum + next X
// split), [2] MFMAs, [3] accumulators -> LDS + barrier, [4] the epilogue row
// loop (LDS reads, element-wise, store issue)
static void walk(const char* tag, int nblocks) {
  std::vector<unsigned long long> h(nblocks * 8);
  hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_ph), h.size() * 8);
  double d[5] = {0, 0, 0, 0, 0};
  for (int b = 0; b < nblocks; ++b)
    for (int i = 1; i <= 4; ++i) d[i] += double(h[b * 8 + i]) / nblocks;
  printf("   %s walk: to-barrier %.0f mfma %.0f acc->lds %.0f epilogue-loop %.0f clk/block\n", tag,
         d[1], d[2], d[3], d[4]);
}
static void phases(const char* tag, int nblocks) {
  std::vector<unsigned long long> h(nblocks * 5);
  hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_st), h.size() * 8);
  unsigned long long t0 = ~0ull, t3 = 0;
  double d[3] = {0, 0, 0};
  for (int b = 0; b < nblocks; ++b) {
    const unsigned long long* s = &h[b * 5];
    t0 = std::min(t0, s[0]);
    t3 = std::max(t3, s[3]);
    for (int i = 0; i < 3; ++i) d[i] += double(s[i + 1] - s[i]) / nblocks;
  }
  // start-time spread: how late the last block starts
  unsigned long long smax = 0;
  for (int b = 0; b < nblocks; ++b) smax = std::max(smax, h[b * 5] - t0);
  printf("   %s: span %llu clk, last start +%llu, per block: stage %.0f mfma %.0f epi %.0f\n", tag,
         t3 - t0, smax, d[0], d[1], d[2]);
}

using namespace ddpg;

typedef void (*tk_fn)(TkArgs);
static tk_fn g_kern = thin_k_kernel<0>;
static int g_rb = 0;  // row blocks of the kernel under test
static float time_it(const TkArgs& a, int nparts, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  int nmax = std::max(a.p[0].N, nparts > 1 ? a.p[1].N : 0);
  dim3 grid((nmax + TK_COLS - 1) / TK_COLS, g_rb, nparts);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(g_kern, grid, dim3(TK_NT), 0, 0, a);
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(g_kern, grid, dim3(TK_NT), 0, 0, a);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  static std::vector<unsigned long long> z(8192 * 8, 0ull);
  hipMemcpyToSymbol(HIP_SYMBOL(g_ph), z.data(), z.size() * 8);
  hipLaunchKernelGGL(g_kern, grid, dim3(TK_NT), 0, 0, a);  // the launch phases() / walk() read
  hipDeviceSynchronize();
  return 1e3f * ms / reps;
}

static void run_all();
int main() {
  printf("== thin_k_kernel, one row tile per block\n");
  g_rb = 4096 / TK_ROWS;
  run_all();
  printf("== thin_k_kernel, 4 row tiles per block\n");
  g_rb = 4096 / TK_ROWS / 4;
  run_all();
  printf("== thin_k_kernel, 6 row tiles per block\n");
  g_rb = (4096 / TK_ROWS + 5) / 6;
  run_all();
  printf("== thin_k_kernel, 8 row tiles per block\n");
  g_rb = 4096 / TK_ROWS / 8;
  run_all();
#ifdef WITH_OLD
  printf("== old thin_k_kernel\n");
  g_kern = old::thin_k_old_kernel;  // (build_variants/, WITH_OLD only)
  g_rb = 4096 / 64;
  run_all();
#endif
  return 0;
}

static void run_all() {
  const int M = 4096, N = 1024;
  float *X, *W, *bias, *out, *aux, *cs;
  hipMalloc(&X, (size_t)M * 64 * 4);
  hipMalloc(&W, (size_t)64 * N * 4);
  hipMalloc(&bias, N * 4);
  hipMalloc(&out, (size_t)M * 2 * N * 4);
  hipMalloc(&aux, (size_t)M * N * 4);
  hipMalloc(&cs, (size_t)64 * N * 4);
  hipMemset(X, 0, (size_t)M * 64 * 4);
  hipMemset(W, 0, (size_t)64 * N * 4);
  hipMemset(bias, 0, N * 4);
  hipMemset(aux, 0, (size_t)M * N * 4);
  TkPart p;
  memset(&p, 0, sizeof p);
  p.X = X; p.ldx = 64; p.K = 64; p.W = W; p.ldw = N; p.N = N; p.bias = bias; p.act = 1;
  p.out = out; p.ldo = 2 * N;
  TkArgs a;
  memset(&a, 0, sizeof a);
  a.M = M;
  a.mt = M / TK_ROWS;
  a.rpb = (a.mt + g_rb - 1) / g_rb;  // row tiles per block for g_rb row blocks
  a.p[0] = p;
  printf("K64 bias+elu+store           %.2f us\n", time_it(a, 1, 200));
  phases("K64", 8 * g_rb);
  walk("K64", 8 * g_rb);
  {
    __bf16* tw;
    hipMalloc(&tw, (size_t)M * 2 * N * 2 * 3);
    a.p[0].outh = tw;
    a.p[0].hps = (long long)M * 2 * N;
    a.p[0].hnp = 3;
    printf("K64 bias+elu+store+3 planes  %.2f us\n", time_it(a, 1, 200));
    phases("K64 twin", 8 * g_rb);
    a.p[0].out = nullptr;
    printf("K64 bias+elu+3 planes only   %.2f us\n", time_it(a, 1, 200));
    a.p[0] = p;
    hipFree(tw);
  }
  a.p[0].act = 0;
  printf("K64 bias+store (no elu)      %.2f us\n", time_it(a, 1, 200));
  a.p[0].out = nullptr;
  printf("K64 no store                 %.2f us\n", time_it(a, 1, 200));
  phases("K64 nostore", 8 * g_rb);
  a.p[0] = p;
  a.p[0].K = 8;
  a.p[0].ldx = 8;
  printf("K8 bias+elu+store            %.2f us\n", time_it(a, 1, 200));
  phases("K8", 8 * g_rb);
  a.p[0] = p;
  a.p[1] = p;
  a.p[1].out = out + N;
  a.p[1].K = 16; a.p[1].ldx = 16;
  printf("2 parts K64|K16              %.2f us\n", time_it(a, 2, 200));
  {  // the large-batch step's five-part first-layer launch: 3-plane twins only
    __bf16* tw;
    const size_t ne = (size_t)M * N;
    hipMalloc(&tw, ne * 2 * 3 * 5);
    TkPart f = p;
    f.out = nullptr;
    f.ldo = N;
    f.hnp = 3;
    f.hps = (long long)ne * 5;
    for (int i = 0; i < 5; ++i) {
      a.p[i] = f;
      a.p[i].outh = tw + ne * i;
      if (i == 4) { a.p[i].K = 16; a.p[i].ldx = 16; }
    }
    printf("5 parts twin-only K64x4|K16  %.2f us\n", time_it(a, 5, 100));
    phases("5 parts", 8 * g_rb * 5);
    walk("5 parts", 8 * g_rb * 5);
    g_kern = thin_k_kernel<1>;
    printf("5 parts twin-only, FWD form  %.2f us\n", time_it(a, 5, 100));
    walk("5 parts FWD", 8 * g_rb * 5);
    g_kern = thin_k_kernel<0>;
    for (int i = 0; i < 5; ++i) a.p[i].act = 0;
    printf("5 parts twin-only, no elu    %.2f us\n", time_it(a, 5, 100));
    walk("5 parts no elu", 8 * g_rb * 5);
    for (int i = 0; i < 5; ++i) a.p[i].act = 1, a.p[i].outh = nullptr;
    printf("5 parts no store             %.2f us\n", time_it(a, 5, 100));
    walk("5 parts no store", 8 * g_rb * 5);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 50; ++i) hipMemsetAsync(tw, 0, ne * 2 * 3 * 5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("hipMemset 126 MB             %.2f us\n", 1e3f * ms / 50);
    hipFree(tw);
    memset(&a.p, 0, sizeof a.p);
  }
  // dz2: K = 16, w_nk, aux, colsum, no bias / act
  TkPart q = p;
  q.K = 16; q.ldx = 16; q.w_nk = 1; q.ldw = 16; q.bias = nullptr; q.act = 0;
  q.aux = aux; q.ldaux = N; q.ldo = N; q.colsum = cs; q.ld_colsum = N;
  a.p[0] = q;
  printf("dz2 K16 w_nk aux colsum      %.2f us\n", time_it(a, 1, 200));
  // pure write of 16 MB for reference
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 50; ++i) hipMemsetAsync(out, 0, (size_t)M * N * 4);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("hipMemset 16 MB              %.2f us\n", 1e3f * ms / 50);
  hipFree(X); hipFree(W); hipFree(bias); hipFree(out); hipFree(aux); hipFree(cs);
  if (hipGetLastError() != hipSuccess) printf("LAUNCH ERROR\n");
}
