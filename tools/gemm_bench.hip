// Microbenchmark (tuning aid, not product code): the learner's GEMM kernels on
// the C3 shapes, plain epilogue (store only), timed back to back with events.
// Prints avg us and fp32-equivalent TFLOP/s (2 M N K / t) per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
__device__ unsigned long long g_st[4096 * 4];
#define S3_STAMP(i)                                                                          \
  if (threadIdx.x == 0) g_st[(blockIdx.x + gridDim.x * blockIdx.y) * 4 + (i)] = __builtin_amdgcn_s_memtime();
#include "../distributed_ddpg_amd/csrc/gemm_s3.h"
#include <algorithm>
#ifdef WITH_OLD
#include "../build_variants/gemm_s3_old.h"
#endif

// per-phase block averages of the LAST launch (core clocks): prologue, loop, epilogue
static void phases(const char* tag, int nblocks) {
  std::vector<unsigned long long> h(nblocks * 4);
  hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_st), h.size() * 8);
  double d[3] = {0, 0, 0};
  unsigned long long t0 = ~0ull, t3 = 0;
  for (int b = 0; b < nblocks; ++b) {
    const unsigned long long* s = &h[b * 4];
    for (int i = 0; i < 3; ++i) d[i] += double(s[i + 1] - s[i]) / nblocks;
    t0 = std::min(t0, s[0]);
    t3 = std::max(t3, s[3]);
  }
  printf("   %s: span %llu clk; per block: prologue %.0f loop %.0f epilogue %.0f\n", tag, t3 - t0,
         d[0], d[1], d[2]);
}
#ifdef WITH_P3
#include "../distributed_ddpg_amd/csrc/gemm_p3.h"
#endif

using namespace ddpg;

// min over 7 rounds of `reps` back-to-back launches (the box's clocks vary)
template <typename F>
static float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) launch();
  float best = 1e30f;
  for (int round = 0; round < 7; ++round) {
    hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, 1e3f * ms / reps);
  }
  return best;
}

static void report(const char* tag, int M, int N, int K, float us) {
  const double tf = 2.0 * M * N * (double)K / (us * 1e-6) / 1e12;
  printf("%-34s M=%d N=%d K=%d  %8.2f us  %6.1f TF  (%.0f%% of 417)\n", tag, M, N, K, us, tf,
         100.0 * tf / 416.7);
}

int main(int argc, char** argv) {
  const int M = 4096, N = 1024, K = argc > 1 ? atoi(argv[1]) : 1024;
  const bool nostore = argc > 2 && atoi(argv[2]) == 1;
  float *A, *B, *C;
  hipMalloc(&A, (size_t)M * (K + 32) * 4);
  hipMalloc(&B, (size_t)(K + 32) * 2048 * 4);
  hipMalloc(&C, (size_t)M * 2048 * 4);
  std::vector<float> h((size_t)M * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f - 0.5f;
  hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), (size_t)K * 1024 * 4, hipMemcpyHostToDevice);
  GemmArgs g;
  memset(&g, 0, sizeof g);
  g.M = M;
  g.N = N;
  g.K = K;
  g.kps = K;
  g.xcd = 1;
  g.e.out = nostore ? nullptr : C;
  g.e.ldo = N;
  // forward: A = X [M][K] (RK), B = W [K][N] (KR)
  g.A = A;
  g.lda = K;
  g.B = B;
  g.ldb = N;
  dim3 grid(N / 128, M / 128, 1);
  auto f1 = [&] { hipLaunchKernelGGL((gemm_s3_kernel<L_RK, L_KR, 3>), grid, dim3(S3_NT), 0, 0, g); };
  report("s3 fwd <RK,KR,3>", M, N, K, time_it(f1, 20));
  phases("s3 fwd", N / 128 * (M / 128));
  auto f2 = [&] { hipLaunchKernelGGL((gemm_s3_kernel<L_RK, L_KR, 1>), grid, dim3(S3_NT), 0, 0, g); };
  report("bf16 fwd <RK,KR,1>", M, N, K, time_it(f2, 20));
  phases("bf16 fwd", N / 128 * (M / 128));
  // dX: B = W [N][K] (RK)
  g.ldb = K;
  auto f3 = [&] { hipLaunchKernelGGL((gemm_s3_kernel<L_RK, L_RK, 3>), grid, dim3(S3_NT), 0, 0, g); };
  report("s3 dx <RK,RK,3>", M, N, K, time_it(f3, 20));
#ifdef WITH_OLD
  g.ldb = N;
  auto f4 = [&] { hipLaunchKernelGGL((gemm_s3old_kernel<L_RK, L_KR, 3>), grid, dim3(S3O_NT), 0, 0, g); };
  report("OLD s3 fwd <RK,KR,3>", M, N, K, time_it(f4, 20));
  auto f5 = [&] { hipLaunchKernelGGL((gemm_s3old_kernel<L_RK, L_KR, 1>), grid, dim3(S3O_NT), 0, 0, g); };
  report("OLD bf16 fwd <RK,KR,1>", M, N, K, time_it(f5, 20));
  g.ldb = K;
  auto f6 = [&] { hipLaunchKernelGGL((gemm_s3old_kernel<L_RK, L_RK, 3>), grid, dim3(S3O_NT), 0, 0, g); };
  report("OLD s3 dx <RK,RK,3>", M, N, K, time_it(f6, 20));
  // wgrad shape: A = X^T (KR), B = dY (KR), M = N = 1024, K = 4096
  {
    GemmArgs w = g;
    w.M = 1024; w.N = 1024; w.K = 4096; w.kps = 4096; w.lda = 1024; w.ldb = 1024;
    dim3 gw(8, 8, 1);
    auto f7 = [&] { hipLaunchKernelGGL((gemm_s3old_kernel<L_KR, L_KR, 3>), gw, dim3(S3O_NT), 0, 0, w); };
    report("OLD s3 wgrad <KR,KR,3> (64 blk)", 1024, 1024, 4096, time_it(f7, 20));
    auto f8 = [&] { hipLaunchKernelGGL((gemm_s3_kernel<L_KR, L_KR, 3>), gw, dim3(S3_NT), 0, 0, w); };
    report("s3 wgrad <KR,KR,3> (64 blk)", 1024, 1024, 4096, time_it(f8, 20));
  }
#endif
#ifdef WITH_P3
  p3_bench(M, N, K, A, B, C);
#endif
  return 0;
}
