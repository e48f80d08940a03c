// Microbenchmark (tuning aid, not product code): the learner's bf16-pipe GEMM
// kernels on the C3 / C5 shapes, plain epilogue (store only), timed back to
// back with events (min over 7 rounds).  Every launch is checked
// (hipGetLastError after each timed batch).  With -DWITH_OLD it also times
// build_variants/gemm_s3_old.h (a snapshot of an earlier gemm_s3.h, made by
// tools/snapshot_s3.sh) and compares the two kernels' outputs bit for bit.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../distributed_ddpg_amd/csrc/gemm_s3.h"
#ifdef WITH_OLD
#include "../build_variants/gemm_s3_old.h"
#endif

using namespace ddpg;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

template <typename F>
static float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int round = 0; round < 7; ++round) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipGetLastError());
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, 1e3f * ms / reps);
  }
  return best;
}

static void report(const char* tag, int M, int N, int K, float us, double peak) {
  const double tf = 2.0 * M * N * (double)K / (us * 1e-6) / 1e12;
  printf("%-36s M=%d N=%d K=%d  %8.2f us  %7.1f TF  (%.1f%% of %.0f)\n", tag, M, N, K, us, tf,
         100.0 * tf / peak, peak);
  fflush(stdout);
}

static void compare(const float* C, const float* C2, size_t n, const char* what) {
  std::vector<float> h1(n), h2(n);
  CHECK(hipMemcpy(h1.data(), C, n * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(h2.data(), C2, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += memcmp(&h1[i], &h2[i], 4) != 0;
  printf("    %s: %zu of %zu outputs differ\n", what, bad, n);
}

struct Case {
  const char* name;
  int al, bl, M, N, K, splits;
};

template <int AL, int BL, int NP>
static void run_case(const Case& c, const float* A, const float* B, float* C, float* C2) {
  GemmArgs g;
  memset(&g, 0, sizeof g);
  g.M = c.M;
  g.N = c.N;
  g.K = c.K;
  g.kps = c.K / c.splits;
  g.xcd = 1;
  g.e.out = C;
  g.e.ldo = c.N;
  g.e.out_split_stride = (long long)c.M * c.N;
  g.A = A;
  g.lda = AL == L_RK ? c.K : c.M;
  g.B = B;
  g.ldb = BL == L_RK ? c.K : c.N;
  dim3 grid(c.N / 128, c.M / 128, c.splits);
  const double peak = NP == 3 ? 2500.0 / 6 : 2500.0;
  char tag[96];
  snprintf(tag, sizeof tag, "%s NP=%d", c.name, NP);
  auto f = [&] { hipLaunchKernelGGL((gemm_s3_kernel<AL, BL, NP>), grid, dim3(S3_NT), 0, 0, g); };
  report(tag, c.M, c.N, c.K, time_it(f, 20), peak);
#ifdef WITH_OLD
  g.e.out = C2;
  auto fo = [&] { hipLaunchKernelGGL((gemm_s3old_kernel<AL, BL, NP>), grid, dim3(S3O_NT), 0, 0, g); };
  snprintf(tag, sizeof tag, "  old %s NP=%d", c.name, NP);
  report(tag, c.M, c.N, c.K, time_it(fo, 20), peak);
  compare(C, C2, (size_t)c.M * c.N * c.splits, "new vs old");
#endif
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;  // run only cases whose name contains it
  const size_t maxe = (size_t)4096 * 4096;
  float *A, *B, *C, *C2;
  CHECK(hipMalloc(&A, maxe * 4));
  CHECK(hipMalloc(&B, maxe * 4));
  CHECK(hipMalloc(&C, maxe * 4 * 2));
  CHECK(hipMalloc(&C2, maxe * 4 * 2));
  std::vector<float> h(maxe);
  for (size_t i = 0; i < h.size(); ++i)
    h[i] = (float)((i * 2654435761u) % 1000003) / 1000003.f - 0.5f;
  CHECK(hipMemcpy(A, h.data(), maxe * 4, hipMemcpyHostToDevice));
  std::reverse(h.begin(), h.end());
  CHECK(hipMemcpy(B, h.data(), maxe * 4, hipMemcpyHostToDevice));
  const Case cases[] = {
      {"fwd K=1024 <RK,KR>", L_RK, L_KR, 4096, 1024, 1024, 1},
      {"fwd K=2048 <RK,KR>", L_RK, L_KR, 4096, 1024, 2048, 1},
      {"dx  N=2048 <RK,RK>", L_RK, L_RK, 4096, 2048, 1024, 1},
      {"dx  K=1024 <RK,RK>", L_RK, L_RK, 4096, 1024, 1024, 1},
      {"wgrad 2048x1024 K=4096/4 <KR,KR>", L_KR, L_KR, 2048, 1024, 4096, 4},
      {"wgrad 1024x1024 K=4096/8 <KR,KR>", L_KR, L_KR, 1024, 1024, 4096, 8},
  };
  for (const Case& c : cases) {
    if (only && !strstr(c.name, only)) continue;
    if (c.al == L_RK && c.bl == L_KR) run_case<L_RK, L_KR, 3>(c, A, B, C, C2);
    if (c.al == L_RK && c.bl == L_RK) run_case<L_RK, L_RK, 3>(c, A, B, C, C2);
    if (c.al == L_KR && c.bl == L_KR) run_case<L_KR, L_KR, 3>(c, A, B, C, C2);
  }
  // bf16 configuration (C5 shapes)
  const Case c5[] = {{"c5 fwd K=2048 <RK,KR>", L_RK, L_KR, 4096, 2048, 2048, 1},
                     {"c5 fwd K=4096 <RK,KR>", L_RK, L_KR, 4096, 2048, 4096, 1}};
  for (const Case& c : c5)
    if (!only || strstr(c.name, only)) run_case<L_RK, L_KR, 1>(c, A, B, C, C2);
  printf("done\n");
  return 0;
}
