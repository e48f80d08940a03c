// Microbenchmark + correctness check (tuning aid, not product code) of the
// 128 x 64-wave-tile bf16 GEMM (csrc/gemm_hw.h) against the product's bf16
// kernels (gemm_h16i_kernel for RK A operands, gemm_h16_kernel for KR) on the
// C5 shapes.  Operands: pseudo-random uniform fp32 rounded to bf16; reference:
// the exact-fp32 MFMA kernel on the rounded values.  Kernels timed
// interleaved in one process (cdna_hip_programming.md rule 24).
//   ./hw_bench [case-substring]    env HW_EPI=1: the dX epilogue (EluGrad, colsums, twin)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../distributed_ddpg_amd/csrc/gemm_f32.h"
#include "../distributed_ddpg_amd/csrc/gemm_h3.h"
#include "../distributed_ddpg_amd/csrc/gemm_hw.h"

using namespace ddpg;

// gemm_h16i_kernel with the spread-read schedule (SPR = 1)
template <int AL, int BL>
__global__ __launch_bounds__(HG_NT, 1) void h16i_spr_kernel(GemmHArgs g) {
  gemm_h16i_body<AL, BL, 1>(g, blockIdx.z);
}

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ void round_kernel(float* x, size_t n, __bf16* dst) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const __bf16 h = (__bf16)x[i];
  dst[i] = h;
  x[i] = (float)h;
}

template <typename F>
static float time_it(F launch, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 3; ++i) launch();
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int round = 0; round < 5; ++round) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipGetLastError());
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    best = std::min(best, 1e3f * ms / reps);
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return best;
}

struct Case {
  const char* name;
  int al, bl, M, N, K;
};

static float *gA, *gB, *gC, *gR, *gCs, *gBias;
static __bf16 *hA, *hB, *gTw;

static double check(const float* ref, const float* out, size_t nc) {
  double maxref = 0, maxerr = 0;
  for (size_t i = 0; i < nc; ++i) {
    maxref = std::max(maxref, (double)fabs(ref[i]));
    maxerr = std::max(maxerr, fabs((double)out[i] - ref[i]));
  }
  return maxerr / maxref;
}

template <int AL, int BL>
static void run_case(const Case& c) {
  const size_t na = (size_t)c.M * c.K, nb = (size_t)c.K * c.N, nc = (size_t)c.M * c.N;
  std::vector<float> h(std::max(na, nb));
  for (size_t i = 0; i < na; ++i) h[i] = (float)((i * 2654435761u) % 1000003) / 1000003.f - 0.5f;
  CHECK(hipMemcpy(gA, h.data(), na * 4, hipMemcpyHostToDevice));
  for (size_t i = 0; i < nb; ++i) h[i] = (float)((i * 40503u + 17) % 999983) / 999983.f - 0.5f;
  CHECK(hipMemcpy(gB, h.data(), nb * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(round_kernel, dim3((na + 255) / 256), dim3(256), 0, 0, gA, na, hA);
  hipLaunchKernelGGL(round_kernel, dim3((nb + 255) / 256), dim3(256), 0, 0, gB, nb, hB);
  CHECK(hipGetLastError());
  const int lda = AL == L_RK ? c.K : c.M, ldb = BL == L_RK ? c.K : c.N;
  GemmArgs r;
  memset(&r, 0, sizeof r);
  r.A = gA;
  r.B = gB;
  r.M = c.M;
  r.N = c.N;
  r.K = c.K;
  r.lda = lda;
  r.ldb = ldb;
  r.kps = c.K;
  r.e.out = gR;
  r.e.ldo = c.N;
  hipLaunchKernelGGL((gemm_f32_kernel<AL, BL, 4, 4, 128, 128>),
                     dim3((c.N + 127) / 128, (c.M + 127) / 128, 1), dim3(GNT), 0, 0, r);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  std::vector<float> ref(nc), out(nc);
  CHECK(hipMemcpy(ref.data(), gR, nc * 4, hipMemcpyDeviceToHost));

  const char* ev = getenv("HW_EPI");
  const bool epi = ev && atoi(ev) && AL == L_RK && BL == L_RK;
  GemmHArgs g;
  memset(&g, 0, sizeof g);
  g.A = hA;
  g.B = hB;
  g.M = c.M;
  g.N = c.N;
  g.K = c.K;
  g.lda = lda;
  g.ldb = ldb;
  g.kps = c.K;
  g.xcd = 1;
  g.e.out = gC;
  g.e.ldo = c.N;
  if (epi) {  // the dX epilogue: EluGrad factor of aux, bias column sums, bf16 twin
    g.e.post = 1;
    g.e.aux = gA;
    g.e.ldaux = c.N;
    g.e.colsum = gCs;
    g.e.ld_colsum = c.N;
    g.e.outh = gTw;
    g.e.h_plane_stride = (long long)nc;
    g.e.h_planes = 1;
  }
  // first-layer cases (K = 384): the forward epilogue (bias, elu, bf16 twin only)
  const bool l1 = c.K == 384;
  if (l1) {
    g.e.bias = gBias;
    g.e.act = 1;
    g.e.out = nullptr;
    g.e.outh = gTw;
    g.e.h_plane_stride = (long long)nc;
    g.e.h_planes = 1;
  }
  auto fprod = [&] {
    dim3 grid((c.N + 127) / 128, (c.M + 255) / 256, 1);
    if constexpr (AL == L_RK)
      hipLaunchKernelGGL((gemm_h16i_kernel<AL, BL>), grid, dim3(HG_NT), 0, 0, g);
    else
      hipLaunchKernelGGL((gemm_h16_kernel<AL, BL, 1, 256, 64>), grid, dim3(HG_NT), 0, 0, g);
  };
  auto f128 = [&] {
    hipLaunchKernelGGL((gemm_hw_kernel<AL, BL, 128, 4, 0, -1, false>), dim3(c.N / 128, (c.M + 255) / 256, 1),
                       dim3(HwCfg<128, 4>::NT), 0, 0, g);
  };
  // variant 3: gemm_h16i_kernel with spread fragment reads (RK A only)
  auto f256 = [&] {
    if constexpr (AL == L_RK)
      hipLaunchKernelGGL((h16i_spr_kernel<AL, BL>), dim3((c.N + 127) / 128, (c.M + 255) / 256, 1),
                         dim3(HG_NT), 0, 0, g);
  };
  const double flop = 2.0 * c.M * c.N * (double)c.K;
  for (int rep = 0; rep < 2; ++rep) {
    float us[3];
    double err[3];
    const char* nm[3] = {"prod", "hw128", "spr"};
    for (int v = 0; v < 3; ++v) {
      CHECK(hipMemset(gC, 0, nc * 4));
      us[v] = v == 0 ? time_it(fprod, 10) : v == 1 ? time_it(f128, 10) : time_it(f256, 10);
      CHECK(hipMemcpy(out.data(), gC, nc * 4, hipMemcpyDeviceToHost));
      err[v] = (epi || l1) ? -1.0 : check(ref.data(), out.data(), nc);
    }
    printf("%-16s M=%d N=%d K=%d %s", c.name, c.M, c.N, c.K, epi ? "EPI" : "   ");
    for (int v = 0; v < 3; ++v)
      printf(" | %s %7.2f us %6.1f TF err %.1e", nm[v], us[v], flop / (us[v] * 1e-6) / 1e12,
             err[v]);
    printf(" | hw128 %.2fx spr %.2fx\n", us[0] / us[1], us[0] / us[2]);
    fflush(stdout);
  }
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  const size_t maxe = (size_t)16384 * 2048;
  CHECK(hipMalloc(&gA, maxe * 4));
  CHECK(hipMalloc(&gB, maxe * 4));
  CHECK(hipMalloc(&gC, maxe * 4));
  CHECK(hipMalloc(&gR, maxe * 4));
  CHECK(hipMalloc(&hA, maxe * 2));
  CHECK(hipMalloc(&hB, maxe * 2));
  CHECK(hipMalloc(&gTw, maxe * 2));
  CHECK(hipMalloc(&gCs, 64 * 4096 * 4));
  CHECK(hipMalloc(&gBias, 4096 * 4));
  CHECK(hipMemset(gBias, 0, 4096 * 4));
  const Case cases[] = {
      {"c5 l1x4 <RK,KR>", L_RK, L_KR, 16384, 2048, 384},
      {"c5 fwd <RK,KR>", L_RK, L_KR, 4096, 2048, 2048},
      {"c5 fwd <RK,KR>", L_RK, L_KR, 4096, 2048, 4096},
      {"c5 dx <RK,RK>", L_RK, L_RK, 4096, 4096, 2048},
      {"c5 dx <RK,RK>", L_RK, L_RK, 4096, 2048, 2048},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 4096, 2048, 4096},
      {"c5 wgrad dWs <KR,KR>", L_KR, L_KR, 376, 2048, 512},
  };
  for (const Case& c : cases) {
    char full[96];
    snprintf(full, sizeof full, "%s M=%d N=%d K=%d", c.name, c.M, c.N, c.K);
    if (only && !strstr(full, only)) continue;
    if (c.al == L_RK && c.bl == L_KR) run_case<L_RK, L_KR>(c);
    if (c.al == L_RK && c.bl == L_RK) run_case<L_RK, L_RK>(c);
    if (c.al == L_KR && c.bl == L_KR) run_case<L_KR, L_KR>(c);
  }
  printf("done\n");
  return 0;
}
