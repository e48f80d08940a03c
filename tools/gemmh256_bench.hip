// Microbenchmark + correctness check (tuning aid, not product code) of the
// 256 x 256 bf16 GEMM (csrc/gemm_h256.h) against gemm_h16_kernel (256 x 128)
// on the C5 shapes it takes (N = 4096 dX; split-K weight gradients).  Operands are random fp32 rounded to bf16; the reference
// is the exact-fp32 MFMA kernel on the rounded values.  Every variant's
// output (split slabs summed on the host) is checked; the two kernels are
// timed interleaved in one process (cdna_hip_programming.md rule 24).
//   ./gemmh256_bench [case-substring]     env H2_EPI=1: the dX epilogue (EluGrad, colsums, twin)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../distributed_ddpg_amd/csrc/gemm_f32.h"
#include "../distributed_ddpg_amd/csrc/gemm_h256.h"

using namespace ddpg;

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
  return best;
}

struct Case {
  const char* name;
  int al, bl, M, N, K, splits;  // wgrad: h16 split count (h256: twice as many)
  bool wgrad;                   // split slabs
};

static float *gA, *gB, *gC, *gR, *gBias, *gCs;
static __bf16 *hA, *hB, *gTw;

static double check(const float* ref, const float* out, size_t nc, int slabs) {
  double maxref = 0, maxerr = 0;
  for (size_t i = 0; i < nc; ++i) {
    double s = 0;
    for (int z = 0; z < slabs; ++z) s += out[z * nc + i];
    maxref = std::max(maxref, (double)fabs(ref[i]));
    maxerr = std::max(maxerr, fabs(s - ref[i]));
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
  std::vector<float> ref(nc), out(nc * 8);
  CHECK(hipMemcpy(ref.data(), gR, nc * 4, hipMemcpyDeviceToHost));

  const char* ev = getenv("H2_EPI");
  const bool epi = ev && atoi(ev) && !c.wgrad;
  auto args = [&](int splits) {
    GemmHArgs g;
    memset(&g, 0, sizeof g);
    g.A = hA;
    g.B = hB;
    g.M = c.M;
    g.N = c.N;
    g.K = c.K;
    g.lda = lda;
    g.ldb = ldb;
    g.kps = c.K / splits;
    g.xcd = 1;
    g.e.out = gC;
    g.e.ldo = c.N;
    g.e.out_split_stride = c.wgrad ? (long long)nc : 0;
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
    return g;
  };
  // gemm_h16_kernel (the product's bf16 kernel)
  const int s16 = c.wgrad ? c.splits : 1;
  GemmHArgs g16 = args(s16);
  dim3 grid16((c.N + 127) / 128, (c.M + 255) / 256, s16);
  auto f16 = [&] {
    hipLaunchKernelGGL((gemm_h16_kernel<AL, BL, 1, 256, 64>), grid16, dim3(HG_NT), 0, 0, g16);
  };
  // gemm_h256_kernel: wgrad -> split slabs (MODE 0); plain -> one split (MODE 1)
  const int s2 = c.wgrad ? 2 * c.splits : 1;
  GemmHArgs g2 = args(s2);
  dim3 grid2((c.N + 255) / 256, (c.M + 255) / 256, s2);
  auto f2 = [&] {
    if (c.wgrad)
      hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 0>), grid2, dim3(H2_NT), 0, 0, g2);
    else
      hipLaunchKernelGGL((gemm_h256_kernel<AL, BL, 1>), grid2, dim3(H2_NT), 0, 0, g2);
  };
  const double flop = 2.0 * c.M * c.N * (double)c.K;
  for (int rep = 0; rep < 2; ++rep) {
    CHECK(hipMemset(gC, 0, nc * 4 * 8));
    const float u16 = time_it(f16, 10);
    double e16 = -1;
    if (!epi) {
      CHECK(hipMemcpy(out.data(), gC, nc * s16 * 4, hipMemcpyDeviceToHost));
      e16 = check(ref.data(), out.data(), nc, s16);
    }
    CHECK(hipMemset(gC, 0, nc * 4 * 8));
    const float u2 = time_it(f2, 10);
    double e2 = -1;
    const int sl2 = c.wgrad ? s2 : 1;
    if (!epi) {
      CHECK(hipMemcpy(out.data(), gC, nc * sl2 * 4, hipMemcpyDeviceToHost));
      e2 = check(ref.data(), out.data(), nc, sl2);
    }
    printf("%-22s M=%d N=%d K=%d %s | h16 s=%d %8.2f us %7.1f TF err %.2e | h256 s=%d%s %8.2f us "
           "%7.1f TF err %.2e | %.2fx\n",
           c.name, c.M, c.N, c.K, epi ? "EPI" : "   ", s16, u16, flop / (u16 * 1e-6) / 1e12, e16,
           s2, " ", u2, flop / (u2 * 1e-6) / 1e12, e2, u16 / u2);
    fflush(stdout);
  }
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  const size_t maxe = (size_t)4096 * 4096;
  CHECK(hipMalloc(&gA, maxe * 4));
  CHECK(hipMalloc(&gB, maxe * 4));
  CHECK(hipMalloc(&gC, maxe * 4 * 8));
  CHECK(hipMalloc(&gR, maxe * 4));
  CHECK(hipMalloc(&hA, maxe * 2));
  CHECK(hipMalloc(&hB, maxe * 2));
  CHECK(hipMalloc(&gTw, maxe * 2));
  CHECK(hipMalloc(&gBias, 4096 * 4));
  CHECK(hipMemset(gBias, 0, 4096 * 4));
  CHECK(hipMalloc(&gCs, 64 * 4096 * 4));
  const Case cases[] = {
      {"c5 dx <RK,RK>", L_RK, L_RK, 4096, 4096, 2048, 1, false},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 4096, 2048, 4096, 1, true},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 2048, 2048, 4096, 2, true},
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
