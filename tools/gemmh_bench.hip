// Microbenchmark + correctness check (tuning aid, not product code) of the
// bf16-operand GEMM (gemm_h.h) on the learner's C3 / C5 shapes.  Operands are
// random fp32, split into NP bf16 planes on the device; the reference is the
// exact-fp32 MFMA kernel (gemm_f32.h) on the same values (for NP = 1: on the
// bf16-rounded values), so the reported error is the accumulation-order /
// plane-truncation difference only.  Every launch is checked.
//   ./gemmh_bench [case-substring]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../distributed_ddpg_amd/csrc/gemm_f32.h"
#include "../distributed_ddpg_amd/csrc/gemm_h.h"

using namespace ddpg;

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

// x -> NP planes (dst, plane stride n); NP = 1 also rounds x to bf16 in place
__global__ void split_kernel(float* x, size_t n, __bf16* dst, int np) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const __bf16 h = (__bf16)v;
  dst[i] = h;
  if (np == 3) {
    const float r1 = v - (float)h;
    const __bf16 m = (__bf16)r1;
    dst[n + i] = m;
    dst[2 * n + i] = (__bf16)(r1 - (float)m);
  } else {
    x[i] = (float)h;
  }
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
  int al, bl, np, M, N, K, splits;
};

static float *gA, *gB, *gC, *gR, *gBias;
static __bf16 *hA, *hB, *gTw;

template <int AL, int BL, int NP, int BM, int BK, int MF, int SCH = 0, int WGN = 4>
static void run_case(const Case& c) {
  const size_t na = (size_t)c.M * c.K, nb = (size_t)c.K * c.N, nc = (size_t)c.M * c.N;
  // fresh operands (NP = 1 rounds them), planes
  std::vector<float> h(std::max(na, nb));
  for (size_t i = 0; i < na; ++i) h[i] = (float)((i * 2654435761u) % 1000003) / 1000003.f - 0.5f;
  CHECK(hipMemcpy(gA, h.data(), na * 4, hipMemcpyHostToDevice));
  for (size_t i = 0; i < nb; ++i) h[i] = (float)((i * 40503u + 17) % 999983) / 999983.f - 0.5f;
  CHECK(hipMemcpy(gB, h.data(), nb * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(split_kernel, dim3((na + 255) / 256), dim3(256), 0, 0, gA, na, hA, NP);
  hipLaunchKernelGGL(split_kernel, dim3((nb + 255) / 256), dim3(256), 0, 0, gB, nb, hB, NP);
  CHECK(hipGetLastError());
  const int lda = AL == L_RK ? c.K : c.M, ldb = BL == L_RK ? c.K : c.N;
  // reference: exact fp32 MFMA, no split
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

  GemmHArgs g;
  memset(&g, 0, sizeof g);
  g.A = hA;
  g.B = hB;
  g.pa = (long long)na;
  g.pb = (long long)nb;
  g.M = c.M;
  g.N = c.N;
  g.K = c.K;
  g.lda = lda;
  g.ldb = ldb;
  g.kps = c.K / c.splits;
  g.xcd = 1;
  g.e.out = gC;
  g.e.ldo = c.N;
  g.e.out_split_stride = (long long)nc;
  // env GH_EPI (unsplit cases): 1 = fp32 out + bf16 twin (NP planes) + bias + elu
  // (the learner's forward epilogue), 2 = the twin only + bias + elu
  const char* ev = getenv("GH_EPI");
  const int epi = (ev && c.splits == 1) ? atoi(ev) : 0;
  if (epi) {
    g.e.bias = gBias;
    g.e.act = 1;
    g.e.outh = gTw;
    g.e.h_plane_stride = (long long)nc;
    g.e.h_planes = NP;
    if (epi == 2) g.e.out = nullptr;
  }
  dim3 grid((c.N + HG_BN - 1) / HG_BN, (c.M + BM - 1) / BM, c.splits);
  auto f = [&] {
    if constexpr (MF == 16)
      hipLaunchKernelGGL((gemm_h16_kernel<AL, BL, NP, BM, BK, SCH>), grid, dim3(HG_NT), 0, 0, g);
    else
      hipLaunchKernelGGL((gemm_h_kernel<AL, BL, NP, BM, BK, SCH, WGN>), grid, dim3(128 * WGN), 0, 0, g);
  };
  const float us = time_it(f, 10);
  if (epi) {  // elu'd outputs: timing only
    printf("%-26s MF%d S%d W%d NP=%d BM=%d BK=%d M=%d N=%d K=%d s=%d EPI%d  %8.2f us %7.1f TF\n", c.name,
           MF, SCH, WGN, NP, BM, BK, c.M, c.N, c.K, c.splits, epi, us,
           2.0 * c.M * c.N * (double)c.K / (us * 1e-6) / 1e12);
    fflush(stdout);
    return;
  }
  // check: sum the split slabs on the host
  std::vector<float> out(nc * c.splits), ref(nc);
  CHECK(hipMemcpy(out.data(), gC, nc * c.splits * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(ref.data(), gR, nc * 4, hipMemcpyDeviceToHost));
  double maxref = 0, maxerr = 0;
  for (size_t i = 0; i < nc; ++i) {
    double s = 0;
    for (int z = 0; z < c.splits; ++z) s += out[z * nc + i];
    maxref = std::max(maxref, (double)fabs(ref[i]));
    maxerr = std::max(maxerr, fabs(s - ref[i]));
  }
  // fp64 reference on a sample of outputs (inputs as the kernels saw them)
  std::vector<float> ha(na), hb(nb);
  CHECK(hipMemcpy(ha.data(), gA, na * 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(hb.data(), gB, nb * 4, hipMemcpyDeviceToHost));
  double e64h = 0, e64r = 0, m64 = 0;
  for (int sidx = 0; sidx < 2048; ++sidx) {
    const size_t i = ((size_t)sidx * 2654435761u) % nc;
    const int m = (int)(i / c.N), n = (int)(i % c.N);
    double d = 0;
    for (int k = 0; k < c.K; ++k) {
      const double a = AL == L_RK ? ha[(size_t)m * lda + k] : ha[(size_t)k * lda + m];
      const double b = BL == L_RK ? hb[(size_t)n * ldb + k] : hb[(size_t)k * ldb + n];
      d += a * b;
    }
    double s = 0;
    for (int z = 0; z < c.splits; ++z) s += out[z * nc + i];
    m64 = std::max(m64, fabs(d));
    e64h = std::max(e64h, fabs(s - d));
    e64r = std::max(e64r, fabs((double)ref[i] - d));
  }
  const double flop = 2.0 * c.M * c.N * (double)c.K;
  const double tf = flop / (us * 1e-6) / 1e12;
  const double peak = NP == 3 ? 2500.0 / 6 : 2500.0;
  printf("%-26s MF%d S%d W%d NP=%d BM=%d BK=%d M=%d N=%d K=%d s=%d  %8.2f us %7.1f TF (%5.1f%% of %.0f)  "
         "vs f32 %.2e | vs f64: gemm_h %.2e, f32 MFMA %.2e | out %.9e\n",
         c.name, MF, SCH, WGN, NP, BM, BK, c.M, c.N, c.K, c.splits, us, tf, 100.0 * tf / peak, peak,
         maxerr / maxref, e64h / m64, e64r / m64, (double)out[nc / 3 + 7]);
  fflush(stdout);
}

template <int NP, int BM, int BK, int MF, int SCH = 0, int WGN = 4>
static void dispatch1(const Case& c) {
  if (c.al == L_RK && c.bl == L_KR) run_case<L_RK, L_KR, NP, BM, BK, MF, SCH, WGN>(c);
  if (c.al == L_RK && c.bl == L_RK) run_case<L_RK, L_RK, NP, BM, BK, MF, SCH, WGN>(c);
  if (c.al == L_KR && c.bl == L_KR) run_case<L_KR, L_KR, NP, BM, BK, MF, SCH, WGN>(c);
}
// the 32x32x16 kernel (both schedules) and the 16x16x32 kernel on the same
// case, interleaved
template <int NP, int BM, int BK>
static void dispatch(const Case& c) {
  for (int rep = 0; rep < 2; ++rep) {
    dispatch1<NP, BM, BK, 32, 0>(c);
    dispatch1<NP, BM, BK, 32, 1>(c);
    // env GH_W2=1: also the 4-wave form (WGN = 2, wave tile BM/2 x 64)
    if (getenv("GH_W2") && atoi(getenv("GH_W2"))) {
      dispatch1<NP, BM, BK, 32, 0, 2>(c);
      dispatch1<NP, BM, BK, 32, 1, 2>(c);
    }
    if constexpr (NP == 1) {
      dispatch1<NP, BM, BK, 16, 0>(c);
      dispatch1<NP, BM, BK, 16, 1>(c);
    }
  }
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;
  const size_t maxe = (size_t)4096 * 4096;
  CHECK(hipMalloc(&gA, maxe * 4));
  CHECK(hipMalloc(&gB, maxe * 4));
  CHECK(hipMalloc(&gC, maxe * 4 * 8));
  CHECK(hipMalloc(&gR, maxe * 4));
  CHECK(hipMalloc(&hA, maxe * 2 * 3));
  CHECK(hipMalloc(&hB, maxe * 2 * 3));
  CHECK(hipMalloc(&gTw, maxe * 2 * 3));
  CHECK(hipMalloc(&gBias, 4096 * 4));
  CHECK(hipMemset(gBias, 0, 4096 * 4));
  const Case cases[] = {
      // C5 (bf16): forward, dX, weight gradients
      {"c5 first fwd <RK,KR>", L_RK, L_KR, 1, 4096, 2048, 384, 1},
      {"c5 fwd <RK,KR>", L_RK, L_KR, 1, 4096, 2048, 2048, 1},
      {"c5 fwd <RK,KR>", L_RK, L_KR, 1, 4096, 2048, 4096, 1},
      {"c5 dx <RK,RK>", L_RK, L_RK, 1, 4096, 4096, 2048, 1},
      {"c5 dx <RK,RK>", L_RK, L_RK, 1, 4096, 2048, 2048, 1},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 1, 4096, 2048, 4096, 1},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 1, 2048, 2048, 4096, 2},
      {"c5 wgrad <KR,KR>", L_KR, L_KR, 1, 376, 2048, 4096, 8},
      // C3 (fp32 via three planes)
      {"c3 fwd <RK,KR>", L_RK, L_KR, 3, 4096, 1024, 1024, 1},
      {"c3 fwd <RK,KR>", L_RK, L_KR, 3, 4096, 1024, 2048, 1},
      {"c3 dx <RK,RK>", L_RK, L_RK, 3, 4096, 2048, 1024, 1},
      {"c3 dx <RK,RK>", L_RK, L_RK, 3, 4096, 1024, 1024, 1},
      {"c3 wgrad <KR,KR>", L_KR, L_KR, 3, 2048, 1024, 4096, 2},
      {"c3 wgrad <KR,KR>", L_KR, L_KR, 3, 1024, 1024, 4096, 4},
      {"c3 thin fwd <RK,KR>", L_RK, L_KR, 3, 4096, 1024, 64, 1},
      {"c3 thin fwd <RK,KR>", L_RK, L_KR, 3, 4096, 1024, 32, 1},
      {"c3 thin wgrad <KR,KR>", L_KR, L_KR, 3, 64, 1024, 4096, 16},
      {"c3 thin wgrad <KR,KR>", L_KR, L_KR, 3, 64, 1024, 4096, 32},
  };
  // env GH_TILES=1: the bf16 cases on the 16x16x32 kernel at every (BM, BK)
  const bool tiles = getenv("GH_TILES") && atoi(getenv("GH_TILES"));
  for (const Case& c : cases) {
    char full[96];
    snprintf(full, sizeof full, "%s M=%d N=%d K=%d", c.name, c.M, c.N, c.K);
    if (only && !strstr(full, only)) continue;
    if (c.np == 1 && tiles) {
      for (int rep = 0; rep < 2; ++rep) {
        // (BK = 32 builds of the 16x16x32 kernel fail tools/isa_check.py:
        // with one k-step per tile the register sets alternate by tile parity
        // and hipcc copies in-flight fragment registers -- never run them)
        dispatch1<1, 256, 64, 16>(c);
        dispatch1<1, 128, 64, 16>(c);
      }
    } else if (c.np == 1) {
      dispatch<1, 256, 64>(c);
    } else {
      dispatch<3, 128, 32>(c);
    }
  }
  printf("done\n");
  return 0;
}
