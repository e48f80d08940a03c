// Microbenchmark (tuning aid, not product code): where the time of one
// full-size C3 twin-GEMM launch goes.  gemm_h3_kernel<RK,KR> at M = 4096,
// N = 1024, K = 1024 / 2048 (the forward shapes of the C3 step) with three
// epilogues: none (accumulators dropped), the forward epilogue (bias, elu,
// three bf16 planes) and the same plus the fp32 copy.  Per launch: the
// back-to-back event time, and from per-block s_memrealtime stamps (100 MHz)
// the dispatch skew (last block start), the k-loop and the epilogue spans.
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/h3_phase_bench.hip -o tools/h3_phase_bench
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define DDPG_KC_STAMPS 1
#define DDPG_STAMPS8 1
#define DDPG_H3_STAMP_PROLOGUE 1
#include "../distributed_ddpg_amd/csrc/gemm_h3m.h"


using namespace ddpg;

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void split3(const float* x, size_t n, __bf16* dst) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const __bf16 h = (__bf16)v;
  const float r1 = v - (float)h;
  const __bf16 m = (__bf16)r1;
  dst[i] = h;
  dst[n + i] = m;
  dst[2 * n + i] = (__bf16)(r1 - (float)m);
}

template <int KSEL>
void launch(dim3 grid, const GemmHArgs& g) {
  if (KSEL == 16)
    hipLaunchKernelGGL((gemm_h3m_kernel<L_RK, L_KR>), grid, dim3(HG_NT), 0, 0, g);
  else
    hipLaunchKernelGGL((gemm_h3_kernel<L_RK, L_KR>), grid, dim3(HG_NT), 0, 0, g);
}
#define KERN_LAUNCH(grid, g) (ksel == 16 ? launch<16>(grid, g) : launch<32>(grid, g))

int main(int argc, char** argv) {
  const bool one = argc > 1 && atoi(argv[1]) > 0;  // one K (argv[1]), no epilogue: the ablation builds
  const int ksel = argc > 2 ? atoi(argv[2]) : 32;   // 32: gemm_h3_kernel, 16: gemm_h3m_kernel
  const int M = 4096, N = 1024, KMAX = 4096;
  std::vector<float> ha((size_t)M * KMAX), hb((size_t)KMAX * N), hbias(N);
  srand(1);
  for (auto& v : ha) v = (rand() / (float)RAND_MAX) * 2.f - 1.f;
  for (auto& v : hb) v = ((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.03f;
  for (auto& v : hbias) v = (rand() / (float)RAND_MAX) * 0.1f;
  float *da, *db, *dbias, *out;
  __bf16 *ta, *tb, *outh;
  CHECK(hipMalloc(&da, ha.size() * 4));
  CHECK(hipMalloc(&db, hb.size() * 4));
  CHECK(hipMalloc(&dbias, N * 4));
  CHECK(hipMalloc(&ta, ha.size() * 6));
  CHECK(hipMalloc(&tb, hb.size() * 6));
  CHECK(hipMalloc(&out, (size_t)M * N * 4));
  CHECK(hipMalloc(&outh, (size_t)M * N * 6));
  unsigned long long* stamps;
  CHECK(hipMalloc(&stamps, 1024 * 8 * 8));
  CHECK(hipMemcpy(da, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dbias, hbias.data(), N * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(split3, dim3((ha.size() + 255) / 256), dim3(256), 0, 0, da, ha.size(), ta);
  hipLaunchKernelGGL(split3, dim3((hb.size() + 255) / 256), dim3(256), 0, 0, db, hb.size(), tb);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  if (argc > 1 && atoi(argv[1]) == 0) {
    // correctness: both kernels, K = 2048, bias + elu + fp32 out, against a
    // double reference on 64 rows (the h/m/l planes reconstruct the fp32 inputs)
    const int K = 2048, R = 64;
    std::vector<float> o32((size_t)M * N), o16((size_t)M * N);
    for (int ks : {32, 16}) {
      GemmHArgs g;
      memset(&g, 0, sizeof g);
      g.A = ta; g.B = tb; g.pa = (long long)ha.size(); g.pb = (long long)hb.size();
      g.M = M; g.N = N; g.K = K; g.lda = K; g.ldb = N; g.kps = K; g.xcd = 1;
      g.e.ldo = N; g.e.bias = dbias; g.e.act = 1; g.e.out = out;
      g.e.outh = outh; g.e.h_plane_stride = (long long)M * N; g.e.h_planes = 3;
      CHECK(hipMemset(out, 0, (size_t)M * N * 4));
      if (ks == 16) launch<16>(dim3(N / 128, M / 128), g); else launch<32>(dim3(N / 128, M / 128), g);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(ks == 16 ? o16.data() : o32.data(), out, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    }
    double e32 = 0, e16 = 0, mx = 0, d = 0;
    for (int r = 0; r < R; ++r) {
      const int m = r * (M / R) + (r % 7);
      for (int n = 0; n < N; ++n) {
        double acc = hbias[n];
        for (int k = 0; k < K; ++k) acc += (double)ha[(size_t)m * K + k] * hb[(size_t)k * N + n];
        const double y = acc < 0 ? expm1(acc) : acc;
        mx = std::max(mx, fabs(y));
        e32 = std::max(e32, fabs(o32[(size_t)m * N + n] - y));
        e16 = std::max(e16, fabs(o16[(size_t)m * N + n] - y));
      }
    }
    for (size_t i = 0; i < o32.size(); ++i) d = std::max(d, (double)fabs(o32[i] - o16[i]));
    printf("check K=2048 bias+elu: max|ref| %.3f  gemm_h3 err %.3e  gemm_h3m err %.3e  (rel %.2e / %.2e)  "
           "max|h3 - h3m| over all %.3e\n", mx, e32, e16, e32 / mx, e16 / mx, d);
    return 0;
  }
  static const char* en[3] = {"no epilogue      ", "bias+elu+3 planes", "  + fp32 copy    "};
  for (int K : {256, 512, 1024, 2048, 4096}) {
    if (one && K != atoi(argv[1])) continue;
    for (int epi = 0; epi < (one ? 1 : 2); ++epi) {
      GemmHArgs g;
      g.A = ta;
      g.B = tb;
      g.pa = (long long)ha.size();
      g.pb = (long long)hb.size();
      g.M = M;
      g.N = N;
      g.K = K;
      g.lda = K;
      g.ldb = N;
      g.kps = K;
      g.xcd = 1;
      memset(&g.e, 0, sizeof g.e);
      g.e.ldo = N;
      if (epi >= 1) {
        g.e.bias = dbias;
        g.e.act = 1;
        g.e.outh = outh;
        g.e.h_plane_stride = (long long)M * N;
        g.e.h_planes = 3;
      }
      if (epi == 2) g.e.out = out;
      const dim3 grid(N / 128, M / 128, 1);
      for (int i = 0; i < 5; ++i)
        KERN_LAUNCH(grid, g);
      CHECK(hipDeviceSynchronize());
      const int reps = 50;
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i)
        KERN_LAUNCH(grid, g);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      // stamped launches right behind a normal one (the same back-to-back state)
      const int nb = grid.x * grid.y;
      double skew = 0, pro = 0, loop = 0, lmin = 1e30, lmax = 0, epis = 0, span = 0, lend = 0;
      double cyc = 0, clk = 0;
      const int sreps = 5;
      for (int r = 0; r < sreps; ++r) {
        CHECK(hipMemset(stamps, 0, (size_t)nb * 8 * 8));
        KERN_LAUNCH(grid, g);
        g.stamps = stamps;
        KERN_LAUNCH(grid, g);
        g.stamps = nullptr;
        CHECK(hipDeviceSynchronize());
        std::vector<unsigned long long> st((size_t)nb * 8);
        CHECK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t00 = ~0ull, s0max = 0, tend = 0;
        for (int b = 0; b < nb; ++b) {
          t00 = std::min(t00, st[b * 8]);
          s0max = std::max(s0max, st[b * 8]);
          tend = std::max(tend, st[b * 8 + 3]);
        }
        skew += (double)(s0max - t00);
        span += (double)(tend - t00);
        double le = 0;
        for (int b = 0; b < nb; ++b) {
          const unsigned long long* q = &st[b * 8];
          const double l = (double)(q[1] - q[2]);  // k-loop after the prologue (realtime)
          const double lc = (double)(q[5] - q[6]);  // same, shader cycles
          pro += (double)(q[2] - q[0]);
          loop += l;
          cyc += lc;
          clk += lc / l / 10.0;  // GHz (realtime ticks are 10 ns)
          lmin = std::min(lmin, l);
          lmax = std::max(lmax, l);
          epis += (double)(q[3] - q[1]);
          le = std::max(le, (double)(q[1] - t00));
        }
        lend += le;
      }
      const double us = 1e3 * ms / reps, fl = 2.0 * M * N * K;
      const int nk = K / 32;
      printf("K=%d %s %7.2f us/launch (%.0f TF-eq, %.3f of 417) | start skew %.2f, prologue %.2f, "
             "k-loop %.2f us [%.2f..%.2f] = %.0f cyc/k-tile at %.2f GHz (MFMA-bound 1536), "
             "epilogue %.2f, span %.2f\n",
             K, en[epi], us, fl / us * 1e-6, fl / us * 1e-6 / 417, skew / sreps / 100,
             pro / nb / sreps / 100, loop / nb / sreps / 100, lmin / 100, lmax / 100,
             cyc / nb / sreps / (nk - 1), clk / nb / sreps, epis / nb / sreps / 100,
             span / sreps / 100);
      fflush(stdout);
    }
  }
  return 0;
}
