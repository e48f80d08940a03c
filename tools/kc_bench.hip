// Microbenchmark (tuning aid, not product code): the small-M plan's
// in-launch K split (ksplit_combine, gemm_common.h) on gemm_h3_kernel at the
// strong-scaling per-rank shapes of C3: M = 512 / 1024 / 2048 rows, N = 1024,
// K = 1024 / 2048, with the forward epilogue (bias, elu, fp32 out + three
// bf16 planes).  For each shape: unsplit (M/128 x 8 blocks) and S = 2, 3, 4
// splits (skipping any whose partials exceed the buffer, as the product does); prints avg us per launch and checks every split result against
// the unsplit one (max abs diff; the split sums in another order).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/kc_bench.hip -o tools/kc_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <vector>
#define DDPG_KC_STAMPS 1
#include "../distributed_ddpg_amd/csrc/gemm_h3.h"

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

int main() {
  const int N = 1024, KMAX = 2048, MMAX = 2048;
  std::vector<float> ha((size_t)MMAX * KMAX), hb((size_t)KMAX * N), hbias(N);
  srand(1);
  for (auto& v : ha) v = (rand() / (float)RAND_MAX) * 2.f - 1.f;
  for (auto& v : hb) v = ((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.03f;
  for (auto& v : hbias) v = (rand() / (float)RAND_MAX) * 0.1f;
  float *da, *db, *dbias, *out, *ref, *part;
  __bf16 *ta, *tb, *outh;
  unsigned* tick;
  CHECK(hipMalloc(&da, ha.size() * 4));
  CHECK(hipMalloc(&db, hb.size() * 4));
  CHECK(hipMalloc(&dbias, N * 4));
  CHECK(hipMalloc(&ta, ha.size() * 6));
  CHECK(hipMalloc(&tb, hb.size() * 6));
  CHECK(hipMalloc(&out, (size_t)MMAX * N * 4));
  CHECK(hipMalloc(&ref, (size_t)MMAX * N * 4));
  CHECK(hipMalloc(&outh, (size_t)MMAX * N * 6));
  const size_t part_n = (size_t)(256 + 200) * 128 * 128;
  CHECK(hipMalloc(&part, part_n * 4));
  CHECK(hipMalloc(&tick, 1024 * 4));
  unsigned long long* stamps;
  CHECK(hipMalloc(&stamps, 1024 * 4 * 8));
  CHECK(hipMemset(tick, 0, 1024 * 4));
  CHECK(hipMemcpy(da, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dbias, hbias.data(), N * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(split3, dim3((ha.size() + 255) / 256), dim3(256), 0, 0, da, ha.size(), ta);
  hipLaunchKernelGGL(split3, dim3((hb.size() + 255) / 256), dim3(256), 0, 0, db, hb.size(), tb);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  // mode 0: the in-launch combine (forward epilogue); 1: the same splits
  // writing plain fp32 slabs (no combine, no epilogue work: the compute and
  // partial-store floor); 2: one unsplit launch over K / S (the per-block
  // k-slice alone, forward epilogue)
  for (int M : {512, 1024}) {
    for (int K : {1024, 2048}) {
      for (int S0 : {1, 2, 3, 4}) {
        const int nkt = K / 32, kps = (nkt + S0 - 1) / S0 * 32, S = (K + kps - 1) / kps;
        if ((size_t)S * (M / 128) * (N / 128) * 128 * 128 > part_n || S > KC_MAXS) continue;
        for (int mode = 0; mode < (S > 1 ? 3 : 1); ++mode) {
          GemmHArgs g;
          g.A = ta;
          g.B = tb;
          g.pa = (long long)ha.size();
          g.pb = (long long)hb.size();
          g.M = M;
          g.N = N;
          g.K = mode == 2 ? kps : K;
          g.lda = K;  // A [M][K] row-major (RK) -- uses the first M*K of ha's planes
          g.ldb = N;
          g.kps = mode == 2 ? kps : kps;
          g.xcd = 1;
          memset(&g.e, 0, sizeof g.e);
          g.e.out = S == 1 ? ref : mode == 1 ? part : out;
          g.e.ldo = N;
          if (mode != 1) {
            g.e.bias = dbias;
            g.e.act = 1;
            g.e.outh = outh;
            g.e.h_plane_stride = (long long)MMAX * N;
            g.e.h_planes = 3;
          } else {
            g.e.out_split_stride = (long long)M * N;  // S slabs of M x N in the partial buffer
          }
          g.kpart = S > 1 && mode == 0 ? part : nullptr;
          g.kticket = S > 1 && mode == 0 ? tick : nullptr;
          const dim3 grid(N / 128, M / 128, mode == 2 ? 1 : S);
          for (int i = 0; i < 3; ++i)
            hipLaunchKernelGGL((gemm_h3_kernel<L_RK, L_KR>), grid, dim3(HG_NT), 0, 0, g);
          CHECK(hipDeviceSynchronize());
          const int reps = 20;
          CHECK(hipEventRecord(e0));
          for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL((gemm_h3_kernel<L_RK, L_KR>), grid, dim3(HG_NT), 0, 0, g);
          CHECK(hipEventRecord(e1));
          CHECK(hipEventSynchronize(e1));
          float ms;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          double diff = 0;
          if (S > 1 && mode == 0) {
            std::vector<float> a((size_t)M * N), b((size_t)M * N);
            CHECK(hipMemcpy(a.data(), out, a.size() * 4, hipMemcpyDeviceToHost));
            CHECK(hipMemcpy(b.data(), ref, b.size() * 4, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < a.size(); ++i) diff = fmax(diff, fabs((double)a[i] - b[i]));
          }
          // one more launch with phase stamps (s_memrealtime, 100 MHz): per tile,
          // from the launch's first block start: the last split's main-loop end,
          // the combine end and the epilogue end (the tile's last block)
          const int nb = grid.x * grid.y * grid.z;
          CHECK(hipMemset(stamps, 0, (size_t)nb * 4 * 8));
          g.stamps = stamps;
          hipLaunchKernelGGL((gemm_h3_kernel<L_RK, L_KR>), grid, dim3(HG_NT), 0, 0, g);
          CHECK(hipDeviceSynchronize());
          g.stamps = nullptr;
          std::vector<unsigned long long> st((size_t)nb * 4);
          CHECK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
          unsigned long long t00 = ~0ull, tend = 0;
          for (int b = 0; b < nb; ++b) t00 = std::min(t00, st[b * 4]), tend = std::max(tend, st[b * 4 + 3]);
          const int tiles = grid.x * grid.y, sz = grid.z;
          double loop = 0, s0max = 0, lend = 0, cend = 0, eend = 0;
          for (int t = 0; t < tiles; ++t) {
            unsigned long long l = 0, c = 0, e = 0, s0 = 0;
            for (int zz = 0; zz < sz; ++zz) {
              const unsigned long long* q = &st[((size_t)zz * tiles + t) * 4];
              l = std::max(l, q[1]);
              s0 = std::max(s0, q[0]);
              c = std::max(c, q[2]);
              e = std::max(e, q[3]);
              loop += (double)(q[1] - q[0]);
            }
            s0max += (double)(s0 - t00);
            lend += (double)(l - t00);
            cend += (double)(c - t00);
            eend += (double)(e - t00);
          }
          const double us = 1e3 * ms / reps;
          static const char* mn[3] = {"combine", "slabs  ", "k-slice"};
          printf("M=%4d N=%d K=%d S=%d %s blocks=%3d  %7.2f us  maxdiff %.2e | stamps us: "
                 "last start %.2f, block loop %.2f, loops done %.2f, combined %.2f, epilogue %.2f, "
                 "span %.2f\n",
                 M, N, K, S, S > 1 ? mn[mode] : "unsplit", nb, us, diff, s0max / tiles / 100,
                 loop / nb / 100, lend / tiles / 100, cend / tiles / 100, eend / tiles / 100,
                 (double)(tend - t00) / 100);
          fflush(stdout);
        }
      }
    }
  }
  return 0;
}
