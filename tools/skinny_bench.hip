// Standalone timing + correctness check of skinny_wgrad_kernel (skinny.h) on
// the large-batch path's skinny weight-gradient shapes.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/skinny_bench tools/skinny_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
#include "../distributed_ddpg_amd/csrc/skinny.h"

using namespace ddpg;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Case { const char* name; int K, nn, ldn, nw, ldw, narrow_rows, cap; };

int main() {
  Case cases[] = {
    {"c3 dW1/dWs  s[4096][64] x dz1[4096][1024]", 4096, 64, 64, 1024, 1024, 1, 32},
    {"c3 dWa      a[4096][16] x dcat[4096][1024]", 4096, 16, 16, 1024, 2048, 1, 32},
    {"c3 dW3      h2[4096][1024] x dz3[4096][16]", 4096, 16, 16, 1024, 1024, 0, 32},
    {"c5 dW3      h2[4096][2048] x dz3[4096][17]", 4096, 17, 24, 2048, 2048, 0, 32},
    {"c5 dWa      a[4096][17] x dcat[4096][2048]", 4096, 17, 24, 2048, 4096, 1, 32},
    {"ragged      [1000][40] x [1000][520]", 1000, 40, 48, 520, 520, 1, 32},
  };
  CK(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(8)));
  CK(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<8, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(8)));
  CK(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<16, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(16)));
  CK(hipFuncSetAttribute((const void*)skinny_wgrad_kernel<16, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, sk_lds_bytes(16)));
  int bad = 0;
  for (auto& cs : cases) {
    const int K = cs.K;
    std::vector<float> hn((size_t)K * cs.ldn), hw((size_t)K * cs.ldw);
    srand(7);
    for (auto& x : hn) x = (rand() / (float)RAND_MAX - 0.5f);
    for (auto& x : hw) x = (rand() / (float)RAND_MAX - 0.5f);
    float *dn, *dw, *out;
    CK(hipMalloc(&dn, hn.size() * 4)); CK(hipMalloc(&dw, hw.size() * 4));
    CK(hipMemcpy(dn, hn.data(), hn.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
    int ng = (cs.nn > 16 && (cs.nn + 15) / 16 * 16 <= cs.ldn) ? 16 : 8;  // as wgrad_launch
    if (getenv("SK_NG")) ng = atoi(getenv("SK_NG"));
    if ((cs.nn + ng - 1) / ng * ng > cs.ldn) ng = 8;  // reads stay inside the row
    const int RR = getenv("SK_RR") ? atoi(getenv("SK_RR")) : 4;
    const int target = getenv("SK_BLOCKS") ? atoi(getenv("SK_BLOCKS")) : ng == 8 ? 512 : 256;
    const int ntn = (cs.nn + ng - 1) / ng, ntw = (cs.nw + SK_WT - 1) / SK_WT;
    const int tiles = ntn * ntw;
    int splits = std::min(cs.cap, std::max(1, target / tiles));
    int kc = ((K + splits - 1) / splits + SK_WAVES - 1) / SK_WAVES * SK_WAVES;
    splits = (K + kc - 1) / kc;
    const size_t MN = (size_t)cs.nn * cs.nw;
    CK(hipMalloc(&out, MN * splits * 4));
    SkArgs a{dn, cs.ldn, cs.nn, dw, cs.ldw, cs.nw, K, kc, ntw, ntn, cs.narrow_rows, out, (long long)MN};
    auto launch = [&]() {
      const dim3 g(tiles * splits), t(SK_NT);
      if (ng == 8 && RR == 4) hipLaunchKernelGGL((skinny_wgrad_kernel<8, 4>), g, t, sk_lds_bytes(8), 0, a);
      else if (ng == 8) hipLaunchKernelGGL((skinny_wgrad_kernel<8, 8>), g, t, sk_lds_bytes(8), 0, a);
      else if (RR == 4) hipLaunchKernelGGL((skinny_wgrad_kernel<16, 4>), g, t, sk_lds_bytes(16), 0, a);
      else hipLaunchKernelGGL((skinny_wgrad_kernel<16, 8>), g, t, sk_lds_bytes(16), 0, a);
    };
    launch(); CK(hipGetLastError()); CK(hipDeviceSynchronize());
    std::vector<float> ho(MN * splits);
    CK(hipMemcpy(ho.data(), out, ho.size() * 4, hipMemcpyDeviceToHost));
    double maxe = 0, maxr = 0;
    for (int i = 0; i < cs.nn; ++i)
      for (int j = 0; j < cs.nw; ++j) {
        double ref = 0, mag = 0;
        for (int b = 0; b < K; ++b) { double p = (double)hn[(size_t)b * cs.ldn + i] * hw[(size_t)b * cs.ldw + j]; ref += p; mag += fabs(p); }
        double got = 0;
        const size_t o = cs.narrow_rows ? (size_t)i * cs.nw + j : (size_t)j * cs.nn + i;
        for (int z = 0; z < splits; ++z) got += ho[z * MN + o];
        maxe = std::max(maxe, fabs(got - ref) / (mag + 1e-30));
      }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 5; ++i) launch();
    const int reps = 50;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps, fl = 2.0 * K * cs.nn * cs.nw;
    printf("%-46s NG=%2d R=%d grid=%4d splits=%3d  %7.2f us  %6.1f TF/s  err/|sum| %.2e %s\n", cs.name, ng, RR, tiles * splits, splits, us, fl / us * 1e-6, maxe, maxe < 1e-6 ? "ok" : "BAD");
    if (!(maxe < 1e-6)) bad = 1;
    CK(hipFree(dn)); CK(hipFree(dw)); CK(hipFree(out));
  }
  printf(bad ? "FAIL\n" : "done\n");
  return bad;
}
