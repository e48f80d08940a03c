// Microbenchmark (tuning aid, not product code): the NP = 3 twin GEMM's
// matrix work on the two bf16 MFMA shapes under the chip's power limit.
// One 512-thread block per CU (256 blocks, 2 waves per SIMD), operands in
// registers from random bf16 planes, one s_barrier per "k-tile" as in
// gemm_h3_kernel.  Per k-tile and wave the same 786,432 flop:
//   32x32x16: 2 (M) x 1 (N) output blocks x 2 k-steps x 6 plane products = 24 MFMAs
//   16x16x32: 4 (M) x 2 (N) output blocks x 1 k-step  x 6 plane products = 48 MFMAs
// Prints us per launch, TF-eq (6 products = one fp32 MAC) and the in-kernel
// clock (s_memtime / s_memrealtime) for both.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_power_bench.hip -o tools/mfma_power_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

template <int SHAPE>
__global__ __launch_bounds__(512, 1) void mfma_loop(const bf16x8* __restrict__ src, int ntiles,
                                                    float* out, unsigned long long* clk) {
  const int tid = threadIdx.x;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  if constexpr (SHAPE == 32) {
    bf16x8 a[3][2], b[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      b[p] = src[(p * 3) * 512 + tid];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[p][i] = src[(p * 3 + 1 + i) * 512 + tid];
    }
    f32x16 acc[2], acs[2];
    for (int i = 0; i < 2; ++i)
      for (int r = 0; r < 16; ++r) acc[i][r] = acs[i][r] = 0.f;
    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2][i], b[0], acs[i], 0, 0, 0);
          acs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[1], acs[i], 0, 0, 0);
          acs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[2], acs[i], 0, 0, 0);
          acs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1][i], b[0], acs[i], 0, 0, 0);
          acs[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[1], acs[i], 0, 0, 0);
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][i], b[0], acc[i], 0, 0, 0);
        }
      __builtin_amdgcn_s_barrier();
      // keep the operands live and opaque (a reload per tile would be hoisted)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        asm volatile("" : "+v"(b[p]));
        for (int i = 0; i < 2; ++i) asm volatile("" : "+v"(a[p][i]));
      }
    }
    for (int i = 0; i < 2; ++i)
      for (int r = 0; r < 16; ++r) sum += acc[i][r] + acs[i][r];
  } else {
    bf16x8 a[3][4], b[3][2];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int j = 0; j < 2; ++j) b[p][j] = src[(p * 6 + j) * 512 + tid];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[p][i] = src[(p * 6 + 2 + i) * 512 + tid];
    }
    f32x4 acc[4][2], acs[4][2];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j) acc[i][j] = acs[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < ntiles; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2][i], b[0][j], acs[i][j], 0, 0, 0);
          acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[1][j], acs[i][j], 0, 0, 0);
          acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[2][j], acs[i][j], 0, 0, 0);
          acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1][i], b[0][j], acs[i][j], 0, 0, 0);
          acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[1][j], acs[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0][i], b[0][j], acc[i][j], 0, 0, 0);
        }
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        for (int j = 0; j < 2; ++j) asm volatile("" : "+v"(b[p][j]));
        for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(a[p][i]));
      }
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 4; ++r) sum += acc[i][j][r] + acs[i][j][r];
  }
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + tid] = sum;
  if (tid == 0) {
    clk[2 * blockIdx.x] = r1 - r0;
    clk[2 * blockIdx.x + 1] = c1 - c0;
  }
}

int main() {
  const int nb = 256, ntiles = 2000;
  std::vector<unsigned short> h(18 * 512 * 8);
  srand(3);
  // random bf16 planes of a unit-scale value: h plane O(1), m ~2^-8, l ~2^-16
  for (size_t i = 0; i < h.size(); ++i) {
    const int plane = (int)((i / (512 * 8)) % 3);
    const unsigned sign = rand() & 1, man = rand() & 127;
    const unsigned ex = 127 - 8 * plane - (rand() & 3);
    h[i] = (unsigned short)((sign << 15) | (ex << 7) | man);
  }
  bf16x8* src;
  float* out;
  unsigned long long* clk;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, nb * 512 * 4));
  CHECK(hipMalloc(&clk, nb * 2 * 8));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int round = 0; round < 3; ++round) {
    for (int shape : {32, 16}) {
      auto launch = [&]() {
        if (shape == 32)
          hipLaunchKernelGGL(mfma_loop<32>, dim3(nb), dim3(512), 0, 0, src, ntiles, out, clk);
        else
          hipLaunchKernelGGL(mfma_loop<16>, dim3(nb), dim3(512), 0, 0, src, ntiles, out, clk);
      };
      for (int i = 0; i < 3; ++i) launch();
      CHECK(hipDeviceSynchronize());
      const int reps = 10;
      CHECK(hipEventRecord(e0));
      for (int i = 0; i < reps; ++i) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<unsigned long long> c(nb * 2);
      CHECK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
      double ghz = 0, cyc = 0;
      for (int b = 0; b < nb; ++b) {
        ghz += (double)c[2 * b + 1] / (double)c[2 * b] / 10.0;
        cyc += (double)c[2 * b + 1];
      }
      const double us = 1e3 * ms / reps;
      const double fl = (double)nb * 8 * ntiles * 786432.0 / 6.0;  // fp32-eq flop
      printf("round %d %dx%d MFMA: %8.1f us/launch, %6.1f TF-eq (%.3f of 417), %.0f cyc/tile "
             "(MFMA-bound 1536), clock %.2f GHz\n",
             round, shape, shape, us, fl / us * 1e-6, fl / us * 1e-6 / 417.0,
             cyc / nb / ntiles, ghz / nb);
      fflush(stdout);
    }
  }
  return 0;
}
