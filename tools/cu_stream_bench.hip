// Microbenchmark (tuning aid, not product code): how fast can ONE workgroup
// of 1024 threads stream a weight matrix into registers, cold vs L2-warm,
// with U float4 loads in flight per thread.  Prints cycles per pass.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(1024) void stream_kernel(const f32x4* __restrict__ w, int n4, int passes,
                                                      unsigned long long* out, float* sink, int active_mod) {
  if (blockIdx.x % active_mod) return;
  float acc = 0.f;
  for (int p = 0; p < passes; ++p) {
    __syncthreads();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i0 = threadIdx.x; i0 < n4; i0 += 1024 * U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = w[min(i0 + u * 1024, n4 - 1)];
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u][0] + v[u][1] + v[u][2] + v[u][3];
    }
    __syncthreads();
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) out[p] = t1 - t0;
  }
  if (acc == 12345.f) sink[threadIdx.x] = acc;
}

int main() {
  const int n4 = 205 * 1024 / 16;  // 205 KB (critic Wh at C2)
  f32x4* w; unsigned long long* out; float* sink; float* big;
  hipMalloc(&w, n4 * 16); hipMalloc(&out, 64 * 8); hipMalloc(&sink, 4096 * 4);
  hipMalloc(&big, 512ull << 20);
  hipMemset(w, 0, n4 * 16);
  unsigned long long h[8];
  for (int blocks : {1, 16, 128}) for (int mod : {1, 8}) {
    if (blocks == 1 && mod == 8) continue;
    hipMemset(big, 1, 512ull << 20);  // evict caches (L2 + MALL)
    hipLaunchKernelGGL(stream_kernel<8>, dim3(blocks), dim3(1024), 0, 0, w, n4, 4, out, sink, mod);
    hipMemcpy(h, out, 4 * 8, hipMemcpyDeviceToHost);
    printf("U=8 blocks=%d active_mod=%d: cold %llu, warm %llu %llu %llu cycles (205 KB) -> %.1f / %.1f B/clk\n",
           blocks, mod, h[0], h[1], h[2], h[3], 205.0 * 1024 / h[0], 205.0 * 1024 / h[1]);
  }
  // write from another kernel on all CUs, then read (the learner's situation)
  for (int U : {4, 8, 16}) {
    hipMemset(w, 0, n4 * 16);  // written by a fill kernel on every XCD
    if (U == 4) hipLaunchKernelGGL(stream_kernel<4>, dim3(16), dim3(1024), 0, 0, w, n4, 3, out, sink, 1);
    if (U == 8) hipLaunchKernelGGL(stream_kernel<8>, dim3(16), dim3(1024), 0, 0, w, n4, 3, out, sink, 1);
    if (U == 16) hipLaunchKernelGGL(stream_kernel<16>, dim3(16), dim3(1024), 0, 0, w, n4, 3, out, sink, 1);
    hipMemcpy(h, out, 3 * 8, hipMemcpyDeviceToHost);
    printf("after memset, 16 blocks U=%d: first %llu, then %llu %llu cycles\n", U, h[0], h[1], h[2]);
  }
  hipDeviceSynchronize();
  return 0;
}
