// Microbenchmark (tuning aid, not product code): duration of near-empty
// kernels vs block size, LDS size and grid size (run under rocprofv3
// --kernel-trace to read the per-kernel durations).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int NT, int LDSF>
__global__ __launch_bounds__(NT) void empty_kernel(float* out, int flag) {
  __shared__ float s[LDSF > 0 ? LDSF : 1];
  if (flag == 12345) {  // never true: keeps the LDS allocation
    s[threadIdx.x] = 1.f;
    __syncthreads();
    out[threadIdx.x] = s[(threadIdx.x + 1) % NT];
  }
}

template <int NT, int LDSF>
static void run(int blocks, float* out) {
  for (int i = 0; i < 20; ++i)
    hipLaunchKernelGGL((empty_kernel<NT, LDSF>), dim3(blocks), dim3(NT), 0, 0, out, 0);
  hipDeviceSynchronize();
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 20);
  run<512, 0>(256, out);
  run<512, 30720>(256, out);
  run<256, 0>(256, out);
  run<256, 30720>(256, out);
  run<512, 0>(2048, out);
  run<64, 0>(256, out);
  printf("done\n");
  return 0;
}
