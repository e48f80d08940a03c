// Microbenchmark (tuning aid, not product code): the cost of the in-launch
// K-split hand-off alone (ksplit_combine's protocol, gemm_common.h) without
// the GEMM around it.  T tiles x S splits of 512-lane blocks, each holding a
// 128 x 128 fp32 partial in registers (32 floats per lane):
//   null    : every block writes its partial to out (no hand-off)
//   ticket  : the ticket round trip only (no partial stores / loads)
//   full<st,ld>: partial stores with cache policy st, vmcnt(0), barrier, one
//             lane's agent-scope atomic, barrier, the last block loads the
//             other S - 1 partials with cache policy ld and writes the sum
// cache policy bits: 1 = sc0, 2 = nt, 16 = sc1.  Prints avg us per launch and
// whether the sums are right (the hand-off is only valid where they are on
// every run; a wrong sum means the policy does not publish across XCDs).
//   hipcc -O3 --offload-arch=gfx950 tools/kc_comb_bench.hip -o tools/kc_comb_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int NT = 512, NQ = 8;  // 8 x 16 B per lane = the 128 x 128 fp32 tile

__device__ inline f32x4 val(int tile, int z, int tid, int q) {
  const float b = (float)(tile * 131 + z * 7 + tid + q);
  return f32x4{b, b + 0.25f, b + 0.5f, b + 0.75f};
}

template <int MODE, int ST, int LD>
__global__ __launch_bounds__(NT) void comb(float* part, unsigned* ticket, float* out, int S) {
  const int tid = threadIdx.x, tile = blockIdx.x, z = blockIdx.y;
  f32x4 acc[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) acc[q] = val(tile, z, tid, q);
  __shared__ unsigned last_s;
  if constexpr (MODE == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      *(f32x4*)(out + ((size_t)(tile * S + z) * NQ * NT + q * NT + tid) * 4) = acc[q];
    return;
  } else {
    const unsigned slab = NQ * NT * 16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(part + (size_t)tile * S * (slab / 4)), 0, 0x7fffffff, 0x00020000);
    if constexpr (MODE == 2) {
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[q]), rs,
                                               z * slab + (unsigned)(q * NT + tid) * 16, 0, ST);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (tid == 0) {
      const unsigned old =
          __hip_atomic_fetch_add(ticket + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned l = old == (unsigned)(S - 1);
      if (l) __hip_atomic_store(ticket + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_s = l;
    }
    __syncthreads();
    if (!last_s) return;
    f32x4 x[3][NQ];
    if constexpr (MODE == 2) {
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int zz = j + (j >= z);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          x[j][q] = zz < S ? __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                           rs, zz * slab + (unsigned)(q * NT + tid) * 16,
                                                           0, LD))
                           : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
#pragma unroll
      for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int q = 0; q < NQ; ++q) x[j][q] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      f32x4 t = acc[q];
#pragma unroll
      for (int j = 0; j < 3; ++j) t += x[j][q];
      *(f32x4*)(out + ((size_t)tile * NQ * NT + q * NT + tid) * 4) = t;
    }
  }
}

int main() {
  const int TMAX = 256, SMAX = 4;
  float *part, *out;
  unsigned* tick;
  CHECK(hipMalloc(&part, (size_t)TMAX * SMAX * NQ * NT * 16));
  CHECK(hipMalloc(&out, (size_t)TMAX * SMAX * NQ * NT * 16));
  CHECK(hipMalloc(&tick, TMAX * 4));
  CHECK(hipMemset(tick, 0, TMAX * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct V {
    const char* name;
    void (*k)(float*, unsigned*, float*, int);
  } vs[] = {{"null          ", comb<0, 0, 0>},   {"ticket        ", comb<1, 0, 0>},
            {"full st16 ld16", comb<2, 16, 16>}, {"full st16 ld17", comb<2, 16, 17>},
            {"full st17 ld17", comb<2, 17, 17>}, {"full st16 ld1 ", comb<2, 16, 1>},
            {"full st18 ld16", comb<2, 18, 16>}, {"full st0  ld16", comb<2, 0, 16>},
            {"full st0  ld0 ", comb<2, 0, 0>}};
  for (int T : {32, 64}) {
    for (int S : {2, 4}) {
      for (auto& v : vs) {
        const dim3 grid(T, S);
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(v.k, grid, dim3(NT), 0, 0, part, tick, out, S);
        CHECK(hipDeviceSynchronize());
        const int reps = 50;
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < reps; ++i)
          hipLaunchKernelGGL(v.k, grid, dim3(NT), 0, 0, part, tick, out, S);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        int bad = -1;
        if (v.k != comb<0, 0, 0> && v.k != comb<1, 0, 0>) {
          // the sum of val() over z for every tile / lane / element
          std::vector<float> h((size_t)T * NQ * NT * 4);
          CHECK(hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost));
          bad = 0;
          for (int tile = 0; tile < T; ++tile)
            for (int q = 0; q < NQ; ++q)
              for (int tid = 0; tid < NT; ++tid)
                for (int e = 0; e < 4; ++e) {
                  float s = 0.f;
                  for (int z = 0; z < S; ++z) s += (float)(tile * 131 + z * 7 + tid + q) + 0.25f * e;
                  const float g = h[((size_t)tile * NQ * NT + q * NT + tid) * 4 + e];
                  bad += fabsf(g - s) > 1e-3f * fabsf(s) + 1e-3f;
                }
        }
        printf("T=%3d S=%d %s  %7.2f us  wrong %d\n", T, S, v.name, 1e3 * ms / reps, bad);
        fflush(stdout);
      }
    }
  }
  return 0;
}
