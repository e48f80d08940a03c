// Microbenchmark (tuning aid, not product code): how much of the NP = 3 twin
// GEMM's clock the LDS fragment reads cost under the chip's power limit, and
// whether a 64 x 64 wave tile (a third fewer fragment bytes per MFMA) would
// hold a higher clock than gemm_h3m's 64 x 32.  One block per CU (256
// blocks), v_mfma_f32_16x16x32_bf16 with the six plane products; per k-tile
// and SIMD the same 96 MFMAs (786,432 x 2 flop) in every mode:
//   mode 0: 8 waves x 64x32 wave tile, operands in registers (no LDS reads)
//   mode 1: 8 waves x 64x32, 18 fragment reads (ds_read_b128) per wave and tile
//   mode 2: 4 waves x 64x64, 24 fragment reads per wave and tile
//   mode 3: mode 1 with the reads in the tile's first 18 MFMA gaps (gemm_h3m's placement)
//   modes 4-6: mode 1 plus the LDS-DMA (buffer_load ... lds, 1 KiB per wave
//   and piece, L2-resident source) of 6 pieces per wave and tile (gemm_h3m's
//   128 x 128 tile: 48 KiB per k-tile), 4 pieces (a 256 x 128 tile's bytes per
//   flop: 36 KiB per 128 x 128 equivalent, rounded to 32) and 3 pieces
//   mode 7: registers (no reads) plus the 6-piece DMA
//   modes 8-10: modes 4 / 7 / 4 with the pieces of each SIMD's second wave
//   (waves 4-7) 2 gaps later / 2 gaps later / 14 gaps earlier
//   mode 11: mode 4 with global_load_lds instead of buffer_load ... lds
// Prints us per launch, TF-eq and the in-kernel clock (s_memtime / s_memrealtime).
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_lds_power_bench.hip -o tools/mfma_lds_power_bench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <utility>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

// fragment read R (of 3 * (4 + TB)) goes before MFMA M when R * NMF / NRD == M
// (spread over the tile), or when R == M (FRONT: gemm_h3m's placement)
template <int TB, bool FRONT, int M, int R>
__device__ __forceinline__ void rd_step(bf16x8 (&na)[3][4], bf16x8 (&nb)[3][TB], unsigned lbase) {
  constexpr int NMF = 6 * 4 * TB, NRD = 3 * (4 + TB);
  if constexpr (R < NRD) {
    if constexpr ((FRONT ? R : R * NMF / NRD) == M) {
      constexpr int p = R / (4 + TB), f = R % (4 + TB);
      if constexpr (f < 4)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(na[p][f]) : "v"(lbase), "n"(R * 1024));
      else
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=v"(nb[p][f - 4]) : "v"(lbase), "n"(R * 1024));
    }
    rd_step<TB, FRONT, M, R + 1>(na, nb, lbase);
  }
}

// MFMA M of the tile's 6 * 4 * TB (product-outer: 4 * TB independent MFMAs
// between dependent ones), accumulators pinned in AGPRs (the compiler's own
// allocation shuffles them through VGPRs at 4 x 4 blocks)
// DMA piece d goes after MFMA gap 20 + 4 d (gemm_h3m's DG0 / DGS, scaled with TB)
struct Dma {
  __amdgpu_buffer_rsrc_t rs;
  const char* g;  // GLOBAL: this lane's source for global_load_lds
  unsigned voff, soff;
  char* dst;  // this wave's LDS pieces
};
template <int TB, bool READ, bool FRONT, int DMA, int DOFF, bool GLOBAL, int M>
__device__ __forceinline__ void mm_step(bf16x8 (&fa)[3][4], bf16x8 (&fb)[3][TB],
                                        bf16x8 (&na)[3][4], bf16x8 (&nb)[3][TB],
                                        f32x4 (&acc)[4][TB], f32x4 (&acs)[4][TB], unsigned lbase,
                                        const Dma& dm) {
  constexpr int NMF = 6 * 4 * TB;
  if constexpr (M < NMF) {
    constexpr int DG0 = 20 * TB / 2 + DOFF, DGS = 4 * TB / 2;
    if constexpr (M >= DG0 && (M - DG0) % DGS == 0 && (M - DG0) / DGS < DMA) {
      constexpr int d = (M - DG0) / DGS;
      if constexpr (GLOBAL)
        __builtin_amdgcn_global_load_lds((const void*)(dm.g + dm.soff + d * 65536),
                                         (lds_void*)(dm.dst + d * 1024), 16, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(dm.rs, (lds_void*)(dm.dst + d * 1024), 16,
                                                 dm.voff, dm.soff + d * 65536, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    constexpr int q = M / (4 * TB), i = (M / TB) % 4, j = M % TB;
    constexpr int PA[6] = {2, 1, 0, 1, 0, 0}, PB[6] = {0, 1, 2, 0, 1, 0};
    if constexpr (READ) rd_step<TB, FRONT, M, 0>(na, nb, lbase);
    if constexpr (q < 5)
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                   : "+a"(acs[i][j]) : "v"(fa[PA[q]][i]), "v"(fb[PB[q]][j]));
    else
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                   : "+a"(acc[i][j]) : "v"(fa[PA[q]][i]), "v"(fb[PB[q]][j]));
    mm_step<TB, READ, FRONT, DMA, DOFF, GLOBAL, M + 1>(fa, fb, na, nb, acc, acs, lbase, dm);
  }
}

// TB 16-column B fragments, 4 16-row A fragments per wave; READ: reload every
// fragment from LDS each tile (else keep the registers); DMA pieces per wave
// and tile.  All waves read the same fragment image (bank behaviour is per
// wave), so the DMA region fits beside it.
template <int TB, bool READ, bool FRONT = false, int DMA = 0, int STAG = 0, bool GLOBAL = false>
__global__ __launch_bounds__(TB == 2 ? 512 : 256, 1) void loop(const bf16x8* __restrict__ src,
                                                               const char* __restrict__ dsrc,
                                                               int ntiles, float* out,
                                                               unsigned long long* clk) {
  constexpr int NT = TB == 2 ? 512 : 256;
  constexpr int NF = 3 * (4 + TB);  // fragments per wave and tile
  __shared__ bf16x8 lds[NF * 64];
  __shared__ __attribute__((aligned(16))) char dlds[DMA > 0 ? (NT / 64) * DMA * 1024 : 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bf16x8 a[3][4], b[3][TB];
  for (int i = tid; i < NF * 64; i += NT) lds[i] = src[i % (18 * 512)];
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 3; ++p) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[p][i] = lds[(p * (4 + TB) + i) * 64 + lane];
#pragma unroll
    for (int j = 0; j < TB; ++j) b[p][j] = lds[(p * (4 + TB) + 4 + j) * 64 + lane];
  }
  // DMA source: 64 KiB per piece index, 3 MiB window shared by all blocks
  // (L2 / MALL resident like the product's re-read operand tiles)
  Dma dm;
  dm.rs = __builtin_amdgcn_make_buffer_rsrc((void*)dsrc, 0, 0x7fffffff, 0x00020000);
  dm.voff = (unsigned)((wave * 64 + lane) * 16 + (blockIdx.x % 8) * 8192);
  dm.dst = (char*)dlds + wave * DMA * 1024;
  dm.g = dsrc + dm.voff;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), c0 = __builtin_amdgcn_s_memtime();
  f32x4 acc[4][TB], acs[4][TB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = acs[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // READ: double-buffered like the product kernel: tile t+1's fragments are
  // read (hand-issued ds_read_b128, spread evenly between tile t's MFMAs so
  // the 15-deep lgkmcnt never stalls the MFMA chain) and waited for at the
  // tile's end; the tile's DMA pieces may stay in flight one tile.  The same
  // slot every tile: the LDS traffic, not the data, is measured.
  const unsigned lbase = (unsigned)(size_t)&lds[lane];  // fragment r at + r KiB
  // the whole k-loop per placement, chosen by a wave-uniform (scalar) branch
  // outside it, so each copy keeps its own register assignment
  bf16x8 a2[3][4], b2[3][TB];
  auto kloop = [&](auto doff_c) {
    constexpr int DOFF = decltype(doff_c)::value;
    auto mm_ld = [&](int t, bf16x8 (&fa)[3][4], bf16x8 (&fb)[3][TB], bf16x8 (&na)[3][4],
                     bf16x8 (&nb)[3][TB]) {
      dm.soff = (unsigned)(t % 48) * 65536u / 4u;
      mm_step<TB, READ, FRONT, DMA, DOFF, GLOBAL, 0>(fa, fb, na, nb, acc, acs, lbase, dm);
      if constexpr (READ) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr (DMA > 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA) : "memory");
    };
    for (int t = 0; t < ntiles; t += 2) {
      mm_ld(t, a, b, a2, b2);
      __builtin_amdgcn_s_barrier();
      mm_ld(t + 1, READ ? a2 : a, READ ? b2 : b, a, b);
      __builtin_amdgcn_s_barrier();
      if constexpr (!READ) {
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          for (int j = 0; j < TB; ++j) asm volatile("" : "+v"(b[p][j]));
          for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(a[p][i]));
        }
      }
    }
  };
  // the SIMD's second wave (waves NT/128 ..) puts its pieces STAG gaps later
  if (STAG != 0 && __builtin_amdgcn_readfirstlane(wave) >= NT / 128)
    kloop(std::integral_constant<int, STAG>{});
  else
    kloop(std::integral_constant<int, 0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), c1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < TB; ++j)
      for (int r = 0; r < 4; ++r) sum += acc[i][j][r] + acs[i][j][r];
  out[blockIdx.x * NT + tid] = sum;
  if (tid == 0) {
    clk[2 * blockIdx.x] = r1 - r0;
    clk[2 * blockIdx.x + 1] = c1 - c0;
  }
}

int main() {
  const int nb = 256, ntiles = 2000;
  std::vector<unsigned short> h(18 * 512 * 8);
  srand(3);
  for (size_t i = 0; i < h.size(); ++i) {
    const int plane = (int)((i / (512 * 8)) % 3);
    const unsigned sign = rand() & 1, man = rand() & 127;
    const unsigned ex = 127 - 8 * plane - (rand() & 3);
    h[i] = (unsigned short)((sign << 15) | (ex << 7) | man);
  }
  bf16x8* src;
  float* out;
  unsigned long long* clk;
  char* dsrc;  // DMA window: 48 piece indices x 64 KiB / 4 apart + 8 KiB x 8 + 512 x 16 B
  const size_t dbytes = 48 * 16384 + 8 * 8192 + 8 * 1024 * 6 + 4096;
  CHECK(hipMalloc(&dsrc, dbytes + 6 * 65536));
  CHECK(hipMemset(dsrc, 0x3c, dbytes + 6 * 65536));
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, nb * 512 * 4));
  CHECK(hipMalloc(&clk, nb * 2 * 8));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  static const char* names[12] = {
      "8 waves 64x32, registers          ", "8 waves 64x32, 18 reads/tile      ",
      "4 waves 64x64, 24 reads/tile      ", "8 waves 64x32, 18 front-read      ",
      "8 waves 64x32, 18 reads + 6 DMA   ", "8 waves 64x32, 18 reads + 4 DMA   ",
      "8 waves 64x32, 18 reads + 3 DMA   ", "8 waves 64x32, registers + 6 DMA  ",
      "8 w, 18 reads + 6 DMA, stagger 2  ", "8 w, registers + 6 DMA, stagger 2 ",
      "8 w, 18 reads + 6 DMA, stagger 14 ", "8 w, 18 reads + 6 global_load_lds"};
  for (int round = 0; round < 3; ++round) {
    for (int mode = 0; mode < 12; ++mode) {
      auto launch = [&]() {
#define L(TB, ...) hipLaunchKernelGGL((loop<TB, __VA_ARGS__>), dim3(nb), dim3(TB == 2 ? 512 : 256), 0, 0, \
                                      src, dsrc, ntiles, out, clk)
        switch (mode) {
          case 0: L(2, false); break;
          case 1: L(2, true); break;
          case 2: L(4, true); break;
          case 3: L(2, true, true); break;
          case 4: L(2, true, false, 6); break;
          case 5: L(2, true, false, 4); break;
          case 6: L(2, true, false, 3); break;
          case 7: L(2, false, false, 6); break;
          case 8: L(2, true, false, 6, 2); break;
          case 9: L(2, false, false, 6, 2); break;
          case 10: L(2, true, false, 6, -14); break;
          default: L(2, true, false, 6, 0, true); break;
        }
#undef L
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
      // per block and tile: 8 waves x 48 or 4 waves x 96 MFMAs of 16x16x32 = 16384 flop each
      const double fl = (double)nb * 384 * ntiles * 16384.0 / 6.0;  // fp32-eq flop
      printf("round %d %s: %8.1f us/launch, %6.1f TF-eq (%.3f of 417), %.0f cyc/tile (MFMA-bound "
             "1536), clock %.2f GHz\n",
             round, names[mode], us, fl / us * 1e-6, fl / us * 1e-6 / 417.0, cyc / nb / ntiles,
             ghz / nb);
      fflush(stdout);
    }
  }
  return 0;
}
