// bf16-configuration GEMM with 128 x 64 wave tiles (gfx950,
// v_mfma_f32_16x16x32_bf16, fp32 accumulation): block tile 256 x BN, waves
// 2 along M x BN / 64 along N (BN = 128: 4 waves, one per SIMD).
//
// Why: gemm_h16i_kernel's 256 x 128 tile runs 8 waves of 128 x 32, so a
// 32-deep k-step reads 10 fragments (8 A + 2 B) for 16 MFMAs -- 0.625 reads
// per MFMA, with the LDS-DMA writes about 80 % of the CU's LDS cycles at the
// MFMA rate (profiles/r6: MFMA busy 0.32-0.41 in the C5 step).  A 128 x 64
// wave tile reads 12 fragments per 32 MFMAs (0.375) -- the wave tile of
// gemm_h256_kernel and of the 256^2 template (cdna_hip_programming.md) --
// while BN = 128 keeps one block per CU on the C5 shapes (4096 x 2048
// outputs = 256 tiles).
//
// Staging: a ring of NS LDS slots, each one 32-deep k-step (A 256 x 32 and B
// 32 x BN bf16), filled by buffer_load ... lds (16 B per lane, 1-KiB pieces,
// gemm_h.h's swizzled source addresses); steps s+1 .. s+NS-1 in flight while
// step s is computed.  Per step each wave waits for its own fragment reads of
// s, retires its LDS-DMA of s+1 with a counted vmcnt, passes one barrier,
// then issues the fragment reads of s+1 and the DMA of s+NS into slot s in the
// gaps of its 32 MFMAs (gemm_h256.h's schedule).  The loop is unrolled by the
// NS slots so every LDS address is a base register + an immediate.
//
// Any fused epilogue of gemm_common.h, or split-K slabs (blockIdx.z = split,
// kps deep each); full tiles: the host checks M % 256 == N % BN == 0 and
// kps % (32 NS) == 0 == K % kps.  The product runs it on the bf16
// configuration's weight gradients (KR x KR), 1.2x gemm_h16_kernel isolated
// (tools/hw_bench.hip, profiles/r6/hw_bench.txt); on RK A operands the
// 8-wave gemm_h16i_kernel stays faster (0.91-0.99x).
#pragma once
#include "gemm_h256.h"

namespace ddpg {

// one 16-B-per-lane LDS-DMA piece (buffer_load ... lds).  A plain device
// function: called with template-dependent arguments straight from the
// kernel template, the builtin kept hipcc's host pass from emitting the
// kernel's launch stub.
DDPG_DEV void glds16(__amdgpu_buffer_rsrc_t r, lds_void* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
}

template <int BN, int NS, int PR_ = 0>
struct HwCfg {
  static constexpr int BM = 256, BK = 32;
  static constexpr int NW = 2 * (BN / 64);  // waves
  static constexpr int NT = 64 * NW;  // = 2 BN (the launch bounds)
  static constexpr int A_BYTES = BM * BK * 2;  // 16 KB
  static constexpr int B_BYTES = BN * BK * 2;
  static constexpr int A_PW = A_BYTES / 1024 / NW;  // 1-KiB pieces per wave
  static constexpr int B_PW = B_BYTES / 1024 / NW;
  static constexpr int G = A_PW + B_PW;  // LDS-DMA instructions per wave per step
  static constexpr int RING = NS * (A_BYTES + B_BYTES);
  // gemm_epilogue<256, BN, BN / 64, 16, PR>: PR rows x (BN + 4) + projection
  // panel + reduction (+ at PR = 128 the narrow rows of a fused weight
  // gradient); BN = 256 stages 64 rows per pass, as gemm_h256
  static constexpr int PR = PR_ ? PR_ : (BN == 256 ? 64 : 128);
  static constexpr int EPI_BYTES =
      (PR * (BN + 4) + BN * PROJ_MAX + 2 * GNT + (PR == 128 ? 128 * 64 : 0)) * 4;
  static constexpr int SMEM_BYTES = RING > EPI_BYTES ? RING : EPI_BYTES;
  static_assert(SMEM_BYTES <= 160 * 1024, "LDS");
  static_assert(A_PW * NW * 1024 == A_BYTES && B_PW * NW * 1024 == B_BYTES, "whole pieces");
};

// PR: epilogue rows per LDS pass (0: 128, or 64 at BN = 256); PR = 64 at
// NS = 2 fits two blocks per CU (52 KB of epilogue LDS), without the fused
// narrow weight gradient (it needs PR = 128)
// ONLY >= 0: compile one element-wise epilogue variant (gemm_epilogue's),
// which the two-blocks-per-CU form needs to stay within 256 registers
// FULL = false: M need not be a multiple of 256 (rows past M are read
// clamped and never stored: the epilogue's bounds checks)
template <int AL, int BL, int BN, int NS, int PR, int ONLY, bool FULL>
DDPG_DEV void gemm_hw_body(const GemmHArgs& g, int z) {
  using C = HwCfg<BN, NS, PR>;
  constexpr int BM = C::BM, BK = C::BK;
  constexpr int WGN = BN / 64;  // waves along N
  constexpr int TA = 8;         // 16-row A fragments per wave (128 rows)
  constexpr int TB = 4;         // 16-column B fragments per wave (64 columns)
  constexpr int NM = TA * TB;   // MFMAs per step
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_BYTES / 4];
  char* const lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * BN, m0 = by * BM;
  const int kbeg = z * g.kps;  // split-K: each split's fp32 slab at out + z out_split_stride
  const int nk = g.kps / BK;   // host: kps % (BK NS) == 0, every split full

  f32x4 acc[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, 0x00020000);
  unsigned oa[C::A_PW], ob[C::B_PW];
#pragma unroll
  for (int i = 0; i < C::A_PW; ++i)
    oa[i] = (unsigned)((const char*)hg_src<AL, BM, BK, 16>(g.A, g.lda, g.M, m0, kbeg,
                                                          wave * C::A_PW + i, lane) -
                       (const char*)g.A);
#pragma unroll
  for (int i = 0; i < C::B_PW; ++i)
    ob[i] = (unsigned)((const char*)hg_src<BL, BN, BK, 16>(g.B, g.ldb, g.N, n0, kbeg,
                                                          wave * C::B_PW + i, lane) -
                       (const char*)g.B);
  const unsigned stepA = 2u * (AL == L_RK ? BK : (unsigned)BK * g.lda);  // bytes per step
  const unsigned stepB = 2u * (BL == L_RK ? BK : (unsigned)BK * g.ldb);

  // LDS: the NS slots' A images first, then their B images
  constexpr unsigned BREG = NS * C::A_BYTES;
  auto piece = [&](int s, int slot, int q) {
    if (q < C::A_PW)
      glds16(ra, (lds_void*)(lds + slot * C::A_BYTES + (wave * C::A_PW + q) * 1024), oa[q],
             s * stepA);
    else
      glds16(rb, (lds_void*)(lds + BREG + slot * C::B_BYTES + (wave * C::B_PW + q - C::A_PW) * 1024),
             ob[q - C::A_PW], s * stepB);
  };
  auto bcol = [&](int j) { return wn * 64 + 16 * j; };

  // fragment-read bases (gemm_h256.h): RK one base per operand, KR one per
  // fragment and k-row half; slots and fragments are immediates
  const unsigned lbase = (unsigned)(uintptr_t)(lds_char*)lds;
  auto rk_base = [&](int row0) {
    const int r = row0 + (lane & 15);
    return (unsigned)(r * 64 + 16 * ((lane >> 4) ^ ((r >> 2) & 2)));
  };
  auto kr_addr = [&](int col0, int half) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 4 * p;
    const int ch = (col & 127) >> 3;
    const int k = 8 * (lane >> 4) + q + 4 * half;
    return (unsigned)((col >> 7) * (BK * 256) + k * 256 + 16 * (ch ^ kr_swz(k)) + 8 * (p & 1));
  };
  constexpr int NAB = AL == L_RK ? 1 : 2 * TA;
  constexpr int NBB = BL == L_RK ? 1 : 2 * TB;
  unsigned abase[NAB], bbase[NBB];
  if constexpr (AL == L_RK) {
    abase[0] = lbase + rk_base(wm * 128);
  } else {
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) abase[2 * i + hh] = lbase + kr_addr(wm * 128 + 16 * i, hh);
  }
  if constexpr (BL == L_RK) {
    bbase[0] = lbase + BREG + rk_base(wn * 64);
  } else {
#pragma unroll
    for (int j = 0; j < TB; ++j)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) bbase[2 * j + hh] = lbase + BREG + kr_addr(bcol(j), hh);
  }
  // read group J of a step from slot SL: B fragment J (J < TB), then A
  // fragment J - TB
  auto read_one = [&](auto sl_c, auto j_c, bf16x8 (&av)[1][TA], bf16x8 (&bv)[1][TB]) {
    constexpr int SL = decltype(sl_c)::value, J = decltype(j_c)::value;
    if constexpr (J < TB) {
      if constexpr (BL == L_RK) {
        constexpr int OFF = SL * C::B_BYTES + 16 * J * 64;
        bv[0][J] = b128_read_off<OFF>(bbase[0]);
      } else {
        constexpr int OFF = SL * C::B_BYTES;
        bv[0][J] = __builtin_shufflevector(tr_read_off<OFF>(bbase[2 * J]),
                                           tr_read_off<OFF>(bbase[2 * J + 1]), 0, 1, 2, 3, 4, 5,
                                           6, 7);
      }
    } else {
      constexpr int I = J - TB;
      if constexpr (AL == L_RK) {
        constexpr int OFF = SL * C::A_BYTES + I * 16 * 64;
        av[0][I] = b128_read_off<OFF>(abase[0]);
      } else {
        constexpr int OFF = SL * C::A_BYTES;
        av[0][I] = __builtin_shufflevector(tr_read_off<OFF>(abase[2 * I]),
                                           tr_read_off<OFF>(abase[2 * I + 1]), 0, 1, 2, 3, 4, 5,
                                           6, 7);
      }
    }
  };

  // A fragments: one register set, each refilled for step s+1 one MFMA row
  // after its last use in step s; B fragments: two sets alternating by step
  bf16x8 fa[1][TA], fb[2][1][TB];
  // one k-step s in ring slot SL.  NEXT: step s+1 exists; INF: LDS-DMA
  // groups of steps beyond s+1 that may stay in flight; ST: stage step s+NS
  // into this slot
  auto step = [&](int s, auto sl_c, auto next_c, auto inf_c, auto st_c) {
    constexpr int SL = decltype(sl_c)::value;
    constexpr int SET = SL & 1;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr int INF = decltype(inf_c)::value;
    constexpr bool ST = decltype(st_c)::value;
    static_assert(NS % 2 == 0, "B sets alternate with the slot's parity");
    hg_wait16<1, TA, TB>(fa, fb[SET]);
    if constexpr (NEXT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF * C::G) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int RS = (SL + 1) % NS;  // slot of step s+1
    static_for<NM>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      constexpr int i = q / TB, j = q % TB;
      mfma_inplace(acc[i][j], fa[0][i], fb[SET][0][j]);
      if constexpr (NEXT) {
        if constexpr (q < TB)
          read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, q>{}, fa,
                   fb[SET ^ 1]);
        if constexpr (q >= TB && j == 0)
          read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, TB + i - 1>{},
                   fa, fb[SET ^ 1]);
        if constexpr (q == NM - 1)
          read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, TB + TA - 1>{},
                   fa, fb[SET ^ 1]);
      }
      // LDS-DMA of step s+NS: one piece per other gap from the second MFMA row
      if constexpr (ST && q >= TB + 1 && ((q - TB - 1) & 1) == 0 && (q - TB - 1) / 2 < C::G)
        piece(s + NS, SL, (q - TB - 1) / 2);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  // prologue: steps 0 .. NS-1 into the NS slots, wait for step 0
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(s, s, q);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NS - 1) * C::G) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  static_for<TA + TB>(
      [&](auto j_c) { read_one(std::integral_constant<int, 0>{}, j_c, fa, fb[0]); });
  __builtin_amdgcn_sched_barrier(0);

  // steady state: NS steps per trip, every step stages s+NS (host: nk % NS
  // == 0, so the loop leaves exactly the last NS steps)
  int s = 0;
  for (; s + NS < nk; s += NS)
    static_for<NS>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      step(s + k, std::integral_constant<int, k>{}, T_{},
           std::integral_constant<int, NS - 2>{}, T_{});
    });
  // the last NS steps: nothing more to stage; steps staged beyond s+k+1 that
  // may stay in flight: NS - 2 - k
  static_for<NS>([&](auto k_c) {
    constexpr int k = decltype(k_c)::value;
    if constexpr (k + 1 < NS)
      step(s + k, std::integral_constant<int, k>{}, T_{},
           std::integral_constant<int, NS - 2 - k>{}, F_{});
    else
      step(s + k, std::integral_constant<int, k>{}, F_{}, std::integral_constant<int, 0>{}, F_{});
  });

  mfma_drain();
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) asm volatile("" : "+v"(acc[i][j]));
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // staging slots are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  // the epilogue's 32 x 32 register blocks (acc_row / acc_col<16>): block
  // (I, J) = 16 x 16 fragments (2I + tr, 2J + tc)
  f32x16 out[4][2];
#pragma unroll
  for (int I = 0; I < 4; ++I)
#pragma unroll
    for (int J = 0; J < 2; ++J)
#pragma unroll
      for (int tr = 0; tr < 2; ++tr)
#pragma unroll
        for (int tc = 0; tc < 2; ++tc)
#pragma unroll
          for (int q = 0; q < 4; ++q) out[I][J][4 * (2 * tr + tc) + q] = acc[2 * I + tr][2 * J + tc][q];
  gemm_epilogue<256, BN, WGN, 16, C::PR, FULL, ONLY>(out, smem, ge, tid, n0, m0, z, bx, by);
}

template <int AL, int BL, int BN, int NS, int PR = 0, int ONLY = -1, bool FULL = true>
__global__ __launch_bounds__(BN * 2, NS == 2 ? 2 : 1) void gemm_hw_kernel(GemmHArgs g) {
  gemm_hw_body<AL, BL, BN, NS, PR, ONLY, FULL>(g, blockIdx.z);
}

// Up to GH_MAXP independent GEMMs of one grid shape in one launch (part =
// blockIdx.z, one split each), as gemm_h16i_pack_kernel: the bf16
// configuration's batch-only first layers (K = S = 376 -> 384).  At NS = 2 /
// PR = 64 with the forward epilogue only, two 4-wave blocks share a CU, so
// one block's prologue and epilogue stores run beside the other's k-loop:
// 1.18x gemm_h16i_pack_kernel's form isolated on the four C5 first layers
// (tools/hw_bench.hip, profiles/r6/hw_bench_2x.txt).
template <int AL, int BL, int BN, int NS, int PR = 0, int ONLY = -1>
__global__ __launch_bounds__(BN * 2, NS == 2 ? 2 : 1) void gemm_hw_pack_kernel(GemmHPack pk) {
  gemm_hw_body<AL, BL, BN, NS, PR, ONLY, true>(pk.p[blockIdx.z], 0);
}

}  // namespace ddpg
