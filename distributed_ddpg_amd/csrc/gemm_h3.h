// The fp32-context twin GEMM (three exact bf16 planes, six plane products
// per MAC: gemm_h.h's gemm_h_kernel<AL, BL, NP = 3, 128, 32, SCH = 1>) with
// its k-loop addressing reduced to immediates.
//
// gemm_h_kernel computes every fragment-read address and every LDS-DMA
// source per k-tile: with the ring slot t % 3 a runtime value, a k-tile of 24
// MFMAs carried 24 v_subrev + 26 v_add + 6 v_lshl_add_u64 + ~12 SALU of
// address arithmetic beside its 24 LDS reads and 6 LDS-DMAs -- about five
// issue slots per MFMA gap, the limit one 32x32x16 gap hides
// (MI355X_MICROARCH.md, "single-issue instructions hidden per gap").  Here:
//   * the k-loop is unrolled by the three ring slots, so the slot is a
//     compile-time constant;
//   * the LDS holds the three slots' A images (3 planes each) in one region
//     and their B images in the next, and every fragment read is one of a
//     few per-lane base registers + an immediate offset (ds_read offset:, 16
//     bits: slots 0 / 1 from one base, slot 2 from a second).  The distinct
//     bases per operand are the lane patterns the swizzles leave: RK images
//     one per k-step parity (the chunk index 2 ks + h is XORed with the row
//     swizzle), KR images one per k-row octet half (k0 / k0 + 4) and, for
//     the A operand of a weight gradient, per 32-column fragment (its chunk
//     bit 2 meets the swizzle);
//   * the LDS-DMA goes through buffer_load ... lds with the plane and k-tile
//     advance in the scalar soffset and a 32-bit per-lane voffset.
// Same staging ring, counted vmcnt, barrier placement, read / MFMA / DMA
// interleave (SCH = 1) and MFMA order as gemm_h_kernel: the results are
// bitwise equal (tested: DDPG_GEMM_H3=0 selects gemm_h_kernel).
#pragma once
#include "gemm_h256.h"

namespace ddpg {

template <int AL, int BL>
#if defined(DDPG_KC_STAMPS) && defined(DDPG_STAMPS8)  // tools/h3_phase_bench.hip: + shader clock
#define KC_STAMP(i)                                                                    \
  if (g.stamps && threadIdx.x == 0) {                                                  \
    const unsigned b_ = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x; \
    g.stamps[b_ * 8 + (i)] = __builtin_amdgcn_s_memrealtime();                         \
    g.stamps[b_ * 8 + 4 + (i)] = __builtin_amdgcn_s_memtime();                         \
  }
#elif defined(DDPG_KC_STAMPS)  // tools/kc_bench.hip: s_memrealtime per phase, lane 0 of each block
#define KC_STAMP(i)                                                                    \
  if (g.stamps && threadIdx.x == 0)                                                    \
    g.stamps[((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 + (i)] = \
        __builtin_amdgcn_s_memrealtime();
#else
#define KC_STAMP(i)
#endif
__global__ __launch_bounds__(HG_NT, 1) void gemm_h3_kernel(GemmHArgs g) {
  KC_STAMP(0)
  constexpr int NP = 3, BM = 128, BK = 32, WGN = 4;
  using C = HgCfg<BM, BK, NP, 8>;
  constexpr int TM = BM / 64;  // 2 32-row A fragments per wave
  constexpr int TN = 1;        // 1 32-column B fragment per wave
  constexpr int KS = BK / 16;  // 2 k-steps per tile
  constexpr int AREG = HG_STAGES * NP * C::A_BYTES;  // A region: 72 KB
  constexpr int ASLOT = NP * C::A_BYTES, BSLOT = NP * C::B_BYTES;
  static_assert(C::A_PW == 1 && C::B_PW == 1, "one 1-KiB piece per wave per plane");
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_BYTES / 4];
  char* const lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * HG_BN, m0 = by * BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

  f32x16 acc[TM][TN], acs[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[i][0][r] = 0.f;
      acs[i][0][r] = 0.f;
    }

  // LDS-DMA: buffer descriptors over plane 0 of each operand; lane offsets
  // 32-bit; plane and k-tile advance in the scalar soffset
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, 0x00020000);
  const unsigned oa =
      (unsigned)((const char*)hg_src<AL, BM, BK>(g.A, g.lda, g.M, m0, kbeg, wave, lane) -
                 (const char*)g.A);
  const unsigned ob =
      (unsigned)((const char*)hg_src<BL, HG_BN, BK>(g.B, g.ldb, g.N, n0, kbeg, wave, lane) -
                 (const char*)g.B);
  const unsigned stepA = 2u * (AL == L_RK ? BK : (unsigned)BK * g.lda);  // bytes per k-tile
  const unsigned stepB = 2u * (BL == L_RK ? BK : (unsigned)BK * g.ldb);
  const unsigned psA = 2u * (unsigned)g.pa, psB = 2u * (unsigned)g.pb;  // plane strides
  // DMA piece q of k-tile t into slot SL: q = 2 p + (0: A, 1: B)
  auto piece = [&](int t, auto sl_c, int q) {
    constexpr int SL = decltype(sl_c)::value;
#ifdef DDPG_H3_ABL_NODMA  // tools/h3_phase_bench.hip ablation only: no staging after the prologue
    if (t > 1) return;
#endif
    const int p = q >> 1;
    if ((q & 1) == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (lds_void*)(lds + SL * ASLOT + p * C::A_BYTES + wave * 1024), 16, oa,
          t * stepA + p * psA, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (lds_void*)(lds + AREG + SL * BSLOT + p * C::B_BYTES + wave * 1024), 16, ob,
          t * stepB + p * psB, 0, 0);
  };

  // ---- fragment-read bases (see the header).  RK: row r = rb + li, chunk
  // (2 ks + h) ^ ((r >> 2) & 3); rb % 32 == 0 leaves the swizzle to li.
  const unsigned lbase = (unsigned)(uintptr_t)(lds_char*)lds;
  const int h = lane >> 5, li = lane & 31;
  auto rk_pat = [&](int rb, int ks) {
    const int r = rb + li;
    return (unsigned)(r * (2 * BK) + 16 * ((2 * ks + h) ^ ((r >> 2) & 3)));
  };
  // KR ([BK][128] image): lane 4q + p of each 16-lane group g addresses k-row
  // k0 = 16 ks + 8 h + q (half 0) or k0 + 4 (half 1), columns col .. +3
  auto kr_pat = [&](int rb, int half) {
    const int gq = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 16 * gq + 4 * p;
    const int ch = (col & 127) >> 3;
    const int k = 8 * h + q + 4 * half;  // ks = 0; ks = 1 adds 16 rows (4 KB)
    return (unsigned)(k * 256 + 16 * (ch ^ kr_swz(k)) + 8 * (p & 1));
  };
  constexpr int NAB = AL == L_RK ? 2 : 2 * TM;  // A patterns
  constexpr int NBB = 2;                        // B patterns
  unsigned abase[2][NAB], bbase[2][NBB];       // [region: slots 0-1 / slot 2]
#pragma unroll
  for (int reg = 0; reg < 2; ++reg) {
    const unsigned ao = lbase + (reg ? 2 * ASLOT : 0);
    const unsigned bo = lbase + AREG + (reg ? 2 * BSLOT : 0);
#pragma unroll
    for (int x = 0; x < NAB; ++x)
      abase[reg][x] = ao + (AL == L_RK ? rk_pat(wm * (BM / 2), x)
                                       : kr_pat(wm * (BM / 2) + 32 * (x >> 1), x & 1));
#pragma unroll
    for (int x = 0; x < NBB; ++x)
      bbase[reg][x] = bo + (BL == L_RK ? rk_pat(wn * 32, x) : kr_pat(wn * 32, x));
  }
  // read group J (of NP (TM + TN)) of k-step KSR from slot SL: plane J / 3,
  // fragment J % 3 (0: B, 1 .. TM: A row block f - 1)
  auto read_one = [&](auto sl_c, auto ks_c, auto j_c, bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP][TN]) {
    constexpr int SL = decltype(sl_c)::value, KSR = decltype(ks_c)::value;
    constexpr int J = decltype(j_c)::value;
    constexpr int P = J / (TM + TN), F = J % (TM + TN);
    constexpr int REG = SL == 2 ? 1 : 0;
    constexpr int SO = SL == 2 ? 0 : SL;  // slot within the region
#ifdef DDPG_H3_ABL_NOREAD  // tools/h3_phase_bench.hip ablation only
    return;
#endif
    if constexpr (F < TN) {
      constexpr int OFF = SO * BSLOT + P * C::B_BYTES;
      if constexpr (BL == L_RK) {
        bv[P][0] = b128_read_off<OFF>(bbase[REG][KSR]);
      } else {
        constexpr int O2 = OFF + KSR * 16 * 256;
        bv[P][0] = __builtin_shufflevector(tr_read_off<O2>(bbase[REG][0]),
                                           tr_read_off<O2>(bbase[REG][1]), 0, 1, 2, 3, 4, 5, 6,
                                           7);
      }
    } else {
      constexpr int I = F - TN;
      constexpr int OFF = SO * ASLOT + P * C::A_BYTES;
      if constexpr (AL == L_RK) {
        av[P][I] = b128_read_off<OFF + I * 32 * (2 * BK)>(abase[REG][KSR]);
      } else {
        constexpr int O2 = OFF + KSR * 16 * 256;
        av[P][I] = __builtin_shufflevector(tr_read_off<O2>(abase[REG][2 * I]),
                                           tr_read_off<O2>(abase[REG][2 * I + 1]), 0, 1, 2, 3,
                                           4, 5, 6, 7);
      }
    }
  };
  // the 6 plane products of output block i, in gemm_h_kernel's order
  auto mfma_q = [&](int i, int q, bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP][TN]) {
#ifdef DDPG_H3_ABL_NOMFMA  // tools/h3_phase_bench.hip ablation only
    return;
#endif
    if (q == 0) acs[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0][0], acs[i][0], 0, 0, 0);
    if (q == 1) acs[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1][0], acs[i][0], 0, 0, 0);
    if (q == 2) acs[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2][0], acs[i][0], 0, 0, 0);
    if (q == 3) acs[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][0], acs[i][0], 0, 0, 0);
    if (q == 4) acs[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][0], acs[i][0], 0, 0, 0);
    if (q == 5) acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][0], acc[i][0], 0, 0, 0);
  };

  bf16x8 fa[2][NP][TM], fb[2][NP][TN];
  constexpr int NRG = NP * (TM + TN);  // 9 read groups per k-step
  constexpr int NMF = TM * TN * 6;     // 12 MFMAs per k-step
  // one k-tile t in slot SL.  ST: stage tile t+2 (into slot (SL + 2) % 3);
  // NX: tile t+1 exists
  auto tile = [&](int t, auto sl_c, auto st_c, auto nx_c) {
    constexpr int SL = decltype(sl_c)::value;
    constexpr bool ST = decltype(st_c)::value;
    constexpr bool NX = decltype(nx_c)::value;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      auto& av = fa[ks & 1];
      auto& bv = fb[ks & 1];
      constexpr bool RD = ks + 1 < KS || NX;  // reads to issue in this step
      constexpr int RSL = ks + 1 < KS ? SL : (SL + 1) % 3;
      constexpr int RKS = ks + 1 < KS ? ks + 1 : 0;
      auto& nav = fa[(ks + 1) & 1];
      auto& nbv = fb[(ks + 1) & 1];
      hg_wait16<NP, TM, TN>(av, bv);
      if constexpr (ks + 1 == KS && NX) {
        if constexpr (ST)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      constexpr bool GL = ST && ks == 0;  // the tile's DMA goes into step 0's gaps
      constexpr int g0 = (NRG + 1) / 2;   // first MFMA gap without reads
      static_for<NMF>([&](auto q_c) {
        constexpr int q = decltype(q_c)::value;
        mfma_q(q / 6, q % 6, av, bv);
        if constexpr (RD) {
          if constexpr (2 * q < NRG)
            read_one(std::integral_constant<int, RSL>{}, std::integral_constant<int, RKS>{},
                     std::integral_constant<int, 2 * q>{}, nav, nbv);
          if constexpr (2 * q + 1 < NRG)
            read_one(std::integral_constant<int, RSL>{}, std::integral_constant<int, RKS>{},
                     std::integral_constant<int, 2 * q + 1>{}, nav, nbv);
        }
        if constexpr (GL && q >= g0 && q - g0 < C::G)
          piece(t + 2, std::integral_constant<int, (SL + 2) % 3>{}, q - g0);
        if constexpr (GL && q == NMF - 1 && C::G > NMF - g0) {
#pragma unroll
          for (int r = NMF - g0; r < C::G; ++r)
            piece(t + 2, std::integral_constant<int, (SL + 2) % 3>{}, r);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;

  if (nk > 0) {
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(0, S0{}, q);
    if (nk > 1) {
#pragma unroll
      for (int q = 0; q < C::G; ++q) piece(1, S1{}, q);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    static_for<NRG>([&](auto j_c) { read_one(S0{}, std::integral_constant<int, 0>{}, j_c, fa[0], fb[0]); });
    __builtin_amdgcn_sched_barrier(0);
#ifdef DDPG_H3_STAMP_PROLOGUE
    KC_STAMP(2)
#endif
    int t = 0;
    // full trips of three tiles (slots 0, 1, 2), each staging t + 2
    for (; t + 4 < nk; t += 3) {
      tile(t, S0{}, T_{}, T_{});
      tile(t + 1, S1{}, T_{}, T_{});
      tile(t + 2, S2{}, T_{}, T_{});
    }
    // the last 1 .. 4 tiles (slots 0, 1, 2, 0)
    switch (nk - t) {
      case 4:
        tile(t, S0{}, T_{}, T_{});
        tile(t + 1, S1{}, T_{}, T_{});
        tile(t + 2, S2{}, F_{}, T_{});
        tile(t + 3, S0{}, F_{}, F_{});
        break;
      case 3:
        tile(t, S0{}, T_{}, T_{});
        tile(t + 1, S1{}, F_{}, T_{});
        tile(t + 2, S2{}, F_{}, F_{});
        break;
      case 2:
        tile(t, S0{}, F_{}, T_{});
        tile(t + 1, S1{}, F_{}, F_{});
        break;
      default:
        tile(t, S0{}, F_{}, F_{});
        break;
    }
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) acc[i][0] += acs[i][0];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  KC_STAMP(1)
  int ze = z;
  if (g.kpart) {  // small-M plan: this launch's splits are combined here
    if (!ksplit_combine<TM>(&acc[0][0], g.kpart, g.kticket, by * gridDim.x + bx, z, gridDim.z,
                            tid, HG_NT))
      return;
    ze = 0;
  }
#ifndef DDPG_H3_STAMP_PROLOGUE
  KC_STAMP(2)
#endif
  __syncthreads();  // staging buffers are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  // the whole 128-row tile in one LDS pass (fits the 144-KB staging region)
  static_assert((BM * (HG_BN + 4) + HG_BN * PROJ_MAX + 2 * GNT + BM * 64) * 4 <= C::SMEM_BYTES,
                "epilogue LDS (+ the narrow rows of a fused weight gradient)");
  gemm_epilogue<BM, HG_BN, WGN, 32, BM>(acc, smem, ge, tid, n0, m0, ze, bx, by);
  KC_STAMP(3)
}

}  // namespace ddpg

namespace ddpg {

// The bf16-configuration GEMM gemm_h16_kernel<AL, BL, 1, 256, 64> (SCH = 0)
// with cheaper addressing.  Its loop carried 24 v_subrev + 26 v_add + 10
// v_lshl_add_u64 per 32 MFMAs, and a v_mfma_f32_16x16x32_bf16 gap hides only
// about two VALU issues.  Here the ring slot stays a runtime value (a loop
// unrolled by the three slots, as gemm_h3_kernel, spilled at 16x16x32's
// register count) but is applied once per tile: every fragment read is a
// per-lane base + the slot's byte offset (one v_add per base and tile) + an
// immediate offset, and the LDS-DMA goes through buffer_load ... lds with the
// k-tile advance in the scalar soffset.  RK A operands (forward, dX).  Same
// schedule and MFMA order: bitwise equal to gemm_h16_kernel
// (DDPG_GEMM_H3=0 selects it).
// SPR = 1: the fragment reads of step ks+1 go one read group per MFMA gap of
// step ks instead of as one burst ahead of its MFMAs (schedule knob)
template <int AL, int BL, int SPR = 0>
DDPG_DEV void gemm_h16i_body(const GemmHArgs& g, int z) {
  static_assert(AL == L_RK, "RK A operand");
  constexpr int NP = 1, BM = 256, BK = 64;
  using C = HgCfg<BM, BK, NP>;
  constexpr int TM = BM / 64;   // 32-row blocks per wave (epilogue layout)
  constexpr int TA = BM / 32;   // 16-row A fragments per wave
  constexpr int TB = 2;         // 16-column B fragments per wave
  constexpr int KS = BK / 32;   // 2 32-deep steps per tile
  static_assert(C::A_PW == 4 && C::B_PW == 2 && KS == 2, "tile shape");
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_BYTES / 4];
  char* const lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * HG_BN, m0 = by * BM;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

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
    ob[i] = (unsigned)((const char*)hg_src<BL, HG_BN, BK, 16>(g.B, g.ldb, g.N, n0, kbeg,
                                                             wave * C::B_PW + i, lane) -
                       (const char*)g.B);
  const unsigned stepA = 2u * BK;  // RK A
  const unsigned stepB = 2u * (BL == L_RK ? BK : (unsigned)BK * g.ldb);
  // stage layout as gemm_h16_kernel: [A image | B image] per slot
  auto piece = [&](int t, int buf, int q) {
    char* base = lds + buf * C::STAGE;
    if (q < C::A_PW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (lds_void*)(base + (wave * C::A_PW + q) * 1024), 16, oa[q], t * stepA, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (lds_void*)(base + C::A_BYTES + (wave * C::B_PW + q - C::A_PW) * 1024), 16,
          ob[q - C::A_PW], t * stepB, 0, 0);
  };
  auto stage = [&](int t, int buf) {
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(t, buf, q);
  };

  // per-lane bases in slot 0.  RK image rows of 128 B, chunk
  // (4 ks + (lane >> 4)) ^ ((r >> 1) & 7); rb % 16 == 0 leaves the swizzle to
  // lane & 15 -> one pattern per ks.  KR B image ([64][128], kr_swz): per
  // 16-column fragment j and k-row half.
  const unsigned lbase = (unsigned)(uintptr_t)(lds_char*)lds;
  auto rk_pat = [&](int rb, int ks) {
    const int r = rb + (lane & 15);
    return (unsigned)(r * (2 * BK) + 16 * ((4 * ks + (lane >> 4)) ^ ((r >> 1) & 7)));
  };
  auto kr_pat = [&](int rb, int half) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 4 * p;
    const int ch = (col & 127) >> 3;
    const int k = 8 * (lane >> 4) + q + 4 * half;  // ks = 0; ks = 1 adds 32 rows (8 KB)
    return (unsigned)((col >> 7) * (BK * 256) + k * 256 + 16 * (ch ^ kr_swz(k)) + 8 * (p & 1));
  };
  constexpr int NBB = BL == L_RK ? 2 : 2 * TB;
  unsigned abase[2], bbase[NBB];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) abase[ks] = lbase + rk_pat(wm * (BM / 2), ks);
#pragma unroll
  for (int x = 0; x < NBB; ++x)
    bbase[x] = lbase + C::A_BYTES +
               (BL == L_RK ? rk_pat(wn * 32, x) : kr_pat(wn * 32 + 16 * (x >> 1), x & 1));
  // the fragments of k-step KSR from the slot at byte offset so
  auto read = [&](unsigned so, auto ks_c, bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
    constexpr int KSR = decltype(ks_c)::value;
    if constexpr (BL == L_RK) {
      const unsigned b = bbase[KSR] + so;
      static_for<TB>([&](auto j_c) {
        constexpr int J = decltype(j_c)::value;
        bv[0][J] = b128_read_off<J * 16 * (2 * BK)>(b);
      });
    } else {
      static_for<TB>([&](auto j_c) {
        constexpr int J = decltype(j_c)::value;
        constexpr int OFF = KSR * 32 * 256;
        bv[0][J] = __builtin_shufflevector(tr_read_off<OFF>(bbase[2 * J] + so),
                                           tr_read_off<OFF>(bbase[2 * J + 1] + so), 0, 1, 2, 3,
                                           4, 5, 6, 7);
      });
    }
    const unsigned a = abase[KSR] + so;
    static_for<TA>([&](auto i_c) {
      constexpr int I = decltype(i_c)::value;
      av[0][I] = b128_read_off<I * 16 * (2 * BK)>(a);
    });
  };
  // one read group of read(): B fragment R (R < TB), else A fragment R - TB
  auto read_group = [&](unsigned so, auto ks_c, auto r_c, bf16x8 (&av)[NP][TA],
                        bf16x8 (&bv)[NP][TB]) {
    constexpr int KSR = decltype(ks_c)::value, R = decltype(r_c)::value;
    if constexpr (R < TB) {
      if constexpr (BL == L_RK) {
        bv[0][R] = b128_read_off<R * 16 * (2 * BK)>(bbase[KSR] + so);
      } else {
        constexpr int OFF = KSR * 32 * 256;
        bv[0][R] = __builtin_shufflevector(tr_read_off<OFF>(bbase[2 * R] + so),
                                           tr_read_off<OFF>(bbase[2 * R + 1] + so), 0, 1, 2, 3,
                                           4, 5, 6, 7);
      }
    } else {
      av[0][R - TB] = b128_read_off<(R - TB) * 16 * (2 * BK)>(abase[KSR] + so);
    }
  };
  auto mfma_all = [&](bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
  };

  bf16x8 fa[2][NP][TA], fb[2][NP][TB];
  constexpr int NM = TA * TB;
  // gemm_h16_kernel's tile: STAGE3: stage tile t+3 after X_t into tile t's
  // slot; NEXT: tile t+1 exists; G2: tile t+2 was staged (vmcnt(G) at X_t)
  auto tile = [&](int t, auto stage_c, auto next_c, auto g2_c) {
    constexpr bool STAGE3 = decltype(stage_c)::value;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr bool G2 = decltype(g2_c)::value;
    const int slot = t % HG_STAGES;
    const unsigned so = (unsigned)slot * C::STAGE;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      constexpr int cs = ks & 1, ns = (ks + 1) & 1;
      hg_wait16<NP, TA, TB>(fa[cs], fb[cs]);
      if constexpr (ks + 1 == KS && NEXT) {
        if constexpr (G2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      constexpr bool RD = ks + 1 < KS || NEXT;  // this step reads the next one's fragments
      const unsigned rso =
          ks + 1 < KS ? so : (unsigned)((slot + 1) % HG_STAGES) * C::STAGE;
      constexpr int RKS = ks + 1 < KS ? ks + 1 : 0;
      if constexpr (!SPR && RD) read(rso, std::integral_constant<int, RKS>{}, fa[ns], fb[ns]);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (SPR && RD) {
        // read group r (B fragment r < TB, then A fragment r - TB) after MFMA r
        static_for<TA * TB>([&](auto q_c) {
          constexpr int q = decltype(q_c)::value, i = q / TB, j = q % TB;
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cs][0][i], fb[cs][0][j],
                                                              acc[i][j], 0, 0, 0);
          if constexpr (q < TA + TB) read_group(rso, std::integral_constant<int, RKS>{},
                                                std::integral_constant<int, q>{}, fa[ns], fb[ns]);
          // the tile-(t+3) LDS-DMA in the gaps after the reads
          if constexpr (ks + 1 == KS && STAGE3 && q >= TA + TB && q - (TA + TB) < C::G)
            piece(t + 3, slot, q - (TA + TB));
          __builtin_amdgcn_sched_barrier(0);
        });
      } else {
        mfma_all(fa[cs], fb[cs]);
      }
      if constexpr (ks + 1 == KS && STAGE3 && !(SPR && RD)) {
        stage(t + 3, slot);
        constexpr int NG = C::G, MPG = NM / NG > 0 ? NM / NG : 1;
        static_for<NG>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, MPG, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        });
        if constexpr (NM - MPG * NG > 0)
          __builtin_amdgcn_sched_group_barrier(0x008, NM - MPG * NG, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  if (nk > 0) {
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    if (nk > 2) {
      stage(2, 2);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C::G) : "memory");
    } else if (nk > 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(0u, std::integral_constant<int, 0>{}, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    int t = 0;
    for (; t + 3 < nk; ++t) tile(t, T_{}, T_{}, T_{});  // stages t+3; t+2 in flight
    if (t + 2 < nk) tile(t++, F_{}, T_{}, T_{});         // t+2 in flight
    if (t + 1 < nk) tile(t++, F_{}, T_{}, F_{});
    tile(t, F_{}, F_{}, F_{});
  }
  // repack into the 32x32 register layout of gemm_epilogue<..., 16>
  f32x16 out[TM][1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int tr = 0; tr < 2; ++tr)
#pragma unroll
      for (int tc = 0; tc < 2; ++tc)
#pragma unroll
        for (int q = 0; q < 4; ++q) out[i][0][4 * (2 * tr + tc) + q] = acc[2 * i + tr][tc][q];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  int ze = z;
  if (g.kpart) {  // small-M plan: this launch's splits are combined here
    if (!ksplit_combine<TM>(&out[0][0], g.kpart, g.kticket, by * gridDim.x + bx, z, gridDim.z,
                            tid, HG_NT))
      return;
    ze = 0;
  }
  __syncthreads();  // staging buffers are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  static_assert(((BM / 2) * (HG_BN + 4) + HG_BN * PROJ_MAX + 2 * GNT + (BM / 2) * 64) * 4 <=
                    C::SMEM_BYTES,
                "epilogue LDS (+ the narrow rows of a fused weight gradient)");
  gemm_epilogue<BM, HG_BN, 4, 16>(out, smem, ge, tid, n0, m0, ze, bx, by);
}

template <int AL, int BL>
__global__ __launch_bounds__(HG_NT, 1) void gemm_h16i_kernel(GemmHArgs g) {
  gemm_h16i_body<AL, BL>(g, blockIdx.z);
}

// Up to GH_MAXP independent GEMMs of one grid shape in one launch, part =
// blockIdx.z (one split each, no in-launch combine): the batch-only first
// layers of the bf16 configuration (K = S > 64, so not thin_k's).  A CU's
// next block (the next part's tile) stages and computes while the previous
// block's epilogue stores drain, where separate launches wrote every output
// in one burst at the end of each.
template <int AL, int BL>
__global__ __launch_bounds__(HG_NT, 1) void gemm_h16i_pack_kernel(GemmHPack pk) {
  gemm_h16i_body<AL, BL>(pk.p[blockIdx.z], 0);
}

}  // namespace ddpg
