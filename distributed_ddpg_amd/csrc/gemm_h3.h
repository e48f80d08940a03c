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
__global__ __launch_bounds__(HG_NT, 1) void gemm_h3_kernel(GemmHArgs g) {
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
  __syncthreads();  // staging buffers are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  gemm_epilogue<BM, HG_BN, WGN>(acc, smem, ge, tid, n0, m0, z, bx, by);
}

}  // namespace ddpg
