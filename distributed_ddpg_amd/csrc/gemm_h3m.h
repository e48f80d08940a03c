// The fp32-context twin GEMM (three exact bf16 planes, six plane products per
// MAC) on v_mfma_f32_16x16x32_bf16.
//
// Why the MFMA shape matters here.  gemm_h3_kernel (32x32x16) issues its
// MFMAs at 95 % of the pipe's cycle budget (1 600 of 1 536 cycles per k-tile,
// s_memtime stamps, profiles/r5/h3_phase_*.txt) when launched back to back in
// isolation, where the chip holds 1.2-1.3 GHz.  The same matrix work on the
// 16x16x32 shape (same cycles per flop) holds a 15-17 % higher clock: a bare
// MFMA loop with gemm_h3's per-k-tile work and barrier runs 2.05-2.09 GHz vs
// 1.75-1.78 GHz, 343 vs 300 TF-eq (tools/mfma_power_bench.hip,
// profiles/r5/mfma_power.txt; MI355X_MICROARCH.md "DVFS give-back" item 7).
// Inside the learner step the chip holds >= 1.9 GHz under this kernel
// (round 6 PMC wave clock, profiles/r6/clock_c3.txt), where it issues MFMAs
// <= 0.59 of the time and its waves wait on staging / barriers a third of
// their lifetime (profiles/r6/stall_c3.txt).
//
// Tile 128 x 128 x 32 as gemm_h3_kernel: 8 waves (2 along M x 4 along N),
// wave tile 64 x 32 = 4 x 2 16x16 output blocks, one 32-deep k-step per
// k-tile: 48 MFMAs (8 blocks x 6 plane products) and 18 fragment-plane reads
// per wave and k-tile.  Same staging (buffer_load ... lds into a 3-slot ring,
// 48 KB per slot), same LDS images except the RK chunk swizzle
// (rk_swz<32, 16>: a 16x16x32 fragment read has lane l on row l & 15, chunk
// l >> 4).  With one k-step per tile the fragment sets alternate per tile,
// so the loop is unrolled by 6 (slot x parity compile-time), and every
// fragment read is a per-lane base + a ds_read immediate as in gemm_h3.
// Schedule per tile t (slot s): wait own reads of t | vmcnt (t+1 landed,
// t+2 in flight) | barrier X_t | 48 MFMAs with the 18 reads of tile t+1 in
// the first gaps and the LDS-DMA of tile t+3 into slot s (every fragment of
// tile t is in registers once X_t is passed) in later gaps.
// The 16x16x32 MFMA sums 32 products per instruction (16 for 32x32x16), so
// results differ from gemm_h3_kernel in fp32 rounding only; both are
// fp32-accurate (DDPG_GEMM_M16=0 selects gemm_h3_kernel).
#pragma once
#include "gemm_h3.h"

namespace ddpg {

template <int AL, int BL>
DDPG_DEV void gemm_h3m_body(const GemmHArgs& g, int z) {
  KC_STAMP(0)
  constexpr int NP = 3, BM = 128, BK = 32;
  using C = HgCfg<BM, BK, NP, 8>;
  constexpr int TM = BM / 64;  // 32-row blocks per wave (epilogue layout)
  constexpr int TA = BM / 32;  // 4 16-row A fragments per wave
  constexpr int TB = 2;        // 2 16-column B fragments per wave
  constexpr int AREG = HG_STAGES * NP * C::A_BYTES;  // A region: 72 KB
  constexpr int ASLOT = NP * C::A_BYTES, BSLOT = NP * C::B_BYTES;
  static_assert(C::A_PW == 1 && C::B_PW == 1 && C::G == 6, "one 1-KiB piece per wave per plane");
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

  f32x4 acc[TA][TB], acs[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = acs[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, 0x00020000);
  const unsigned oa =
      (unsigned)((const char*)hg_src<AL, BM, BK, 16>(g.A, g.lda, g.M, m0, kbeg, wave, lane) -
                 (const char*)g.A);
  const unsigned ob =
      (unsigned)((const char*)hg_src<BL, HG_BN, BK, 16>(g.B, g.ldb, g.N, n0, kbeg, wave, lane) -
                 (const char*)g.B);
  const unsigned stepA = 2u * (AL == L_RK ? BK : (unsigned)BK * g.lda);  // bytes per k-tile
  const unsigned stepB = 2u * (BL == L_RK ? BK : (unsigned)BK * g.ldb);
  const unsigned psA = 2u * (unsigned)g.pa, psB = 2u * (unsigned)g.pb;  // plane strides
  // LDS-DMA piece q of k-tile t into slot SL: q = 2 p + (0: A, 1: B)
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

  // ---- fragment-read bases.  RK ([rows][32] image, 64-B rows): lane row
  // rb + (l & 15), chunk (l >> 4) ^ rk_swz<32, 16>(row); rb % 16 == 0, so one
  // pattern per operand and fragment i at + 1 KiB i.
  const unsigned lbase = (unsigned)(uintptr_t)(lds_char*)lds;
  auto rk_pat = [&](int rb) {
    const int r = rb + (lane & 15);
    return (unsigned)(r * (2 * BK) + 16 * ((lane >> 4) ^ rk_swz<BK, 16>(r)));
  };
  // KR ([32][128] image): lane 4q + p of each 16-lane group g addresses k-row
  // 8 g + q (half 0) or + 4 (half 1), columns rb + 4 p .. +3 (hg_frag16)
  auto kr_pat = [&](int rb, int half) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 4 * p;
    const int ch = (col & 127) >> 3;
    const int k = 8 * (lane >> 4) + q + 4 * half;
    return (unsigned)(k * 256 + 16 * (ch ^ kr_swz(k)) + 8 * (p & 1));
  };
  constexpr int NAB = AL == L_RK ? 1 : 2 * TA;  // A patterns per region
  constexpr int NBB = BL == L_RK ? 1 : 2 * TB;  // B patterns per region
  unsigned abase[2][NAB], bbase[2][NBB];        // [region: slots 0-1 / slot 2]
#pragma unroll
  for (int reg = 0; reg < 2; ++reg) {
    const unsigned ao = lbase + (reg ? 2 * ASLOT : 0);
    const unsigned bo = lbase + AREG + (reg ? 2 * BSLOT : 0);
#pragma unroll
    for (int x = 0; x < NAB; ++x)
      abase[reg][x] = ao + (AL == L_RK ? rk_pat(wm * (BM / 2)) : kr_pat(wm * (BM / 2) + 16 * (x >> 1), x & 1));
#pragma unroll
    for (int x = 0; x < NBB; ++x)
      bbase[reg][x] = bo + (BL == L_RK ? rk_pat(wn * 32) : kr_pat(wn * 32 + 16 * (x >> 1), x & 1));
  }
  // KR operands (the weight gradient's KR x KR) hold 2 TA + 2 TB per-lane
  // bases per region; the slot-2 region's are the slots-0-1 region's plus a
  // constant (2 slots), added at the read (an asm add the compiler cannot
  // hoist back into long-lived registers) -- 12 VGPRs fewer at the 256 limit
  auto kr_base = [&](unsigned b, auto reg_c, auto add_c) -> unsigned {
    constexpr int REG = decltype(reg_c)::value;
    constexpr unsigned ADD = decltype(add_c)::value;
    if constexpr (REG == 0) {
      return b;
    } else {
      unsigned r;
      asm volatile("v_add_u32 %0, %1, %2" : "=v"(r) : "n"(ADD), "v"(b));
      return r;
    }
  };
  // read group J (of NP (TA + TB)) from slot SL: plane J / 6, fragment
  // J % 6 (0 .. TB-1: B fragment, then the A fragments)
  auto read_one = [&](auto sl_c, auto j_c, bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
    constexpr int SL = decltype(sl_c)::value;
    constexpr int J = decltype(j_c)::value;
    constexpr int P = J / (TA + TB), F = J % (TA + TB);
    constexpr int REG = SL == 2 ? 1 : 0;
    constexpr int SO = SL == 2 ? 0 : SL;  // slot within the region
    if constexpr (F < TB) {
      constexpr int OFF = SO * BSLOT + P * C::B_BYTES;
      if constexpr (BL == L_RK) {
        bv[P][F] = b128_read_off<OFF + F * 16 * (2 * BK)>(bbase[REG][0]);
      } else {
        using RC = std::integral_constant<int, REG>;
        using AC = std::integral_constant<unsigned, 2u * BSLOT>;
        bv[P][F] = __builtin_shufflevector(tr_read_off<OFF>(kr_base(bbase[0][2 * F], RC{}, AC{})),
                                           tr_read_off<OFF>(kr_base(bbase[0][2 * F + 1], RC{}, AC{})), 0, 1, 2, 3,
                                           4, 5, 6, 7);
      }
    } else {
      constexpr int I = F - TB;
      constexpr int OFF = SO * ASLOT + P * C::A_BYTES;
      if constexpr (AL == L_RK) {
        av[P][I] = b128_read_off<OFF + I * 16 * (2 * BK)>(abase[REG][0]);
      } else {
        using RC = std::integral_constant<int, REG>;
        using AC = std::integral_constant<unsigned, 2u * ASLOT>;
        av[P][I] = __builtin_shufflevector(tr_read_off<OFF>(kr_base(abase[0][2 * I], RC{}, AC{})),
                                           tr_read_off<OFF>(kr_base(abase[0][2 * I + 1], RC{}, AC{})), 0, 1, 2, 3,
                                           4, 5, 6, 7);
      }
    }
  };
  // MFMA Q of a k-tile: product Q / 8 (the small terms lh, mm, hl, mh, hm
  // into acs, then hh into acc -- gemm_h3's per-block order), output block
  // Q % 8 = (i, j): eight independent accumulators between dependent MFMAs
  auto mfma_q = [&](auto q_c, bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
    constexpr int Q = decltype(q_c)::value;
    constexpr int PR = Q / (TA * TB), BQ = Q % (TA * TB), i = BQ / TB, j = BQ % TB;
    if constexpr (PR == 0) acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2][i], bv[0][j], acs[i][j], 0, 0, 0);
    if constexpr (PR == 1) acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[1][j], acs[i][j], 0, 0, 0);
    if constexpr (PR == 2) acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[2][j], acs[i][j], 0, 0, 0);
    if constexpr (PR == 3) acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[0][j], acs[i][j], 0, 0, 0);
    if constexpr (PR == 4) acs[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[1][j], acs[i][j], 0, 0, 0);
    if constexpr (PR == 5) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
  };

  bf16x8 fa[2][NP][TA], fb[2][NP][TB];
  constexpr int NRG = NP * (TA + TB);  // 18 read groups per k-tile
  constexpr int NMF = TA * TB * 6;     // 48 MFMAs per k-tile
#ifndef H3M_DG0  // schedule knobs (tools/h3_phase_bench.hip sweeps them)
#define H3M_DG0 (NRG + 2)
#define H3M_DGS 4
#define H3M_RPG 1
#endif
  constexpr int DG0 = H3M_DG0, DGS = H3M_DGS;  // LDS-DMA pieces in gaps DG0, DG0 + DGS, ...
  constexpr int RPG = H3M_RPG;                  // read groups per MFMA gap
  static_assert(DG0 + DGS * (C::G - 1) < NMF, "DMA gaps");
  // k-tile t in slot SL with fragment set PAR.  st: stage tile t+3 into slot
  // SL after X_t; nx: tile t+1 exists (read in this tile's gaps); g2: tile
  // t+2 is in flight (vmcnt(G) at X_t leaves it there)
  auto tile = [&](int t, auto sl_c, auto par_c, bool st, bool nx, bool g2) __attribute__((always_inline)) {
    constexpr int SL = decltype(sl_c)::value;
    constexpr int PAR = decltype(par_c)::value;
    auto& av = fa[PAR];
    auto& bv = fb[PAR];
    auto& nav = fa[PAR ^ 1];
    auto& nbv = fb[PAR ^ 1];
    hg_wait16<NP, TA, TB>(av, bv);
    if (nx) {
      if (g2)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    static_for<NMF>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      mfma_q(q_c, av, bv);
#ifdef H3M_RSPAN  // reads spread over the first H3M_RSPAN gaps (bench knob)
      static_for<NRG>([&](auto j_c) {
        constexpr int J = decltype(j_c)::value;
        if constexpr (J * H3M_RSPAN / NRG == q) {
          if (nx) read_one(std::integral_constant<int, (SL + 1) % 3>{}, j_c, nav, nbv);
        }
      });
#else
      static_for<RPG>([&](auto r_c) {
        constexpr int J = RPG * q + decltype(r_c)::value;
        if constexpr (J < NRG) {
          if (nx)
            read_one(std::integral_constant<int, (SL + 1) % 3>{}, std::integral_constant<int, J>{},
                     nav, nbv);
        }
      });
#endif
      if constexpr (q >= DG0 && (q - DG0) % DGS == 0 && (q - DG0) / DGS < C::G) {
        if (st) piece(t + 3, sl_c, (q - DG0) / DGS);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  using S2 = std::integral_constant<int, 2>;

  if (nk > 0) {
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(0, S0{}, q);
    if (nk > 1)
#pragma unroll
      for (int q = 0; q < C::G; ++q) piece(1, S1{}, q);
    if (nk > 2) {
#pragma unroll
      for (int q = 0; q < C::G; ++q) piece(2, S2{}, q);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * C::G) : "memory");
    } else if (nk > 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    static_for<NRG>([&](auto j_c) { read_one(S0{}, j_c, fa[0], fb[0]); });
    __builtin_amdgcn_sched_barrier(0);
#ifdef DDPG_H3_STAMP_PROLOGUE
    KC_STAMP(2)
#endif
#if defined(H3M_PRIO) && H3M_PRIO
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);  // schedule knob (bench only)
#endif
    int t = 0;
    // full trips of six tiles (slots 0 1 2 0 1 2, sets 0 1 0 1 0 1), every
    // tile staging t + 3
    for (; t + 8 < nk; t += 6) {
      tile(t, S0{}, S0{}, true, true, true);
      tile(t + 1, S1{}, S1{}, true, true, true);
      tile(t + 2, S2{}, S0{}, true, true, true);
      tile(t + 3, S0{}, S1{}, true, true, true);
      tile(t + 4, S1{}, S0{}, true, true, true);
      tile(t + 5, S2{}, S1{}, true, true, true);
    }
    // the last 1 .. 8 tiles, continuing the slot / set pattern
    static_for<8>([&](auto k_c) {
      constexpr int k = decltype(k_c)::value;
      const int tt = t + k;
      if (tt < nk)
        tile(tt, std::integral_constant<int, k % 3>{}, std::integral_constant<int, k & 1>{},
             tt + 3 < nk, tt + 1 < nk, tt + 2 < nk);
    });
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
        for (int q = 0; q < 4; ++q)
          out[i][0][4 * (2 * tr + tc) + q] = acc[2 * i + tr][tc][q] + acs[2 * i + tr][tc][q];
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  KC_STAMP(1)
  int ze = z;
  if (g.kpart) {  // small-M plan: this launch's splits are combined here
    if (!ksplit_combine<TM>(&out[0][0], g.kpart, g.kticket, by * gridDim.x + bx, z, gridDim.z,
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
  static_assert((BM * (HG_BN + 4) + HG_BN * PROJ_MAX + 2 * GNT + BM * 64) * 4 <= C::SMEM_BYTES,
                "epilogue LDS (+ the narrow rows of a fused weight gradient)");
  gemm_epilogue<BM, HG_BN, 4, 16, BM>(out, smem, ge, tid, n0, m0, ze, bx, by);
  KC_STAMP(3)
}

template <int AL, int BL>
__global__ __launch_bounds__(HG_NT, 1) void gemm_h3m_kernel(GemmHArgs g) {
  gemm_h3m_body<AL, BL>(g, blockIdx.z);
}

// Up to GH_MAXP independent GEMMs of one grid shape in one launch, part =
// blockIdx.z (one split each, no in-launch combine): the fp32 context's
// forward layers that read only the first layers' outputs (target actor W2,
// online actor W2, online critic Wh; learner_step_dev).  A CU's next block,
// the next part's tile, starts while the previous block's epilogue drains,
// instead of each launch's ramp and tail on its own.
template <int AL, int BL>
__global__ __launch_bounds__(HG_NT, 1) void gemm_h3m_pack_kernel(GemmHPack pk) {
  gemm_h3m_body<AL, BL>(pk.p[blockIdx.z], 0);
}

}  // namespace ddpg
