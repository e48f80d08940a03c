// GEMM on bf16 operands that are already bf16 in HBM (gfx950,
// v_mfma_f32_32x32x16_bf16, fp32 accumulation), with the fused epilogues of
// gemm_common.h.  The operands are the bf16 "twins" the producers write next
// to their fp32 outputs (GEMM epilogues, gather, Adam, soft update):
//   NP = 1: bf16(x)                      -- the bf16 configuration (C5)
//   NP = 3: the exact h/m/l split of x   -- fp32-accurate (six plane products,
//           x y ~ hh + hm + mh + hl + mm + lh, as gemm_s3.h but split once by
//           the producer instead of in every GEMM's staging loop)
// so the staging path moves 2 B per element and does no conversion work.
//
// Block tile BM x 128 x BK, 512 threads = 8 waves (2 along M x 4 along N),
// wave tile (BM/2) x 32 = BM/64 MFMA tiles.  Staging is global_load_lds
// (16 B per lane, 1 KiB per wave instruction) into a 3-stage LDS ring with a
// counted vmcnt, so tile t+1's loads stay in flight across the one barrier
// per k-tile while tile t is consumed.  LDS images (per plane):
//   RK operand (rows contiguous in k): [rows][BK], 16-B chunk c of row r at
//     chunk c ^ swz(r) -- every 16-lane ds_read_b128 group of a fragment read
//     hits 16 distinct bank slots;
//   KR operand (k-major): [BK][128] sub-images with 256-B rows, chunk c of
//     k-row r at c ^ ((r & 3) << 2 | (r >> 2) & 3), read as the MFMA operand by
//     two ds_read_b64_tr_b16 (hardware transpose) per fragment, conflict-free.
// global_load_lds writes lane-linear LDS, so the swizzle is applied to each
// lane's SOURCE address.  Rows / columns past M or N are clamped (their
// outputs are discarded by the epilogue); K must be a multiple of BK per split.
#pragma once
#include <type_traits>
#include <utility>
#include "gemm_bf16.h"

namespace ddpg {

// f(std::integral_constant<int, 0>{}) ... f(std::integral_constant<int, N-1>{})
template <typename F, int... I>
DDPG_DEV void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
DDPG_DEV void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// GemmHArgs: types.h


constexpr int HG_NT = 512, HG_BN = 128, HG_STAGES = 3;

template <int BM, int BK, int NP, int NW = 8>
struct HgCfg {
  static constexpr int A_BYTES = BM * BK * 2;  // one plane, one stage
  static constexpr int B_BYTES = HG_BN * BK * 2;
  static constexpr int STAGE = NP * (A_BYTES + B_BYTES);
  static constexpr int A_PW = A_BYTES / 1024 / NW;  // 1-KiB pieces per wave per plane
  static constexpr int B_PW = B_BYTES / 1024 / NW;
  static constexpr int G = NP * (A_PW + B_PW);  // glds instructions per wave per k-tile
  static constexpr int EPI_BYTES = TileCfg<BM, HG_BN>::EPI * 4;
  static constexpr int SMEM_BYTES =
      HG_STAGES * STAGE > EPI_BYTES ? HG_STAGES * STAGE : EPI_BYTES;
  static_assert(A_PW >= 1 && B_PW >= 1 && A_PW * 1024 * NW == A_BYTES &&
                    B_PW * 1024 * NW == B_BYTES,
                "tile must split into whole 1-KiB pieces per wave");
  static_assert(SMEM_BYTES <= 160 * 1024, "LDS");
};

// RK image: rows of 2*BK bytes; chunk swizzle spreading 16 consecutive rows
// over the 16 slots of a 256-B bank row
// MF = 16 (16x16x32 fragments: lane l reads row l & 15, 16-B chunk l >> 4 of
// the 32-k step) at BK = 32 needs a different spread over the ds_read_b128
// lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...: (row >> 2) & 2.
template <int BK, int MF = 32>
DDPG_DEV int rk_swz(int row) {
  if constexpr (BK == 64)
    return (row >> 1) & 7;
  else if constexpr (MF == 16)
    return (row >> 2) & 2;
  else
    return (row >> 2) & 3;
}
DDPG_DEV int kr_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Source address of this lane's 16 B of piece `piece` (1 KiB of the image).
// R = row extent of the operand (M or N), r0 = the block's first row,
// BR = image rows (BM or 128).
template <int L, int BR, int BK, int MF = 32>
DDPG_DEV const __bf16* hg_src(const __bf16* P, int ld, int R, int r0, int kbeg, int piece,
                              int lane) {
  const int off = piece * 1024 + 16 * lane;
  if constexpr (L == L_RK) {
    constexpr int RB = 2 * BK;
    const int row = off / RB, pc = (off % RB) >> 4;
    const int c = pc ^ rk_swz<BK, MF>(row);
    const int gr = min(r0 + row, R - 1);
    return P + (size_t)gr * ld + kbeg + 8 * c;
  } else {
    constexpr int SUB = BK * 256;  // one [BK][128] sub-image
    const int sub = off / SUB, o2 = off % SUB;
    const int row = o2 >> 8, pc = (o2 & 255) >> 4;
    const int c = pc ^ kr_swz(row);
    const int col = min(r0 + 128 * sub + 8 * c, R - 8);  // R % 8 == 0
    return P + (size_t)(kbeg + row) * ld + col;
  }
}

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;

// Fragment reads as inline asm: the builtin ds_read_b64_tr_b16 makes hipcc
// wait vmcnt(0) before it (it cannot rule out an overlap with the in-flight
// global_load_lds writes), which would drain the staging pipeline every
// k-tile; with every fragment read in asm the k-step loop is software
// pipelined by hand (counted lgkmcnt, hg_wait).
DDPG_DEV bf16x4 tr_read(const char* p) {
  bf16x4 r;
  const unsigned a = (unsigned)(uintptr_t)(lds_char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

DDPG_DEV bf16x8 b128_read(const char* p) {
  bf16x8 r;
  const unsigned a = (unsigned)(uintptr_t)(lds_char*)p;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// MFMA fragment (lane: row/col li of the operand tile starting at image row
// `rb`, k = 16 ks + 8 h .. +7) from one plane image.
template <int L, int BK>
DDPG_DEV bf16x8 hg_frag(const char* img, int rb, int ks, int lane) {
  const int h = lane >> 5, li = lane & 31;
  if constexpr (L == L_RK) {
    const int r = rb + li;
    const int c = (2 * ks + h) ^ rk_swz<BK>(r);
    return b128_read(img + r * (2 * BK) + 16 * c);
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of a 16-lane group addresses k-row q,
    // columns 4p..4p+3 of the group's 16 columns; lane i receives column i.
    const int g = (lane >> 4) & 1, q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 16 * g + 4 * p;
    const char* sub = img + (col >> 7) * (BK * 256);
    const int ch = (col & 127) >> 3;
    const int k0 = 16 * ks + 8 * h + q, k1 = k0 + 4;
    const char* a0 = sub + k0 * 256 + 16 * (ch ^ kr_swz(k0)) + 8 * (p & 1);
    const char* a1 = sub + k1 * 256 + 16 * (ch ^ kr_swz(k1)) + 8 * (p & 1);
    return __builtin_shufflevector(tr_read(a0), tr_read(a1), 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// 16x16x32 MFMA fragment (lane: row/col l & 15 of the operand tile starting
// at image row `rb`, k = 32 ks + 8 (l >> 4) .. +7).  KR: the same
// ds_read_b64_tr_b16 pair as hg_frag, with the four 16-lane groups on four
// k-row octets (conflict-free under kr_swz).
template <int L, int BK>
DDPG_DEV bf16x8 hg_frag16(const char* img, int rb, int ks, int lane) {
  if constexpr (L == L_RK) {
    const int r = rb + (lane & 15);
    const int c = (4 * ks + (lane >> 4)) ^ rk_swz<BK, 16>(r);
    return b128_read(img + r * (2 * BK) + 16 * c);
  } else {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int col = rb + 4 * p;
    const char* sub = img + (col >> 7) * (BK * 256);
    const int ch = (col & 127) >> 3;
    const int k0 = 32 * ks + 8 * (lane >> 4) + q, k1 = k0 + 4;
    const char* a0 = sub + k0 * 256 + 16 * (ch ^ kr_swz(k0)) + 8 * (p & 1);
    const char* a1 = sub + k1 * 256 + 16 * (ch ^ kr_swz(k1)) + 8 * (p & 1);
    return __builtin_shufflevector(tr_read(a0), tr_read(a1), 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// lgkmcnt(0) tied to the fragments, so no MFMA reading them is scheduled
// above the wait
template <int N, int NP, int TM>
DDPG_DEV void hg_wait(bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP]) {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    asm volatile("" : "+v"(bv[p]));
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(av[p][i]));
  }
}
template <int NP, int TA, int TB>
DDPG_DEV void hg_wait16(bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int p = 0; p < NP; ++p) {
#pragma unroll
    for (int j = 0; j < TB; ++j) asm volatile("" : "+v"(bv[p][j]));
#pragma unroll
    for (int i = 0; i < TA; ++i) asm volatile("" : "+v"(av[p][i]));
  }
}

// Main loop (software-pipelined across k-tiles; every phase boundary is a
// sched_barrier so hipcc cannot sink the MFMAs below the next step's waits):
//   k-step ks < KS-1: wait own reads of ks | issue reads of ks+1 | MFMAs of ks,
//                     with this tile's share of the tile-(t+2) glds between them
//   k-step KS-1:      wait own reads | vmcnt (tile t+1 landed) | s_barrier |
//                     issue reads of tile t+1 k-step 0 | MFMAs of KS-1
// so the barrier and the next tile's first LDS reads sit under one k-step of
// MFMAs.  Ring of 3 LDS stages: tile t+2 is staged into tile t-1's buffer,
// whose reads every wave finished before the barrier that ended tile t-1.
//
// Measured alternative (tools/gemmh_bench.hip, round 2): one tile in flight
// with waves 4-7 staggered KS/2 k-steps behind waves 0-3 (so SIMD partners
// are in different phases) is 15-25 % SLOWER on every C3/C5 shape than two
// tiles in flight without a stagger: the glds latency under full load, not
// the phase pairing, is what the second tile in flight covers.
//
// SCH = 1: the fragment reads of step ks+1 are spread between the MFMAs of
// step ks (two read groups per MFMA gap, in program order pinned by
// sched_barriers) instead of issued as one burst ahead of them, and the
// tile-(t+2) glds sit in the MFMA gaps after the reads.
//
// WGN: waves along N.  4 (default): 8 waves, wave tile (BM/2) x 32.  2: 4
// waves (one per SIMD), wave tile (BM/2) x 64 -- every A fragment feeds two
// B fragments: a k-step reads NP (TM + TN) fragments for 6 TM TN MFMAs (NP =
// 3, BM = 128: 12 reads per 24 MFMAs instead of 9 per 12, so 2/3 of the LDS
// read bytes per MFMA).
template <int AL, int BL, int NP, int BM, int BK, int SCH = 0, int WGN = 4>
__global__ __launch_bounds__(128 * WGN, 1) void gemm_h_kernel(GemmHArgs g) {
  constexpr int NW = 2 * WGN;
  using C = HgCfg<BM, BK, NP, NW>;
  constexpr int TM = BM / 64;
  constexpr int TN = 4 / WGN;      // 32-column MFMA tiles per wave
  constexpr int WCOL = HG_BN / WGN;  // columns per wave
  constexpr int KS = BK / 16;
  static_assert(KS % 2 == 0, "fragment register sets alternate by k-step parity");
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

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // NP = 3: the five small plane products go to their own accumulators, so
  // the main (hh) chain takes one rounding per k-step instead of six
  f32x16 acs[NP == 3 ? TM : 1][NP == 3 ? TN : 1];
  if constexpr (NP == 3) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acs[i][j][r] = 0.f;
  }

  const __bf16* sa[C::A_PW];
  const __bf16* sb[C::B_PW];
#pragma unroll
  for (int i = 0; i < C::A_PW; ++i)
    sa[i] = hg_src<AL, BM, BK>(g.A, g.lda, g.M, m0, kbeg, wave * C::A_PW + i, lane);
#pragma unroll
  for (int i = 0; i < C::B_PW; ++i)
    sb[i] = hg_src<BL, HG_BN, BK>(g.B, g.ldb, g.N, n0, kbeg, wave * C::B_PW + i, lane);
  const long long stepA = AL == L_RK ? BK : (long long)BK * g.lda;
  const long long stepB = BL == L_RK ? BK : (long long)BK * g.ldb;

  // glds piece q (0 .. G-1) of k-tile t into stage buffer `buf`
  auto piece = [&](int t, int buf, int q) {
    char* base = lds + buf * C::STAGE;
    const int p = q / (C::A_PW + C::B_PW), r = q % (C::A_PW + C::B_PW);
    if (r < C::A_PW)
      __builtin_amdgcn_global_load_lds(
          (const void*)(sa[r] + p * g.pa + t * stepA),
          (lds_void*)(base + p * C::A_BYTES + (wave * C::A_PW + r) * 1024), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds(
          (const void*)(sb[r - C::A_PW] + p * g.pb + t * stepB),
          (lds_void*)(base + NP * C::A_BYTES + p * C::B_BYTES +
                      (wave * C::B_PW + r - C::A_PW) * 1024),
          16, 0, 0);
  };
  auto stage = [&](int t, int buf) {
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(t, buf, q);
  };

  auto read = [&](const char* base, int ks, bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP][TN]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[p][j] = hg_frag<BL, BK>(base + NP * C::A_BYTES + p * C::B_BYTES, wn * WCOL + 32 * j,
                                   ks, lane);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[p][i] = hg_frag<AL, BK>(base + p * C::A_BYTES, wm * (BM / 2) + 32 * i, ks, lane);
    }
  };
  auto mfma_i = [&](int i, bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP][TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (NP == 3) {
        // small terms, smallest first: lh, mm, hl, mh, hm  (planes 0 = h, 1 = m, 2 = l)
        f32x16 c = acs[i][j];
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][j], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][j], c, 0, 0, 0);
        acs[i][j] = c;
      }
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
    }
  };

  // read group j (0 .. NP * (TM + TN) - 1) of step ks: plane j / (TM + TN),
  // fragment f = j % (TM + TN) (f < TN: B fragment f, then A fragment f - TN)
  auto read_one = [&](const char* base, int ks, int j, bf16x8 (&av)[NP][TM],
                      bf16x8 (&bv)[NP][TN]) {
    const int p = j / (TM + TN), f = j % (TM + TN);
    if (f < TN)
      bv[p][f] = hg_frag<BL, BK>(base + NP * C::A_BYTES + p * C::B_BYTES, wn * WCOL + 32 * f, ks,
                                 lane);
    else
      av[p][f - TN] =
          hg_frag<AL, BK>(base + p * C::A_BYTES, wm * (BM / 2) + 32 * (f - TN), ks, lane);
  };
  // the 6 (NP = 3) or 1 MFMAs of output block b = (i, j) as a flat list
  auto mfma_q = [&](int b, int q, bf16x8 (&av)[NP][TM], bf16x8 (&bv)[NP][TN]) {
    const int i = b / TN, j = b % TN;
    if constexpr (NP == 3) {
      if (q == 0) acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0][j], acs[i][j], 0, 0, 0);
      if (q == 1) acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1][j], acs[i][j], 0, 0, 0);
      if (q == 2) acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2][j], acs[i][j], 0, 0, 0);
      if (q == 3) acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][j], acs[i][j], 0, 0, 0);
      if (q == 4) acs[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][j], acs[i][j], 0, 0, 0);
    }
    if (q == (NP == 3 ? 5 : 0))
      acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
  };

  bf16x8 fa[2][NP][TM], fb[2][NP][TN];
  // glds of the next-but-one tile are spread over the first KS-1 k-steps
  constexpr int GSEG = KS - 1;
  // one k-tile; STAGE_NEXT2: stage tile t+2; HAS_NEXT: tile t+1 exists
  auto tile = [&](int t, auto stage_c, auto next_c) {
    constexpr bool STAGE_NEXT2 = decltype(stage_c)::value;
    constexpr bool HAS_NEXT = decltype(next_c)::value;
    const char* base = lds + (t % HG_STAGES) * C::STAGE;
    const int sbuf = (t + 2) % HG_STAGES;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      auto& av = fa[ks & 1];
      auto& bv = fb[ks & 1];
      hg_wait16<NP, TM, TN>(av, bv);
      if constexpr (ks + 1 < KS) {
        read(base, ks + 1, fa[(ks + 1) & 1], fb[(ks + 1) & 1]);
      } else if constexpr (HAS_NEXT) {
        if constexpr (STAGE_NEXT2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        read(lds + ((t + 1) % HG_STAGES) * C::STAGE, 0, fa[0], fb[0]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i) mfma_i(i, av, bv);
      if constexpr (STAGE_NEXT2 && ks < GSEG) {
        constexpr int lo = ks * C::G / GSEG, hi = (ks + 1) * C::G / GSEG;
#pragma unroll
        for (int q = lo; q < hi; ++q) piece(t + 2, sbuf, q);
        // MFMAs and glds alternate (MPG MFMAs, one glds, ...)
        constexpr int NM = TM * TN * (NP == 3 ? 6 : 1), NG = hi - lo;
        constexpr int MPG = NG > 0 ? NM / NG : NM;
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

  // SCH = 1 k-tile: per k-step, wait own reads | (last step: vmcnt, barrier) |
  // MFMA q, then read groups / glds in its gap, in pinned program order
  constexpr int NRG = NP * (TM + TN);       // read groups per k-step
  constexpr int NMF = TM * TN * (NP == 3 ? 6 : 1);  // MFMAs per k-step
  auto tile_il = [&](int t, auto stage_c, auto next_c) {
    constexpr bool STAGE_NEXT2 = decltype(stage_c)::value;
    constexpr bool HAS_NEXT = decltype(next_c)::value;
    const char* base = lds + (t % HG_STAGES) * C::STAGE;
    const int sbuf = (t + 2) % HG_STAGES;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      auto& av = fa[ks & 1];
      auto& bv = fb[ks & 1];
      constexpr bool RD = ks + 1 < KS || HAS_NEXT;  // reads to issue in this step
      const char* rbase = ks + 1 < KS ? base : lds + ((t + 1) % HG_STAGES) * C::STAGE;
      constexpr int rks = ks + 1 < KS ? ks + 1 : 0;
      auto& nav = fa[(ks + 1) & 1];
      auto& nbv = fb[(ks + 1) & 1];
      hg_wait16<NP, TM, TN>(av, bv);
      if constexpr (ks + 1 == KS && HAS_NEXT) {
        if constexpr (STAGE_NEXT2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      // glds of this step (tile t+2), placed after the reads
      constexpr bool GL = STAGE_NEXT2 && ks < GSEG;
      constexpr int glo = GL ? ks * C::G / GSEG : 0, ghi = GL ? (ks + 1) * C::G / GSEG : 0;
      static_for<NMF>([&](auto q_c) {
        constexpr int q = decltype(q_c)::value;
        mfma_q(q / (NP == 3 ? 6 : 1), q % (NP == 3 ? 6 : 1), av, bv);
        if constexpr (RD) {
          // two read groups per gap from the first gap on
          if constexpr (2 * q < NRG) read_one(rbase, rks, 2 * q, nav, nbv);
          if constexpr (2 * q + 1 < NRG) read_one(rbase, rks, 2 * q + 1, nav, nbv);
        }
        // then one glds per gap
        constexpr int g0 = (NRG + 1) / 2;  // first gap without reads
        if constexpr (q >= g0 && q - g0 < ghi - glo) piece(t + 2, sbuf, glo + q - g0);
        if constexpr (q == NMF - 1 && ghi - glo > NMF - g0) {
          for (int r = glo + NMF - g0; r < ghi; ++r) piece(t + 2, sbuf, r);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  };

  if (nk > 0) {
    stage(0, 0);
    if (nk > 1) {
      stage(1, 1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    read(lds, 0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    using T_ = std::true_type;
    using F_ = std::false_type;
    int t = 0;
    if constexpr (SCH == 1) {
      for (; t + 2 < nk; ++t) tile_il(t, T_{}, T_{});
      if (t + 1 < nk) tile_il(t++, F_{}, T_{});
      tile_il(t, F_{}, F_{});
    } else {
      for (; t + 2 < nk; ++t) tile(t, T_{}, T_{});
      if (t + 1 < nk) tile(t++, F_{}, T_{});
      tile(t, F_{}, F_{});
    }
  }
  if constexpr (NP == 3) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += acs[i][j];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // staging buffers are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  gemm_epilogue<BM, HG_BN, WGN>(acc, smem, ge, tid, n0, m0, z, bx, by);
}

// The same GEMM on v_mfma_f32_16x16x32_bf16 (MI355X_MICROARCH.md "DVFS
// give-back" item 7: at equal cycles per FLOP the chip holds a higher clock on
// the 16x16 shape under random data).  Wave tile (BM/2) x 32 = TA x 2 16x16
// tiles; one 32-deep k-step per 32 of BK (KS32 = BK / 32).  Schedule as in
// gemm_h_kernel: k-step j waits its own reads, issues j+1's, then its MFMAs;
// the tile barrier X_t sits in the last k-step of tile t behind the reads of
// tile t.  Because every fragment of tile t is in registers once X_t is passed,
// tile t's buffer is free then: glds of tile t+3 go there right after X_t
// (three buffers: t+1 being read, t+2 in flight, t+3 issued), interleaved with
// the MFMAs of that last k-step.  The accumulators are repacked into the 32x32
// register layout of gemm_epilogue<..., 16> (see acc_row / acc_col there).
// SCH = 1: as gemm_h_kernel's SCH = 1, the next step's fragment reads (and
// the tile-(t+3) glds) go into the gaps of this step's MFMAs.
template <int AL, int BL, int NP, int BM, int BK, int SCH = 0>
__global__ __launch_bounds__(HG_NT, 1) void gemm_h16_kernel(GemmHArgs g) {
  using C = HgCfg<BM, BK, NP>;
  constexpr int TM = BM / 64;        // 32-row blocks per wave (epilogue layout)
  constexpr int TA = BM / 32;        // 16-row A fragments per wave
  constexpr int TB = 2;              // 16-column B fragments per wave
  constexpr int KS = BK / 32;
  // NP = 3 holds 2 x 3 planes x 6 fragments of a 32-deep step: past 256 VGPRs.
  // It spilled, and the spills touched fragment registers whose inline-asm LDS
  // reads were still in flight: the late LDS return overwrote a register the
  // allocator had reused for a staging address -> the round-2 aperture
  // violation (profiles/r3/np3_h16_fault_cause.txt).  tools/isa_check.py now
  // rejects any build with scratch or such a hazard; the fp32 configuration
  // keeps gemm_h_kernel.
  static_assert(NP == 1, "16x16x32 variant: one plane (bf16 configuration) only");
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_BYTES / 4];
  char* const lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * HG_BN, m0 = by * BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

  f32x4 acc[TA][TB], acs[NP == 3 ? TA : 1][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) {
      acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if constexpr (NP == 3) acs[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

  const __bf16* sa[C::A_PW];
  const __bf16* sb[C::B_PW];
#pragma unroll
  for (int i = 0; i < C::A_PW; ++i)
    sa[i] = hg_src<AL, BM, BK, 16>(g.A, g.lda, g.M, m0, kbeg, wave * C::A_PW + i, lane);
#pragma unroll
  for (int i = 0; i < C::B_PW; ++i)
    sb[i] = hg_src<BL, HG_BN, BK, 16>(g.B, g.ldb, g.N, n0, kbeg, wave * C::B_PW + i, lane);
  const long long stepA = AL == L_RK ? BK : (long long)BK * g.lda;
  const long long stepB = BL == L_RK ? BK : (long long)BK * g.ldb;

  auto piece = [&](int t, int buf, int q) {
    char* base = lds + buf * C::STAGE;
    const int p = q / (C::A_PW + C::B_PW), r = q % (C::A_PW + C::B_PW);
    if (r < C::A_PW)
      __builtin_amdgcn_global_load_lds(
          (const void*)(sa[r] + p * g.pa + t * stepA),
          (lds_void*)(base + p * C::A_BYTES + (wave * C::A_PW + r) * 1024), 16, 0, 0);
    else
      __builtin_amdgcn_global_load_lds(
          (const void*)(sb[r - C::A_PW] + p * g.pb + t * stepB),
          (lds_void*)(base + NP * C::A_BYTES + p * C::B_BYTES +
                      (wave * C::B_PW + r - C::A_PW) * 1024),
          16, 0, 0);
  };
  auto stage = [&](int t, int buf) {
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(t, buf, q);
  };
  auto read = [&](const char* base, int ks, bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) {
#pragma unroll
      for (int j = 0; j < TB; ++j)
        bv[p][j] = hg_frag16<BL, BK>(base + NP * C::A_BYTES + p * C::B_BYTES, wn * 32 + 16 * j,
                                     ks, lane);
#pragma unroll
      for (int i = 0; i < TA; ++i)
        av[p][i] = hg_frag16<AL, BK>(base + p * C::A_BYTES, wm * (BM / 2) + 16 * i, ks, lane);
    }
  };
  auto mfma_all = [&](bf16x8 (&av)[NP][TA], bf16x8 (&bv)[NP][TB]) {
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) {
        if constexpr (NP == 3) {
          // small terms, smallest first: lh, mm, hl, mh, hm
          f32x4 c = acs[i][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[2][i], bv[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[1][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[2][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[1][i], bv[0][j], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[1][j], c, 0, 0, 0);
          acs[i][j] = c;
        }
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[0][i], bv[0][j], acc[i][j], 0, 0, 0);
      }
  };

  // SCH = 1 pieces: read group j (B fragments first, then A), MFMA q = (i, j)
  auto read_one = [&](const char* base, int ks, int j, bf16x8 (&av)[NP][TA],
                      bf16x8 (&bv)[NP][TB]) {
    if (j < TB)
      bv[0][j] = hg_frag16<BL, BK>(base + NP * C::A_BYTES, wn * 32 + 16 * j, ks, lane);
    else
      av[0][j - TB] = hg_frag16<AL, BK>(base, wm * (BM / 2) + 16 * (j - TB), ks, lane);
  };

  bf16x8 fa[2][NP][TA], fb[2][NP][TB];
  constexpr int NM = TA * TB * (NP == 3 ? 6 : 1);  // MFMAs per k-step
  // one k-tile whose first k-step uses register set P0; STAGE3: stage tile
  // t+3 after X_t; NEXT: tile t+1 exists; G2: tile t+2 was staged (vmcnt(G))
  auto tile = [&](int t, auto p0_c, auto stage_c, auto next_c, auto g2_c) {
    constexpr int P0 = decltype(p0_c)::value;
    constexpr bool STAGE3 = decltype(stage_c)::value;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr bool G2 = decltype(g2_c)::value;
    const char* base = lds + (t % HG_STAGES) * C::STAGE;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      constexpr int cs = (P0 + ks) & 1, ns = (P0 + ks + 1) & 1;
      hg_wait16<NP, TA, TB>(fa[cs], fb[cs]);
      if constexpr (ks + 1 < KS) {
        read(base, ks + 1, fa[ns], fb[ns]);
      } else if constexpr (NEXT) {
        if constexpr (G2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        read(lds + ((t + 1) % HG_STAGES) * C::STAGE, 0, fa[ns], fb[ns]);
      }
      __builtin_amdgcn_sched_barrier(0);
      mfma_all(fa[cs], fb[cs]);
      if constexpr (ks + 1 == KS && STAGE3) {
        stage(t + 3, t % HG_STAGES);
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
  constexpr int NRG = TA + TB;  // read groups per k-step (NP = 1)
  auto tile_il = [&](int t, auto p0_c, auto stage_c, auto next_c, auto g2_c) {
    constexpr int P0 = decltype(p0_c)::value;
    constexpr bool STAGE3 = decltype(stage_c)::value;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr bool G2 = decltype(g2_c)::value;
    const char* base = lds + (t % HG_STAGES) * C::STAGE;
    static_for<KS>([&](auto ks_c) {
      constexpr int ks = decltype(ks_c)::value;
      constexpr int cs = (P0 + ks) & 1, ns = (P0 + ks + 1) & 1;
      constexpr bool RD = ks + 1 < KS || NEXT;
      const char* rbase = ks + 1 < KS ? base : lds + ((t + 1) % HG_STAGES) * C::STAGE;
      constexpr int rks = ks + 1 < KS ? ks + 1 : 0;
      hg_wait16<NP, TA, TB>(fa[cs], fb[cs]);
      if constexpr (ks + 1 == KS && NEXT) {
        if constexpr (G2)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(C::G) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      constexpr int NG = (ks + 1 == KS && STAGE3) ? C::G : 0;
      constexpr int g0 = (NRG + 1) / 2;  // first MFMA gap without reads
      static_for<NM>([&](auto q_c) {
        constexpr int q = decltype(q_c)::value;
        constexpr int i = q / TB, j = q % TB;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[cs][0][i], fb[cs][0][j], acc[i][j],
                                                           0, 0, 0);
        if constexpr (RD) {
          if constexpr (2 * q < NRG) read_one(rbase, rks, 2 * q, fa[ns], fb[ns]);
          if constexpr (2 * q + 1 < NRG) read_one(rbase, rks, 2 * q + 1, fa[ns], fb[ns]);
        }
        if constexpr (q >= g0 && q - g0 < NG) piece(t + 3, t % HG_STAGES, q - g0);
        if constexpr (q == NM - 1 && NG > NM - g0) {
          for (int r = NM - g0; r < NG; ++r) piece(t + 3, t % HG_STAGES, r);
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  // tile t with its register-set parity (KS odd: sets alternate per tile)
  auto run = [&](int t, auto stage_c, auto next_c, auto g2_c) {
    auto go = [&](auto p0) {
      if constexpr (SCH == 1 && NP == 1)
        tile_il(t, p0, stage_c, next_c, g2_c);
      else
        tile(t, p0, stage_c, next_c, g2_c);
    };
    if constexpr (KS % 2 == 0) {
      go(std::integral_constant<int, 0>{});
    } else {
      if (t & 1)
        go(std::integral_constant<int, 1>{});
      else
        go(std::integral_constant<int, 0>{});
    }
  };

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
    read(lds, 0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    int t = 0;
    for (; t + 3 < nk; ++t) run(t, T_{}, T_{}, T_{});   // stages t+3; t+2 in flight
    if (t + 2 < nk) run(t++, F_{}, T_{}, T_{});          // t+2 in flight
    if (t + 1 < nk) run(t++, F_{}, T_{}, F_{});
    run(t, F_{}, F_{}, F_{});
  }
  // repack into the 32x32 register layout: 32-row block i = fragments 2i, 2i+1;
  // register 4 (2 tr + tc) + q of block i = row 16 tr + 4 (l >> 4) + q,
  // column 16 tc + (l & 15)
  f32x16 out[TM][1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int tr = 0; tr < 2; ++tr)
#pragma unroll
      for (int tc = 0; tc < 2; ++tc)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v = acc[2 * i + tr][tc][q];
          if constexpr (NP == 3) v += acs[2 * i + tr][tc][q];
          out[i][0][4 * (2 * tr + tc) + q] = v;
        }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();  // staging buffers are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  gemm_epilogue<BM, HG_BN, 4, 16>(out, smem, ge, tid, n0, m0, z, bx, by);
}

}  // namespace ddpg
