// bf16-configuration GEMM on 256 x 256 block tiles (gfx950,
// v_mfma_f32_16x16x32_bf16, fp32 accumulation) for the large C5 contractions.
//
// Why a second tile: the 256 x 128 tile of gemm_h16_kernel gives each wave a
// 128 x 32 output, so a 32-deep k-step reads 12 fragments (8 A + 4 B halves)
// for 16 MFMAs, and the block stages 48 KB per 64-deep k-tile.  With both
// SIMD partners streaming, that is ~156 B/clk/CU of ds_read plus ~47 B/clk of
// LDS-DMA writes at the MFMA peak, against 256 B/clk of LDS: the loop runs at
// about half the MFMA rate in isolation.  A 256 x 256 tile with
// 128 x 64 wave tiles reads 12 fragments per 32 MFMAs and stages 32 KB per
// 32-deep step per block: ~94 + ~31 B/clk at the peak
// (cdna_hip_programming.md, "The 256^2 8-phase template", measured there at
// 1.3-1.5 PF on 4096^3).
//
// Block: 512 threads = 8 waves, 2 along M x 4 along N, wave tile 128 x 64.
// The fused epilogue of gemm_common.h runs on the whole tile, staging 64
// rows per LDS pass (a 128-row wave row would not fit beside the projection
// weights).
//
// Staging: a ring of 4 LDS slots, each one 32-deep k-step (A 256 x 32 and B
// 32 x 256 bf16 = 32 KB; 128 KB in all), filled by global_load_lds (16 B per
// lane, buffer_load ... lds, 2 + 2 pieces per wave per step; the swizzles of
// gemm_h.h applied to the source addresses).  Steps s+1 .. s+3 are in flight while step s is
// computed: at step s each wave waits for its own reads of s (issued during
// s-1), retires its LDS-DMA of s+1 with a counted vmcnt (s+2, s+3 stay in
// flight), passes one barrier (after which every wave has finished reading
// slot s and every DMA of s+1 has landed), then issues the fragment reads of
// s+1 and the DMA of s+4 into slot s between the 32 MFMAs of step s.  The
// loop is unrolled by the 4 slots so every LDS address is an immediate
// offset and the two fragment register sets alternate statically.
//
// The product instantiates MODE 0 only, behind the opt-in DDPG_GEMM256=1: the
// split-K weight gradients (each split's fp32 slab reduced by the Adam-side
// slab reduction).  MODE 1 / 2 (fused epilogues, one split) are built by
// tools/gemmh256_bench.hip alone: 1.19x gemm_h16 on the N = 4096 dX in
// isolation, no faster inside the C5 step.
// The 128-tile C5 shapes (4096 x 2048 outputs) stay on gemm_h16_kernel: an
// in-launch combine of two K-halves (ticketed first / last arriver, the first
// arriver's fp32 partial through write-through stores) measured 0.75-0.92x
// of gemm_h16_kernel there -- 64 MB of partials per launch
// (profiles/r3/gemm_h256.txt).
#pragma once
#include "gemm_h.h"

namespace ddpg {

constexpr int H2_BM = 256, H2_BN = 256, H2_BK = 32, H2_SLOTS = 4, H2_NT = 512;

struct H2Cfg {
  static constexpr int A_BYTES = H2_BM * H2_BK * 2;  // 16 KB
  static constexpr int B_BYTES = H2_BN * H2_BK * 2;  // 16 KB
  static constexpr int SLOT = A_BYTES + B_BYTES;
  static constexpr int A_PW = A_BYTES / 1024 / 8;  // 1-KiB pieces per wave
  static constexpr int B_PW = B_BYTES / 1024 / 8;
  static constexpr int G = A_PW + B_PW;  // LDS-DMA instructions per wave per step
  // gemm_epilogue<256, 256, 4, 16, 64>: 64 rows x (256 + 4) + projection panel + reduction
  static constexpr int EPI_BYTES = (64 * TileCfg<256, 256>::VS_LD + 256 * PROJ_MAX + 2 * GNT) * 4;
  static constexpr int SMEM_BYTES = H2_SLOTS * SLOT > EPI_BYTES ? H2_SLOTS * SLOT : EPI_BYTES;
  static_assert(SMEM_BYTES <= 160 * 1024, "LDS");
  static_assert(A_PW * 8 * 1024 == A_BYTES && B_PW * 8 * 1024 == B_BYTES, "whole pieces");
};

// LDS fragment reads at base + immediate offset (inline asm, as gemm_h.h's)
template <int OFF>
DDPG_DEV bf16x8 b128_read_off(unsigned a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int OFF>
DDPG_DEV bf16x4 tr_read_off(unsigned a) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}

// v_mfma_f32_16x16x32_bf16 with D == C forced (the accumulators stay in
// place: with the builtin, hipcc rotated the 128 accumulator registers
// through fresh ones every step and spilled).  hipcc does not model an asm
// statement's hazards (cdna_hip_programming.md §5.7 item 2): the leading
// s_nop 1 covers a VALU write of an A/B operand just before; the D -> read
// hazard after the last MFMA is covered by mfma_drain() before the epilogue;
// D -> the same accumulator as C of the next MFMA needs none.
DDPG_DEV void mfma_inplace(f32x4& d, const bf16x8& a, const bf16x8& b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(a), "v"(b));
}
DDPG_DEV void mfma_drain() { asm volatile("s_nop 15\n\ts_nop 15" ::: "memory"); }

// MODE 1: fused epilogue (gemm_common.h) of the dX GEMMs (no bias, no
// activation, EluGrad factor of aux: post 1; column sums, projection, twin),
// one split.  MODE 2: any epilogue the learner uses (runtime dispatch), one
// split.  MODE 0: split-K weight
// gradients: each split stores its fp32 slab (out + z * out_split_stride)
// straight from the registers, nothing else.  Full tiles only (the host
// checks M % 256 == N % 256 == 0 and kps % 128 == 0).
template <int AL, int BL, int MODE>
__global__ __launch_bounds__(H2_NT, 1) void gemm_h256_kernel(GemmHArgs g) {
  using C = H2Cfg;
  constexpr int TA = 8;  // 16-row A fragments per wave (128 rows)
  constexpr int TB = 4;  // 16-column B fragments per wave (two 32-column strips)
  constexpr int NRG = TA + TB;
  constexpr int NM = TA * TB;  // MFMAs per step
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM_BYTES / 4];
  char* const lds = reinterpret_cast<char*>(smem);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * H2_BN, m0 = by * H2_BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int nk = g.kps / H2_BK;  // host: kps % (4 * H2_BK) == 0, every split full

  f32x4 acc[TA][TB];
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // LDS-DMA sources: buffer descriptors over the operands (uniform, SGPRs) +
  // each lane's 32-bit byte offset; the k-step advance is the scalar soffset
  // (cdna_hip_programming.md T8: half the address registers of 64-bit
  // global_load_lds addressing)
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.A, 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc((void*)g.B, 0, 0x7fffffff, 0x00020000);
  unsigned oa[C::A_PW], ob[C::B_PW];
#pragma unroll
  for (int i = 0; i < C::A_PW; ++i)
    oa[i] = (unsigned)((const char*)hg_src<AL, H2_BM, H2_BK, 16>(g.A, g.lda, g.M, m0, kbeg,
                                                                 wave * C::A_PW + i, lane) -
                       (const char*)g.A);
#pragma unroll
  for (int i = 0; i < C::B_PW; ++i)
    ob[i] = (unsigned)((const char*)hg_src<BL, H2_BN, H2_BK, 16>(g.B, g.ldb, g.N, n0, kbeg,
                                                                 wave * C::B_PW + i, lane) -
                       (const char*)g.B);
  const unsigned stepA = 2u * (AL == L_RK ? H2_BK : (unsigned)H2_BK * g.lda);  // bytes
  const unsigned stepB = 2u * (BL == L_RK ? H2_BK : (unsigned)H2_BK * g.ldb);

  // LDS: the four slots' A images in the first 64 KB, their B images in the
  // second, so every fragment read is one base register + an immediate offset
  auto aimg = [&](int slot) { return lds + slot * C::A_BYTES; };
  auto bimg = [&](int slot) { return lds + H2_SLOTS * C::A_BYTES + slot * C::B_BYTES; };
  // LDS-DMA piece q (0 .. G-1) of k-step s into slot `slot`
  auto piece = [&](int s, int slot, int q) {
    if (q < C::A_PW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (lds_void*)(aimg(slot) + (wave * C::A_PW + q) * 1024), 16, oa[q], s * stepA, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (lds_void*)(bimg(slot) + (wave * C::B_PW + q - C::A_PW) * 1024), 16,
          ob[q - C::A_PW], s * stepB, 0, 0);
  };
  auto bcol = [&](int j) { return wn * 64 + 16 * j; };

  // Fragment-read addresses: per-lane LDS bases computed once, everything
  // that varies with the slot / fragment an immediate offset (hipcc kept one
  // register per slot and fragment otherwise, and spilled them).
  //   RK image (rows of 64 B, chunk swizzle (row >> 2) & 2): fragment rows
  //     differ by multiples of 16, which leave the swizzle unchanged -> one
  //     base per operand.
  //   KR image ([32][128] sub-images, kr_swz): the column chunk of fragment f
  //     is XORed with a lane-dependent swizzle, so the two k-row octets of
  //     each distinct chunk pattern get their own base (A: 8 fragments x 2,
  //     B: (j & 1) x 2); sub-images and slots are immediates.
  const unsigned lbase = (unsigned)(uintptr_t)(lds_char*)lds;
  constexpr unsigned BREG = H2_SLOTS * C::A_BYTES;  // B region
  auto rk_base = [&](int row0) {
    const int r = row0 + (lane & 15);
    return (unsigned)(r * 64 + 16 * ((lane >> 4) ^ ((r >> 2) & 2)));
  };
  auto kr_addr = [&](int col0, int half) {
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int col = col0 + 4 * p;
    const int ch = (col & 127) >> 3;
    const int k = 8 * (lane >> 4) + q + 4 * half;
    return (unsigned)((col >> 7) * (H2_BK * 256) + k * 256 + 16 * (ch ^ kr_swz(k)) + 8 * (p & 1));
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

  // A fragments: one register set, each refilled for step s+1 one MFMA after
  // its last use in step s (the MFMAs run A-fragment-major: i outer, j inner);
  // B fragments (used by every MFMA row): two sets alternating by step.  The
  // refill of A fragment 7 follows the step's last MFMA.
  bf16x8 fa[1][TA], fb[2][1][TB];
  // one k-step s in ring slot SL (B set SL & 1).  NEXT: step s+1 exists; INF:
  // LDS-DMA groups issued for steps beyond s+1 that may stay in flight
  // (0, 1, 2); ST4: stage step s+4 into this slot.
  auto step = [&](int s, auto sl_c, auto next_c, auto inf_c, auto st4_c) {
    constexpr int SL = decltype(sl_c)::value;
    constexpr int SET = SL & 1;
    constexpr bool NEXT = decltype(next_c)::value;
    constexpr int INF = decltype(inf_c)::value;
    constexpr bool ST4 = decltype(st4_c)::value;
    hg_wait16<1, TA, TB>(fa, fb[SET]);
    if constexpr (NEXT) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(INF * C::G) : "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    constexpr int RS = (SL + 1) & 3;  // slot of step s+1
    static_for<NM>([&](auto q_c) {
      constexpr int q = decltype(q_c)::value;
      constexpr int i = q / TB, j = q % TB;
      mfma_inplace(acc[i][j], fa[0][i], fb[SET][0][j]);
      if constexpr (NEXT) {
        // B fragments of s+1 in the first gaps, A fragment i-1 one MFMA into row i
        if constexpr (q < TB) read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, q>{}, fa, fb[SET ^ 1]);
        if constexpr (q >= TB && j == 0) read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, TB + i - 1>{}, fa, fb[SET ^ 1]);
        if constexpr (q == NM - 1) read_one(std::integral_constant<int, RS>{}, std::integral_constant<int, TB + TA - 1>{}, fa, fb[SET ^ 1]);
      }
      // LDS-DMA of step s+4: one piece per gap from the second MFMA row
      if constexpr (ST4 && q >= TB + 1 && ((q - TB - 1) & 1) == 0 && (q - TB - 1) / 2 < C::G)
        piece(s + 4, SL, (q - TB - 1) / 2);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // prologue: steps 0..3 into the four slots, wait for step 0
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int q = 0; q < C::G; ++q) piece(s, s, q);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * C::G) : "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  static_for<NRG>([&](auto j_c) { read_one(std::integral_constant<int, 0>{}, j_c, fa, fb[0]); });
  __builtin_amdgcn_sched_barrier(0);

  // steady state: 4 steps per trip, every step stages s+4
  int s = 0;
  for (; s + 8 <= nk; s += 4) {
    step(s, I0{}, T_{}, I2{}, T_{});
    step(s + 1, I1{}, T_{}, I2{}, T_{});
    step(s + 2, I2{}, T_{}, I2{}, T_{});
    step(s + 3, I3{}, T_{}, I2{}, T_{});
  }
  // last four steps (s = nk - 4): nothing more to stage; in flight after
  // step s+1's group: 2, 1, 0
  step(s, I0{}, T_{}, I2{}, F_{});
  step(s + 1, I1{}, T_{}, I1{}, F_{});
  step(s + 2, I2{}, T_{}, I0{}, F_{});
  step(s + 3, I3{}, F_{}, I0{}, F_{});

  mfma_drain();
#pragma unroll
  for (int i = 0; i < TA; ++i)
#pragma unroll
    for (int j = 0; j < TB; ++j) asm volatile("" : "+v"(acc[i][j]));
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if constexpr (MODE == 0) {
    // slab store: lane holds rows 4 (lane >> 4) + q, column lane & 15 of each
    // 16 x 16 fragment (64-B row pieces per store instruction)
    float* o = g.e.out + (size_t)z * g.e.out_split_stride;
#pragma unroll
    for (int i = 0; i < TA; ++i)
#pragma unroll
      for (int j = 0; j < TB; ++j) {
        const int n = n0 + bcol(j) + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = m0 + wm * 128 + 16 * i + 4 * (lane >> 4) + q;
          o[(size_t)m * g.e.ldo + n] = acc[i][j][q];  // full tiles (host)
        }
      }
    return;
  }
  __syncthreads();  // staging slots are reused by the epilogue
  GemmArgs ge;
  ge.M = g.M;
  ge.N = g.N;
  ge.e = g.e;
  // the epilogue's 32 x 32 register blocks (acc_row / acc_col<16>): block
  // (I, J) = 16 x 16 fragments (2I + tr, 2J + tc); 64 tile rows per LDS pass
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
  gemm_epilogue<256, 256, 4, 16, 64, true, MODE == 1 ? 3 : -1>(out, smem, ge, tid, n0, m0, 0, bx, by);
}

}  // namespace ddpg
