// EXPERIMENT (not built into the product): producer/consumer variant of
// gemm_s3_kernel -- waves 0-3 MFMA only (64x64 quadrants), waves 4-7 stage
// (global loads S3_NS-1 k-tiles ahead, split, LDS stores).  Measured on MI355X
// (tools/gemm_bench.hip, 4096x1024x1024 fwd <RK,KR,3>, new epilogue): 67.5 us
// vs 57 us for the 8-wave lockstep kernel in distributed_ddpg_amd/csrc/gemm_s3.h,
// so the product keeps the lockstep kernel.  Kept for reference.
// fp32-accurate GEMM on the bf16 MFMA pipe (gfx950, v_mfma_f32_32x32x16_bf16):
// every fp32 operand x is split exactly into three bf16 planes
//   h = bf16(x),  m = bf16(x - h),  l = bf16(x - h - m)      (x = h + m + l + O(2^-27 |x|))
// (both differences are exact in fp32), and each product is the sum of the
// six plane products that reach fp32 precision,
//   x y ~ hh + hm + mh + hl + mm + lh                         (dropped: O(2^-27 |x y|)),
// each an exact 8x8-bit product accumulated in fp32 by the MFMA.  The result
// is an fp32 GEMM whose per-product error is below fp32 rounding (2^-24);
// only the accumulation order differs from the fp32-input MFMA (both are fp32
// sums).  The bf16 pipe's dense rate is 16x the fp32 one, so six bf16 MFMAs
// per fp32 MAC group still run at up to 16/6 = 2.7x the fp32 MFMA peak.
//
// Tile 128 x 128 x 32, 512 threads = 4 MFMA waves (2 x 2, each 64 x 64 = 2 x 2
// MFMA 32x32 tiles, two 16-deep k-steps per k-tile) + 4 staging waves; 1 block
// per CU (LDS: 3 planes x 2 operands x 2 stages).  The split happens while staging (fp32
// global -> registers -> split -> three bf16 LDS planes, [row][k] with 40-bf16
// rows as in gemm_bf16.h), so the operands stay fp32 in HBM and every epilogue
// of gemm_common.h applies unchanged.
#pragma once
#include "gemm_bf16.h"

// Phase timestamp hook for tools/gemm_bench.hip; empty in the product build.
#ifndef S3_STAMP
#define S3_STAMP(i)
#endif

namespace ddpg {

constexpr int S3_PLANE = 128 * H_ROW;  // bf16 per plane (one operand, one stage)
// NP = 3: fp32 via the three-plane split; NP = 1: plain bf16 operands (the
// bf16 configuration), same kernel with one plane and one product.
template <int NP>
struct S3Cfg {
  static constexpr int STAGE = NP * S3_PLANE;      // one operand, one stage (bf16)
  static constexpr int HALFS = 2 * 2 * STAGE;      // 2 operands x 2 stages
  static constexpr int SMEM = (HALFS / 2 > TileCfg<128, 128>::EPI) ? HALFS / 2
                                                                   : TileCfg<128, 128>::EPI;
};

constexpr int S3_NT = 512;   // 4 MFMA waves + 4 staging waves
constexpr int S3_PT = 256;   // staging (producer) threads
constexpr int S3_NS = 4;     // register sets: global loads run S3_NS - 1 k-tiles ahead

// (x0, x1) -> packed (h, m, l) bf16 pairs: three v_cvt_pk_bf16_f32, the
// widening of a bf16 pair is two bit operations, the residuals packed f32 subs.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
DDPG_DEV f32x2v widen(bf16x2 b) {
  const unsigned u = __builtin_bit_cast(unsigned, b);
  return f32x2v{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xFFFF0000u)};
}
DDPG_DEV void split3_pair(f32x2v x, bf16x2& h, bf16x2& m, bf16x2& l) {
#ifdef S3_TIMING_NOSPLIT  // tuning experiment only: wrong results
  h = m = l = __builtin_convertvector(x, bf16x2);
  return;
#endif
  h = __builtin_convertvector(x, bf16x2);
  const f32x2v r1 = x - widen(h);  // exact
  m = __builtin_convertvector(r1, bf16x2);
  const f32x2v r2 = r1 - widen(m);  // exact
  l = __builtin_convertvector(r2, bf16x2);
}

// 128 rows x 32 k of fp32 for the S3_PT staging threads, 16 floats each
// (ptid = staging thread index).
//   RK (rows contiguous in k): float4 f = i*256 + ptid -> row f>>3, k quad f&7.
//   KR (k-major): thread (k pair kp = ptid&15, row quad rq = ptid>>4) loads
//   rows 4rq..4rq+3 and 64+4rq..64+4rq+3 of k = 2kp, 2kp+1 (load j = 2 g + kb:
//   row group g, k bit kb); the transposed bf16x2 stores are at most 2-way
//   bank-conflicted (free for ds_write_b32).
// Per-thread pointers are set once and advanced one k-tile per load; rows out
// of range read the zero quad s3_zero4 (no branches), and only a partial last
// k-tile checks k.
struct S3Vals {
  f32x4 q[4];
};

__device__ f32x4 s3_zero4 = {0.f, 0.f, 0.f, 0.f};
typedef __attribute__((address_space(1))) f32x4 s3_glb_v4;

template <int L, int NP>
struct StageS3 {
  const float* p[4];
  bool rok[4];
  int kof[4];      // k offset of each load within the k-tile
  long long step;  // floats between consecutive k-tiles

  DDPG_DEV void init(const float* __restrict__ P, int ld, int R, int r0, int kbeg, int ptid) {
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f = i * S3_PT + ptid, r = f >> 3, kq = f & 7;
        rok[i] = r0 + r < R;
        p[i] = P + (size_t)(rok[i] ? r0 + r : 0) * ld + kbeg + 4 * kq;
        kof[i] = 4 * kq;
      }
      step = GBK;
    } else {
      const int kp = ptid & 15, rq = ptid >> 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int g = j >> 1, kb = j & 1, r = r0 + 64 * g + 4 * rq;
        rok[j] = r < R;
        p[j] = P + (size_t)(kbeg + 2 * kp + kb) * ld + (rok[j] ? r : 0);
        kof[j] = 2 * kp + kb;
      }
      step = (long long)GBK * ld;
    }
  }

  // k-tile t; krem = k extent left from this tile's start (>= GBK: full tile).
  // Masked loads read a zero quad instead of selecting on the loaded data:
  // a select after the load would make the compiler wait for every load in
  // flight at the loop back edge.
  DDPG_DEV void load(S3Vals& d, int t, int krem) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = rok[i] && (krem >= GBK || kof[i] < krem);
      const s3_glb_v4* q = ok ? (const s3_glb_v4*)(p[i] + t * step) : (const s3_glb_v4*)&s3_zero4;
      d.q[i] = *q;
    }
  }

  // split into the three bf16 planes [row][H_ROW] of one stage
  DDPG_DEV void store(const S3Vals& d, __bf16* __restrict__ lds, int ptid) const {
    float v[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int c = 0; c < 4; ++c) v[4 * i + c] = d.q[i][c];
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f = i * S3_PT + ptid, r = f >> 3, kq = f & 7;
        __bf16* q = lds + r * H_ROW + 4 * kq;
        if constexpr (NP == 1) {
          const bf16x2 h0 = __builtin_convertvector(f32x2v{v[4 * i], v[4 * i + 1]}, bf16x2);
          const bf16x2 h1 = __builtin_convertvector(f32x2v{v[4 * i + 2], v[4 * i + 3]}, bf16x2);
          *reinterpret_cast<bf16x4*>(q) = bf16x4{h0[0], h0[1], h1[0], h1[1]};
        } else {
          bf16x2 h0, m0, l0, h1, m1, l1;
          split3_pair(f32x2v{v[4 * i], v[4 * i + 1]}, h0, m0, l0);
          split3_pair(f32x2v{v[4 * i + 2], v[4 * i + 3]}, h1, m1, l1);
          *reinterpret_cast<bf16x4*>(q) = bf16x4{h0[0], h0[1], h1[0], h1[1]};
          *reinterpret_cast<bf16x4*>(q + S3_PLANE) = bf16x4{m0[0], m0[1], m1[0], m1[1]};
          *reinterpret_cast<bf16x4*>(q + 2 * S3_PLANE) = bf16x4{l0[0], l0[1], l1[0], l1[1]};
        }
      }
    } else {
      const int kp = ptid & 15, rq = ptid >> 4;
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // row 64g+4rq+i gets k = 2kp, 2kp+1
          __bf16* q = lds + (64 * g + 4 * rq + i) * H_ROW + 2 * kp;
          const f32x2v x = f32x2v{v[8 * g + i], v[8 * g + 4 + i]};
          if constexpr (NP == 1) {
            *reinterpret_cast<bf16x2*>(q) = __builtin_convertvector(x, bf16x2);
          } else {
            bf16x2 hh, mm, ll;
            split3_pair(x, hh, mm, ll);
            *reinterpret_cast<bf16x2*>(q) = hh;
            *reinterpret_cast<bf16x2*>(q + S3_PLANE) = mm;
            *reinterpret_cast<bf16x2*>(q + 2 * S3_PLANE) = ll;
          }
        }
    }
  }
};

// Producer / consumer split: waves 0-3 (one per SIMD) only read LDS and issue
// MFMAs, each owning a 64 x 64 quadrant (2 x 2 MFMA 32x32 tiles); waves 4-7
// only stage (global loads S3_NS - 1 k-tiles ahead, split, LDS stores one k-tile
// ahead).  One barrier per k-tile; on every SIMD the staging wave's VALU and
// LDS-store work runs beside the MFMA wave's matrix work instead of in
// lockstep with it.
template <int AL, int BL, int NP>
__global__ __launch_bounds__(S3_NT, 1) void gemm_s3_kernel(GemmArgs g) {
  using C = S3Cfg<NP>;
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  __bf16* const As0 = reinterpret_cast<__bf16*>(smem);   // [stage][plane][128][H_ROW]
  __bf16* const Bs0 = As0 + 2 * C::STAGE;
  __bf16* const A1 = As0 + C::STAGE;
  __bf16* const B1 = Bs0 + C::STAGE;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const bool producer = wave >= 4;
  const int ptid = tid - S3_PT;
  const int wm = (wave >> 1) & 1, wn = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * H_BN, m0 = by * H_BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;
  const int klen = kend - kbeg;
  S3_STAMP(0);

  auto mfma_tile = [&](f32x16(&acc)[2][2], const __bf16* As, const __bf16* Bs) {
    const __bf16* a_s = As + (wm * 64 + li) * H_ROW + 8 * h;
    const __bf16* b_s = Bs + (wn * 64 + li) * H_ROW + 8 * h;
#pragma unroll
    for (int ks = 0; ks < GBK / 16; ++ks) {
      bf16x8 av[NP][2], bv[NP][2];  // [plane][tile]
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          av[p][i] =
              *reinterpret_cast<const bf16x8*>(a_s + p * S3_PLANE + i * 32 * H_ROW + ks * 16);
          bv[p][i] =
              *reinterpret_cast<const bf16x8*>(b_s + p * S3_PLANE + i * 32 * H_ROW + ks * 16);
        }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x16 c = acc[i][j];
          if constexpr (NP == 3) {
            // small terms first: lh, mm, hl, mh, hm, hh  (planes 0 = h, 1 = m, 2 = l)
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0][j], c, 0, 0, 0);
            c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1][j], c, 0, 0, 0);
          }
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0][j], c, 0, 0, 0);
          acc[i][j] = c;
        }
    }
  };

  // The two wave groups run separate loops with the same barrier count (one
  // per k-tile), so their registers are allocated independently.
  if (producer) {
    // k-tile t: global loads into register set t % S3_NS (issued S3_NS - 1
    // k-tiles ahead of its LDS store), LDS stage t & 1 one k-tile ahead of
    // its MFMAs.
    if (nk > 0) {
      StageS3<AL, NP> sa;
      StageS3<BL, NP> sb;
      S3Vals va[S3_NS], vb[S3_NS];
      sa.init(g.A, g.lda, g.M, m0, kbeg, ptid);
      sb.init(g.B, g.ldb, g.N, n0, kbeg, ptid);
#pragma unroll
      for (int u = 0; u < S3_NS; ++u) {
        sa.load(va[u], u, klen - u * GBK);
        sb.load(vb[u], u, klen - u * GBK);
      }
      sa.store(va[0], As0, ptid);
      sb.store(vb[0], Bs0, ptid);
      __syncthreads();
      for (int t = 0; t < nk; t += S3_NS) {
#pragma unroll
        for (int u = 0; u < S3_NS; ++u) {
          const int tt = t + u;
          __bf16* const Anext = (u & 1) ? As0 : A1;
          __bf16* const Bnext = (u & 1) ? Bs0 : B1;
          // set u held k-tile tt (stored last iteration): refill with tt + S3_NS
#ifndef S3_TIMING_NOSTAGE  // tuning experiment only: MFMAs on stale tiles
#ifndef S3_TIMING_NOLOAD  // tuning experiment only: split + store stale registers
          sa.load(va[u], tt + S3_NS, klen - (tt + S3_NS) * GBK);
          sb.load(vb[u], tt + S3_NS, klen - (tt + S3_NS) * GBK);
#endif
          if (tt + 1 < nk) {
            sa.store(va[(u + 1) % S3_NS], Anext, ptid);
            sb.store(vb[(u + 1) % S3_NS], Bnext, ptid);
          }
#endif
          __syncthreads();
          if (tt + 1 >= nk) break;
        }
      }
    }
    gemm_epilogue_barriers(g.e);
  } else {
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    if (nk > 0) {
      __syncthreads();
      S3_STAMP(1);
      for (int t = 0; t < nk; ++t) {
#ifndef S3_TIMING_NOMFMA  // tuning experiment only: staging alone
        mfma_tile(acc, (t & 1) ? A1 : As0, (t & 1) ? B1 : Bs0);
#endif
        __syncthreads();
      }
    }
    S3_STAMP(2);
    gemm_epilogue<128, 128, 2>(acc, smem, g, tid, n0, m0, z, bx, by);
    S3_STAMP(3);
  }
}

}  // namespace ddpg
