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
// Tile 128 x 128 x 32, 512 threads = 8 waves (2 along M x 4 along N), each
// wave 64 x 32 = 2 MFMA 32x32 tiles, two 16-deep k-steps per k-tile; 1 block
// per CU (LDS: 3 planes x 2 operands x 2 stages), 2 waves per SIMD.  The split happens while staging (fp32
// global -> registers -> split -> three bf16 LDS planes, [row][k] with 40-bf16
// rows as in gemm_bf16.h), so the operands stay fp32 in HBM and every epilogue
// of gemm_common.h applies unchanged.
#pragma once
#include "gemm_bf16.h"

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

constexpr int S3_NT = 512;  // 8 waves: 2 along M x 4 along N, wave tile 64 x 32

// 128 rows x 32 k of fp32 for S3_NT threads, 8 floats each.
//   RK (rows contiguous in k): float4 f = i*512 + tid -> row f>>3, k quad f&7.
//   KR (k-major): thread (k pair kp = tid&15, row quad rq = tid>>4) loads rows
//   4rq..4rq+3 of k = 2kp, 2kp+1 (each wave reads 16 k-rows x 64 B), and the
//   transposed bf16x2 stores of a wave cover all 64 LDS banks.
// Per-thread pointers are set once and advanced one k-tile per load; rows out
// of range read a clamped address and are zeroed (no branches), and only a
// partial last k-tile checks k.
template <int L, int NP>
struct StageS3 {
  float v[8];
  const float* p[2];
  const float* base;  // 16-B aligned matrix start: the address of masked loads
  bool rok[2];
  int kof[2];    // k offset of each load within the k-tile
  long long step;  // floats between consecutive k-tiles

  DDPG_DEV void init(const float* __restrict__ P, int ld, int R, int r0, int kbeg, int tid) {
    base = P;
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int f = i * S3_NT + tid, r = f >> 3, kq = f & 7;
        rok[i] = r0 + r < R;
        p[i] = P + (size_t)(rok[i] ? r0 + r : 0) * ld + kbeg + 4 * kq;
        kof[i] = 4 * kq;
      }
      step = GBK;
    } else {
      const int kp = tid & 15, rq = tid >> 4;
      const bool ok = r0 + 4 * rq < R;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        rok[j] = ok;
        p[j] = P + (size_t)(kbeg + 2 * kp + j) * ld + (ok ? r0 + 4 * rq : 0);
        kof[j] = 2 * kp + j;
      }
      step = (long long)GBK * ld;
    }
  }

  // k-tile t; krem = k extent left from this tile's start (>= GBK: full tile)
  DDPG_DEV void load(int t, int krem) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool ok = rok[i] && (krem >= GBK || kof[i] < krem);
      const float* q = ok ? p[i] + t * step : base;
      const float4 x = *reinterpret_cast<const float4*>(q);
      v[4 * i] = ok ? x.x : 0.f;
      v[4 * i + 1] = ok ? x.y : 0.f;
      v[4 * i + 2] = ok ? x.z : 0.f;
      v[4 * i + 3] = ok ? x.w : 0.f;
    }
  }

  // split into the three bf16 planes [row][H_ROW] of one stage
  DDPG_DEV void store(__bf16* __restrict__ lds, int tid) const {
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int f = i * S3_NT + tid, r = f >> 3, kq = f & 7;
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
      const int kp = tid & 15, rq = tid >> 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // row 4rq+i gets k = 2kp, 2kp+1
        __bf16* q = lds + (4 * rq + i) * H_ROW + 2 * kp;
        if constexpr (NP == 1) {
          *reinterpret_cast<bf16x2*>(q) = __builtin_convertvector(f32x2v{v[i], v[4 + i]}, bf16x2);
        } else {
          bf16x2 hh, mm, ll;
          split3_pair(f32x2v{v[i], v[4 + i]}, hh, mm, ll);
          *reinterpret_cast<bf16x2*>(q) = hh;
          *reinterpret_cast<bf16x2*>(q + S3_PLANE) = mm;
          *reinterpret_cast<bf16x2*>(q + 2 * S3_PLANE) = ll;
        }
      }
    }
  }
};

template <int AL, int BL, int NP>
__global__ __launch_bounds__(S3_NT, 1) void gemm_s3_kernel(GemmArgs g) {
  using C = S3Cfg<NP>;
  __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
  __bf16* const As0 = reinterpret_cast<__bf16*>(smem);   // [stage][plane][128][H_ROW]
  __bf16* const Bs0 = As0 + 2 * C::STAGE;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 2, wn = wave & 3;
  const int h = lane >> 5, li = lane & 31;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * H_BN, m0 = by * H_BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;

  f32x16 acc[2][1];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][0][r] = 0.f;

  // k-tile t lives in LDS stage t & 1.  Registers hold the fp32 loads of the
  // next two k-tiles (sets 0 and 1, alternating): tile t+1's split + LDS
  // store and tile t+2's global loads are issued before tile t's MFMAs, and
  // with two waves per SIMD one wave's MFMAs overlap the other's LDS reads
  // and split VALU work.  Loads past kend read zeros.
  auto mfma_tile = [&](const __bf16* As, const __bf16* Bs) {
    const __bf16* a_s = As + (wm * 64 + li) * H_ROW + 8 * h;
    const __bf16* b_s = Bs + (wn * 32 + li) * H_ROW + 8 * h;
#pragma unroll
    for (int ks = 0; ks < GBK / 16; ++ks) {
      bf16x8 av[NP][2], bv[NP];  // [plane][tile]
#pragma unroll
      for (int p = 0; p < NP; ++p) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
          av[p][i] =
              *reinterpret_cast<const bf16x8*>(a_s + p * S3_PLANE + i * 32 * H_ROW + ks * 16);
        bv[p] = *reinterpret_cast<const bf16x8*>(b_s + p * S3_PLANE + ks * 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f32x16 c = acc[i][0];
        if constexpr (NP == 3) {
          // small terms first: lh, mm, hl, mh, hm, hh  (planes 0 = h, 1 = m, 2 = l)
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2][i], bv[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1][i], bv[0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[1], c, 0, 0, 0);
        }
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0][i], bv[0], c, 0, 0, 0);
        acc[i][0] = c;
      }
    }
  };
  if (nk > 0) {
    StageS3<AL, NP> sa0, sa1;
    StageS3<BL, NP> sb0, sb1;
    sa0.init(g.A, g.lda, g.M, m0, kbeg, tid);
    sb0.init(g.B, g.ldb, g.N, n0, kbeg, tid);
    sa1 = sa0;
    sb1 = sb0;
    const int klen = kend - kbeg;
    __bf16* const A1 = As0 + C::STAGE;
    __bf16* const B1 = Bs0 + C::STAGE;
    sa0.load(0, klen);
    sb0.load(0, klen);
    sa1.load(1, klen - GBK);
    sb1.load(1, klen - GBK);
    sa0.store(As0, tid);
    sb0.store(Bs0, tid);
    __syncthreads();
    for (int t = 0; t < nk; t += 2) {
      sa1.store(A1, tid);
      sb1.store(B1, tid);
      sa0.load(t + 2, klen - (t + 2) * GBK);
      sb0.load(t + 2, klen - (t + 2) * GBK);
      mfma_tile(As0, Bs0);
      __syncthreads();
      if (t + 1 >= nk) break;
      sa0.store(As0, tid);
      sb0.store(Bs0, tid);
      sa1.load(t + 3, klen - (t + 3) * GBK);
      sb1.load(t + 3, klen - (t + 3) * GBK);
      mfma_tile(A1, B1);
      __syncthreads();
    }
  }
  gemm_epilogue<128, 128, 4>(acc, smem, g, tid, n0, m0, z, bx, by);
}

}  // namespace ddpg
