// bf16 MFMA GEMM kernel (gfx950, v_mfma_f32_32x32x16_bf16) for the bf16
// configuration: fp32 operands in HBM (fp32 master weights
// and activations), converted to bf16 (round-to-nearest-even,
// v_cvt_pk_bf16_f32) while staging into LDS, fp32 accumulation, and the same
// fused fp32 epilogues as the fp32 kernel (gemm_common.h).
//
// Tile 128 x 128 x 32, 256 threads = 4 waves (2x2), each wave 64x64 = 2x2
// MFMA 32x32 tiles, two 16-deep k-steps per k-tile.  LDS holds both operands
// as [row][k] bf16 with 40-element (80 B) rows: the 32x32x16 fragment of lane
// l is 8 consecutive k of row l&31 (one ds_read_b128), and the 80-B stride
// spreads every 16-lane ds_read_b128 group over all 16 slots of a bank row.
// k-contiguous sources (RK) store 4 k of one row per lane (ds_write_b64);
// row-contiguous sources (KR) load a 4k x 4row block per lane and write it
// transposed as four 4-k runs; lanes are ordered k-quad fastest so each
// 16-lane write group covers all 32 banks, while every load instruction still
// reads whole 128-B lines (8 lanes x 16 B per k row).
#pragma once
#include "gemm_common.h"

namespace ddpg {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int H_BM = 128, H_BN = 128;
constexpr int H_ROW = 40;  // bf16 per LDS row (32 k + 8 pad)
constexpr int H_STAGE_HALFS = 2 * 2 * 128 * H_ROW;  // 2 buffers x (A + B)
constexpr int H_SMEM = (H_STAGE_HALFS / 2 > TileCfg<128, 128>::EPI) ? H_STAGE_HALFS / 2
                                                                    : TileCfg<128, 128>::EPI;

DDPG_DEV bf16x4 cvt4(float a, float b, float c, float d) {
  bf16x4 r;
  r[0] = (__bf16)a;
  r[1] = (__bf16)b;
  r[2] = (__bf16)c;
  r[3] = (__bf16)d;
  return r;
}

// 128 rows x 32 k, fp32 global -> bf16 LDS [row][H_ROW]
template <int L>
struct Stage16 {
  float v[16];

  DDPG_DEV void load(const float* __restrict__ P, int ld, int R, int kend, int r0, int k0,
                     int tid) {
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f = i * GNT + tid, r = f >> 3, kq = f & 7;
        const int gr = r0 + r, gk = k0 + 4 * kq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < R && gk < kend) x = *reinterpret_cast<const float4*>(P + (size_t)gr * ld + gk);
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else {
      const int rq = ((tid & 63) >> 3) + 8 * (tid >> 6), kq = tid & 7;
      const int gr = r0 + 4 * rq;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int gk = k0 + 4 * kq + j;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < kend && gr < R) x = *reinterpret_cast<const float4*>(P + (size_t)gk * ld + gr);
        v[4 * j] = x.x; v[4 * j + 1] = x.y; v[4 * j + 2] = x.z; v[4 * j + 3] = x.w;
      }
    }
  }

  DDPG_DEV void store(__bf16* __restrict__ lds, int tid) const {
    if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int f = i * GNT + tid, r = f >> 3, kq = f & 7;
        *reinterpret_cast<bf16x4*>(lds + r * H_ROW + 4 * kq) =
            cvt4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      }
    } else {
      const int rq = ((tid & 63) >> 3) + 8 * (tid >> 6), kq = tid & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i)  // row 4rq+i gets k = 4kq .. 4kq+3
        *reinterpret_cast<bf16x4*>(lds + (4 * rq + i) * H_ROW + 4 * kq) =
            cvt4(v[i], v[4 + i], v[8 + i], v[12 + i]);
    }
  }
};

template <int AL, int BL>
__global__ __launch_bounds__(GNT, 2) void gemm_bf16_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float smem[H_SMEM];
  __bf16* const As0 = reinterpret_cast<__bf16*>(smem);
  __bf16* const Bs0 = As0 + 2 * 128 * H_ROW;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * H_BN, m0 = by * H_BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    Stage16<AL> sa;
    Stage16<BL> sb;
    sa.load(g.A, g.lda, g.M, kend, m0, kbeg, tid);
    sb.load(g.B, g.ldb, g.N, kend, n0, kbeg, tid);
    sa.store(As0, tid);
    sb.store(Bs0, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      const int cur = t & 1;
      const bool more = (t + 1) < nk;
      if (more) {
        sa.load(g.A, g.lda, g.M, kend, m0, kbeg + (t + 1) * GBK, tid);
        sb.load(g.B, g.ldb, g.N, kend, n0, kbeg + (t + 1) * GBK, tid);
      }
      const __bf16* a_s = As0 + cur * 128 * H_ROW + (wm * 64 + li) * H_ROW + 8 * h;
      const __bf16* b_s = Bs0 + cur * 128 * H_ROW + (wn * 64 + li) * H_ROW + 8 * h;
#pragma unroll
      for (int ks = 0; ks < GBK / 16; ++ks) {
        bf16x8 av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          av[i] = *reinterpret_cast<const bf16x8*>(a_s + i * 32 * H_ROW + ks * 16);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bv[j] = *reinterpret_cast<const bf16x8*>(b_s + j * 32 * H_ROW + ks * 16);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      if (more) {
        sa.store(As0 + (cur ^ 1) * 128 * H_ROW, tid);
        sb.store(Bs0 + (cur ^ 1) * 128 * H_ROW, tid);
      }
      __syncthreads();
    }
  }
  gemm_epilogue<128, 128>(acc, smem, g, tid, n0, m0, z, bx, by);
}

}  // namespace ddpg
