// fp32 MFMA GEMM kernel (gfx950, v_mfma_f32_32x32x2_f32); arguments and the
// fused epilogue are in gemm_common.h.
//
// C[M,N] = op(A)[M,K] . op(B)[K,N], exact-f32 products and accumulation
// (the f32-input MFMA is a k-ordered fmaf chain).
// Block tile BM x BN x 32 (BM, BN in {64, 128}), 256 threads = 4 waves (2x2),
// each wave (BM/2) x (BN/2) = TM x TN MFMA 32x32 tiles.  Both operands are
// staged k-major into LDS ([k][row], stride BR+1 when the global source is
// k-contiguous so that the transposing scalar LDS writes and the MFMA operand
// reads are both bank-conflict free; stride BR + ds_write_b128 otherwise).
// Register prefetch of tile t+1 overlaps the MFMAs of tile t (one barrier per
// k-tile).
#pragma once
#include "gemm_common.h"

namespace ddpg {

// ---------------------------------------------------------------- staging
// One operand tile of BR rows x GBK k, global -> registers -> LDS [k][row].
template <int L, int VEC, int BR>
struct Stage {
  static constexpr int PAD = (L == L_RK) ? 1 : 0;
  static constexpr int LS = BR + PAD;                  // LDS row stride ([k][row])
  static constexpr int NV = (BR * GBK) / (GNT * VEC);  // vectors per thread
  static constexpr int RQ = BR / 4;                    // float4 per k-row (KR)
  float v[NV * VEC];

  DDPG_DEV void load(const float* __restrict__ P, int ld, int R, int kend, int r0, int k0,
                     int tid) {
    if constexpr (L == L_RK && VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, r = f >> 3, kq = f & 7;
        const int gr = r0 + r, gk = k0 + 4 * kq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < R && gk < kend) x = *reinterpret_cast<const float4*>(P + (size_t)gr * ld + gk);
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, r = f >> 5, k = f & 31;
        const int gr = r0 + r, gk = k0 + k;
        v[i] = (gr < R && gk < kend) ? P[(size_t)gr * ld + gk] : 0.f;
      }
    } else if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, k = f / RQ, rq = f % RQ;
        const int gk = k0 + k, gr = r0 + 4 * rq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < kend && gr < R) x = *reinterpret_cast<const float4*>(P + (size_t)gk * ld + gr);
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, k = f / BR, r = f % BR;
        const int gk = k0 + k, gr = r0 + r;
        v[i] = (gk < kend && gr < R) ? P[(size_t)gk * ld + gr] : 0.f;
      }
    }
  }

  DDPG_DEV void store(float* __restrict__ lds, int tid) const {
    if constexpr (L == L_RK && VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, r = f >> 3, kq = f & 7;
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[(4 * kq + j) * LS + r] = v[4 * i + j];
      }
    } else if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, r = f >> 5, k = f & 31;
        lds[k * LS + r] = v[i];
      }
    } else if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, k = f / RQ, rq = f % RQ;
        *reinterpret_cast<float4*>(lds + k * LS + 4 * rq) =
            make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int f = i * GNT + tid, k = f / BR, r = f % BR;
        lds[k * LS + r] = v[i];
      }
    }
  }
};

// ---------------------------------------------------------------- kernel
// VA / VB: 16-B (4) or scalar (1) global loads for the A / B operand, chosen
// per operand (e.g. K = A = 17 forces scalar k-loads on the activations while
// the weights stay vectorised).
template <int AL, int BL, int VA, int VB, int BM, int BN>
__global__ __launch_bounds__(GNT, 2) void gemm_f32_kernel(GemmArgs g) {
  using TC = TileCfg<BM, BN>;
  __shared__ __attribute__((aligned(16))) float smem[TC::SMEM];
  using SA = Stage<AL, VA, BM>;
  using SB = Stage<BL, VB, BN>;
  constexpr int LSA = SA::LS, LSB = SB::LS;
  constexpr int TM = BM / 64, TN = BN / 64;  // MFMA tiles per wave
  constexpr int WR = BM / 2, WC = BN / 2;    // wave tile
  float* const As0 = smem;
  float* const Bs0 = smem + 2 * GBK * LSA;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  int bx, by;
  xcd_tile(bx, by, g.xcd);
  const int n0 = bx * BN, m0 = by * BM, z = blockIdx.z;
  const int kbeg = z * g.kps;
  const int kend = min(g.K, kbeg + g.kps);
  const int nk = kend > kbeg ? (kend - kbeg + GBK - 1) / GBK : 0;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    SA sa;
    SB sb;
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
      const float* a_s = As0 + cur * GBK * LSA + wm * WR + li;
      const float* b_s = Bs0 + cur * GBK * LSB + wn * WC + li;
#pragma unroll
      for (int kk = 0; kk < GBK / 2; ++kk) {
        const int k = 2 * kk + h;
        float av[TM], bv[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) av[i] = a_s[k * LSA + 32 * i];
#pragma unroll
        for (int j = 0; j < TN; ++j) bv[j] = b_s[k * LSB + 32 * j];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      if (more) {
        sa.store(As0 + (cur ^ 1) * GBK * LSA, tid);
        sb.store(Bs0 + (cur ^ 1) * GBK * LSB, tid);
      }
      __syncthreads();
    }
  }

  gemm_epilogue<BM, BN>(acc, smem, g, tid, n0, m0, z, bx, by);
}

}  // namespace ddpg
