// fp32 MFMA GEMM with fused DDPG epilogues (gfx950, v_mfma_f32_32x32x2_f32).
//
// C[M,N] = op(A)[M,K] . op(B)[K,N], exact-f32 products and accumulation
// (the f32-input MFMA is a k-ordered fmaf chain), used for every dense
// contraction of the learner step:
//   forward      Y  = X . W          A: X  [M=B][K=in]  (RK)   B: W [K=in][N=out]  (KR)
//   dX           dX = dY . W^T       A: dY [M=B][K=out] (RK)   B: W [N=in][K=out]  (RK)
//   weight grad  dW = X^T . dY       A: X  [K=B][M=in]  (KR)   B: dY [K=B][N=out]  (KR)
// Layout codes: RK = operand rows contiguous in k, KR = k-major, rows contiguous.
//
// Block tile BM x BN x 32 (BM, BN in {64, 128}), 256 threads = 4 waves (2x2),
// each wave (BM/2) x (BN/2) = TM x TN MFMA 32x32 tiles.  Both operands are
// staged k-major into LDS ([k][row], stride BR+1 when the global source is
// k-contiguous so that the transposing scalar LDS writes and the MFMA operand
// reads are both bank-conflict free; stride BR + ds_write_b128 otherwise).
// Register prefetch of tile t+1 overlaps the MFMAs of tile t (one barrier per
// k-tile).
//
// Epilogue (all optional, fused so that no thin layer is a separate pass):
//   v = acc (+ bias[n]) -> act (elu) -> post:
//       post 1: v *= EluGrad factor of aux[m,n]      (dX . elu'(y))
//       post 2: v  = pw[n] * EluGrad factor of v     (critic head, grad_ys = 1)
//   -> store out[m,n] (per split slab)
//   -> colsum partial  : sum over the tile's rows of v      (bias gradients)
//   -> proj  partial   : v[m, tile cols] . Wp[tile cols, 0..pn)  (thin output
//                        layers: actor W3, critic Wo, critic Wa^T for dQ/da)
#pragma once
#include "common.h"

namespace ddpg {

enum { L_RK = 0, L_KR = 1 };

constexpr int GBK = 32, GNT = 256;
constexpr int PROJ_MAX = 32;

template <int BM, int BN>
struct TileCfg {
  static constexpr int STAGE = 2 * GBK * (BM + 1) + 2 * GBK * (BN + 1);
  static constexpr int VS_LD = BN + 4;
  static constexpr int EPI = (BM / 2) * VS_LD + BN * PROJ_MAX + GNT;
  static constexpr int SMEM = STAGE > EPI ? STAGE : EPI;
};

struct GemmEpi {
  float* out;
  long long out_split_stride;
  int ldo;
  int act;   // 0 none, 1 elu
  int post;  // 0 none, 1 mul elu'(aux), 2 pw[n] * elu'(v)
  int ldaux;
  const float* bias;
  const float* aux;
  const float* pw;
  float* colsum;  // [split * mtiles + mtile][ld_colsum]
  int ld_colsum;
  int proj_n, proj_sn, proj_sa;
  const float* proj;  // Wp[n][a] = proj[n * proj_sn + a * proj_sa]
  float* proj_out;    // [ntile][M][proj_n]
};

struct GemmArgs {
  const float* A;
  const float* B;
  int M, N, K, lda, ldb;
  int kps;  // k extent per split (multiple of GBK)
  GemmEpi e;
};

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
template <int AL, int BL, int VEC, int BM, int BN>
__global__ __launch_bounds__(GNT, 2) void gemm_f32_kernel(GemmArgs g) {
  using TC = TileCfg<BM, BN>;
  __shared__ __attribute__((aligned(16))) float smem[TC::SMEM];
  using SA = Stage<AL, VEC, BM>;
  using SB = Stage<BL, VEC, BN>;
  constexpr int LSA = SA::LS, LSB = SB::LS;
  constexpr int TM = BM / 64, TN = BN / 64;  // MFMA tiles per wave
  constexpr int WR = BM / 2, WC = BN / 2;    // wave tile
  float* const As0 = smem;
  float* const Bs0 = smem + 2 * GBK * LSA;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, z = blockIdx.z;
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

  // ------------------------------------------------------------ epilogue
  const GemmEpi& e = g.e;
  const int M = g.M, N = g.N;
  float* outp = e.out ? e.out + (size_t)z * e.out_split_stride : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WC + j * 32 + li;
      const bool nok = n < N;
      const float bn = (nok && e.bias) ? e.bias[n] : 0.f;
      const float pwn = (nok && e.post == 2) ? e.pw[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WR + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = acc[i][j][r];
        if (nok && m < M) {
          if (e.bias) v = __fadd_rn(v, bn);
          if (e.act == 1) v = elu_f(v);
          if (e.post == 1) v = __fmul_rn(v, elu_grad_factor(e.aux[(size_t)m * e.ldaux + n]));
          else if (e.post == 2) v = __fmul_rn(pwn, elu_grad_factor(v));
          if (outp) outp[(size_t)m * e.ldo + n] = v;
        } else {
          v = 0.f;
        }
        acc[i][j][r] = v;
      }
    }
  }

  if (!e.colsum && !e.proj_out) return;

  // Row-wise reductions through LDS, WR tile rows (one wave row) per pass.
  constexpr int VS_LD = TC::VS_LD;
  float* Vs = smem;                      // [WR][VS_LD]
  float* Wps = smem + WR * VS_LD;        // [BN][PN]
  float* red = Wps + BN * PROJ_MAX;      // [GNT]
  const int PN = (e.proj_n + 3) & ~3;
  if (e.proj_out) {
    for (int idx = tid; idx < BN * PN; idx += GNT) {
      const int nl = idx / PN, a = idx - nl * PN, n = n0 + nl;
      Wps[idx] = (n < N && a < e.proj_n) ? e.proj[(size_t)n * e.proj_sn + (size_t)a * e.proj_sa]
                                          : 0.f;
    }
  }
  constexpr int CG = GNT / BN;  // column-sum row groups
  float csum = 0.f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            Vs[rl * VS_LD + wn * WC + j * 32 + li] = acc[i][j][r];
          }
    }
    __syncthreads();
    if (e.colsum) {
      const int col = tid % BN, grp = tid / BN;
#pragma unroll 4
      for (int rr = grp; rr < WR; rr += CG) csum += Vs[rr * VS_LD + col];
    }
    if (e.proj_out) {
      const int PG = PN >> 2;
      for (int p = tid; p < WR * PG; p += GNT) {
        const int row = p % WR, ag = p / WR;
        float4 ap = make_float4(0.f, 0.f, 0.f, 0.f);
        // partial unroll: a full unroll makes every Wps load invariant in p
        // and the compiler hoists them all into registers (spills at BN=64)
#pragma unroll 2
        for (int n4 = 0; n4 < BN / 4; ++n4) {
          const float4 vv = *reinterpret_cast<const float4*>(Vs + row * VS_LD + 4 * n4);
          const float vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 w = *reinterpret_cast<const float4*>(Wps + (4 * n4 + q) * PN + 4 * ag);
            ap.x = fmaf(vq[q], w.x, ap.x);
            ap.y = fmaf(vq[q], w.y, ap.y);
            ap.z = fmaf(vq[q], w.z, ap.z);
            ap.w = fmaf(vq[q], w.w, ap.w);
          }
        }
        const int m = m0 + pass * WR + row;
        if (m < M) {
          float* po = e.proj_out + ((size_t)blockIdx.x * M + m) * e.proj_n;
          const float av[4] = {ap.x, ap.y, ap.z, ap.w};
#pragma unroll
          for (int a = 0; a < 4; ++a)
            if (4 * ag + a < e.proj_n) po[4 * ag + a] = av[a];
        }
      }
    }
    __syncthreads();
  }
  if (e.colsum) {
    red[tid] = csum;
    __syncthreads();
    if (tid < BN) {
      float s = 0.f;
#pragma unroll
      for (int gi = 0; gi < CG; ++gi) s += red[tid + gi * BN];
      const int n = n0 + tid;
      if (n < N) e.colsum[((size_t)z * gridDim.y + blockIdx.y) * e.ld_colsum + n] = s;
    }
  }
}

}  // namespace ddpg
