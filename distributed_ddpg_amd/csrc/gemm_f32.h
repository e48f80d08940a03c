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
// Block tile 128x128x32, 256 threads = 4 waves (2x2), each wave 64x64 =
// 2x2 MFMA 32x32 tiles.  Both operands are staged k-major into LDS
// ([k][row], stride 129 when the global source is k-contiguous so that the
// transposing scalar LDS writes and the MFMA operand reads are both
// bank-conflict free; stride 128 + ds_write_b128 otherwise).  Register
// prefetch of tile t+1 overlaps the MFMAs of tile t (one barrier per k-tile).
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

constexpr int GBM = 128, GBN = 128, GBK = 32, GNT = 256;
constexpr int GSMEM = 2 * GBK * (GBM + 1) + 2 * GBK * (GBN + 1);  // 16512 floats
constexpr int VS_LD = 132;                                        // epilogue tile stride
constexpr int PROJ_MAX = 32;

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
template <int L, int VEC>
struct Stage {
  static constexpr int PAD = (L == L_RK) ? 1 : 0;
  static constexpr int LS = GBM + PAD;                // LDS row stride ([k][row])
  static constexpr int NV = (GBM * GBK) / (GNT * VEC);  // vectors per thread
  float v[NV * VEC];

  DDPG_DEV void load(const float* __restrict__ P, int ld, int R, int kend, int r0, int k0,
                     int tid) {
    if constexpr (L == L_RK && VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, r = f >> 3, kq = f & 7;
        int gr = r0 + r, gk = k0 + 4 * kq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gr < R && gk < kend) x = *reinterpret_cast<const float4*>(P + (size_t)gr * ld + gk);
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, r = f >> 5, k = f & 31;
        int gr = r0 + r, gk = k0 + k;
        v[i] = (gr < R && gk < kend) ? P[(size_t)gr * ld + gk] : 0.f;
      }
    } else if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, k = f >> 5, rq = f & 31;
        int gk = k0 + k, gr = r0 + 4 * rq;
        float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
        if (gk < kend && gr < R) x = *reinterpret_cast<const float4*>(P + (size_t)gk * ld + gr);
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, k = f >> 7, r = f & 127;
        int gk = k0 + k, gr = r0 + r;
        v[i] = (gk < kend && gr < R) ? P[(size_t)gk * ld + gr] : 0.f;
      }
    }
  }

  DDPG_DEV void store(float* __restrict__ lds, int tid) const {
    if constexpr (L == L_RK && VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, r = f >> 3, kq = f & 7;
#pragma unroll
        for (int j = 0; j < 4; ++j) lds[(4 * kq + j) * LS + r] = v[4 * i + j];
      }
    } else if constexpr (L == L_RK) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, r = f >> 5, k = f & 31;
        lds[k * LS + r] = v[i];
      }
    } else if constexpr (VEC == 4) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, k = f >> 5, rq = f & 31;
        *reinterpret_cast<float4*>(lds + k * LS + 4 * rq) =
            make_float4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        int f = i * GNT + tid, k = f >> 7, r = f & 127;
        lds[k * LS + r] = v[i];
      }
    }
  }
};

// ---------------------------------------------------------------- kernel
template <int AL, int BL, int VEC>
__global__ __launch_bounds__(GNT, 2) void gemm_f32_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float smem[GSMEM];
  using SA = Stage<AL, VEC>;
  using SB = Stage<BL, VEC>;
  constexpr int LSA = SA::LS, LSB = SB::LS;
  float* const As0 = smem;
  float* const Bs0 = smem + 2 * GBK * LSA;

  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5, li = lane & 31;
  const int n0 = blockIdx.x * GBN, m0 = blockIdx.y * GBM, z = blockIdx.z;
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
      const float* a_s = As0 + cur * GBK * LSA + wm * 64 + li;
      const float* b_s = Bs0 + cur * GBK * LSB + wn * 64 + li;
#pragma unroll
      for (int kk = 0; kk < GBK / 2; ++kk) {
        const int k = 2 * kk + h;
        const float a0 = a_s[k * LSA], a1 = a_s[k * LSA + 32];
        const float b0 = b_s[k * LSB], b1 = b_s[k * LSB + 32];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
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
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + li;
      const bool nok = n < N;
      const float bn = (nok && e.bias) ? e.bias[n] : 0.f;
      const float pwn = (nok && e.post == 2) ? e.pw[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
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

  // Row-wise reductions through LDS, 64 tile rows per pass.
  float* Vs = smem;                 // [64][VS_LD]
  float* Wps = smem + 64 * VS_LD;   // [128][PN]
  float* red = Wps + GBN * PROJ_MAX;  // [256]
  const int PN = (e.proj_n + 3) & ~3;
  if (e.proj_out) {
    for (int idx = tid; idx < GBN * PN; idx += GNT) {
      const int nl = idx / PN, a = idx - nl * PN, n = n0 + nl;
      Wps[idx] = (n < N && a < e.proj_n) ? e.proj[(size_t)n * e.proj_sn + (size_t)a * e.proj_sa]
                                          : 0.f;
    }
  }
  float csum = 0.f;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (wm == pass) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rl = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            Vs[rl * VS_LD + wn * 64 + j * 32 + li] = acc[i][j][r];
          }
    }
    __syncthreads();
    if (e.colsum) {
      const int col = tid & 127, rh = tid >> 7;
#pragma unroll 8
      for (int rr = 0; rr < 32; ++rr) csum += Vs[(rh * 32 + rr) * VS_LD + col];
    }
    if (e.proj_out) {
      const int PG = PN >> 2;
      for (int p = tid; p < 64 * PG; p += GNT) {
        const int row = p & 63, ag = p >> 6;
        float4 ap = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int n4 = 0; n4 < GBN / 4; ++n4) {
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
        const int m = m0 + pass * 64 + row;
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
    if (tid < 128) {
      const int n = n0 + tid;
      if (n < N)
        e.colsum[((size_t)z * gridDim.y + blockIdx.y) * e.ld_colsum + n] = red[tid] + red[tid + 128];
    }
  }
}

}  // namespace ddpg
