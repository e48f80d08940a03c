// Shared pieces of the DDPG GEMMs (fp32 and bf16 MFMA variants): arguments,
// tile configuration and the fused epilogue.  Kernel-specific comments live
// in gemm_f32.h / gemm_bf16.h.
//
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
  static constexpr int EPI = (BM / 2) * VS_LD + BN * PROJ_MAX + 2 * GNT;  // red: up to 512 threads
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
  int xcd;  // 1: XCD-aware tile order (xcd_tile)
  GemmEpi e;
};


// ---------------------------------------------------------------- epilogue
// Accumulator layout (32x32 MFMA, dtype independent on gfx950): lane l holds
// column l&31 of tile (i, j); register r holds row (r&3) + 8(r>>2) + 4(l>>5).
// smem must hold TileCfg<BM,BN>::EPI floats and be free (all staging reads
// done) on entry.
// XCD-aware tile order (guide T1, bijective form): hardware deals workgroups
// round-robin over the 8 XCDs, so consecutive linear ids land on different
// L2s.  Remap so each XCD owns a contiguous run of row-major tiles (whole
// rows of m-tiles share their A panel in one L2).  Speed only; any placement
// is correct.
DDPG_DEV void xcd_tile(int& bx, int& by, int on) {
  if (!on) {
    bx = blockIdx.x;
    by = blockIdx.y;
    return;
  }
  const int nx = gridDim.x;
  const int nwg = gridDim.x * gridDim.y;
  const int lin = blockIdx.x + blockIdx.y * nx;
  const int xcd = lin & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
  by = wgid / nx;
  bx = wgid - by * nx;
}

// WGN: waves along N (2 for the 4-wave kernels, 4 for the 8-wave gemm_s3);
// the block always has 2 waves along M, each owning BM/2 rows.
template <int BM, int BN, int WGN = 2>
DDPG_DEV void gemm_epilogue(f32x16 (&acc)[BM / 64][BN / (32 * WGN)], float* smem,
                            const GemmArgs& g,
                            int tid, int n0, int m0, int z, int bx, int by) {
  using TC = TileCfg<BM, BN>;
  constexpr int NT = 2 * WGN * 64;  // threads
  constexpr int TM = BM / 64, TN = BN / (32 * WGN);
  constexpr int WR = BM / 2, WC = BN / WGN;
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WGN, wn = wave % WGN;
  const int h = lane >> 5, li = lane & 31;
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
  float* red = Wps + BN * PROJ_MAX;      // [NT]
  const int PN = (e.proj_n + 3) & ~3;
  if (e.proj_out) {
    for (int idx = tid; idx < BN * PN; idx += NT) {
      const int nl = idx / PN, a = idx - nl * PN, n = n0 + nl;
      Wps[idx] = (n < N && a < e.proj_n) ? e.proj[(size_t)n * e.proj_sn + (size_t)a * e.proj_sa]
                                          : 0.f;
    }
  }
  constexpr int CG = NT / BN;  // column-sum row groups
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
      for (int p = tid; p < WR * PG; p += NT) {
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
          float* po = e.proj_out + ((size_t)bx * M + m) * e.proj_n;
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
      if (n < N) e.colsum[((size_t)z * gridDim.y + by) * e.ld_colsum + n] = s;
    }
  }
}

}  // namespace ddpg
