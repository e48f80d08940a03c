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
#include "types.h"

namespace ddpg {

// XCD-aware tile order (guide T1, bijective form): hardware deals workgroups
// round-robin over the 8 XCDs, so consecutive linear ids land on different
// L2s.  Remap so each XCD owns a contiguous run of row-major tiles (whole
// rows of m-tiles share their A panel in one L2).  Speed only; any placement
// is correct.
// on >= 16: each XCD owns a W x H rectangle of tiles (W = on - 16 columns,
// H = tiles per XCD / W rows; the host checks that 8 rectangles tile the
// grid), so it reads H row panels of A and W column panels of B instead of
// the whole B panel.
DDPG_DEV void xcd_tile(int& bx, int& by, int on) {
  if (!on) {
    bx = blockIdx.x;
    by = blockIdx.y;
    return;
  }
  if (on >= 16) {
    const int W = on - 16, nx = gridDim.x;
    const int lin = blockIdx.x + blockIdx.y * nx;
    const int x = lin & 7, idx = lin >> 3;
    const int H = ((nx * gridDim.y) >> 3) / W, rx = nx / W;
    bx = (x % rx) * W + idx % W;
    by = (x / rx) * H + idx / W;
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
// The __syncthreads() that gemm_epilogue executes for these epilogue flags:
// waves of a block that hold no accumulators (gemm_s3's staging waves) call
// this instead so that every wave passes the same barriers.  Keep in step
// with the barriers in gemm_epilogue below.
DDPG_DEV void gemm_epilogue_barriers(const GemmEpi& e) {
  if (!e.out && !e.outh && !e.colsum && !e.proj_out) return;
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();
    __syncthreads();
  }
  if (e.colsum) __syncthreads();
}

// Row / column (within the wave's 32x32 block) of accumulator register r of
// lane l: MF = 32 is the v_mfma_f32_32x32x* layout; MF = 16 is four 16x16
// tiles packed as register 4 (2 tr + tc) + q = row 16 tr + 4 (l >> 4) + q,
// column 16 tc + (l & 15) (gemm_h16_kernel).
template <int MF>
DDPG_DEV int acc_row(int r, int lane) {
  return MF == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
                  : 16 * (r >> 3) + 4 * (lane >> 4) + (r & 3);
}
template <int MF>
DDPG_DEV int acc_col(int r, int lane) {
  return MF == 32 ? (lane & 31) : 16 * ((r >> 2) & 1) + (lane & 15);
}

// Element-wise part of the epilogue on one wave's accumulators, specialised
// on the flag combinations the learner uses (BIAS: + bias[n]; ACT 1: elu;
// POST 1: * EluGrad factor of aux[m][n]; POST 2: pw[n] * EluGrad factor of v).
// Values outside the M x N range become 0 (they feed the row reductions).
// FULL: the tile lies inside M x N (the caller checked), no range tests.
template <int BM, int BN, int WGN, bool BIAS, int ACT, int POST, int MF, bool FULL = false>
DDPG_DEV void epi_apply(f32x16 (&acc)[BM / 64][BN / (32 * WGN)], const GemmEpi& e, int M, int N,
                        int n0, int m0, int wm, int wn, int lane) {
  constexpr int TM = BM / 64, TN = BN / (32 * WGN);
  constexpr int WR = BM / 2, WC = BN / WGN;
  constexpr int NC = MF == 32 ? 1 : 2;  // distinct columns per lane in a block
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int ncol[NC];
      float bnc[NC], pwc[NC];
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        ncol[u] = n0 + wn * WC + j * 32 + acc_col<MF>(4 * u, lane);
        bnc[u] = (BIAS && (FULL || ncol[u] < N)) ? e.bias[ncol[u]] : 0.f;
        pwc[u] = (POST == 2 && (FULL || ncol[u] < N)) ? e.pw[ncol[u]] : 0.f;
      }
      float av[16];
      if constexpr (POST == 1) {  // all 16 loads in flight before the first use
        if (e.auxh) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int n = ncol[NC == 1 ? 0 : (r >> 2) & 1];
            const int m = m0 + wm * WR + i * 32 + acc_row<MF>(r, lane);
            const __bf16* q = e.auxh + ((FULL || (n < N && m < M)) ? (size_t)m * e.ldaux + n : 0);
            av[r] = ((float)q[0] + (float)q[e.auxh_ps]) + (float)q[2 * e.auxh_ps];
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int n = ncol[NC == 1 ? 0 : (r >> 2) & 1];
            const int m = m0 + wm * WR + i * 32 + acc_row<MF>(r, lane);
            const float* q = (FULL || (n < N && m < M)) ? e.aux + (size_t)m * e.ldaux + n : e.aux;
            av[r] = *q;
          }
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int u = NC == 1 ? 0 : (r >> 2) & 1;
        const int n = ncol[u];
        const bool nok = n < N;
        const float bn = bnc[u], pwn = pwc[u];
        const int m = m0 + wm * WR + i * 32 + acc_row<MF>(r, lane);
        float v = acc[i][j][r];
        if constexpr (BIAS) v = __fadd_rn(v, bn);
        if constexpr (ACT == 1) v = elu_f(v);
        if constexpr (POST == 1) v = __fmul_rn(v, elu_grad_factor(av[r]));
        if constexpr (POST == 2) v = __fmul_rn(pwn, elu_grad_factor(v));
        acc[i][j][r] = (FULL || (nok && m < M)) ? v : 0.f;
      }
    }
  }
}

DDPG_DEV void store_twin(const GemmEpi& e, size_t i, float4 v) {
  store_twin4(e.outh + i, e.h_plane_stride, e.h_planes, v);
}

// Narrow weight-gradient partial of a staged tile (GemmEpi.nw_*): Vs holds
// PR = 128 rows of final values (the whole tile of gemm_h3 / gemm_h3m, one
// of the two passes of gemm_h16i's 256-row tile), Xs receives the narrow
// operand's rows.  Thread t: column quad nq = t % (BN / 4), narrow quad iq
// and row group g from t / (BN / 4); every thread sums its rows r = g, g +
// RG, ... in order with fp32 FMAs, and stores its 4 x 4 block to slab
// (rt * RG + g), rt = the 128-row block's index.
template <int PR, int BN, int NT>
DDPG_DEV void nw_load(const GemmEpi& e, int set, float* Xs, int tid, int m0) {
  const int K4 = (e.nw_k[set] + 3) >> 2;
  const f32x4* X = reinterpret_cast<const f32x4*>(e.nw_x[set]);
  f32x4* X4 = reinterpret_cast<f32x4*>(Xs);
  const int ld4 = e.nw_ldx[set] >> 2;
  for (int f = tid; f < PR * K4; f += NT) {
    const int r = f / K4, q = f - r * K4;
    X4[f] = X[(size_t)(m0 + r) * ld4 + q];
  }
}
template <int PR, int BN, int NT, int VS_LD>
DDPG_DEV void nw_partial(const GemmEpi& e, int set, const float* Vs, const float* Xs, int tid,
                         int n0, int rt) {
  const int K = e.nw_k[set], K4 = (K + 3) >> 2, RG = e.nw_rg[set];
  constexpr int NQ = BN / 4;
  const int nq = tid % NQ, rest = tid / NQ;
  const int iq = rest % K4, g = rest / K4;
  if (g >= RG) return;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4* X4 = reinterpret_cast<const f32x4*>(Xs);
#pragma unroll 4
  for (int r = g; r < PR; r += RG) {
    const f32x4 x = X4[r * K4 + iq];
    const f32x4 v = *reinterpret_cast<const f32x4*>(Vs + r * VS_LD + 4 * nq);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(x[i], v[j], acc[i][j]);
  }
  float* o = e.nw_out[set] + (size_t)(rt * RG + g) * e.nw_slab[set] + n0 + 4 * nq;
  if (set == 1) o -= e.nw_col1;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * iq + i < K) *reinterpret_cast<f32x4*>(o + (size_t)(4 * iq + i) * e.nw_ld[set]) = acc[i];
}

// ---------------------------------------------------------------- epilogue
// Accumulator layout (32x32 MFMA, dtype independent on gfx950): lane l holds
// column l&31 of tile (i, j); register r holds row (r&3) + 8(r>>2) + 4(l>>5).
// smem must hold TileCfg<BM,BN>::EPI floats and be free (all staging reads
// done) on entry.  WGN: waves along N; the accumulator waves are 2 x WGN
// (threads 0 .. 2*WGN*64-1), each owning BM/2 rows.
//
// The element-wise ops run in registers; the tile then goes through LDS one
// wave row (BM/2 rows) at a time, from where it is stored as float4 rows
// (1 KiB per wave instruction instead of 128-B column pieces) and reduced
// (bias-gradient column sums, thin projections).
// PR: tile rows staged through LDS per pass (default BM / 2, one wave row;
// BM / 4 for the 256 x 256 tile of gemm_h256.h, whose full wave row would not
// fit beside the projection weights; BM for gemm_h3_kernel's 128-row tile:
// one pass, every thread busy in the projection): smem must hold
// PR * (BN + 4) + BN * PROJ_MAX + 2 * GNT floats.
// ONLY >= 0: compile just that element-wise variant (the order of the
// dispatch below; the caller guarantees the flags), fewer live registers.
template <int BM, int BN, int WGN = 2, int MF = 32, int PR = BM / 2, bool FULL = false,
          int ONLY = -1>
DDPG_DEV void gemm_epilogue(f32x16 (&acc)[BM / 64][BN / (32 * WGN)], float* smem,
                            const GemmArgs& g,
                            int tid, int n0, int m0, int z, int bx, int by) {
  using TC = TileCfg<BM, BN>;
  constexpr int NT = 2 * WGN * 64;  // threads
  constexpr int TM = BM / 64, TN = BN / (32 * WGN);
  constexpr int WR = BM / 2, WC = BN / WGN;
  constexpr int NPASS = BM / PR;
  static_assert(BM % PR == 0 && PR % 32 == 0, "pass rows");
  const int wave = tid >> 6, lane = tid & 63;
  const int wm = wave / WGN, wn = wave % WGN;
  const GemmEpi& e = g.e;
  const int M = g.M, N = g.N;
  float* outp = e.out ? e.out + (size_t)z * e.out_split_stride : nullptr;

  const bool bias = e.bias != nullptr;
  if constexpr (ONLY == 0)
    epi_apply<BM, BN, WGN, false, 0, 0, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if constexpr (ONLY == 1)
    epi_apply<BM, BN, WGN, true, 1, 0, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if constexpr (ONLY == 3)
    epi_apply<BM, BN, WGN, false, 0, 1, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if (!bias && e.act == 0 && e.post == 0)
    epi_apply<BM, BN, WGN, false, 0, 0, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if (bias && e.act == 1 && e.post == 0)
    epi_apply<BM, BN, WGN, true, 1, 0, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if (bias && e.act == 1 && e.post == 2)
    epi_apply<BM, BN, WGN, true, 1, 2, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if (!bias && e.act == 0 && e.post == 1)
    epi_apply<BM, BN, WGN, false, 0, 1, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else if (bias && e.act == 0 && e.post == 0)
    epi_apply<BM, BN, WGN, true, 0, 0, MF, FULL>(acc, e, M, N, n0, m0, wm, wn, lane);
  else  // not used by the learner; the host rejects other combinations
    __builtin_trap();

  if (!outp && !e.outh && !e.colsum && !e.proj_out && !e.nw_out[0] && !e.nw_out[1]) return;

  constexpr int VS_LD = TC::VS_LD;
  float* Vs = smem;                      // [PR][VS_LD]
  float* Wps = smem + PR * VS_LD;        // [BN][PN]
  float* red = Wps + BN * PROJ_MAX;      // [NT]
  float* Xs = red + 2 * GNT;             // [PR][<= 64] narrow rows (nw_*, PR == 128)
  // narrow set of this tile by its column range: set 0 below nw_col1, set 1
  // from it (nw_col1 = 0: one set over every column); a null set's tiles
  // carry no partial
  const int nws = (e.nw_col1 > 0 && n0 >= e.nw_col1) ? 1 : 0;
  const bool nw = PR == 128 && e.nw_out[nws] != nullptr;
  const int PN = (e.proj_n + 3) & ~3;
  if (e.proj_out) {
    for (int idx = tid; idx < BN * PN; idx += NT) {
      const int nl = idx / PN, a = idx - nl * PN, n = n0 + nl;
      Wps[idx] = ((FULL || n < N) && a < e.proj_n) ? e.proj[(size_t)n * e.proj_sn + (size_t)a * e.proj_sa]
                                          : 0.f;
    }
  }
  // float4 row stores need 4-aligned widths / leading dims and a 16-B base
  const bool vst = outp && ((N | e.ldo) & 3) == 0 && (e.out_split_stride & 3) == 0 &&
                   ((uintptr_t)outp & 15) == 0;
  constexpr int C4 = BN / 4, RPR = NT / C4;  // float4 columns per row, rows per round
  // 8-column rows (16-B twin stores) when every row start is 16-B aligned
  const bool oct = (N & 7) == 0 && (!outp || (vst && (e.ldo & 7) == 0)) &&
                   (!e.outh || ((e.ldo & 7) == 0 && (e.h_plane_stride & 7) == 0 &&
                                (e.out_split_stride & 7) == 0 &&
                                ((uintptr_t)e.outh & 15) == 0)) &&
                   BN % 8 == 0 && NT % (BN / 8) == 0;
  constexpr int CG = NT / BN;  // column-sum row groups
  float csum = 0.f;
  // one LDS pass of PR rows (unrolled: a runtime pass index sends the
  // accumulators to scratch)
  auto do_pass = [&](int pass) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int r0 = wm * WR + i * 32;  // this 32-row block's first tile row
      if (r0 / PR != pass) continue;     // (wave-uniform) not in this pass
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = r0 - pass * PR + acc_row<MF>(r, lane);
          Vs[rl * VS_LD + wn * WC + j * 32 + acc_col<MF>(r, lane)] = acc[i][j][r];
        }
    }
    if (nw) nw_load<PR, BN, NT>(e, nws, Xs, tid, m0 + pass * PR);
    __syncthreads();
    if (nw) nw_partial<PR, BN, NT, VS_LD>(e, nws, Vs, Xs, tid, n0, (m0 + pass * PR) / PR);
    if ((outp || e.outh) && oct) {
      // 8 columns per thread: 16-B stores for the fp32 rows and every twin plane
      constexpr int C8 = BN / 8, RPR8 = NT / C8;
      const int c8 = tid % C8, rr0 = tid / C8, n = n0 + 8 * c8;
      if (FULL || n < N) {
#pragma unroll 2
        for (int rr = rr0; rr < PR; rr += RPR8) {
          const int m = m0 + pass * PR + rr;
          if (!FULL && m >= M) continue;
          const float4 va = *reinterpret_cast<const float4*>(Vs + rr * VS_LD + 8 * c8);
          const float4 vb = *reinterpret_cast<const float4*>(Vs + rr * VS_LD + 8 * c8 + 4);
          const size_t o = (size_t)m * e.ldo + n;
          if (e.outh)
            store_twin8(e.outh + (size_t)z * e.out_split_stride + o, e.h_plane_stride,
                        e.h_planes, va, vb);
          if (outp && n >= e.out_col0) {
            *reinterpret_cast<float4*>(outp + o) = va;
            *reinterpret_cast<float4*>(outp + o + 4) = vb;
          }
        }
      }
    } else if (outp || e.outh) {
      const int c4 = tid % C4, rr0 = tid / C4, n = n0 + 4 * c4;
#pragma unroll 4
      for (int rr = rr0; rr < PR; rr += RPR) {
        const int m = m0 + pass * PR + rr;
        if (m < M) {
          const float4 v = *reinterpret_cast<const float4*>(Vs + rr * VS_LD + 4 * c4);
          float* o = outp ? outp + (size_t)m * e.ldo + n : nullptr;
          if (e.outh && n < N) store_twin(e, (size_t)z * e.out_split_stride + (size_t)m * e.ldo + n, v);
          if (!outp || n < e.out_col0) continue;
          if (vst) {
            if (n < N) *reinterpret_cast<float4*>(o) = v;
          } else {
            if (n < N) o[0] = v.x;
            if (n + 1 < N) o[1] = v.y;
            if (n + 2 < N) o[2] = v.z;
            if (n + 3 < N) o[3] = v.w;
          }
        }
      }
    }
    if (e.colsum) {
      const int col = tid % BN, grp = tid / BN;
#pragma unroll 4
      for (int rr = grp; rr < PR; rr += CG) csum += Vs[rr * VS_LD + col];
    }
    if (e.proj_out) {
      const int PG = PN >> 2;
      for (int p = tid; p < PR * PG; p += NT) {
        const int row = p % PR, ag = p / PR;
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
        const int m = m0 + pass * PR + row;
        if (FULL || m < M) {
          float* po = e.proj_out + ((size_t)bx * M + m) * e.proj_n;
          const float av[4] = {ap.x, ap.y, ap.z, ap.w};
#pragma unroll
          for (int a = 0; a < 4; ++a)
            if (4 * ag + a < e.proj_n) po[4 * ag + a] = av[a];
        }
      }
    }
    __syncthreads();
  };
#pragma unroll
  for (int pass = 0; pass < NPASS; ++pass) do_pass(pass);
  if (e.colsum) {
    red[tid] = csum;
    __syncthreads();
    if (tid < BN) {
      float s = 0.f;
#pragma unroll
      for (int gi = 0; gi < CG; ++gi) s += red[tid + gi * BN];
      const int n = n0 + tid;
      if (FULL || n < N) e.colsum[((size_t)z * gridDim.y + by) * e.ld_colsum + n] = s;
    }
  }
}

// ---------------------------------------------------------------- in-launch K split
// Small-M plan (per-rank batches of a strong-scaling run: M = B <= 2048): a
// plain GEMM whose output tiles do not fill the chip runs its K range as
// gridDim.z splits, and the splits of each tile are combined inside the same
// launch before the fused epilogue.  Every block stores its fp32 partial
// (each lane's accumulator registers as 64-B runs: coalesced) to its slot of
// `part` ([tile][split][NV][threads][16]), then takes a ticket on the tile;
// the block that draws the last ticket adds the partials in split order
// 0 .. S-1 (its own from registers), so the sum does not depend on which
// split arrives last (bitwise reproducible), resets the ticket for the next
// launch and returns true; the other blocks return false and exit.
// Cross-XCD hand-off without cache flushes (MI355X_MICROARCH.md, the sc1
// hand-off table, first row): the partials are stored and loaded with sc1
// (16 B per lane, lane-linear so that one wave instruction covers 1 KiB of
// whole lines -- a 64-B lane stride made every instruction a 64-line partial
// write and tripled the hand-off, 7-10 -> 2-3 us; written through past the
// storing XCD's L2, read past the reading CU's caches), every storing wave waits vmcnt(0) before the
// workgroup barrier, then ONE lane's agent-scope atomic add on the tile's
// counter; the block whose add returns S - 1 loads after a barrier.  (An
// agent fence per wave instead -- buffer_wbl2 + buffer_inv -- cost more than
// the split saved.)  The sc1 accesses are the buffer intrinsics with cache
// policy 16 (sc1), which the compiler sees, so it orders and waits for them
// and keeps the store-data hazards (an inline-asm store whose data registers
// were rewritten one cycle later gave run-to-run differences).
constexpr int KC_SC1 = 16;  // CPol SC1

template <int NV>
DDPG_DEV bool ksplit_combine(f32x16* acc, float* part, unsigned* ticket, int tile, int z, int S,
                             int tid, int nt) {
  __shared__ unsigned last_s;
  const unsigned slab = (unsigned)(NV * nt * 16 * 4);  // bytes per (tile, split)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(part + (size_t)tile * S * (slab / 4)), 0, 0x7fffffff, 0x00020000);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_raw_buffer_store_b128(
          __builtin_bit_cast(u32x4, f32x4{acc[v][4 * q], acc[v][4 * q + 1], acc[v][4 * q + 2],
                                          acc[v][4 * q + 3]}),
          rs, z * slab + (unsigned)(((v * 4 + q) * nt + tid) * 16), 0, KC_SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial has left
  __syncthreads();
  if (tid == 0) {
    const unsigned old =
        __hip_atomic_fetch_add(ticket + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned l = old == (unsigned)(S - 1);
    if (l) __hip_atomic_store(ticket + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = l;
  }
  __syncthreads();
  if (!last_s) return false;
  auto ld = [&](int zz, int v, int q) {
    return __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                   rs, zz * slab + (unsigned)(((v * 4 + q) * nt + tid) * 16), 0, KC_SC1));
  };
  if constexpr (NV <= 2) {
    // the other splits' partials in flight four at a time (one memory round
    // trip per four splits, not one per split), summed in split order 0 ..
    // S-1 (own partial from the registers); the host caps S at KC_MAXS
    f32x4 t[NV][4];
#pragma unroll
    for (int c0 = 0; c0 < KC_MAXS; c0 += 4) {
      if (c0 >= S) break;
      f32x4 x[4][NV][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int zz = c0 + j;
#pragma unroll
        for (int v = 0; v < NV; ++v)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            x[j][v][q] = zz < S && zz != z
                             ? ld(zz, v, q)
                             : f32x4{acc[v][4 * q], acc[v][4 * q + 1], acc[v][4 * q + 2],
                                     acc[v][4 * q + 3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int zz = c0 + j;
        if (zz < S)
#pragma unroll
          for (int v = 0; v < NV; ++v)
#pragma unroll
            for (int q = 0; q < 4; ++q) t[v][q] = zz == 0 ? x[j][v][q] : t[v][q] + x[j][v][q];
      }
    }
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[v][4 * q + e] = t[v][q][e];
  } else {
    // 256-row tiles (64 accumulators per lane): no registers for S - 1
    // partials at once -- one split per round trip, in split order
    f32x16 own[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) own[v] = acc[v];
    for (int zz = 0; zz < S; ++zz) {
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        f32x16 p = own[v];
        if (zz != z)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x4 y = ld(zz, v, q);
#pragma unroll
            for (int e = 0; e < 4; ++e) p[4 * q + e] = y[e];
          }
        acc[v] = zz == 0 ? p : acc[v] + p;
      }
    }
  }
  return true;
}

}  // namespace ddpg
