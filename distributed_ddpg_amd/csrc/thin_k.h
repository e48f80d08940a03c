// Thin-K dense layers (K <= 64) of the large-batch path: the input layers
// (actor W1: K = S, critic Ws / Wa: K = S / A, networks.py:54,151-152) and the
// dz2 = dz3 . W3^T layer (K = A, networks.py:44).  At B = 4096 these are
// output-write-bound (16 MB per 1024-wide layer) with a few hundred MFLOP, so
// a tiled GEMM spends its time in prologue, epilogue and launch, and a VALU
// kernel is LDS-bandwidth-bound (every fmaf operand pair comes from LDS).
//
// Here a workgroup (4 waves) owns a 64-row x TK_COLS-column output block
// (TK_COLS = 128, or 64 for a 48-KB block, three per CU).  The
// K x TK_COLS weight panel and the 64 x K input tile are split once into their
// exact three bf16 planes (x = h + m + l) in LDS; each wave owns 32 rows x
// TK_COLS / 2 columns (TK_TPW 32x32 tiles) and takes the six plane products of the twin GEMM
// (gemm_h.h) per 16-deep step on v_mfma_f32_32x32x16_bf16 with fp32
// accumulation -- 2.7x the fp32-input MFMA rate at the same accuracy class as
// the large GEMMs.  The fused epilogue has the gemm_common.h semantics (bias,
// elu, EluGrad multiply, bias-gradient column sums).  Up to TK_MAXP
// independent layers share one launch (blockIdx.z selects the part): the
// critic's [state | action] concat, and the large-batch step's five
// batch-only first layers (target actor, target critic state branch, actor,
// critic state and action branches).
#pragma once
#include "common.h"
#include "types.h"

// Phase timestamp hook for tools/thin_k_bench.hip; empty in the product build.
#ifndef TK_STAMP
#define TK_STAMP(i)
#endif

namespace ddpg {

// Three-plane bf16 images (the exact split x = h + m + l of every fp32
// operand, as the twins of gemm_h.h): [plane][row][64 k] with 128-B rows, 16-B
// chunk c of row r at c ^ ((r >> 1) & 7) -- every 32x32x16 fragment read
// (lane: row l & 31, chunk 2 ks + (l >> 5)) is bank-conflict-free.  X rows are
// batch rows; W rows are output columns (W^T), so both operands are read the
// same way.
DDPG_DEV int tk_swz(int r) { return (r >> 1) & 7; }
// hipcc's waitcnt insertion treats an asm operand as a use: the wait for a
// register's pending global load goes here instead of at its first real use
// (where, behind branches and conditional stores, it becomes vmcnt(0) and
// waits for every store issued since)
#define TK_LANDED(x) asm volatile("" ::"v"(x))
DDPG_DEV int tk_off(int r, int k) { return r * 128 + 16 * ((k >> 3) ^ tk_swz(r)) + 2 * (k & 7); }
// output tile: float (r, n) -- the MFMA write of lanes h = 0 / 1 (rows r, r + 4)
// lands in opposite 128-B halves of the banks; the quad's low bit is XORed
// with bit 4 of the quad index, so the epilogue's 8-column row reads (quads
// 2 c8 and 2 c8 + 1, lanes of a ds_read_b128 group spanning c8 and c8 + 8)
// hit 16 distinct 16-B bank slots instead of 8 twice (SQ_LDS_BANK_CONFLICT
// was 16-23 % of thin_k's LDS cycles, profiles/r4/lds_conflicts.txt)
DDPG_DEV int tk_oidx(int r, int n) {
  const int q = n >> 2;
  return r * TK_COLS + ((q ^ (((r >> 2) & 1) << 3) ^ ((q >> 4) & 1)) << 2) + (n & 3);
}

// Block (column block x, row tiles [rpb y, rpb y + rpb), part z): the W panel
// is loaded and split once; each row tile's X tile is loaded one tile ahead
// (its global loads in flight under the current tile's MFMAs and epilogue
// stores), so the stream of output stores -- what bounds these layers -- is
// not interrupted by a fresh W-panel round trip per 64 rows.
// MODE 0: every part's flags read at run time.  MODE 1, the forward form:
// every part has bias, elu, the twin as whole 8-column octets, an fp32 copy
// or none, no aux, no column sums, full row and column tiles.  MODE 2, the
// backward form (dz2 = dz3 . W3^T): no bias, no activation, the EluGrad aux,
// column sums, full tiles.  thin_k_launch checks; the folded flags and bounds
// matter because the epilogue row loop is VALU-bound.
// DW: the fused weight gradient (TkPart.dw) compiled in (MODE != 1).
template <int MODE, bool DW = false>
__global__ __launch_bounds__(TK_NT) void thin_k_kernel(TkArgs args) {
  __shared__ __attribute__((aligned(16))) char lds[TK_LDS];
  char* const wimg = lds;
  char* const ximg = lds + 3 * TK_WIMG;
  float* const Os = reinterpret_cast<float*>(ximg);   // output tile (after the MFMAs)
  float* const red = reinterpret_cast<float*>(ximg);  // column-sum scratch (after the stores)
  const TkPart P = args.p[blockIdx.z];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, h = lane >> 5;
  const int wr = wave & 1, wc = wave >> 1;  // 32-row half, column half
  const int n0 = blockIdx.x * TK_COLS;
  const int rt0 = blockIdx.y * args.rpb, rt1 = min(args.mt, rt0 + args.rpb);
  if (n0 >= P.N || rt0 >= rt1) return;
  TK_STAMP(0);
  const int K = P.K, M = args.M;
  const int KS = (K + 15) >> 4;  // 16-deep MFMA steps; k in [K, 16 KS) are zeros
  const int KP = 16 * KS;
  // ---- X tile loads (64 rows x 16 quads, 4 float4 per thread)
  f32x4 xg[4];
  auto load_x = [&](int rt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = tid + TK_NT * j, r = f >> 4, k = 4 * (f & 15), m = rt * TK_ROWS + r;
      xg[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < K && m < M) xg[j] = *reinterpret_cast<const f32x4*>(P.X + (size_t)m * P.ldx + k);
    }
  };
  load_x(rt0);
  // ---- W panel: thread (column c, k quads kq + 2 j), split into its image once
  const int wcol = tid % TK_COLS, kq = tid / TK_COLS, wn = n0 + wcol;
  auto put4 = [&](char* img, int plane_bytes, int r, int k, f32x4 v) {
    bf16x2 h0, m0_, l0, h1, m1, l1;
    split3_pair(f32x2v{v[0], v[1]}, h0, m0_, l0);
    split3_pair(f32x2v{v[2], v[3]}, h1, m1, l1);
    const int off = tk_off(r, k);
    *reinterpret_cast<bf16x4*>(img + off) = bf16x4{h0[0], h0[1], h1[0], h1[1]};
    *reinterpret_cast<bf16x4*>(img + plane_bytes + off) = bf16x4{m0_[0], m0_[1], m1[0], m1[1]};
    *reinterpret_cast<bf16x4*>(img + 2 * plane_bytes + off) = bf16x4{l0[0], l0[1], l1[0], l1[1]};
  };
  {
    // every load unconditional (clamped into the panel, masked after): behind
    // per-load branches hipcc put a vmcnt(0) before each group, one round
    // trip per k quad
    f32x4 wv[TK_WJ];
    const bool wvec = P.w_nk && ((P.ldw & 3) == 0) && (((uintptr_t)P.W & 15) == 0);
    const int wnc = min(wn, P.N - 1);
    if (wvec) {  // W[n][k], 16-B rows: 4 consecutive k per load
#pragma unroll
      for (int j = 0; j < TK_WJ; ++j) {
        const int k = 4 * (kq + TK_KQS * j);
        wv[j] = *reinterpret_cast<const f32x4*>(P.W + (size_t)wnc * P.ldw + min(k, K - 4));
      }
    } else if (P.w_nk) {  // W[n][k] of an unaligned stride: scalars
#pragma unroll
      for (int j = 0; j < TK_WJ; ++j) {
        const float* q = P.W + (size_t)wnc * P.ldw + min(4 * (kq + TK_KQS * j), K - 4);
        wv[j] = f32x4{q[0], q[1], q[2], q[3]};
      }
    } else {  // W[k][n]: 4 rows of column n (each load coalesced over the 128 columns)
#pragma unroll
      for (int j = 0; j < TK_WJ; ++j) {
        const int k = min(4 * (kq + TK_KQS * j), K - 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) wv[j][e] = P.W[(size_t)(k + e) * P.ldw + wnc];
      }
    }
#pragma unroll
    for (int j = 0; j < TK_WJ; ++j)
      if (4 * (kq + TK_KQS * j) >= K || wn >= P.N) wv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < TK_WJ; ++j) {
      const int k = 4 * (kq + TK_KQS * j);
      if (k < KP) put4(wimg, TK_WIMG, wcol, k, wv[j]);
    }
  }
  // per-thread epilogue constants: column octet c8, rows rg + TK_RG i
  const int c8 = tid % TK_OCT, rg = tid / TK_OCT, n = n0 + 8 * c8;
  const bool q0 = n < P.N, q1 = n + 4 < P.N;  // N % 4 == 0: quads all in or all out
  const bool oct = q1 && ((P.ldo & 7) == 0) && ((P.hps & 7) == 0) &&
                   (((uintptr_t)P.outh & 15) == 0);
  f32x4 bq0 = f32x4{0.f, 0.f, 0.f, 0.f}, bq1 = bq0;
  if (P.bias && q0) bq0 = *reinterpret_cast<const f32x4*>(P.bias + n);
  if (P.bias && q1) bq1 = *reinterpret_cast<const f32x4*>(P.bias + n + 4);
  const int ra = 32 * wr + li;
#pragma unroll
  for (int j = 0; j < 4; ++j) TK_LANDED(xg[j]);
  TK_LANDED(bq0);
  TK_LANDED(bq1);

  for (int rt = rt0; rt < rt1; ++rt) {
    const int m0 = rt * TK_ROWS;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int f = tid + TK_NT * j, r = f >> 4, k = 4 * (f & 15);
      if (k < KP) put4(ximg, TK_XIMG, r, k, xg[j]);
    }
    __syncthreads();  // X image (and, first trip, the W image) complete
    TK_STAMP(1);
    if (rt + 1 < rt1) load_x(rt + 1);  // next tile's loads in flight from here
    // ---- MFMA (v_mfma_f32_32x32x16_bf16, fp32 accumulation): per 16-deep
    // step the six plane products hh, hm, mh, hl, lh, mm of gemm_h.h, the five
    // small ones in their own accumulator.  Wave (wr, wc): rows 32 wr + li,
    // columns (TK_COLS / 2) wc + 32 t + li (t < TK_TPW).
    f32x16 acc[TK_TPW], acs[TK_TPW];
#pragma unroll
    for (int t = 0; t < TK_TPW; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = acs[t][r] = 0.f;
    for (int ks = 0; ks < KS; ++ks) {
      const int kk = 16 * ks + 8 * h;
      bf16x8 a[3], b[TK_TPW][3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        a[p] = *reinterpret_cast<const bf16x8*>(ximg + p * TK_XIMG + tk_off(ra, kk));
#pragma unroll
        for (int t = 0; t < TK_TPW; ++t)
          b[t][p] = *reinterpret_cast<const bf16x8*>(
              wimg + p * TK_WIMG + tk_off((TK_COLS / 2) * wc + 32 * t + li, kk));
      }
#pragma unroll
      for (int t = 0; t < TK_TPW; ++t) {
        f32x16 q = acs[t];
        q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[t][0], q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[t][1], q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t][2], q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[t][0], q, 0, 0, 0);
        q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t][1], q, 0, 0, 0);
        acs[t] = q;
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[t][0], acc[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < TK_TPW; ++t) acc[t] += acs[t];
    TK_STAMP(2);
    // ---- epilogue.  The raw tile goes through LDS (lane li of tile t holds
    // column li, register r row (r & 3) + 8 (r >> 2) + 4 h) so that every
    // element-wise op, the aux loads and the output stores run on float4 rows.
    __syncthreads();  // every wave done reading the X image
    {
      const int rb = 32 * wr + 4 * h;
#pragma unroll
      for (int t = 0; t < TK_TPW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          Os[tk_oidx(rb + (r & 3) + 8 * (r >> 2), (TK_COLS / 2) * wc + 32 * t + li)] = acc[t][r];
    }
    __syncthreads();
    TK_STAMP(3);
    float csum[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) csum[e] = 0.f;
    constexpr int RPT = TK_ROWS / TK_RG;  // rows per thread
    f32x4 aq[RPT][2];
    if (MODE == 2 || (MODE == 0 && P.aux)) {  // all aux loads in flight before the first use
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int m = m0 + rg + TK_RG * i;
        aq[i][0] = aq[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m < M) {
          const float* ap = P.aux + (size_t)m * P.ldaux + n;
          if (q0) aq[i][0] = *reinterpret_cast<const f32x4*>(ap);
          if (q1) aq[i][1] = *reinterpret_cast<const f32x4*>(ap + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        TK_LANDED(aq[i][0]);
        TK_LANDED(aq[i][1]);
      }
    }
    // every load this tile's stores could be ordered behind (the aux rows
    // above, the next X tile) has landed here, before the first store: the
    // row loop below then carries no vmcnt wait, and the next trip's put4 of
    // xg none either -- the stores stream while the next tile's MFMAs run
#pragma unroll
    for (int j = 0; j < 4; ++j) TK_LANDED(xg[j]);
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int rl = rg + TK_RG * i, m = m0 + rl;
      if (MODE == 0 && (!q0 || m >= M)) continue;
      f32x4 v[2];
      v[0] = *reinterpret_cast<const f32x4*>(Os + tk_oidx(rl, 8 * c8));
      v[1] = *reinterpret_cast<const f32x4*>(Os + tk_oidx(rl, 8 * c8 + 4));
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x = v[u][e];
          if (MODE == 1 || (MODE == 0 && P.bias)) x = __fadd_rn(x, u ? bq1[e] : bq0[e]);
          if (MODE == 1 || (MODE == 0 && P.act == 1)) x = elu_f(x);
          if (MODE == 2 || (MODE == 0 && P.aux)) x = __fmul_rn(x, elu_grad_factor(aq[i][u][e]));
          v[u][e] = x;
          if (MODE == 2 || (MODE == 0 && (u == 0 || q1))) csum[4 * u + e] += x;
        }
      const size_t o = (size_t)m * P.ldo + n;
      const float4 va = make_float4(v[0][0], v[0][1], v[0][2], v[0][3]);
      const float4 vb = make_float4(v[1][0], v[1][1], v[1][2], v[1][3]);
      if (MODE != 0) {
        if (P.out) {
          *reinterpret_cast<f32x4*>(P.out + o) = v[0];
          *reinterpret_cast<f32x4*>(P.out + o + 4) = v[1];
        }
        if (MODE == 1 || P.outh) store_twin8(P.outh + o, P.hps, P.hnp, va, vb);
        continue;
      }
      if (P.out) {
        *reinterpret_cast<f32x4*>(P.out + o) = v[0];
        if (q1) *reinterpret_cast<f32x4*>(P.out + o + 4) = v[1];
      }
      if (P.outh) {
        if (oct) {
          store_twin8(P.outh + o, P.hps, P.hnp, va, vb);
        } else {
          store_twin4(P.outh + o, P.hps, P.hnp, va);
          if (q1) store_twin4(P.outh + o + 4, P.hps, P.hnp, vb);
        }
      }
    }
    TK_STAMP(4);
    __syncthreads();  // output tile read: the region is next the column-sum scratch / X image
    if (MODE == 2 || (MODE == 0 && P.colsum)) {
#pragma unroll
      for (int e = 0; e < 8; ++e) red[rg * TK_COLS + 8 * c8 + e] = csum[e];
      __syncthreads();
      if (tid < TK_COLS && n0 + tid < P.N) {
        float s = 0.f;
#pragma unroll
        for (int g = 0; g < TK_RG; ++g) s += red[g * TK_COLS + tid];
        P.colsum[(size_t)rt * P.ld_colsum + n0 + tid] = s;
      }
      __syncthreads();
    }
    // backward / generic form: the fused weight gradient aux^T X of this row
    // tile (dW3 = h2^T dz3, networks.py:44's dW beside its dX) on the fp32
    // MFMA (v_mfma_f32_16x16x4_f32: exact f32 products, an fmaf chain): the aux
    // rows this thread holds (aq) and the tile's X rows are staged in LDS 32
    // rows at a time; wave w owns the dw rows (output columns) of 16-column
    // blocks NBW w .. NBW w + NBW - 1, every 16-wide block of dw's columns;
    // one fp32 partial per row tile
    if (DW && MODE != 1 && P.dw) {
      constexpr int NBW = TK_COLS / 64;         // 16-column blocks per wave
      float* const Hs = Os;                     // [32][TK_COLS] aux rows
      float* const Ds = Os + 32 * TK_COLS;      // [32][K] X rows (fp32)
      const int NAB = (P.dw_k + 15) >> 4;       // 16-wide blocks of dw columns (<= 2)
      const int li16 = lane & 15, lq = lane >> 4;
      f32x4 dacc[NBW][2];
#pragma unroll
      for (int b = 0; b < NBW; ++b) dacc[b][0] = dacc[b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int half = 0; half < 2; ++half) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          const int rl = rg + TK_RG * i;
          if ((rl >> 5) != half) continue;
          *reinterpret_cast<f32x4*>(Hs + (rl & 31) * TK_COLS + 8 * c8) = aq[i][0];
          *reinterpret_cast<f32x4*>(Hs + (rl & 31) * TK_COLS + 8 * c8 + 4) = aq[i][1];
        }
        const int K4 = K >> 2;
        for (int f = tid; f < 32 * K4; f += TK_NT) {
          const int r = f / K4, q = f - r * K4, m = m0 + 32 * half + r;
          f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
          if (m < M) v = *reinterpret_cast<const f32x4*>(P.X + (size_t)m * P.ldx + 4 * q);
          *reinterpret_cast<f32x4*>(Ds + r * K + 4 * q) = v;
        }
        __syncthreads();
#pragma unroll
        for (int st = 0; st < 8; ++st) {  // 4 rows per MFMA k-step
          const int r = 4 * st + lq;
          float av[NBW], bv[2];
#pragma unroll
          for (int b = 0; b < NBW; ++b) av[b] = Hs[r * TK_COLS + (NBW * wave + b) * 16 + li16];
#pragma unroll
          for (int ab = 0; ab < 2; ++ab)
            bv[ab] = (ab < NAB && ab * 16 + li16 < K) ? Ds[r * K + ab * 16 + li16] : 0.f;
#pragma unroll
          for (int b = 0; b < NBW; ++b)
#pragma unroll
            for (int ab = 0; ab < 2; ++ab)
              if (ab < NAB)
                dacc[b][ab] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[b], bv[ab], dacc[b][ab], 0, 0, 0);
        }
        __syncthreads();
      }
      // D[i][j]: i = dw row (output column) 4 lq + e of the block, j = dw column li16
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int ab = 0; ab < 2; ++ab) {
          const int a = ab * 16 + li16;
          if (ab >= NAB || a >= P.dw_k) continue;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int n = n0 + (NBW * wave + b) * 16 + 4 * lq + e;
            if (n < P.N) P.dw[(size_t)rt * P.dw_slab + (size_t)n * P.dw_k + a] = dacc[b][ab][e];
          }
        }
    }
  }
}

}  // namespace ddpg
