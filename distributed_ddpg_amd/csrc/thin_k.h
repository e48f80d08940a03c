// Thin-K dense layers (K <= 64) of the large-batch path: the input layers
// (actor W1: K = S, critic Ws / Wa: K = S / A, networks.py:54,151-152) and the
// dz2 = dz3 . W3^T layer (K = A, networks.py:44).  At B = 4096 these are
// output-write-bound (16 MB per 1024-wide layer) with a few hundred MFLOP, so
// a tiled GEMM spends its time in prologue, epilogue and launch, and a VALU
// kernel is LDS-bandwidth-bound (every fmaf operand pair comes from LDS).
//
// Here a workgroup (4 waves) owns a 64-row x 128-column output block.  The
// K x 128 weight panel is staged once in LDS; each wave owns 32 rows x 64
// columns (two 32x32 fp32 MFMA tiles, v_mfma_f32_32x32x2_f32: exact fp32
// products, fp32 accumulation) and feeds its A operand straight from global
// memory: lane l holds row l&31 and the k half (l>>5) -- the MFMA's two k
// slots walk k = h*K/2 + j, j = 0 .. K/2-1, so each lane's X operands are
// K/2 consecutive floats (float4 loads).  The fused epilogue has the
// gemm_common.h semantics (bias, elu, EluGrad multiply, bias-gradient column
// sums).  Two independent layers writing different column ranges of one
// output (the critic's [state | action] concat) share one launch (blockIdx.z
// selects the part).
#pragma once
#include "common.h"

// Phase timestamp hook for tools/thin_k_bench.hip; empty in the product build.
#ifndef TK_STAMP
#define TK_STAMP(i)
#endif

namespace ddpg {

constexpr int TK_MAXK = 64;
constexpr int TK_ROWS = 64, TK_COLS = 128, TK_NT = 256;
constexpr int TK_KALIGN = 8;

struct TkPart {
  const float* X;   // [M][ldx], 16-byte aligned, ldx % 4 == 0
  int ldx, K;       // K % 8 == 0
  const float* W;   // w_nk ? W[n][k] (ldw) : W[k][n] (ldw); 16-byte aligned, ldw % 4 == 0
  int ldw, w_nk;
  int N;              // N % 4 == 0
  const float* bias;  // [N] or null
  int act;            // 1: elu
  const float* aux;   // v *= EluGrad factor of aux[m][n] (ldaux), or null
  int ldaux;
  float* out;         // out[m * ldo + n]
  int ldo;
  __bf16* outh;       // bf16 twin of out (same offsets; hnp planes, hps apart), or null
  long long hps;
  int hnp;
  float* colsum;      // [row block][ld_colsum] partial column sums of v, or null
  int ld_colsum;
};

struct TkArgs {
  TkPart p[2];
  int M;
};

typedef float tk_f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) tk_f32x2 tk_lds_v2;


constexpr int TK_VLD = TK_COLS + 4;  // LDS row stride of the output tile (floats)
constexpr int TK_SMEM =
    TK_MAXK * TK_COLS > TK_ROWS * TK_VLD ? TK_MAXK * TK_COLS : TK_ROWS * TK_VLD;

__global__ __launch_bounds__(TK_NT) void thin_k_kernel(TkArgs args) {
  // W panel as [k][wave column half][col 0..31][tile 0..1]: one ds_read_b64
  // per MFMA step gives a lane both of its B operands; after the MFMAs the
  // same LDS holds the raw output tile [64 rows][TK_VLD]
  __shared__ __attribute__((aligned(16))) float Ws[TK_SMEM];
  __shared__ float red[8 * TK_COLS];
  __shared__ __attribute__((aligned(16))) float Xs[TK_ROWS * (TK_MAXK + 4)];
  const TkPart P = blockIdx.z ? args.p[1] : args.p[0];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int li = lane & 31, h = lane >> 5;
  const int wr = wave & 1, wc = wave >> 1;  // 32-row half, 64-column half
  const int m0 = blockIdx.y * TK_ROWS, n0 = blockIdx.x * TK_COLS;
  if (n0 >= P.N) return;
  TK_STAMP(0);
  const int K = P.K, M = args.M, K4 = K >> 2, KH = K >> 1, K8 = K >> 3;
  // ---- global loads: W panel (<= 8 float4 per thread) and this lane's X row
  f32x4 wv[8], xv[8];
  if (!P.w_nk) {  // W[k][n]: float4 of 4 columns, rows k = (tid >> 5) + 8 j
    const int c4 = tid & 31, kr = tid >> 5, n = n0 + 4 * c4;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kr + 8 * j;
      wv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < K && n < P.N) wv[j] = *reinterpret_cast<const f32x4*>(P.W + (size_t)k * P.ldw + n);
    }
  } else {  // W[n][k]: 4 k per load, column c = tid & 127, k quads (tid >> 7) + 2 j
    // (rows of an unaligned stride, e.g. W3 [H2][A = 17], load as scalars)
    const int c = tid & 127, kq = tid >> 7, n = n0 + c;
    const bool wvec = ((P.ldw & 3) == 0) && (((uintptr_t)P.W & 15) == 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k4 = kq + 2 * j;
      wv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k4 < K4 && n < P.N) {
        const float* q = P.W + (size_t)n * P.ldw + 4 * k4;
        wv[j] = wvec ? *reinterpret_cast<const f32x4*>(q) : f32x4{q[0], q[1], q[2], q[3]};
      }
    }
  }
  // X tile [64 rows][K] -> LDS with coalesced float4 loads (a lane's own row
  // would otherwise be 8 loads touching 64 different rows per instruction)
  const int XLD = K + 4;  // padded row stride: conflict-free ds_read_b128 below
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int f = tid + TK_NT * j, r = f / K4, k4 = f - r * K4, m = m0 + r;
    if (r < TK_ROWS) {
      f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < M) x = *reinterpret_cast<const f32x4*>(P.X + (size_t)m * P.ldx + 4 * k4);
      *reinterpret_cast<f32x4*>(Xs + r * XLD + 4 * k4) = x;
    }
  }
  // ---- W panel -> LDS: column nl -> (half nl >> 6, tile (nl >> 5) & 1, col nl & 31)
  auto ws_at = [](int k, int nl) { return ((k * 2 + (nl >> 6)) * 32 + (nl & 31)) * 2 + ((nl >> 5) & 1); };
  if (!P.w_nk) {
    const int c4 = tid & 31, kr = tid >> 5;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kr + 8 * j;
      if (k < K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) Ws[ws_at(k, 4 * c4 + e)] = wv[j][e];
      }
    }
  } else {
    const int c = tid & 127, kq = tid >> 7;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k4 = kq + 2 * j;
      if (k4 < K4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) Ws[ws_at(4 * k4 + e, c)] = wv[j][e];
      }
    }
  }
  __syncthreads();
  {
    const float* xr = Xs + (32 * wr + li) * XLD + h * KH;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < K8) xv[q] = *reinterpret_cast<const f32x4*>(xr + 4 * q);
    }
  }
  TK_STAMP(1);
  // ---- MFMA: step j contracts k = j (lanes 0-31) and k = KH + j (lanes 32-63)
  f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const tk_lds_v2* Wb = reinterpret_cast<const tk_lds_v2*>(LDS(Ws)) + (h * KH * 2 + wc) * 32 + li;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    if (q < K8) {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const tk_f32x2 b = Wb[(4 * q + jj) * 64];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[q][jj], b[0], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv[q][jj], b[1], acc[1], 0, 0, 0);
      }
    }
  }
  TK_STAMP(2);
  // ---- epilogue.  The raw tile goes through LDS (lane li of tile t holds
  // column li, register r row (r & 3) + 8 (r >> 2) + 4 h) so that every
  // element-wise op, the aux loads and the output stores run on float4 rows:
  // one 16-B access per lane instead of 32 scalar 4-B stores per lane.
  __syncthreads();  // all waves done reading the W panel
  {
    const int rb = 32 * wr + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        Ws[(rb + (r & 3) + 8 * (r >> 2)) * TK_VLD + 64 * wc + 32 * t + li] = acc[t][r];
  }
  __syncthreads();
  TK_STAMP(3);
  // thread -> column quad c4 = tid & 31, rows rg, rg + 8, ... (rg = tid >> 5)
  const int c4 = tid & 31, rg = tid >> 5, n = n0 + 4 * c4;
  const bool nok = n < P.N;  // N % 4 == 0: a quad is all in or all out
  f32x4 bq = f32x4{0.f, 0.f, 0.f, 0.f};
  if (P.bias && nok) bq = *reinterpret_cast<const f32x4*>(P.bias + n);
  f32x4 csum = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int RPT = TK_ROWS / 8;  // rows per thread
  f32x4 aq[RPT];
  if (P.aux) {  // all aux loads in flight before the first use
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int m = m0 + rg + 8 * i;
      aq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (nok && m < M) aq[i] = *reinterpret_cast<const f32x4*>(P.aux + (size_t)m * P.ldaux + n);
    }
  }
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int rl = rg + 8 * i, m = m0 + rl;
    if (!nok || m >= M) continue;
    f32x4 v = *reinterpret_cast<const f32x4*>(Ws + rl * TK_VLD + 4 * c4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e];
      if (P.bias) x = __fadd_rn(x, bq[e]);
      if (P.act == 1) x = elu_f(x);
      if (P.aux) x = __fmul_rn(x, elu_grad_factor(aq[i][e]));
      v[e] = x;
      csum[e] += x;
    }
    if (P.out) *reinterpret_cast<f32x4*>(P.out + (size_t)m * P.ldo + n) = v;
    if (P.outh) store_twin4(P.outh + (size_t)m * P.ldo + n, P.hps, P.hnp, make_float4(v[0], v[1], v[2], v[3]));
  }
  if (P.colsum) {
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rg * TK_COLS + 4 * c4 + e] = csum[e];
    __syncthreads();
    if (tid < TK_COLS && n0 + tid < P.N) {
      float s = 0.f;
#pragma unroll
      for (int g = 0; g < 8; ++g) s += red[g * TK_COLS + tid];
      P.colsum[(size_t)blockIdx.y * P.ld_colsum + n0 + tid] = s;
    }
  }
}

}  // namespace ddpg
