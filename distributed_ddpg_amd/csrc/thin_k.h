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
  float* colsum;      // [row block][ld_colsum] partial column sums of v, or null
  int ld_colsum;
};

struct TkArgs {
  TkPart p[2];
  int M;
};

typedef float tk_f32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) tk_f32x2 tk_lds_v2;

__global__ __launch_bounds__(TK_NT) void thin_k_kernel(TkArgs args) {
  // W panel as [k][wave column half][col 0..31][tile 0..1]: one ds_read_b64
  // per MFMA step gives a lane both of its B operands
  __shared__ __attribute__((aligned(16))) float Ws[TK_MAXK * TK_COLS];
  __shared__ float red[2 * TK_COLS];
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
  } else {  // W[n][k]: float4 of 4 k, column c = tid & 127, k quads (tid >> 7) + 2 j
    const int c = tid & 127, kq = tid >> 7, n = n0 + c;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k4 = kq + 2 * j;
      wv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k4 < K4 && n < P.N)
        wv[j] = *reinterpret_cast<const f32x4*>(P.W + (size_t)n * P.ldw + 4 * k4);
    }
  }
  {
    const int m = m0 + 32 * wr + li;
    const float* xr = P.X + (size_t)m * P.ldx + h * KH;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      xv[q] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (q < K8 && m < M) xv[q] = *reinterpret_cast<const f32x4*>(xr + 4 * q);
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
  // ---- epilogue: lane holds column li of tile t, register r holds row
  // (r & 3) + 8 (r >> 2) + 4 h
  const int mb = m0 + 32 * wr + 4 * h;
  float cs[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + 64 * wc + 32 * t + li;
    const bool nok = n < P.N;
    const float bn = (nok && P.bias) ? P.bias[n] : 0.f;
    float av[16];
    if (P.aux) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + (r & 3) + 8 * (r >> 2);
        av[r] = (nok && m < M) ? P.aux[(size_t)m * P.ldaux + n] : 0.f;
      }
    }
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = mb + (r & 3) + 8 * (r >> 2);
      float v = acc[t][r];
      if (nok && m < M) {
        if (P.bias) v = __fadd_rn(v, bn);
        if (P.act == 1) v = elu_f(v);
        if (P.aux) v = __fmul_rn(v, elu_grad_factor(av[r]));
        if (P.out) P.out[(size_t)m * P.ldo + n] = v;
        sum += v;
      }
    }
    cs[t] = sum;
  }
  TK_STAMP(3);
  if (P.colsum) {
#pragma unroll
    for (int t = 0; t < 2; ++t) cs[t] += __shfl_xor(cs[t], 32);
    if (h == 0) {
      red[wr * TK_COLS + 64 * wc + li] = cs[0];
      red[wr * TK_COLS + 64 * wc + 32 + li] = cs[1];
    }
    __syncthreads();
    if (tid < TK_COLS && n0 + tid < P.N)
      P.colsum[(size_t)blockIdx.y * P.ld_colsum + n0 + tid] = red[tid] + red[TK_COLS + tid];
  }
}

}  // namespace ddpg
