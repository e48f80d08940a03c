// Skinny weight gradients of the large-batch path: dW = X^T . G over the batch
// (K = B rows) where one side is at most 64 wide -- the input layers' dW1 /
// dWs / dWa (networks.py:44,137 with X = s or a, 64 / 16 columns at C3) and the
// output layer's dW3 (G = dz3, A columns).  A tiled GEMM spends these launches
// in prologue and epilogue (a 64 x 1024 x 4096 product is 0.5 GFLOP); here
// they are fp32 VALU dot products read straight from the fp32 activations,
// no LDS staging and no bf16 planes.
//
// Each wave owns NG narrow columns n0 .. n0 + NG - 1 and 256 wide columns (4
// per lane).  Per batch row the NG narrow values are wave-uniform: one scalar
// load into SGPRs (the vector memory path carries only the wide side, one
// dwordx4 per lane), and the lane does NG x 4 FMAs on packed fp32 (v_pk_fma
// with the SGPR broadcast).  The first version read the narrow side per lane
// and behind per-load branches; the texture data return, not the FMAs, bound
// it (12 floats per 32 FMAs, 43 us for dW1 at C3).
//
// Block = 8 waves on the same (wide, narrow) tile, rows interleaved across the
// waves (row b0 + wave + 8 r); the wide loads run R rows ahead in two register
// sets (loads past the split's end are clamped to its last row and unused).
// The 8 partial tiles meet in LDS and each wave sums its share of the tile
// over the waves in a fixed order (0 .. 7), so the result does not depend on
// timing.  The tile goes to slab `split` of the split-K reduction
// (reduce_slabs_kernel) or, with one split, straight to the gradient.  Columns
// past the narrow width are computed from whatever the row holds there
// (the host guarantees n0 + NG <= ldn) and never stored.
#pragma once
#include "common.h"

namespace ddpg {

#ifndef SK_R_CFG
#define SK_R_CFG 6  // rows per register set (two sets in flight per wave; 4 -> 6: +0.4 % C3)
#endif
constexpr int SK_NT = 512, SK_WAVES = 8, SK_WT = 256, SK_NMAX = 64, SK_R = SK_R_CFG;

struct SkArgs {
  const float* N;  // narrow operand [B][ldn]: columns 0 .. nn-1 used
  int ldn, nn;
  const float* W;  // wide operand [B][ldw]: columns 0 .. nw-1 used (nw % 4 == 0)
  int ldw, nw;
  int B, kc;        // batch rows, rows per split
  int ntw, ntn;     // wide / narrow tiles
  int narrow_rows;  // 1: out[narrow][wide] (X is the narrow side), 0: out[wide][narrow]
  float* out;       // slab z at out + z * split_stride; ld = the out column count
  long long split_stride;
};

typedef const __attribute__((address_space(4))) float* sk_const_f;

static_assert(SK_WAVES == 8, "the reduction splits NG = 8 / 16 rows over 8 waves");

// NL (round 4): the split's narrow rows [b0, b1) x NG are first copied into
// the reduction's LDS region (coalesced float4 loads by the whole block), and
// each row's NG values are read from there as broadcast ds_read_b128s, R rows
// ahead.  The per-row scalar loads of the original form (NL = false) were
// issued one or two rows ahead at most (the SGPR budget), so every row or two
// waited a scalar-load round trip.  Same FMAs in the same order: bitwise equal.
// The host takes NL when (b1 - b0) * NG floats fit the reduction region.
template <int NG, int R = SK_R, bool NL = false>
__global__ __launch_bounds__(SK_NT) void skinny_wgrad_kernel(SkArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sk_red[];  // [8][NG * 4][64]
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // XCD-aware block order: consecutive tiles of one split on one XCD (its L2
  // then holds the split's rows for every tile that reads them)
  const int T = gridDim.x, L = blockIdx.x;
  const int idx = (T & 7) ? L : (L & 7) * (T >> 3) + (L >> 3);
  const int tiles = a.ntw * a.ntn;
  const int split = idx / tiles, tile = idx - split * tiles;
  const int tn = tile / a.ntw, tw = tile - tn * a.ntw;
  const int n0 = tn * NG;
  const int j0 = tw * SK_WT + 4 * lane;
  const bool wok = j0 < a.nw;
  const int jc = wok ? j0 : 0;  // in-bounds column for the idle lanes' loads
  const int b0 = split * a.kc, b1 = min(a.B, b0 + a.kc);
  if (b0 >= b1) return;  // (host sizes the grid so this never happens)
  const int nr = (b1 - b0 - wv + SK_WAVES - 1) / SK_WAVES;  // this wave's rows
  float acc[NG][4];
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;

  auto wrow = [&](int r) {  // batch row of this wave's r-th row, clamped
    return min(b0 + wv + SK_WAVES * r, b1 - 1);
  };
  auto wload = [&](f32x4 (&w)[R], int r) {
#pragma unroll
    for (int u = 0; u < R; ++u)
      w[u] = *reinterpret_cast<const f32x4*>(a.W + (size_t)wrow(r + u) * a.ldw + jc);
  };
  if constexpr (NL) {
    // the split's narrow rows -> LDS [b - b0][NG] (the reduction region is
    // free until the partial tiles are written)
    constexpr int Q = NG / 4;  // float4 per row
    f32x4* nl4 = reinterpret_cast<f32x4*>(sk_red);
    for (int f = threadIdx.x; f < (b1 - b0) * Q; f += SK_NT) {
      const int rr = f / Q, q = f - rr * Q;
      nl4[f] = *reinterpret_cast<const f32x4*>(a.N + (size_t)(b0 + rr) * a.ldn + n0 + 4 * q);
    }
    __syncthreads();
  }
  auto row = [&](const f32x4& w, int b) {
    if constexpr (NL) {
      const f32x4* np = reinterpret_cast<const f32x4*>(sk_red) + (size_t)(b - b0) * (NG / 4);
#pragma unroll
      for (int q = 0; q < NG / 4; ++q) {
        const f32x4 nq = np[q];  // same address in every lane: broadcast
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[4 * q + e][j] = fmaf(nq[e], w[j], acc[4 * q + e][j]);
      }
    } else {
      sk_const_f np = (sk_const_f)(a.N + (size_t)b * a.ldn + n0);
#pragma unroll
      for (int i = 0; i < NG; ++i) {
        const float nv = np[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(nv, w[j], acc[i][j]);
      }
    }
  };
  auto step = [&](const f32x4 (&w)[R], int r) {
#pragma unroll
    for (int u = 0; u < R; ++u) row(w[u], b0 + wv + SK_WAVES * (r + u));
  };
  auto step_tail = [&](const f32x4 (&w)[R], int r) {
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (r + u < nr) row(w[u], b0 + wv + SK_WAVES * (r + u));
  };
  f32x4 wA[R], wB[R];
  wload(wA, 0);
  int r = 0;
  for (; r + 2 * R <= nr; r += 2 * R) {
    wload(wB, r + R);
    step(wA, r);
    wload(wA, r + 2 * R);
    step(wB, r + R);
  }
  if (r < nr) {
    wload(wB, r + R);
    step_tail(wA, r);
    step_tail(wB, r + R);
  }
  // partial tiles -> LDS; wave wv sums narrow rows wv * IPW .. of the tile
  // over the waves 0 .. 7 in order
  constexpr int E = NG * 4, IPW = NG / SK_WAVES;
  if constexpr (NL) __syncthreads();  // every wave done with the narrow rows
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) sk_red[((wv * E) + i * 4 + j) * 64 + lane] = acc[i][j];
  __syncthreads();
  if (!wok) return;
  float* o = a.out + (size_t)split * a.split_stride;
#pragma unroll
  for (int ii = 0; ii < IPW; ++ii) {
    const int i = wv * IPW + ii, ni = n0 + i;
    if (ni >= a.nn) break;
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = sk_red[(i * 4 + j) * 64 + lane];
#pragma unroll
      for (int q = 1; q < SK_WAVES; ++q) s = __fadd_rn(s, sk_red[((q * E) + i * 4 + j) * 64 + lane]);
      v[j] = s;
    }
    if (a.narrow_rows) {  // out[ni][j0 .. j0 + 3], ld = nw
      *reinterpret_cast<f32x4*>(o + (size_t)ni * a.nw + j0) = f32x4{v[0], v[1], v[2], v[3]};
    } else {  // out[j0 + j][ni], ld = nn
#pragma unroll
      for (int j = 0; j < 4; ++j) o[(size_t)(j0 + j) * a.nn + ni] = v[j];
    }
  }
}

// LDS bytes of the cross-wave reduction
constexpr int sk_lds_bytes(int ng) { return SK_WAVES * ng * 4 * 64 * 4; }
// rows of narrow operand the NL form stages (in the same region)
constexpr int sk_nl_rows(int ng) { return sk_lds_bytes(ng) / (ng * 4); }

}  // namespace ddpg
