// Small-batch learner step (the latency-bound B <= ~1k path, SURVEY.md §8 C2:
// InvertedPendulum 4/1/128/200, B = 64).
//
// At these sizes every GEMM of the large-batch path is a few-microsecond,
// few-block launch whose k-loop waits on dependent loads; the step is a
// chain of ~35 such launches.  Here the step is four launches:
//
//   sb_phase1  (row-parallel, one workgroup per R batch rows): target actor
//              fwd -> target critic fwd -> TD target -> online critic fwd ->
//              MSE loss/dQ -> critic head + dX backward -> this workgroup's
//              partial critic gradients (flat layout, one slab per WG).
//              WG 0 also computes the critic Adam step size from the beta
//              powers and advances them (TF AdamOptimizer._finish).
//   sb_reduce_adam(critic): g = sum of slabs -> TF ApplyAdam -> soft update.
//   sb_phase3  (row-parallel): online actor fwd -> updated-critic fwd at
//              (s, mu) -> dQ/da -> actor backward -> partial actor gradients;
//              WG 0 computes the actor step size and advances its powers.
//   sb_reduce_adam(actor).
//
// Every workgroup keeps its R rows of every activation in LDS and streams
// the weights from L2 (the whole parameter set is ~0.3 MB at C2); a dense
// layer is one thread per output column with R accumulators.  Rows beyond B
// are computed on zero inputs and masked out of every gradient and stat.
// The arithmetic is the same TF-semantics fp32 as the large-batch path
// (elu/EluGrad from outputs, TanhGrad, MSE grad, ApplyAdam, soft update);
// only the summation order differs.
#pragma once
#include "common.h"

namespace ddpg {

constexpr int SB_R = 4;      // batch rows per workgroup

// The phase kernels run each layer helper once per call site per workgroup:
// inlined, every call site is a fresh ~5 KB of straight-line code fetched
// cold into the instruction cache.  Out-of-line, one copy serves every call.
#define SB_FN __device__ __attribute__((noinline))

// Diagnostic stamps (env DDPG_SB_STAMPS=1): WG 0 records s_memtime after each
// section; nothing reads them on device and no output depends on them.
#define SB_STAMP(i)                                                           \
  do {                                                                        \
    if (g.stamps && blockIdx.x == 0) {                                        \
      __syncthreads();                                                        \
      if (threadIdx.x == 0) g.stamps[i] = __builtin_amdgcn_s_memtime();       \
    }                                                                         \
  } while (0)
constexpr int SB_NT = 256;   // threads per workgroup

// Per-step arguments (all device pointers; offsets into the flat layout).
struct SbArgs {
  int B;                 // local rows
  int S, A, AH1, AH2, CH1, CH2;
  int ldS, ldA;          // batch buffer strides
  // LDS row strides (floats, multiples of 4)
  int LA, LB, LC, LD, LX;
  float inv_b, gamma, scale, tau, omt, b1, b2, lr_a, lr_c, eps;
  const float *s, *s2, *a, *r, *t;  // gathered batch (device, [B][ld])
  float* theta;
  float* target;
  float* adam_m;
  float* adam_v;
  float* part;           // [G][PT] partial gradient slabs (flat param layout)
  long long PT;          // floats per slab (= layout total)
  float* pw;             // beta powers [actor b1p, b2p, critic b1p, b2p]
  float* alpha;          // [actor, critic] Adam step sizes for this step
  float* stat_part;      // [G][2] loss partial, q max
  float* stats;          // [q_max, loss]
  double* acc;           // [qmax_sum, loss_sum, steps]
  unsigned long long* stamps;  // diagnostic build only: per-section s_memtime (WG 0)
  // tensor offsets
  long long aW1, ab1, aW2, ab2, aW3;
  long long cWs, cbs, cWa, cba, cWh, cbh, cWo, cbo;
  long long actor_begin, actor_end, critic_begin, critic_end;
};

// Y[r][n] = act(sum_k X[r][k] W[k*ldw + n] + b[n]), r < SB_R, n < N.
// X, Y in LDS; W, b global.  act: 0 none, 1 elu, 2 tanh (o), 3 post2 (pw[n]*elu'(elu(.))).
// The weights are cold in this XCD's L2 every phase (another XCD's kernel
// just updated them), so each dependent global round trip costs ~2k cycles:
// a thread issues SB_KC weight loads (clamped addresses, never predicated)
// before consuming any, so a layer costs ceil(K / SB_KC) round trips.
// X rows must be zero beyond K up to the next multiple of 4.
constexpr int SB_KC = 64;

DDPG_DEV void sb_fma_chunk(float (&acc)[SB_R], const lds_f* X, int ldx, int k0, int kn,
                           const float (&w)[SB_KC]) {
#pragma unroll
  for (int q = 0; q < SB_KC / 4; ++q) {
    if (4 * q < kn) {  // uniform; a partial last group meets zero-padded X
#pragma unroll
      for (int r = 0; r < SB_R; ++r) {
        const float x0 = X[r * ldx + k0 + 4 * q], x1 = X[r * ldx + k0 + 4 * q + 1];
        const float x2 = X[r * ldx + k0 + 4 * q + 2], x3 = X[r * ldx + k0 + 4 * q + 3];
        const float4 x = make_float4(x0, x1, x2, x3);
        acc[r] = fmaf(x.x, w[4 * q], acc[r]);
        acc[r] = fmaf(x.y, w[4 * q + 1], acc[r]);
        acc[r] = fmaf(x.z, w[4 * q + 2], acc[r]);
        acc[r] = fmaf(x.w, w[4 * q + 3], acc[r]);
      }
    }
  }
}

SB_FN void sb_dense(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw,
                    const glb_f* __restrict__ b, int N, lds_f* Y, int ldy, int act,
                    const glb_f* __restrict__ pw = nullptr) {
  for (int n = threadIdx.x; n < N; n += SB_NT) {
    const float bn = b ? b[n] : 0.f;
    const float pwn = act == 3 ? pw[n] : 0.f;
    float acc[SB_R];
#pragma unroll
    for (int r = 0; r < SB_R; ++r) acc[r] = 0.f;
    for (int k0 = 0; k0 < K; k0 += SB_KC) {
      float w[SB_KC];
#pragma unroll
      for (int u = 0; u < SB_KC; ++u) w[u] = W[(size_t)min(k0 + u, K - 1) * ldw + n];
      // weights past K are never multiplied by a non-zero x: the padded
      // group reads x = 0 and groups past K are skipped
#pragma unroll
      for (int u = 0; u < SB_KC; ++u) w[u] = (k0 + u < K) ? w[u] : 0.f;
      sb_fma_chunk(acc, X, ldx, k0, min(SB_KC, K - k0), w);
    }
#pragma unroll
    for (int r = 0; r < SB_R; ++r) {
      float v = b ? __fadd_rn(acc[r], bn) : acc[r];
      if (act == 1) v = elu_f(v);
      else if (act == 2) v = tanhf(v);
      else if (act == 3) v = __fmul_rn(pwn, elu_grad_factor(elu_f(v)));
      Y[r * ldy + n] = v;
    }
  }
}

// Y[r][n] = (sum_k X[r][k] W[n*ldw + k]) * (aux ? elu'(aux[r][n]) : 1)   (X . W^T)
SB_FN void sb_dense_t(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw,
                      int N, lds_f* Y, int ldy, const lds_f* aux, int ldaux) {
  for (int n = threadIdx.x; n < N; n += SB_NT) {
    float acc[SB_R];
#pragma unroll
    for (int r = 0; r < SB_R; ++r) acc[r] = 0.f;
    const glb_f* wr = W + (size_t)n * ldw;
    for (int k0 = 0; k0 < K; k0 += SB_KC) {
      float w[SB_KC];
#pragma unroll
      for (int u = 0; u < SB_KC; ++u) w[u] = wr[min(k0 + u, K - 1)];
#pragma unroll
      for (int u = 0; u < SB_KC; ++u) w[u] = (k0 + u < K) ? w[u] : 0.f;
      sb_fma_chunk(acc, X, ldx, k0, min(SB_KC, K - k0), w);
    }
#pragma unroll
    for (int r = 0; r < SB_R; ++r) {
      float v = acc[r];
      if (aux) v = __fmul_rn(v, elu_grad_factor(aux[r * ldaux + n]));
      Y[r * ldy + n] = v;
    }
  }
}

// out[i*N + j] = sum_r X[r][i] dY[r][j]   (i < Kin, j < N), rows masked by the
// caller (masked rows of dY are zero).  bias (optional): db[j] = sum_r dY[r][j].
// Parallel over (4-row block of i, j) pairs: 16 FMAs per 8 LDS reads, no
// serial dependence between outputs.
SB_FN void sb_wgrad(const lds_f* X, int ldx, int Kin, const lds_f* dY, int ldy, int N,
                    glb_f* __restrict__ out, glb_f* __restrict__ db) {
  const int KQ = (Kin + 3) >> 2;
  for (int p = threadIdx.x; p < KQ * N; p += SB_NT) {
    const int iq = p / N, j = p - iq * N, i0 = 4 * iq;
    float d[SB_R];
#pragma unroll
    for (int r = 0; r < SB_R; ++r) d[r] = dY[r * ldy + j];
    float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < SB_R; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[q] = fmaf(X[r * ldx + i0 + q], d[r], s[q]);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i0 + q < Kin) out[(size_t)(i0 + q) * N + j] = s[q];
  }
  if (db)
    for (int jj = threadIdx.x; jj < N; jj += SB_NT) {
      float s = 0.f;
#pragma unroll
      for (int r = 0; r < SB_R; ++r) s += dY[r * ldy + jj];
      db[jj] = s;
    }
}

// Thin layers (N <= SB_NMAX outputs, e.g. W3 / Wo / Wa^T): k-parallel over the
// whole workgroup, then a block reduction.  trans: W is [N][K] (X . W^T).
// Y[r][n] = act(sum_k X[r][k] W(k, n) + b[n]); act 0 none, 2 tanh.
// red: >= SB_NT * SB_R * SB_NMAX / 64 floats of LDS scratch.
constexpr int SB_NMAX = 8;
SB_FN void sb_dense_thin(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw,
                         bool trans, const glb_f* __restrict__ b, int N, lds_f* Y, int ldy,
                         int act, lds_f* red) {
  float acc[SB_R][SB_NMAX];
#pragma unroll
  for (int r = 0; r < SB_R; ++r)
#pragma unroll
    for (int n = 0; n < SB_NMAX; ++n) acc[r][n] = 0.f;
  for (int k = threadIdx.x; k < K; k += SB_NT) {
    float xv[SB_R];
#pragma unroll
    for (int r = 0; r < SB_R; ++r) xv[r] = X[r * ldx + k];
#pragma unroll
    for (int n = 0; n < SB_NMAX; ++n) {
      if (n < N) {
        const float w = trans ? W[(size_t)n * ldw + k] : W[(size_t)k * ldw + n];
#pragma unroll
        for (int r = 0; r < SB_R; ++r) acc[r][n] = fmaf(xv[r], w, acc[r][n]);
      }
    }
  }
  // wave reduction, then across the 4 waves through LDS
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < SB_R; ++r)
#pragma unroll
    for (int n = 0; n < SB_NMAX; ++n) {
      float v = acc[r][n];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0 && n < N) red[(wave * SB_R + r) * SB_NMAX + n] = v;
    }
  __syncthreads();
  if (threadIdx.x < SB_R * N) {
    const int r = threadIdx.x / N, n = threadIdx.x - r * N;
    float v = 0.f;
    for (int w = 0; w < SB_NT / 64; ++w) v += red[(w * SB_R + r) * SB_NMAX + n];
    if (b) v = __fadd_rn(v, b[n]);
    if (act == 2) v = tanhf(v);
    Y[r * ldy + n] = v;
  }
}

// Thin layer dispatch: k-parallel reduction when N <= SB_NMAX, else the
// column-parallel kernels.
DDPG_DEV void sb_thin(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw,
                      bool trans, const glb_f* __restrict__ b, int N, lds_f* Y, int ldy, int act,
                      lds_f* red) {
  if (N <= SB_NMAX) {
    sb_dense_thin(X, ldx, K, W, ldw, trans, b, N, Y, ldy, act, red);
  } else if (trans) {
    sb_dense_t(X, ldx, K, W, ldw, N, Y, ldy, nullptr, 0);
  } else {
    sb_dense(X, ldx, K, W, ldw, b, N, Y, ldy, act);
  }
}

// TF ApplyAdam step size from the beta powers, then _finish's power update.
DDPG_DEV void sb_alpha_and_advance(float* pw, float* alpha, float lr, float b1, float b2) {
  const float b1p = pw[0], b2p = pw[1];
  *alpha = __fdiv_rn(__fmul_rn(lr, __fsqrt_rn(__fsub_rn(1.f, b2p))), __fsub_rn(1.f, b1p));
  pw[0] = __fmul_rn(b1p, b1);
  pw[1] = __fmul_rn(b2p, b2);
}

DDPG_DEV void sb_load_rows(lds_f* dst, int ldd, const float* src, int lds, int cols, int r0,
                           int valid) {
  for (int idx = threadIdx.x; idx < SB_R * ldd; idx += SB_NT) {
    const int r = idx / ldd, k = idx - r * ldd;
    dst[idx] = (r < valid && k < cols) ? src[(size_t)(r0 + r) * lds + k] : 0.f;
  }
}

__global__ __launch_bounds__(SB_NT) void sb_phase1_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * SB_R;
  const int valid = min(SB_R, g.B - r0);
  lds_f* xs = LDS(sm);
  lds_f* xs2 = xs + SB_R * g.LX;
  lds_f* xa = xs2 + SB_R * g.LX;
  lds_f* ta2 = xa + SB_R * g.LX;
  lds_f* bufA = ta2 + SB_R * g.LX;
  lds_f* bufB = bufA + SB_R * g.LA;
  lds_f* bufC = bufB + SB_R * g.LB;
  lds_f* bufD = bufC + SB_R * g.LC;
  lds_f* col = bufD + SB_R * g.LD;  // [SB_R][8]: q', y, q, dq
  lds_f* red = col + SB_R * 8;      // thin-layer reduction scratch
  const glb_f* T = GLB(g.target);
  const glb_f* P = GLB(g.theta);
  glb_f* part = GLB(g.part) + (size_t)blockIdx.x * g.PT;

  if (g.stamps && blockIdx.x == 0 && tid == 0) g.stamps[15] = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && tid == 0) sb_alpha_and_advance(g.pw + 2, g.alpha + 1, g.lr_c, g.b1, g.b2);
  sb_load_rows(xs, g.LX, g.s, g.ldS, g.S, r0, valid);
  sb_load_rows(xs2, g.LX, g.s2, g.ldS, g.S, r0, valid);
  sb_load_rows(xa, g.LX, g.a, g.ldA, g.A, r0, valid);
  // ta2 is written only in its first A columns; the padding up to LX feeds
  // the next layer's zero-padded k group and must be 0, not stale LDS
  for (int idx = tid; idx < SB_R * g.LX; idx += SB_NT) ta2[idx] = 0.f;
  __syncthreads();
  SB_STAMP(0);
  // ---- target actor: ta2 = scale * tanh(elu(elu(s2 W1 + b1) W2 + b2) W3)
  sb_dense(xs2, g.LX, g.S, T + g.aW1, g.AH1, T + g.ab1, g.AH1, bufA, g.LA, 1);
  __syncthreads();
  sb_dense(bufA, g.LA, g.AH1, T + g.aW2, g.AH2, T + g.ab2, g.AH2, bufB, g.LB, 1);
  __syncthreads();
  sb_thin(bufB, g.LB, g.AH2, T + g.aW3, g.A, false, nullptr, g.A, ta2, g.LX, 2, red);
  __syncthreads();
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    ta2[r * g.LX + a] = __fmul_rn(ta2[r * g.LX + a], g.scale);
  }
  __syncthreads();
  SB_STAMP(1);
  // ---- target critic: q' and y = t ? r : r + gamma q'
  sb_dense(xs2, g.LX, g.S, T + g.cWs, g.CH1, T + g.cbs, g.CH1, bufC, g.LC, 1);
  sb_dense(ta2, g.LX, g.A, T + g.cWa, g.CH1, T + g.cba, g.CH1, bufC + g.CH1, g.LC, 1);
  __syncthreads();
  sb_dense(bufC, g.LC, 2 * g.CH1, T + g.cWh, g.CH2, T + g.cbh, g.CH2, bufD, g.LD, 1);
  __syncthreads();
  sb_thin(bufD, g.LD, g.CH2, T + g.cWo, 1, false, T + g.cbo, 1, col + 0, 8, 0, red);
  __syncthreads();
  if (tid < SB_R) {
    const float rr = tid < valid ? g.r[r0 + tid] : 0.f;
    const float tt = tid < valid ? g.t[r0 + tid] : 0.f;
    col[tid * 8 + 1] = tt != 0.f ? rr : __fadd_rn(rr, __fmul_rn(g.gamma, col[tid * 8 + 0]));
  }
  SB_STAMP(2);
  // ---- online critic forward (networks.py:147-162)
  sb_dense(xs, g.LX, g.S, P + g.cWs, g.CH1, P + g.cbs, g.CH1, bufC, g.LC, 1);
  sb_dense(xa, g.LX, g.A, P + g.cWa, g.CH1, P + g.cba, g.CH1, bufC + g.CH1, g.LC, 1);
  __syncthreads();
  sb_dense(bufC, g.LC, 2 * g.CH1, P + g.cWh, g.CH2, P + g.cbh, g.CH2, bufD, g.LD, 1);
  __syncthreads();
  sb_thin(bufD, g.LD, g.CH2, P + g.cWo, 1, false, P + g.cbo, 1, col + 2, 8, 0, red);
  __syncthreads();
  SB_STAMP(3);
  // ---- MSE loss / dQ (networks.py:136): dq = -((1/B) * (2 * (y - q)))
  if (tid == 0) {
    float lsum = 0.f, qmax = -INFINITY;
    for (int r = 0; r < SB_R; ++r) {
      const float q = col[r * 8 + 2];
      const float d = __fsub_rn(col[r * 8 + 1], q);
      const bool ok = r < valid;
      col[r * 8 + 3] = ok ? -__fmul_rn(g.inv_b, __fmul_rn(2.f, d)) : 0.f;
      if (ok) {
        lsum += __fmul_rn(d, d);
        qmax = fmaxf(qmax, q);
      }
    }
    g.stat_part[blockIdx.x * 2 + 0] = lsum;
    g.stat_part[blockIdx.x * 2 + 1] = qmax;
  }
  __syncthreads();
  // ---- critic head backward: dhp = dq * Wo * elu'(h) -> bufB
  for (int idx = tid; idx < SB_R * g.CH2; idx += SB_NT) {
    const int r = idx / g.CH2, j = idx - r * g.CH2;
    bufB[r * g.LB + j] = __fmul_rn(__fmul_rn(col[r * 8 + 3], P[g.cWo + j]),
                                   elu_grad_factor(bufD[r * g.LD + j]));
  }
  __syncthreads();
  // dcat = dhp . Wh^T * elu'(cat) -> bufA
  sb_dense_t(bufB, g.LB, g.CH2, P + g.cWh, g.CH2, 2 * g.CH1, bufA, g.LA, bufC, g.LC);
  __syncthreads();
  SB_STAMP(4);
  // ---- partial critic gradients (this WG's rows)
  sb_wgrad(xs, g.LX, g.S, bufA, g.LA, g.CH1, part + g.cWs, part + g.cbs);
  sb_wgrad(xa, g.LX, g.A, bufA + g.CH1, g.LA, g.CH1, part + g.cWa, part + g.cba);
  sb_wgrad(bufC, g.LC, 2 * g.CH1, bufB, g.LB, g.CH2, part + g.cWh, part + g.cbh);
  for (int j = tid; j < g.CH2; j += SB_NT) {
    float s = 0.f;
    for (int r = 0; r < SB_R; ++r) s = fmaf(bufD[r * g.LD + j], col[r * 8 + 3], s);
    part[g.cWo + j] = s;
  }
  if (tid == 0) {
    float s = 0.f;
    for (int r = 0; r < SB_R; ++r) s += col[r * 8 + 3];
    part[g.cbo] = s;
  }
  SB_STAMP(5);
}

__global__ __launch_bounds__(SB_NT) void sb_phase3_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * SB_R;
  const int valid = min(SB_R, g.B - r0);
  lds_f* xs = LDS(sm);
  lds_f* o = xs + SB_R * g.LX;
  lds_f* mu = o + SB_R * g.LX;
  lds_f* dz3 = mu + SB_R * g.LX;
  lds_f* bufA = dz3 + SB_R * g.LX;
  lds_f* bufB = bufA + SB_R * g.LA;
  lds_f* bufC = bufB + SB_R * g.LB;
  lds_f* bufD = bufC + SB_R * g.LC;
  lds_f* red = bufD + SB_R * g.LD;  // thin-layer reduction scratch
  const glb_f* P = GLB(g.theta);
  glb_f* part = GLB(g.part) + (size_t)blockIdx.x * g.PT;

  if (g.stamps && blockIdx.x == 0 && tid == 0) g.stamps[14] = __builtin_amdgcn_s_memtime();
  if (blockIdx.x == 0 && tid == 0) sb_alpha_and_advance(g.pw, g.alpha, g.lr_a, g.b1, g.b2);
  sb_load_rows(xs, g.LX, g.s, g.ldS, g.S, r0, valid);
  // o / mu / dz3 are written only in their first A columns (see phase 1)
  for (int idx = tid; idx < 3 * SB_R * g.LX; idx += SB_NT) o[idx] = 0.f;
  __syncthreads();
  SB_STAMP(8);
  // ---- online actor forward (current actor params): h1 -> bufA, h2 -> bufB, o, mu
  sb_dense(xs, g.LX, g.S, P + g.aW1, g.AH1, P + g.ab1, g.AH1, bufA, g.LA, 1);
  __syncthreads();
  sb_dense(bufA, g.LA, g.AH1, P + g.aW2, g.AH2, P + g.ab2, g.AH2, bufB, g.LB, 1);
  __syncthreads();
  sb_thin(bufB, g.LB, g.AH2, P + g.aW3, g.A, false, nullptr, g.A, o, g.LX, 2, red);
  __syncthreads();
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    mu[r * g.LX + a] = __fmul_rn(o[r * g.LX + a], g.scale);
  }
  __syncthreads();
  SB_STAMP(9);
  // ---- updated critic at (s, mu): dhp2 = Wo * elu'(h')  (grad_ys = 1)
  sb_dense(xs, g.LX, g.S, P + g.cWs, g.CH1, P + g.cbs, g.CH1, bufC, g.LC, 1);
  sb_dense(mu, g.LX, g.A, P + g.cWa, g.CH1, P + g.cba, g.CH1, bufC + g.CH1, g.LC, 1);
  __syncthreads();
  sb_dense(bufC, g.LC, 2 * g.CH1, P + g.cWh, g.CH2, P + g.cbh, g.CH2, bufD, g.LD, 3, P + g.cWo);
  __syncthreads();
  SB_STAMP(10);
  // dca = dhp2 . Wh[CH1:]^T * elu'(ca), in place over ca (bufC[:, CH1:])
  sb_dense_t(bufD, g.LD, g.CH2, P + g.cWh + (size_t)g.CH1 * g.CH2, g.CH2, g.CH1, bufC + g.CH1,
             g.LC, bufC + g.CH1, g.LC);
  __syncthreads();
  // da = dca . Wa^T -> dz3 (scratch), then dz3 = ((-da) * scale) * (1 - o^2), masked
  sb_thin(bufC + g.CH1, g.LC, g.CH1, P + g.cWa, g.CH1, true, nullptr, g.A, dz3, g.LX, 0, red);
  __syncthreads();
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    const float ov = o[r * g.LX + a];
    const float dy = __fmul_rn(-dz3[r * g.LX + a], g.scale);
    dz3[r * g.LX + a] = r < valid ? __fmul_rn(dy, __fsub_rn(1.f, __fmul_rn(ov, ov))) : 0.f;
  }
  __syncthreads();
  SB_STAMP(11);
  // ---- actor backward (networks.py:44)
  // dz2 = dz3 . W3^T * elu'(h2) -> bufD
  sb_dense_t(dz3, g.LX, g.A, P + g.aW3, g.A, g.AH2, bufD, g.LD, bufB, g.LB);
  __syncthreads();
  sb_wgrad(bufB, g.LB, g.AH2, dz3, g.LX, g.A, part + g.aW3, nullptr);
  sb_wgrad(bufA, g.LA, g.AH1, bufD, g.LD, g.AH2, part + g.aW2, part + g.ab2);
  __syncthreads();
  SB_STAMP(12);
  // dz1 = dz2 . W2^T * elu'(h1), in place over h1 (bufA)
  sb_dense_t(bufD, g.LD, g.AH2, P + g.aW2, g.AH2, g.AH1, bufA, g.LA, bufA, g.LA);
  __syncthreads();
  sb_wgrad(xs, g.LX, g.S, bufA, g.LA, g.AH1, part + g.aW1, part + g.ab1);
  SB_STAMP(13);
}

// g = sum of the per-WG slabs; TF ApplyAdam with this step's alpha; soft
// update of the target.  net: 0 actor, 1 critic.  The critic call also
// finalises the step stats.
__global__ void sb_reduce_adam_kernel(SbArgs g, int net, int nslab) {
  const long long b = net == 0 ? g.actor_begin : g.critic_begin;
  const long long e = net == 0 ? g.actor_end : g.critic_end;
  const float alpha = g.alpha[net];
  const float omb1 = __fsub_rn(1.f, g.b1), omb2 = __fsub_rn(1.f, g.b2);
  for (long long i = b + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < e;
       i += (long long)gridDim.x * blockDim.x) {
    float gv = 0.f;
    for (int w = 0; w < nslab; ++w) gv += g.part[(size_t)w * g.PT + i];
    float m = g.adam_m[i], v = g.adam_v[i], p = g.theta[i];
    m = __fadd_rn(m, __fmul_rn(__fsub_rn(gv, m), omb1));
    v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(gv, gv), v), omb2));
    p = __fsub_rn(p, __fdiv_rn(__fmul_rn(m, alpha), __fadd_rn(__fsqrt_rn(v), g.eps)));
    g.adam_m[i] = m;
    g.adam_v[i] = v;
    g.theta[i] = p;
    g.target[i] = __fadd_rn(__fmul_rn(p, g.tau), __fmul_rn(g.target[i], g.omt));
  }
  if (net == 1 && blockIdx.x == 0 && threadIdx.x == 0) {
    float ls = 0.f, qm = -INFINITY;
    for (int w = 0; w < nslab; ++w) {
      ls += g.stat_part[2 * w];
      qm = fmaxf(qm, g.stat_part[2 * w + 1]);
    }
    const float loss = __fmul_rn(ls, g.inv_b);
    g.stats[0] = qm;
    g.stats[1] = loss;
    g.acc[0] += (double)qm;
    g.acc[1] += (double)loss;
    g.acc[2] += 1.0;
  }
}

}  // namespace ddpg
