// Small-batch learner step (the latency-bound B <= 512 path, SURVEY.md §8 C2:
// InvertedPendulum 4/1/128/200, B = 64).
//
// At these sizes every GEMM of the large-batch path is a few-microsecond,
// few-block launch; the step would be a chain of ~35 of them.  Here it is
// four launches, row-parallel (one workgroup per SB_R batch rows, so the
// forward and backward passes need no inter-workgroup exchange):
//
//   sb_phase1  gather this WG's rows from the replay ring (+ scaler) ->
//              target actor fwd -> target critic fwd -> TD target -> online
//              critic fwd -> MSE loss / dQ -> critic head + dX backward ->
//              this WG's partial critic gradients (one slab per WG, flat
//              parameter layout).  WG 0 also computes the critic Adam step
//              size from the beta powers and advances them (TF
//              AdamOptimizer._finish).
//   sb_reduce_adam(critic): g = ordered sum of the slabs -> TF ApplyAdam ->
//              soft update of the critic target; refreshes the transposed
//              shadow of Wh used by the dX layers.
//   sb_phase3  online actor fwd -> updated-critic fwd at (s, mu) -> dQ/da ->
//              actor backward -> partial actor gradients; WG 0 computes the
//              actor step size and advances its powers.
//   sb_reduce_adam(actor) (+ shadow of W2).
//
// Each dense layer is a skinny [SB_R x K] . [K x N] product: the weights are
// read once per WG straight into VGPRs (the GEMV rule: no LDS round trip),
// every thread owning one 4-column group of one k-slice, all of a slice's
// loads issued before the first FMA, then an ordered LDS reduction over the
// k-slices with the bias / activation / EluGrad epilogue.  Layers whose
// weights would be read transposed (dX = dY . W^T) read a row-major shadow
// W^T instead, so every weight stream is 16-B-per-lane coalesced.  Rows
// beyond B are computed on zero inputs and masked out of every gradient and
// stat.  The arithmetic is the same TF-semantics fp32 as the large-batch
// path (elu / EluGrad from outputs, TanhGrad, MSE grad, ApplyAdam, soft
// update); only the summation order differs.
#pragma once
#include "common.h"

namespace ddpg {

constexpr int SB_R = 4;        // batch rows per workgroup
constexpr int SB_NT = 1024;    // threads per workgroup (16 waves)
constexpr int SB_U = 8;        // weight quads in flight per thread per batch
constexpr int SB_NMAX = 8;     // widest layer handled by the k-parallel thin kernel
constexpr int SB_RED = 4 * SB_R * SB_NT;  // LDS floats of k-slice partials
constexpr int SB_MAXH = 512;   // widest hidden layer of the small path

#define SB_FN __device__ __forceinline__

// native vector (not HIP_vector_type) so that address-space-qualified
// loads / stores compile to global_/ds_ b128 directly
typedef __attribute__((address_space(1))) f32x4 glb_v4;
typedef __attribute__((address_space(3))) f32x4 lds_v4;

// Per-step arguments (device pointers; offsets into the flat layout).
struct SbArgs {
  int B;                 // local rows
  int S, A, AH1, AH2, CH1, CH2;
  int LX, LA, LB, LC, LD;  // LDS row strides (floats, multiples of 4)
  float inv_b, gamma, scale, tau, omt, b1, b2, lr_a, lr_c, eps;
  // replay ring + this step's slots (fused gather)
  const int* slots;
  const float *rs, *ra, *rr, *rt, *rs2;
  const double *mean, *sdev;  // optional scaler
  float* theta;
  float* target;
  float* adam_m;
  float* adam_v;
  float* whT;            // [CH2][2 CH1]  = critic Wh^T
  float* w2T;            // [AH2][AH1]    = actor W2^T
  float* part;           // [G][PT] partial gradient slabs (flat param layout)
  long long PT;          // floats per slab (= layout total)
  float* pw;             // beta powers [actor b1p, b2p, critic b1p, b2p]
  float* alpha;          // [actor, critic] Adam step sizes for this step
  float* stat_part;      // [G][2] loss partial, q max
  float* stats;          // [q_max, loss]
  double* acc;           // [qmax_sum, loss_sum, steps]
  long long aW1, ab1, aW2, ab2, aW3;
  long long cWs, cbs, cWa, cba, cWh, cbh, cWo, cbo;
  long long actor_begin, actor_end, critic_begin, critic_end;
};

// LDS floats a workgroup needs (host side: launch size and eligibility).
inline size_t sb_smem_floats(int LX, int LA, int LB, int LC, int LD) {
  return (size_t)SB_R * (4 * LX + LA + LB + LC + LD + 8) + SB_RED;
}

// Epilogue kinds of sb_dense.
enum { SB_NONE = 0, SB_ELU = 1, SB_POST2 = 2, SB_AUX = 3 };

// Y[r][n] = epi(sum_k X[r][k] W[k*ldw + n]) for r < SB_R, n < N.
// N, ldw multiples of 4, W 16-B aligned, N <= 4 * SB_NT.  X, Y, aux in LDS.
//   SB_NONE  v
//   SB_ELU   elu(v + b[n])
//   SB_POST2 pw[n] * elu'(elu(v + b[n]))     (critic head, grad_ys = 1)
//   SB_AUX   v * elu'(aux[r][n])             (dX . EluGrad)
// Thread t owns column quad q = t % NQ of k-slice s = t / NQ and the k rows
// s, s + S, s + 2S, ...; the SB_U loads of a batch are all issued before any
// is consumed.  The k-slice partials are summed in slice order (fixed,
// deterministic).  Y may alias aux (same element read then written by one
// thread) but not X.  Ends with a barrier.
SB_FN void sb_dense(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw, int N,
                    const glb_f* __restrict__ b, int epi, const glb_f* __restrict__ pw,
                    const lds_f* aux, int ldaux, lds_f* Y, int ldy, lds_f* red) {
  const int tid = threadIdx.x;
  const int NQ = N >> 2;
  const int S = SB_NT / NQ;
  const int q = tid % NQ, s = tid / NQ;
  if (s < S) {
    f32x4 acc[SB_R];
#pragma unroll
    for (int r = 0; r < SB_R; ++r) acc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
    const glb_v4* Wq = reinterpret_cast<const glb_v4*>(W) + q;
    const int ldq = ldw >> 2;
    for (int k0 = s; k0 < K; k0 += SB_U * S) {
      f32x4 w[SB_U];
#pragma unroll
      for (int u = 0; u < SB_U; ++u) w[u] = Wq[(size_t)min(k0 + u * S, K - 1) * ldq];
#pragma unroll
      for (int u = 0; u < SB_U; ++u) {
        const int k = k0 + u * S;
        const int kk = min(k, K - 1);
#pragma unroll
        for (int r = 0; r < SB_R; ++r) {
          const float x = k < K ? X[r * ldx + kk] : 0.f;
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(x, w[u][c], acc[r][c]);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < SB_R; ++r)
      *reinterpret_cast<lds_v4*>(red + (s * SB_R + r) * N + 4 * q) = acc[r];
  }
  __syncthreads();
  for (int idx = tid; idx < SB_R * N; idx += SB_NT) {
    const int r = idx / N, n = idx - r * N;
    float v = 0.f;
    for (int j = 0; j < S; ++j) v += red[(j * SB_R + r) * N + n];
    if (epi == SB_ELU) {
      v = elu_f(__fadd_rn(v, b[n]));
    } else if (epi == SB_POST2) {
      v = __fmul_rn(pw[n], elu_grad_factor(elu_f(__fadd_rn(v, b[n]))));
    } else if (epi == SB_AUX) {
      v = __fmul_rn(v, elu_grad_factor(aux[r * ldaux + n]));
    }
    Y[r * ldy + n] = v;
  }
  __syncthreads();
}

// Thin layers (N <= SB_NMAX outputs: actor W3, critic Wo, critic Wa^T):
// k-parallel over the whole workgroup, then a block reduction.
// trans: W is [N][K] (X . W^T).  Y[r][n] = act(sum_k X[r][k] W(k, n) + b[n]),
// act 0 none, 2 tanh.  Ends with a barrier.
SB_FN void sb_thin(const lds_f* X, int ldx, int K, const glb_f* __restrict__ W, int ldw,
                   bool trans, const glb_f* __restrict__ b, int N, lds_f* Y, int ldy, int act,
                   lds_f* red) {
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
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < SB_R; ++r)
#pragma unroll
    for (int n = 0; n < SB_NMAX; ++n) {
      if (n < N) {
        float v = acc[r][n];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) red[(wave * SB_R + r) * SB_NMAX + n] = v;
      }
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
  __syncthreads();
}

// out[i*N + j] = sum_r X[r][i] dY[r][j] (i < Kin, j < N) into this WG's global
// gradient slab; db[j] = sum_r dY[r][j] when db.  Masked rows of dY are zero.
// N % 4 == 0: one float4 store per (i, column quad); otherwise scalar.
SB_FN void sb_wgrad(const lds_f* X, int ldx, int Kin, const lds_f* dY, int ldy, int N,
                    glb_f* __restrict__ out, glb_f* __restrict__ db) {
  if ((N & 3) == 0) {
    const int NQ = N >> 2;
    for (int p = threadIdx.x; p < Kin * NQ; p += SB_NT) {
      const int i = p / NQ, j = 4 * (p - i * NQ);
      f32x4 sacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < SB_R; ++r) {
        const float x = X[r * ldx + i];
        const f32x4 d = *reinterpret_cast<const lds_v4*>(dY + r * ldy + j);
#pragma unroll
        for (int c = 0; c < 4; ++c) sacc[c] = fmaf(x, d[c], sacc[c]);
      }
      *reinterpret_cast<glb_v4*>(out + (size_t)i * N + j) = sacc;
    }
  } else {
    for (int p = threadIdx.x; p < Kin * N; p += SB_NT) {
      const int i = p / N, j = p - i * N;
      float sacc = 0.f;
#pragma unroll
      for (int r = 0; r < SB_R; ++r) sacc = fmaf(X[r * ldx + i], dY[r * ldy + j], sacc);
      out[p] = sacc;
    }
  }
  if (db)
    for (int j = threadIdx.x; j < N; j += SB_NT) {
      float sacc = 0.f;
#pragma unroll
      for (int r = 0; r < SB_R; ++r) sacc += dY[r * ldy + j];
      db[j] = sacc;
    }
}

// TF ApplyAdam step size from the beta powers, then _finish's power update.
DDPG_DEV void sb_alpha_and_advance(float* pw, float* alpha, float lr, float b1, float b2) {
  const float b1p = pw[0], b2p = pw[1];
  *alpha = __fdiv_rn(__fmul_rn(lr, __fsqrt_rn(__fsub_rn(1.f, b2p))), __fsub_rn(1.f, b1p));
  pw[0] = __fmul_rn(b1p, b1);
  pw[1] = __fmul_rn(b2p, b2);
}

// dst[r][k] = ring[slot(r0 + r)][k] (k < cols), zero beyond cols up to ldd and
// for rows past `valid`; the scaler (x - mean) / scale in fp64 when mean.
DDPG_DEV void sb_gather(lds_f* dst, int ldd, const float* __restrict__ ring, int cols,
                        const int* __restrict__ slots, int r0, int valid,
                        const double* __restrict__ mean, const double* __restrict__ sdev) {
  for (int idx = threadIdx.x; idx < SB_R * ldd; idx += SB_NT) {
    const int r = idx / ldd, k = idx - r * ldd;
    float x = 0.f;
    if (r < valid && k < cols) {
      x = ring[(size_t)slots[r0 + r] * cols + k];
      if (mean) x = (float)(((double)x - mean[k]) / sdev[k]);
    }
    dst[idx] = x;
  }
}

__global__ __launch_bounds__(SB_NT) void sb_phase1_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * SB_R;
  const int valid = min(SB_R, g.B - r0);
  lds_f* red = LDS(sm);
  lds_f* xs = red + SB_RED;
  lds_f* xs2 = xs + SB_R * g.LX;
  lds_f* xa = xs2 + SB_R * g.LX;
  lds_f* ta2 = xa + SB_R * g.LX;
  lds_f* bufA = ta2 + SB_R * g.LX;
  lds_f* bufB = bufA + SB_R * g.LA;
  lds_f* bufC = bufB + SB_R * g.LB;
  lds_f* bufD = bufC + SB_R * g.LC;
  lds_f* col = bufD + SB_R * g.LD;  // [SB_R][8]: q', y, q, dq, r, t
  const glb_f* T = GLB(g.target);
  const glb_f* P = GLB(g.theta);
  glb_f* part = GLB(g.part) + (size_t)blockIdx.x * g.PT;

  if (blockIdx.x == 0 && tid == 0) sb_alpha_and_advance(g.pw + 2, g.alpha + 1, g.lr_c, g.b1, g.b2);
  sb_gather(xs, g.LX, g.rs, g.S, g.slots, r0, valid, g.mean, g.sdev);
  sb_gather(xs2, g.LX, g.rs2, g.S, g.slots, r0, valid, g.mean, g.sdev);
  sb_gather(xa, g.LX, g.ra, g.A, g.slots, r0, valid, nullptr, nullptr);
  // ta2 is written only in its first A columns; the padding up to LX must be 0
  for (int idx = tid; idx < SB_R * g.LX; idx += SB_NT) ta2[idx] = 0.f;
  if (tid < SB_R) {
    const bool ok = tid < valid;
    col[tid * 8 + 4] = ok ? g.rr[g.slots[r0 + tid]] : 0.f;
    col[tid * 8 + 5] = ok ? g.rt[g.slots[r0 + tid]] : 0.f;
  }
  __syncthreads();
  // ---- target actor: ta2 = scale * tanh(elu(elu(s2 W1 + b1) W2 + b2) W3)   ddpg.py:90
  sb_dense(xs2, g.LX, g.S, T + g.aW1, g.AH1, g.AH1, T + g.ab1, SB_ELU, nullptr, nullptr, 0, bufA,
           g.LA, red);
  sb_dense(bufA, g.LA, g.AH1, T + g.aW2, g.AH2, g.AH2, T + g.ab2, SB_ELU, nullptr, nullptr, 0,
           bufB, g.LB, red);
  sb_thin(bufB, g.LB, g.AH2, T + g.aW3, g.A, false, nullptr, g.A, ta2, g.LX, 2, red);
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    ta2[r * g.LX + a] = __fmul_rn(ta2[r * g.LX + a], g.scale);
  }
  __syncthreads();
  // ---- target critic: q' and y = t ? r : r + gamma q'
  sb_dense(xs2, g.LX, g.S, T + g.cWs, g.CH1, g.CH1, T + g.cbs, SB_ELU, nullptr, nullptr, 0, bufC,
           g.LC, red);
  sb_dense(ta2, g.LX, g.A, T + g.cWa, g.CH1, g.CH1, T + g.cba, SB_ELU, nullptr, nullptr, 0,
           bufC + g.CH1, g.LC, red);
  sb_dense(bufC, g.LC, 2 * g.CH1, T + g.cWh, g.CH2, g.CH2, T + g.cbh, SB_ELU, nullptr, nullptr, 0,
           bufD, g.LD, red);
  sb_thin(bufD, g.LD, g.CH2, T + g.cWo, 1, false, T + g.cbo, 1, col + 0, 8, 0, red);
  if (tid < SB_R) {
    const float rr = col[tid * 8 + 4], tt = col[tid * 8 + 5];
    col[tid * 8 + 1] = tt != 0.f ? rr : __fadd_rn(rr, __fmul_rn(g.gamma, col[tid * 8 + 0]));
  }
  // ---- online critic forward (networks.py:147-162)
  sb_dense(xs, g.LX, g.S, P + g.cWs, g.CH1, g.CH1, P + g.cbs, SB_ELU, nullptr, nullptr, 0, bufC,
           g.LC, red);
  sb_dense(xa, g.LX, g.A, P + g.cWa, g.CH1, g.CH1, P + g.cba, SB_ELU, nullptr, nullptr, 0,
           bufC + g.CH1, g.LC, red);
  sb_dense(bufC, g.LC, 2 * g.CH1, P + g.cWh, g.CH2, g.CH2, P + g.cbh, SB_ELU, nullptr, nullptr, 0,
           bufD, g.LD, red);
  sb_thin(bufD, g.LD, g.CH2, P + g.cWo, 1, false, P + g.cbo, 1, col + 2, 8, 0, red);
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
  // dcat = dhp . Wh^T * elu'(cat) -> bufA   (Wh^T read from its row-major shadow)
  sb_dense(bufB, g.LB, g.CH2, GLB(g.whT), 2 * g.CH1, 2 * g.CH1, nullptr, SB_AUX, nullptr, bufC,
           g.LC, bufA, g.LA, red);
  // ---- partial critic gradients (this WG's rows)
  sb_wgrad(xs, g.LX, g.S, bufA, g.LA, g.CH1, part + g.cWs, part + g.cbs);
  sb_wgrad(xa, g.LX, g.A, bufA + g.CH1, g.LA, g.CH1, part + g.cWa, part + g.cba);
  sb_wgrad(bufC, g.LC, 2 * g.CH1, bufB, g.LB, g.CH2, part + g.cWh, part + g.cbh);
  for (int j = tid; j < g.CH2; j += SB_NT) {
    float sacc = 0.f;
    for (int r = 0; r < SB_R; ++r) sacc = fmaf(bufD[r * g.LD + j], col[r * 8 + 3], sacc);
    part[g.cWo + j] = sacc;
  }
  if (tid == 0) {
    float sacc = 0.f;
    for (int r = 0; r < SB_R; ++r) sacc += col[r * 8 + 3];
    part[g.cbo] = sacc;
  }
}

__global__ __launch_bounds__(SB_NT) void sb_phase3_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * SB_R;
  const int valid = min(SB_R, g.B - r0);
  lds_f* red = LDS(sm);
  lds_f* xs = red + SB_RED;
  lds_f* o = xs + SB_R * g.LX;
  lds_f* mu = o + SB_R * g.LX;
  lds_f* dz3 = mu + SB_R * g.LX;
  lds_f* bufA = dz3 + SB_R * g.LX;
  lds_f* bufB = bufA + SB_R * g.LA;
  lds_f* bufC = bufB + SB_R * g.LB;
  lds_f* bufD = bufC + SB_R * g.LC;
  const glb_f* P = GLB(g.theta);
  glb_f* part = GLB(g.part) + (size_t)blockIdx.x * g.PT;

  if (blockIdx.x == 0 && tid == 0) sb_alpha_and_advance(g.pw, g.alpha, g.lr_a, g.b1, g.b2);
  sb_gather(xs, g.LX, g.rs, g.S, g.slots, r0, valid, g.mean, g.sdev);
  // o / mu / dz3 are written only in their first A columns
  for (int idx = tid; idx < 3 * SB_R * g.LX; idx += SB_NT) o[idx] = 0.f;
  __syncthreads();
  // ---- online actor forward (current actor params): h1 -> bufA, h2 -> bufB, o, mu
  sb_dense(xs, g.LX, g.S, P + g.aW1, g.AH1, g.AH1, P + g.ab1, SB_ELU, nullptr, nullptr, 0, bufA,
           g.LA, red);
  sb_dense(bufA, g.LA, g.AH1, P + g.aW2, g.AH2, g.AH2, P + g.ab2, SB_ELU, nullptr, nullptr, 0,
           bufB, g.LB, red);
  sb_thin(bufB, g.LB, g.AH2, P + g.aW3, g.A, false, nullptr, g.A, o, g.LX, 2, red);
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    mu[r * g.LX + a] = __fmul_rn(o[r * g.LX + a], g.scale);
  }
  __syncthreads();
  // ---- updated critic at (s, mu): dhp2 = Wo * elu'(h')  (grad_ys = 1)   networks.py:143
  sb_dense(xs, g.LX, g.S, P + g.cWs, g.CH1, g.CH1, P + g.cbs, SB_ELU, nullptr, nullptr, 0, bufC,
           g.LC, red);
  sb_dense(mu, g.LX, g.A, P + g.cWa, g.CH1, g.CH1, P + g.cba, SB_ELU, nullptr, nullptr, 0,
           bufC + g.CH1, g.LC, red);
  sb_dense(bufC, g.LC, 2 * g.CH1, P + g.cWh, g.CH2, g.CH2, P + g.cbh, SB_POST2, P + g.cWo,
           nullptr, 0, bufD, g.LD, red);
  // dca = dhp2 . Wh[CH1:]^T * elu'(ca), in place over ca (bufC[:, CH1:])
  sb_dense(bufD, g.LD, g.CH2, GLB(g.whT) + g.CH1, 2 * g.CH1, g.CH1, nullptr, SB_AUX, nullptr,
           bufC + g.CH1, g.LC, bufC + g.CH1, g.LC, red);
  // da = dca . Wa^T -> dz3 (scratch), then dz3 = ((-da) * scale) * (1 - o^2), masked
  sb_thin(bufC + g.CH1, g.LC, g.CH1, P + g.cWa, g.CH1, true, nullptr, g.A, dz3, g.LX, 0, red);
  for (int idx = tid; idx < SB_R * g.A; idx += SB_NT) {
    const int r = idx / g.A, a = idx - r * g.A;
    const float ov = o[r * g.LX + a];
    const float dy = __fmul_rn(-dz3[r * g.LX + a], g.scale);
    dz3[r * g.LX + a] = r < valid ? __fmul_rn(dy, __fsub_rn(1.f, __fmul_rn(ov, ov))) : 0.f;
  }
  __syncthreads();
  // ---- actor backward (networks.py:44)
  // dz2 = dz3 . W3^T * elu'(h2) -> bufD   (K = A is tiny: one thread per output)
  for (int idx = tid; idx < SB_R * g.AH2; idx += SB_NT) {
    const int r = idx / g.AH2, n = idx - r * g.AH2;
    float v = 0.f;
    for (int a = 0; a < g.A; ++a) v = fmaf(dz3[r * g.LX + a], P[g.aW3 + (size_t)n * g.A + a], v);
    bufD[r * g.LD + n] = __fmul_rn(v, elu_grad_factor(bufB[r * g.LB + n]));
  }
  __syncthreads();
  sb_wgrad(bufB, g.LB, g.AH2, dz3, g.LX, g.A, part + g.aW3, nullptr);
  sb_wgrad(bufA, g.LA, g.AH1, bufD, g.LD, g.AH2, part + g.aW2, part + g.ab2);
  __syncthreads();
  // dz1 = dz2 . W2^T * elu'(h1), in place over h1 (bufA)
  sb_dense(bufD, g.LD, g.AH2, GLB(g.w2T), g.AH1, g.AH1, nullptr, SB_AUX, nullptr, bufA, g.LA,
           bufA, g.LA, red);
  sb_wgrad(xs, g.LX, g.S, bufA, g.LA, g.AH1, part + g.aW1, part + g.ab1);
}

// g = sum of the per-WG slabs (slab order); TF ApplyAdam with this step's
// alpha; soft update of the target; transposed shadow of the dX weight
// (critic Wh -> whT, actor W2 -> w2T).  net: 0 actor, 1 critic.  The critic
// call also finalises the step stats.
__global__ void sb_reduce_adam_kernel(SbArgs g, int net, int nslab) {
  const long long b = net == 0 ? g.actor_begin : g.critic_begin;
  const long long e = net == 0 ? g.actor_end : g.critic_end;
  const long long sh_off = net == 0 ? g.aW2 : g.cWh;
  const int sh_rows = net == 0 ? g.AH1 : 2 * g.CH1, sh_cols = net == 0 ? g.AH2 : g.CH2;
  float* const sh = net == 0 ? g.w2T : g.whT;
  const long long sh_n = (long long)sh_rows * sh_cols;
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
    const long long si = i - sh_off;
    if (si >= 0 && si < sh_n) {
      const long long rr = si / sh_cols, cc = si - rr * sh_cols;
      sh[cc * sh_rows + rr] = p;
    }
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

// dst[c][r] = src[r][c] for a rows x cols row-major matrix (shadow refresh
// after any parameter write outside the small path).
__global__ void sb_transpose_kernel(const float* __restrict__ src, int rows, int cols,
                                    float* __restrict__ dst) {
  const long long n = (long long)rows * cols;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    const long long r = i / cols, c = i - r * cols;
    dst[c * rows + r] = src[i];
  }
}

}  // namespace ddpg
