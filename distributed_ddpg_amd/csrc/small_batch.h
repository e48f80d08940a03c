// Small-batch learner step (the latency-bound B <= 512 path, SURVEY.md §8 C2:
// InvertedPendulum 4/1/128/200, B = 64).
//
// At these sizes every GEMM of the large-batch path is a few-microsecond,
// few-block launch; the step would be a chain of ~35 of them.  Here it is
// four launches:
//
//   sb_phase1  (row-parallel, one workgroup per SB_R batch rows): gather the
//              rows from the replay ring (+ scaler) -> target actor fwd ->
//              target critic fwd -> TD target -> online critic fwd -> MSE
//              loss / dQ -> critic head + dX backward; saves the activations
//              and output gradients the critic weight gradients need.  WG 0
//              computes the critic Adam step size from the beta powers and
//              advances them (TF AdamOptimizer._finish).  A second set of
//              workgroups, on CUs of their own, runs the online actor's
//              forward on the same rows (its parameters are not updated
//              before phase 3) and saves h1, h2, o.
//   sb_wgrad_adam(critic): every critic weight gradient dW = X^T . dY over
//              the whole batch (one ordered fp32 sum over b per element),
//              TF ApplyAdam, soft update of the critic target, and the
//              transposed shadow of Wh used by the dX layers.
//   sb_phase3  (row-parallel): the saved actor forward -> updated-critic
//              fwd at (s, mu) -> dQ/da -> actor backward; saves what the
//              actor weight gradients need.  WG 0 computes the actor step
//              size.
//   sb_wgrad_adam(actor) (+ shadow of W2).
//
// Inside a phase, independent layers run side by side on disjoint thread
// groups (e.g. the target actor's first layer, both critics' state branches
// and the online critic's action branch are one level), so the dependent
// chain is 8 levels in phase 1 and 5 in phase 3.  Each dense layer is a skinny [SB_R x K] .
// [K x N] product: the weights are read once per WG straight into VGPRs (the
// GEMV rule: no LDS round trip), each thread owning one 4-column group of one
// k-slice, all of a batch's loads issued before the first FMA, then an
// ordered LDS reduction over the k-slices with the bias / activation /
// EluGrad epilogue.  Layers whose weights would be read transposed (dX = dY .
// W^T) read a row-major shadow W^T instead, so every weight stream is
// 16-B-per-lane coalesced.  Rows beyond B are computed on zero inputs and
// never saved.  The arithmetic is the same TF-semantics fp32 as the
// large-batch path (elu / EluGrad from outputs, TanhGrad, MSE grad,
// ApplyAdam, soft update); only the summation order differs.
#pragma once
#include "common.h"
#include "types.h"

namespace ddpg {

constexpr int SB_R = 4;        // batch rows per workgroup
#ifndef SB_NT_DEF
#define SB_NT_DEF 512
#endif
constexpr int SB_NT = SB_NT_DEF;  // threads per workgroup
#ifndef SB_U_DEF
#define SB_U_DEF 8
#endif
#ifndef SB_DBUF
#define SB_DBUF 0  // 1: two register batches (next issued before current consumed)
#endif
constexpr int SB_U = SB_U_DEF;  // weight quads in flight per thread per batch
constexpr int SB_NMAX = 8;     // widest layer handled by the k-parallel thin kernel
constexpr int SB_RED = 4 * SB_R * SB_NT;  // LDS floats of k-slice partials
constexpr int SB_MAXH = 512;   // widest hidden layer of the small path
constexpr int SB_GT = 256;     // threads of the weight-gradient / Adam kernel

#define SB_FN __device__ __forceinline__

// native vector (not HIP_vector_type) so that address-space-qualified
// loads / stores compile to global_/ds_ b128 directly
typedef __attribute__((address_space(1))) f32x4 glb_v4;
typedef __attribute__((address_space(3))) f32x4 lds_v4;



// Per-step arguments (device pointers; offsets into the flat layout).
struct SbArgs {
  int B;                 // local rows
  int S, A, AH1, AH2, CH1, CH2;
  int LX, LW;            // LDS row strides: inputs, hidden buffers (multiples of 4)
  float inv_b, gamma, scale, tau, omt, b1, b2, lr_a, lr_c, eps;
  // replay ring + this step's slots (fused gather)
  const int* slots;
  const float *rs, *ra, *rr, *rt, *rs2;
  const double *rsd, *rs2d, *rrd;  // float64 ring planes (s, s2, r) when the ring keeps them
  const double *mean, *sdev;  // optional scaler (applied to replay rows only)
  float* grad;           // flat gradient buffer (written for ddpg_get_params readback)
  float* theta;
  float* target;
  float* adam_m;
  float* adam_v;
  float* whT;            // [CH2][2 CH1]  = critic Wh^T
  float* w2T;            // [AH2][AH1]    = actor W2^T
  SbSave sv;
  float* pw;             // beta powers [actor b1p, b2p, critic b1p, b2p]
  float* alpha;          // [actor, critic] Adam step sizes for this step
  float* stats;          // [q_max, loss]
  double* acc;           // [qmax_sum, loss_sum, steps]
  long long aW1, ab1, aW2, ab2, aW3;
  long long cWs, cbs, cWa, cba, cWh, cbh, cWo, cbo;
#ifdef DDPG_SB_STAMPS
  unsigned long long* stamps;  // diagnostic build only: WG 0 s_memtime per level
#endif
  // XCD packing: the grid has xstride x G blocks and only every xstride-th
  // works, so with the hardware's round-robin block->XCD dealing all working
  // WGs share one XCD's L2 and the weights stream from it once rather than
  // once per XCD (speed only: any placement computes the same result)
  int xstride;
};

// Diagnostic stamps (a -DDDPG_SB_STAMPS build only; the product compiles
// them away): nothing reads them on device and no output depends on them.
#ifdef DDPG_SB_STAMPS
#define SB_STAMP(i)                                                              \
  do {                                                                           \
    if (g.stamps && blockIdx.x == 0 && threadIdx.x == 0)                         \
      g.stamps[i] = __builtin_amdgcn_s_memtime();                                \
  } while (0)
#define SB_STAMP_SYNC(i)                                                         \
  do {                                                                           \
    if (g.stamps) {                                                              \
      __syncthreads();                                                           \
      SB_STAMP(i);                                                               \
    }                                                                            \
  } while (0)
#else
#define SB_STAMP(i) \
  do {              \
  } while (0)
#define SB_STAMP_SYNC(i) \
  do {                   \
  } while (0)
#endif

// LDS floats a phase workgroup needs (host side: launch size and eligibility).
inline size_t sb_smem_floats(int LX, int LW) {
  return (size_t)SB_R * (4 * LX + 5 * LW + 8) + SB_RED + 2 * 2048;  // + biases / pw
}

// Activation layout in LDS: k-major, the SB_R (= 4) rows of one feature
// contiguous (X[k*4 + r]), so one ds_read_b128 feeds a weight quad's 16 FMAs
// and no index needs a division.  All buffer pointers below are already
// offset to their first feature.
static_assert(SB_R == 4, "k-major activation layout assumes 4 rows per workgroup");
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Epilogue kinds of a dense layer.
enum { SB_NONE = 0, SB_ELU = 1, SB_POST2 = 2, SB_AUX = 3 };

// One skinny layer: Y[n][r] = epi(sum_k X[k][r] W(k, n)) for r < 4, n < N.
//   dense: W(k, n) = W[k*ldw + n]; N, ldw multiples of 4, W 16-B aligned.
//   thin (N <= SB_NMAX): W(k, n) = trans ? W[n*ldw + k] : W[k*ldw + n].
// epi: SB_NONE v | SB_ELU elu(v + b[n]) | SB_POST2 pw[n] * elu'(elu(v + b[n]))
//      (critic head, grad_ys = 1) | SB_AUX v * elu'(aux[n][r]) (dX . EluGrad).
// thin: v (+ b[n]) then tanh when act_tanh.
struct SbOp {
  const lds_f* X;
  int K;
  const glb_f* W;
  int ldw, N;
  const glb_f* b;
  int epi;
  const glb_f* pw;
  const lds_f* aux;
  lds_f* Y;
  bool trans, act_tanh;
};

DDPG_DEV SbOp sb_op(const lds_f* X, int K, const glb_f* W, int ldw, int N, const glb_f* b,
                    int epi, lds_f* Y, const lds_f* aux = nullptr, const glb_f* pw = nullptr) {
  SbOp o;
  o.X = X;
  o.K = K;
  o.W = W;
  o.ldw = ldw;
  o.N = N;
  o.b = b;
  o.epi = epi;
  o.pw = pw;
  o.aux = aux;
  o.Y = Y;
  o.trans = false;
  o.act_tanh = false;
  return o;
}

// acc[c][r] += x[r] * w[c], as packed f32 FMAs (two rows per instruction).
SB_FN void sb_fma4(f32x4 (&acc)[4], f32x4 x, f32x4 w) {
  const f32x2 xl = {x[0], x[1]}, xh = {x[2], x[3]};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const f32x2 wc = {w[c], w[c]};
    f32x2 lo = {acc[c][0], acc[c][1]}, hi = {acc[c][2], acc[c][3]};
    lo = __builtin_elementwise_fma(xl, wc, lo);
    hi = __builtin_elementwise_fma(xh, wc, hi);
    acc[c] = f32x4{lo[0], lo[1], hi[0], hi[1]};
  }
}

// Dense layer, part 1 on threads t < nt of a wave-aligned group: thread t owns
// column quad q = t % NQ of k-slice s = t / NQ (S = min(nt / NQ, K) slices)
// and the k rows s, s + S, ...; the SB_U loads of a batch are all issued
// before any is consumed.  Partials go to red[s][n][r] (f32x4 per n).
SB_FN void sb_dense_part(const SbOp& o, int t, int nt, lds_f* red) {
  const int NQ = o.N >> 2;
  const int S = min(nt / NQ, o.K);
  const int q = t % NQ, s = t / NQ;
  if (s >= S) return;
  f32x4 acc[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int K = o.K;
  const lds_v4* X4 = reinterpret_cast<const lds_v4*>(o.X);
  const glb_v4* Wq = reinterpret_cast<const glb_v4*>(o.W) + q;
  const size_t step = (size_t)S * (o.ldw >> 2);  // float4s between this thread's k rows
  const glb_v4* wp = Wq + (size_t)s * (o.ldw >> 2);
  const int nk = (K - s + S - 1) / S;  // this thread's k rows
  int i = 0;
  for (; i + SB_U <= nk; i += SB_U) {
    f32x4 w[SB_U];
#pragma unroll
    for (int u = 0; u < SB_U; ++u) w[u] = wp[u * step];
#pragma unroll
    for (int u = 0; u < SB_U; ++u) sb_fma4(acc, X4[s + (i + u) * S], w[u]);
    wp += SB_U * step;
  }
  if (i < nk) {  // remainder: clamped loads, masked FMAs
    f32x4 w[SB_U];
    const int rem = nk - i;
#pragma unroll
    for (int u = 0; u < SB_U; ++u) w[u] = wp[min(u, rem - 1) * step];
#pragma unroll
    for (int u = 0; u < SB_U; ++u)
      if (u < rem) sb_fma4(acc, X4[s + (i + u) * S], w[u]);
  }
  lds_v4* r4 = reinterpret_cast<lds_v4*>(red) + (size_t)s * o.N + 4 * q;
#pragma unroll
  for (int c = 0; c < 4; ++c) r4[c] = acc[c];
}

// Dense layer, part 2: output idx = n*4 + r sums its S partials in slice
// order (loads batched 8 at a time, adds sequential) and applies the epilogue.
SB_FN void sb_dense_epi(const SbOp& o, int t, int nt, const lds_f* red, const lds_f* bl,
                        const lds_f* pwl) {
  const int N = o.N;
  const int S = min(nt / (N >> 2), o.K);
  const int stride = 4 * N;
  for (int idx = t; idx < 4 * N; idx += nt) {
    const int n = idx >> 2;
    const lds_f* pr = red + idx;
    float v = 0.f;
    int j = 0;
    for (; j + 8 <= S; j += 8) {
      float p[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) p[u] = pr[(j + u) * stride];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += p[u];
    }
    for (; j < S; ++j) v += pr[j * stride];
    if (o.epi == SB_ELU) {
      v = elu_f(__fadd_rn(v, bl[n]));
    } else if (o.epi == SB_POST2) {
      v = __fmul_rn(pwl[n], elu_grad_factor(elu_f(__fadd_rn(v, bl[n]))));
    } else if (o.epi == SB_AUX) {
      v = __fmul_rn(v, elu_grad_factor(o.aux[idx]));
    }
    o.Y[idx] = v;
  }
}

// Thin layer, part 1: k-parallel over the group, wave reduction, one partial
// per (group wave, output, row) in red.
SB_FN void sb_thin_part(const SbOp& o, int t, int nt, lds_f* red) {
  float acc[SB_NMAX][4];
#pragma unroll
  for (int n = 0; n < SB_NMAX; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[n][r] = 0.f;
  const lds_v4* X4 = reinterpret_cast<const lds_v4*>(o.X);
  for (int k = t; k < o.K; k += nt) {
    const f32x4 x = X4[k];
#pragma unroll
    for (int n = 0; n < SB_NMAX; ++n) {
      if (n < o.N) {
        const float w = o.trans ? o.W[(size_t)n * o.ldw + k] : o.W[(size_t)k * o.ldw + n];
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[n][r] = fmaf(x[r], w, acc[n][r]);
      }
    }
  }
  const int lane = t & 63, wave = t >> 6;
#pragma unroll
  for (int n = 0; n < SB_NMAX; ++n) {
    if (n < o.N) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[n][r];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        if (lane == 0) red[(wave * SB_NMAX + n) * 4 + r] = v;
      }
    }
  }
}

SB_FN void sb_thin_epi(const SbOp& o, int t, int nt, const lds_f* red) {
  if (t < 4 * o.N) {
    const int n = t >> 2;
    float v = 0.f;
    for (int w = 0; w < nt / 64; ++w) v += red[w * SB_NMAX * 4 + t];
    if (o.b) v = __fadd_rn(v, o.b[n]);
    if (o.act_tanh) v = tanhf(v);
    o.Y[t] = v;
  }
}

// One level of NOPS independent layers on NG >= NOPS equal wave-aligned thread
// groups (groups past NOPS idle), each with its own slice of red and of the
// bias area (the bias and pw vectors are loaded before the weights, so their
// round trip hides behind the weights', and parked in LDS for the epilogue).
// Ends with a barrier.
constexpr int SB_BIAS = 2048;  // LDS floats for biases (+ as many for pw)
template <int NOPS, int NG = NOPS>
SB_FN void sb_level(const SbOp (&ops)[NOPS], const bool (&thin)[NOPS], lds_f* red) {
  static_assert(NG >= NOPS, "one thread group per layer");
  constexpr int nt = SB_NT / NG;
  constexpr int rs = SB_RED / NG;
  constexpr int bs = SB_BIAS / NG;
  lds_f* bias = red + SB_RED;
  const int grp = threadIdx.x / nt, t = threadIdx.x - grp * nt;
#pragma unroll
  for (int i = 0; i < NOPS; ++i)
    if (grp == i) {
      if (thin[i]) {
        sb_thin_part(ops[i], t, nt, red + i * rs);
      } else {
        const SbOp& o = ops[i];
        const bool hb = o.epi == SB_ELU || o.epi == SB_POST2;
        float bv[4], pv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = t + j * nt;
          bv[j] = (hb && n < o.N) ? o.b[n] : 0.f;
          pv[j] = (o.epi == SB_POST2 && n < o.N) ? o.pw[n] : 0.f;
        }
        sb_dense_part(o, t, nt, red + i * rs);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = t + j * nt;
          if (n < o.N && n < bs) {
            bias[i * bs + n] = bv[j];
            bias[SB_BIAS + i * bs + n] = pv[j];
          }
        }
      }
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NOPS; ++i)
    if (grp == i) {
      if (thin[i]) sb_thin_epi(ops[i], t, nt, red + i * rs);
      else sb_dense_epi(ops[i], t, nt, red + i * rs, bias + i * bs, bias + SB_BIAS + i * bs);
    }
  __syncthreads();
}

SB_FN void sb_dense1(const SbOp& o, lds_f* red) {
  const SbOp ops[1] = {o};
  const bool th[1] = {false};
  sb_level<1>(ops, th, red);
}

SB_FN void sb_thin1(SbOp o, bool trans, bool act_tanh, lds_f* red) {
  o.trans = trans;
  o.act_tanh = act_tanh;
  const SbOp ops[1] = {o};
  const bool th[1] = {true};
  sb_level<1>(ops, th, red);
}

// TF ApplyAdam step size from the beta powers, then _finish's power update.
DDPG_DEV void sb_alpha_and_advance(float* pw, float* alpha, float lr, float b1, float b2) {
  const float b1p = pw[0], b2p = pw[1];
  *alpha = __fdiv_rn(__fmul_rn(lr, __fsqrt_rn(__fsub_rn(1.f, b2p))), __fsub_rn(1.f, b1p));
  pw[0] = __fmul_rn(b1p, b1);
  pw[1] = __fmul_rn(b2p, b2);
}

// save[k][r0 .. r0 + 3] = src[k][0 .. 3] (feature-major, one float4 per
// feature; rows past B land in the padding that no reader sums).
DDPG_DEV void sb_save(float* __restrict__ save, int Bp, int cols, const lds_f* src, int r0) {
  const lds_v4* s4 = reinterpret_cast<const lds_v4*>(src);
  for (int k = threadIdx.x; k < cols; k += SB_NT)
    *reinterpret_cast<f32x4*>(save + (size_t)k * Bp + r0) = s4[k];
}

// Phase 1's actor-forward workgroups: the online actor's forward on the same
// rows (networks.py:51-63, ddpg.py:106's actor.predict(s)).  The actor's
// parameters do not change until its own Adam step, so this runs beside the
// critic chain on CUs of its own, and phase 3 (after the critic update) reads
// h1, h2 and o back instead of recomputing them on its critical path.  Same
// level shapes as phase 3 used, so the values are the ones it computed.
DDPG_DEV void sb_actor_rows(const SbArgs& g, int r0, int valid, lds_f* red) {
  const int tid = threadIdx.x;
  lds_f* xs = red + SB_RED + 2 * SB_BIAS;  // [LX][4]
  lds_f* o = xs + 4 * g.LX;
  lds_f* h1 = o + 4 * g.LX;  // [LW][4]
  lds_f* h2 = h1 + 4 * g.LW;
  const glb_f* P = GLB(g.theta);
  for (int idx = tid; idx < 4 * g.LX; idx += SB_NT) {  // as phase 1's critic gather
    const int k = idx >> 2, r = idx & 3;
    float x = 0.f;
    if (r < valid && k < g.S) {
      const size_t e = (size_t)g.slots[r0 + r] * g.S + k;
      const double xd = g.rsd ? g.rsd[e] : (double)g.rs[e];
      x = g.mean ? (float)((xd - g.mean[k]) / g.sdev[k]) : (float)xd;
    }
    xs[idx] = x;
  }
  __syncthreads();
  {  // L1 on half the threads: phase 3's former two-group level (its k-slices)
    const SbOp ops[1] = {sb_op(xs, g.S, P + g.aW1, g.AH1, g.AH1, P + g.ab1, SB_ELU, h1)};
    const bool th[1] = {false};
    sb_level<1, 2>(ops, th, red);
  }
  sb_dense1(sb_op(h1, g.AH1, P + g.aW2, g.AH2, g.AH2, P + g.ab2, SB_ELU, h2), red);
  sb_thin1(sb_op(h2, g.AH2, P + g.aW3, g.A, g.A, nullptr, SB_NONE, o), false, true, red);
  sb_save(g.sv.h1, g.sv.Bp, g.AH1, h1, r0);
  sb_save(g.sv.h2, g.sv.Bp, g.AH2, h2, r0);
  sb_save(g.sv.o, g.sv.Bp, g.A, o, r0);
  if (g.A == 1) {
    // one action (the reference's InvertedPendulum): dz3 is a per-row scalar,
    // so the actor backward (networks.py:44) is dz3 times a per-row vector
    // that needs no critic: v2 = W3 * elu'(h2), v1 = (v2 . W2^T) * elu'(h1)
    // (W2^T from its row-major shadow).  Saved in dz2 / dz1's place; the
    // actor's weight-gradient kernel scales them by phase 3's dz3.
    lds_f* v2 = h2 + 4 * g.LW;
    lds_f* v1 = v2 + 4 * g.LW;
    for (int idx = tid; idx < 4 * g.AH2; idx += SB_NT)
      v2[idx] = __fmul_rn(P[g.aW3 + (idx >> 2)], elu_grad_factor(h2[idx]));
    __syncthreads();
    sb_dense1(sb_op(v2, g.AH2, GLB(g.w2T), g.AH1, g.AH1, nullptr, SB_AUX, v1, h1), red);
    sb_save(g.sv.dz2, g.sv.Bp, g.AH2, v2, r0);
    sb_save(g.sv.dz1, g.sv.Bp, g.AH1, v1, r0);
  }
}

// Phase 1's target workgroups: the TD target of the same rows (ddpg.py:90-97)
// -- target actor forward at s2, target critic at (s2, mu'), y = t ? r : r +
// gamma q' -- saved per row for the critic's weight-gradient kernel, which
// forms dQ from it.  Nothing on the online chain waits for it inside the
// launch, so it runs on CUs of its own.
DDPG_DEV void sb_target_rows(const SbArgs& g, int r0, int valid, lds_f* red) {
  const int tid = threadIdx.x;
  const int LX = g.LX, LW = g.LW;
  lds_f* xs2 = red + SB_RED + 2 * SB_BIAS;  // [LX][4]
  lds_f* ta2 = xs2 + 4 * LX;
  lds_f* b1 = ta2 + 4 * LX;  // [LW][4] target h1, then target hh
  lds_f* b2 = b1 + 4 * LW;   // target h2
  lds_f* b3 = b2 + 4 * LW;   // target cat
  lds_f* col = b3 + 4 * LW;  // [8][4]: q', r, t
  const glb_f* T = GLB(g.target);
  // the s2 rows as the online gather does (fp64 planes, scaler in fp64)
  for (int idx = tid; idx < 4 * LX; idx += SB_NT) {
    const int k = idx >> 2, r = idx & 3;
    float x2 = 0.f;
    if (r < valid && k < g.S) {
      const size_t e = (size_t)g.slots[r0 + r] * g.S + k;
      const double x2d = g.rs2d ? g.rs2d[e] : (double)g.rs2[e];
      x2 = g.mean ? (float)((x2d - g.mean[k]) / g.sdev[k]) : (float)x2d;
    }
    xs2[idx] = x2;
  }
  if (tid < 4) {
    const bool ok = tid < valid;
    const int sl = ok ? g.slots[r0 + tid] : 0;
    col[1 * 4 + tid] = ok ? (g.rrd ? (float)g.rrd[sl] : g.rr[sl]) : 0.f;
    col[2 * 4 + tid] = ok ? g.rt[sl] : 0.f;
  }
  __syncthreads();
  {  // L1: target h1 | target state branch
    const SbOp ops[2] = {sb_op(xs2, g.S, T + g.aW1, g.AH1, g.AH1, T + g.ab1, SB_ELU, b1),
                         sb_op(xs2, g.S, T + g.cWs, g.CH1, g.CH1, T + g.cbs, SB_ELU, b3)};
    const bool th[2] = {false, false};
    sb_level<2>(ops, th, red);
  }
  // L2: target h2; L3: o' = tanh(h2' W3'), mu' = scale o'
  sb_dense1(sb_op(b1, g.AH1, T + g.aW2, g.AH2, g.AH2, T + g.ab2, SB_ELU, b2), red);
  sb_thin1(sb_op(b2, g.AH2, T + g.aW3, g.A, g.A, nullptr, SB_NONE, ta2), false, true, red);
  for (int idx = tid; idx < 4 * g.A; idx += SB_NT) ta2[idx] = __fmul_rn(ta2[idx], g.scale);
  __syncthreads();
  // L4: target action branch; L5: target critic hidden; L6: q'
  sb_dense1(sb_op(ta2, g.A, T + g.cWa, g.CH1, g.CH1, T + g.cba, SB_ELU, b3 + 4 * g.CH1), red);
  sb_dense1(sb_op(b3, 2 * g.CH1, T + g.cWh, g.CH2, g.CH2, T + g.cbh, SB_ELU, b1), red);
  sb_thin1(sb_op(b1, g.CH2, T + g.cWo, 1, 1, T + g.cbo, SB_NONE, col), false, false, red);
  // y = t ? r : r + gamma q'  (ddpg.py:92-97)
  if (tid < valid) {
    const float rr = col[1 * 4 + tid], tt = col[2 * 4 + tid];
    g.sv.y[r0 + tid] = tt != 0.f ? rr : __fadd_rn(rr, __fmul_rn(g.gamma, col[tid]));
  }
}

// Phase-1 roles: with XCD packing (xstride > 1) block b works as role b %
// xstride (0: online critic rows, 1: actor rows, 2: target rows; the rest
// exit at once), so each role's workgroups share one XCD's L2; otherwise
// blocks [role G, (role + 1) G) take role `role`.
__global__ __launch_bounds__(SB_NT) void sb_phase1_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int G = (g.B + SB_R - 1) / SB_R;
  int wg, role;
  if (g.xstride > 1) {
    role = blockIdx.x % g.xstride;
    wg = blockIdx.x / g.xstride;
  } else {
    role = blockIdx.x / G;
    wg = blockIdx.x - role * G;
  }
  if (role > 2 || wg >= G) return;
  const int r0 = wg * SB_R;
  const int valid = min(SB_R, g.B - r0);
  if (role == 1) {
    sb_actor_rows(g, r0, valid, LDS(sm));
    return;
  }
  if (role == 2) {
    sb_target_rows(g, r0, valid, LDS(sm));
    return;
  }
  const int LX = g.LX, LW = g.LW;
  lds_f* red = LDS(sm);
  lds_f* xs = red + SB_RED + 2 * SB_BIAS;  // [LX][4]
  lds_f* xa = xs + 4 * LX;
  lds_f* gh = xa + 4 * LX;     // [LW][4] dhp per unit dQ
  lds_f* u = gh + 4 * LW;      // dcat per unit dQ
  lds_f* cat = u + 4 * LW;     // online cat
  lds_f* h = cat + 4 * LW;     // online critic hidden
  lds_f* col = h + 4 * LW;     // [8][4]: q
  const glb_f* P = GLB(g.theta);
  SB_STAMP(0);

  if (wg == 0 && tid == 0) sb_alpha_and_advance(g.pw + 2, g.alpha + 1, g.lr_c, g.b1, g.b2);
  // rows -> xs / xa ([feature][4], zero past S / A and for rows past `valid`)
  // in one pass: one slot read, then every ring read of an element in flight
  // together; from the float64 ring planes when the ring keeps them; the
  // scaler (x - mean) / scale in fp64 before the one rounding to fp32 (the
  // reference's preprocess_input + feed_dict cast); also saved feature-major
  // for the weight gradients
  for (int idx = tid; idx < 4 * LX; idx += SB_NT) {
    const int k = idx >> 2, r = idx & 3;
    float x = 0.f, xv = 0.f;
    if (r < valid) {
      const size_t sl = (size_t)g.slots[r0 + r];
      if (k < g.S) {
        const size_t e = sl * g.S + k;
        const double xd = g.rsd ? g.rsd[e] : (double)g.rs[e];
        x = g.mean ? (float)((xd - g.mean[k]) / g.sdev[k]) : (float)xd;
        g.sv.xs[(size_t)k * g.sv.Bp + r0 + r] = x;
      }
      if (k < g.A) {
        xv = g.ra[sl * g.A + k];
        g.sv.xa[(size_t)k * g.sv.Bp + r0 + r] = xv;
      }
    }
    xs[idx] = x;
    xa[idx] = xv;
  }
  __syncthreads();
  SB_STAMP(1);
  {  // L1: online state branch | online action branch
    const SbOp ops[2] = {sb_op(xs, g.S, P + g.cWs, g.CH1, g.CH1, P + g.cbs, SB_ELU, cat),
                         sb_op(xa, g.A, P + g.cWa, g.CH1, g.CH1, P + g.cba, SB_ELU,
                               cat + 4 * g.CH1)};
    const bool th[2] = {false, false};
    sb_level<2>(ops, th, red);
  }
  SB_STAMP(2);
  // L2: online critic hidden (networks.py:154-156); L3: q = h Wo + bo
  sb_dense1(sb_op(cat, 2 * g.CH1, P + g.cWh, g.CH2, g.CH2, P + g.cbh, SB_ELU, h), red);
  SB_STAMP(3);
  sb_thin1(sb_op(h, g.CH2, P + g.cWo, 1, 1, P + g.cbo, SB_NONE, col), false, false, red);
  SB_STAMP(4);
  // ---- critic backward per unit dQ (networks.py:136's gradient, dQ = -(2/B)(y - q)
  // applied by the weight-gradient kernel): gh = Wo * elu'(h); u = gh . Wh^T * elu'(cat)
  for (int idx = tid; idx < 4 * g.CH2; idx += SB_NT)
    gh[idx] = __fmul_rn(P[g.cWo + (idx >> 2)], elu_grad_factor(h[idx]));
  __syncthreads();
  SB_STAMP(8);
  // L7 (Wh^T read from its row-major shadow)
  sb_dense1(sb_op(gh, g.CH2, GLB(g.whT), 2 * g.CH1, 2 * g.CH1, nullptr, SB_AUX, u, cat), red);
  SB_STAMP(9);
  if (tid < valid) g.sv.q[r0 + tid] = col[tid];
  sb_save(g.sv.cat, g.sv.Bp, 2 * g.CH1, cat, r0);
  sb_save(g.sv.dcat, g.sv.Bp, 2 * g.CH1, u, r0);
  sb_save(g.sv.h, g.sv.Bp, g.CH2, h, r0);
  sb_save(g.sv.dhp, g.sv.Bp, g.CH2, gh, r0);
  SB_STAMP_SYNC(10);
}

__global__ __launch_bounds__(SB_NT) void sb_phase3_kernel(SbArgs g) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  if (blockIdx.x % g.xstride) return;
  const int wg = blockIdx.x / g.xstride;
  const int r0 = wg * SB_R;
  const int valid = min(SB_R, g.B - r0);
  const int LX = g.LX, LW = g.LW;
  lds_f* red = LDS(sm);
  lds_f* xs = red + SB_RED + 2 * SB_BIAS;  // [LX][4]
  lds_f* o = xs + 4 * LX;
  lds_f* mu = o + 4 * LX;
  lds_f* dz3 = mu + 4 * LX;
  lds_f* h1 = dz3 + 4 * LX;    // [LW][4]
  lds_f* h2 = h1 + 4 * LW;
  lds_f* cat = h2 + 4 * LW;    // critic concat at (s, mu); later dz1
  lds_f* dh = cat + 4 * LW;    // dhp2, later dz2
  const glb_f* P = GLB(g.theta);
  SB_STAMP(32);

  if (wg == 0 && tid == 0) sb_alpha_and_advance(g.pw, g.alpha, g.lr_a, g.b1, g.b2);
  // phase 1 saved the (scaled) rows and the actor's forward on them
  // (networks.py:51-63): h1, h2, o; mu = scale o (ddpg.py:106)
  {
    const int Bp = g.sv.Bp;
    auto ld = [&](lds_f* dst, const float* src, int cols, int ld_cols) {
      for (int idx = tid; idx < 4 * ld_cols; idx += SB_NT) {
        const int k = idx >> 2, r = idx & 3;
        dst[idx] = (r < valid && k < cols) ? src[(size_t)k * Bp + r0 + r] : 0.f;
      }
    };
    ld(xs, g.sv.xs, g.S, LX);
    if (g.A != 1) {  // A == 1: phase 1 formed the actor backward per unit dz3
      ld(h1, g.sv.h1, g.AH1, g.AH1);
      ld(h2, g.sv.h2, g.AH2, g.AH2);
    }
    for (int idx = tid; idx < 4 * LX; idx += SB_NT) {
      const int k = idx >> 2, r = idx & 3;
      const float v = (r < valid && k < g.A) ? g.sv.o[(size_t)k * Bp + r0 + r] : 0.f;
      o[idx] = v;
      mu[idx] = __fmul_rn(v, g.scale);
    }
  }
  __syncthreads();
  SB_STAMP(33);
  {  // L1: critic state branch at s | action branch at mu (the updated critic)
    const SbOp ops[2] = {
        sb_op(xs, g.S, P + g.cWs, g.CH1, g.CH1, P + g.cbs, SB_ELU, cat),
        sb_op(mu, g.A, P + g.cWa, g.CH1, g.CH1, P + g.cba, SB_ELU, cat + 4 * g.CH1)};
    const bool th[2] = {false, false};
    sb_level<2>(ops, th, red);
  }
  SB_STAMP(37);
  // L5: dhp2 = Wo * elu'(h')  (updated critic, grad_ys = 1, networks.py:143);
  // L6: dca = dhp2 . Wh[CH1:]^T * elu'(ca), in place over ca
  sb_dense1(sb_op(cat, 2 * g.CH1, P + g.cWh, g.CH2, g.CH2, P + g.cbh, SB_POST2, dh, nullptr,
                  P + g.cWo),
            red);
  SB_STAMP(38);
  sb_dense1(sb_op(dh, g.CH2, GLB(g.whT) + g.CH1, 2 * g.CH1, g.CH1, nullptr, SB_AUX,
                  cat + 4 * g.CH1, cat + 4 * g.CH1),
            red);
  SB_STAMP(39);
  // L7: da = dca . Wa^T -> dz3 (scratch), then dz3 = ((-da) * scale) * (1 - o^2), masked
  sb_thin1(sb_op(cat + 4 * g.CH1, g.CH1, P + g.cWa, g.CH1, g.A, nullptr, SB_NONE, dz3), true,
           false, red);
  for (int idx = tid; idx < 4 * g.A; idx += SB_NT) {
    const float ov = o[idx];
    const float dy = __fmul_rn(-dz3[idx], g.scale);
    dz3[idx] = (idx & 3) < valid ? __fmul_rn(dy, __fsub_rn(1.f, __fmul_rn(ov, ov))) : 0.f;
  }
  __syncthreads();
  if (g.A == 1) {
    sb_save(g.sv.dz3, g.sv.Bp, g.A, dz3, r0);
    SB_STAMP_SYNC(42);
    return;
  }
  // ---- actor backward (networks.py:44)
  // dz2 = dz3 . W3^T * elu'(h2) -> dh   (K = A is tiny: one thread per output)
  for (int idx = tid; idx < 4 * g.AH2; idx += SB_NT) {
    const int n = idx >> 2, r = idx & 3;
    float v = 0.f;
    for (int a = 0; a < g.A; ++a) v = fmaf(dz3[a * 4 + r], P[g.aW3 + (size_t)n * g.A + a], v);
    dh[idx] = __fmul_rn(v, elu_grad_factor(h2[idx]));
  }
  __syncthreads();
  SB_STAMP(40);
  // L8: dz1 = dz2 . W2^T * elu'(h1) -> cat
  sb_dense1(sb_op(dh, g.AH2, GLB(g.w2T), g.AH1, g.AH1, nullptr, SB_AUX, cat, h1), red);
  SB_STAMP(41);
  sb_save(g.sv.dz1, g.sv.Bp, g.AH1, cat, r0);
  sb_save(g.sv.dz2, g.sv.Bp, g.AH2, dh, r0);
  sb_save(g.sv.dz3, g.sv.Bp, g.A, dz3, r0);
  SB_STAMP_SYNC(42);
}

// Action selection (ddpg.py:68-70, actor.predict at B = 1 .. 64): the whole
// actor forward in one launch.  The states travel in the kernel arguments
// (no upload), the scaler is applied in fp64 on device, and mu = scale *
// tanh(elu(elu(s W1 + b1) W2 + b2) W3) is written straight to pinned host
// memory (no download launch); one workgroup per 4 rows.
constexpr int SB_PRED_MAX = 256;  // floats of state in the kernel arguments
constexpr int SB_PRED_BLOCKS = (SB_PRED_MAX + SB_R - 1) / SB_R;  // at most (S >= 1)
struct SbPredIn {
  float s[SB_PRED_MAX];
};
// done (or null): each block, once its actions are visible to the host,
// stores seq to done[blockIdx.x] (pinned coherent memory) -- the host polls
// those words instead of waiting for the kernel's completion signal.
__global__ __launch_bounds__(SB_NT) void sb_actor_predict_kernel(SbArgs g, const float* base,
                                                                 SbPredIn in, float* out,
                                                                 unsigned* done, unsigned seq) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x;
  const int r0 = blockIdx.x * SB_R;
  const int valid = min(SB_R, g.B - r0);
  const int LX = g.LX, LW = g.LW;
  lds_f* red = LDS(sm);
  lds_f* xs = red + SB_RED + 2 * SB_BIAS;  // [LX][4]
  lds_f* o = xs + 4 * LX;
  lds_f* h1 = o + 4 * LX;  // [LW][4]
  lds_f* h2 = h1 + 4 * LW;
  const glb_f* P = GLB(base);
  for (int idx = tid; idx < 4 * LX; idx += SB_NT) {
    const int k = idx >> 2, r = idx & 3;
    float x = 0.f;
    // states arrive preprocessed (the caller's preprocess_input): no scaler here
    if (r < valid && k < g.S) x = in.s[(r0 + r) * g.S + k];
    xs[idx] = x;
  }
  __syncthreads();
  sb_dense1(sb_op(xs, g.S, P + g.aW1, g.AH1, g.AH1, P + g.ab1, SB_ELU, h1), red);
  sb_dense1(sb_op(h1, g.AH1, P + g.aW2, g.AH2, g.AH2, P + g.ab2, SB_ELU, h2), red);
  sb_thin1(sb_op(h2, g.AH2, P + g.aW3, g.A, g.A, nullptr, SB_NONE, o), false, true, red);
  for (int idx = tid; idx < 4 * g.A; idx += SB_NT) {
    const int a = idx >> 2, r = idx & 3;
    if (r < valid) out[(size_t)(r0 + r) * g.A + a] = __fmul_rn(o[idx], g.scale);
  }
  if (done) {
    __threadfence_system();  // this thread's actions written back to host memory
    __syncthreads();
    if (tid == 0) __hip_atomic_store(done + blockIdx.x, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}



// Weight gradients of one network over the whole batch (one ordered fp32
// sum over b per element, no partial slabs), TF ApplyAdam with this step's
// alpha, soft update of the target, and the transposed shadow of the dX
// weight.  net: 0 actor, 1 critic; the critic call also finalises the step
// stats.  A block owns a TK x TN tile of one tensor; its X and dY rows are
// staged through LDS 64 batch rows at a time by coalesced loads (round 6:
// before, every lane streamed its own dY row from global memory, 64 lines
// per load instruction), and thread (k, n) sums its products over b in
// order from LDS; the Adam state is loaded first so that its round trip
// overlaps the gradient's.
constexpr int SB_GC = 64;  // batch rows per staged chunk (16 float4s per tile row)
constexpr int SB_GLD = SB_GC + 4;  // LDS row stride (floats): lanes on different rows
                                   // read 16-B slots 4 banks apart, conflict-free
constexpr int SB_GROWS = SB_GT + 1;  // tile rows TK + TN <= 257 (TK * TN = SB_GT, TN <= 64)
constexpr int SB_GSJ = (SB_GROWS * 16 + SB_GT - 1) / SB_GT;  // staged float4s per thread
// mode 0: gradient + Adam + soft update (+ stats), one launch.  A step with
// a communicator (data parallelism at small batches) splits it around the
// RCCL sum of the gradient buffer: mode 1 computes and stores this rank's
// gradient only (the critic call stores this rank's {max Q, loss share} to
// g.stats for the all-gather, no running sums); mode 2 reads the summed
// gradient back and applies Adam, the soft update and the shadow.
//
// The critic's call forms dQ = -((1/B) * (2 * (y - q))) per row (the MSE
// gradient, networks.py:136, from phase 1's saved q and TD target) into LDS
// first; its tensors' saved output gradients are per unit dQ (sdq), scaled
// by dQ[b] as they are read.  The actor's call at A == 1 does the same with
// phase 3's dz3 (its dz1 / dz2 saved per unit dz3 by phase 1).  Its block 0 also forms the step stats: loss
// partials and max Q per 4-row group in row order, then summed in group order.
constexpr int SB_MAXB = 512;  // rows of the small path (sb_setup's sb_max_b)
__global__ __launch_bounds__(SB_GT) void sb_wgrad_adam_kernel(SbArgs g, SbGradTab tab, int net,
                                                              int nslab, int mode) {
#ifdef DDPG_SB_STAMPS
  const int sbase = net == 1 ? 48 : 56;
#endif
  SB_STAMP(sbase);
  __shared__ float sp[2][SB_MAXB / SB_R];
  __shared__ __attribute__((aligned(16))) float stg[SB_GROWS * SB_GLD];
  const bool crit = net == 1 && mode != 2;  // grid-uniform
  // the actor's call at A == 1: its saved output gradients are per unit dz3
  const bool act1 = net == 0 && mode != 2 && g.A == 1;
  int ti = 0;
#pragma unroll
  for (int i = 1; i < SB_MAXT; ++i)
    if (i < tab.n && (int)blockIdx.x >= tab.t[i].tile0) ti = i;
  const SbGradT T = tab.t[ti];
  const int local = blockIdx.x - T.tile0;
  const int ntn = (T.N + T.TN - 1) / T.TN;
  const int tid = threadIdx.x;
  const int kl = tid / T.TN, nl = tid - kl * T.TN;
  const int k = (local / ntn) * T.TK + kl, n = (local % ntn) * T.TN + nl;
  const bool ok = k < T.K && n < T.N;
  const int kc = min(k, T.K - 1), nc = min(n, T.N - 1);
  const size_t i = (size_t)T.off + (size_t)kc * T.N + nc;
  float m0 = 0.f, v0 = 0.f, p0 = 0.f, t0 = 0.f;
  if (mode != 1) {
    m0 = g.adam_m[i];
    v0 = g.adam_v[i];
    p0 = g.theta[i];
    t0 = g.target[i];
  }
  // X rows [k0, k0 + TK) and dY rows [n0, n0 + TN) of the tile, SB_GC batch
  // rows at a time, staged into LDS by coalesced 16-B loads (the dQ / dz3
  // scaling applied there), then each thread's ordered sum over b from LDS
  const int k0 = (local / ntn) * T.TK, n0 = (local % ntn) * T.TN;
  const int rows = T.TK + T.TN;
  const bool sdq = (crit || act1) && T.sdq;
  const int nB = mode == 2 ? 0 : g.B;
  lds_f* const st = LDS(stg);
  float gv = mode == 2 ? g.grad[i] : 0.f;
  for (int b0 = 0; b0 < nB; b0 += SB_GC) {
    const int nq4 = (min(SB_GC, nB - b0) + 3) >> 2;  // float4s per staged row
    // a thread stages quad qd of every row it touches (SB_GT is a multiple
    // of 16): its rows' per-row scale comes from one float4 of the saves,
    // loaded with the tile in the same round trip
    const int qd = tid & 15, bq = b0 + 4 * qd;
    f32x4 sa = f32x4{0.f, 0.f, 0.f, 0.f}, sb = sa;
    if ((crit || act1) && qd < nq4) {
      if (crit) {
        sa = *reinterpret_cast<const f32x4*>(g.sv.y + bq);
        sb = *reinterpret_cast<const f32x4*>(g.sv.q + bq);
      } else {
        sa = *reinterpret_cast<const f32x4*>(g.sv.dz3 + bq);
      }
    }
    f32x4 v[SB_GSJ];
#pragma unroll
    for (int j = 0; j < SB_GSJ; ++j) {  // every load in flight before the stores
      const int f = tid + SB_GT * j, r = f >> 4, q = f & 15;
      v[j] = f32x4{1.f, 1.f, 1.f, 1.f};
      if (r < rows && q < nq4) {
        const float* src = nullptr;
        if (r < T.TK)
          src = T.X ? T.X + (size_t)min(k0 + r, T.K - 1) * T.ldx : nullptr;
        else
          src = T.dY ? T.dY + (size_t)min(n0 + r - T.TK, T.N - 1) * T.ldy : nullptr;
        if (src) v[j] = *reinterpret_cast<const f32x4*>(src + b0 + 4 * q);
      }
    }
    // dQ = -((1/B) * (2 * (y - q))) (critic; networks.py:136) or dz3
    // (actor, A == 1) per row, 0 past B
    f32x4 d;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      d[e] = bq + e >= nB ? 0.f
             : crit       ? -__fmul_rn(g.inv_b, __fmul_rn(2.f, __fsub_rn(sa[e], sb[e])))
                          : sa[e];
    if (crit && blockIdx.x == 0 && tid < 16 && qd < nq4) {
      // step stats of row group bq / 4: loss partial and max Q, in row order
      float lsum = 0.f, qmax = -INFINITY;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (bq + e < nB) {
          const float dd = __fsub_rn(sa[e], sb[e]);
          lsum += __fmul_rn(dd, dd);
          qmax = fmaxf(qmax, sb[e]);
        }
      sp[0][bq >> 2] = lsum;
      sp[1][bq >> 2] = qmax;
    }
#pragma unroll
    for (int j = 0; j < SB_GSJ; ++j) {
      const int f = tid + SB_GT * j, r = f >> 4;
      if (r < rows && qd < nq4) {
        f32x4 w = v[j];
        if (sdq && r >= T.TK) {
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = __fmul_rn(d[e], w[e]);
        }
        *reinterpret_cast<lds_v4*>(st + r * SB_GLD + 4 * qd) = w;
      }
    }
    __syncthreads();
    const lds_v4* xr = reinterpret_cast<const lds_v4*>(st + kl * SB_GLD);
    const lds_v4* dr = reinterpret_cast<const lds_v4*>(st + (T.TK + nl) * SB_GLD);
    for (int q = 0; q < nq4; ++q) {
      const f32x4 xv = xr[q], dv = dr[q];
#pragma unroll
      for (int e = 0; e < 4; ++e) gv = (b0 + 4 * q + e < nB) ? fmaf(xv[e], dv[e], gv) : gv;
    }
    __syncthreads();  // the next chunk's stores reuse the tile
  }
  SB_STAMP(sbase + 1);
  if (ok && mode == 1) g.grad[i] = gv;
  if (ok && mode != 1) {
    const float alpha = g.alpha[net];
    const float omb1 = __fsub_rn(1.f, g.b1), omb2 = __fsub_rn(1.f, g.b2);
    const float m = __fadd_rn(m0, __fmul_rn(__fsub_rn(gv, m0), omb1));
    const float v = __fadd_rn(v0, __fmul_rn(__fsub_rn(__fmul_rn(gv, gv), v0), omb2));
    const float p =
        __fsub_rn(p0, __fdiv_rn(__fmul_rn(m, alpha), __fadd_rn(__fsqrt_rn(v), g.eps)));
    g.adam_m[i] = m;
    g.adam_v[i] = v;
    g.theta[i] = p;
    if (mode == 0) g.grad[i] = gv;
    g.target[i] = __fadd_rn(__fmul_rn(p, g.tau), __fmul_rn(t0, g.omt));
    if (ti == tab.shadow) tab.sh[(size_t)n * T.K + k] = p;
  }
  SB_STAMP(sbase + 2);
  if (crit && blockIdx.x == 0 && threadIdx.x == 0) {
    float ls = 0.f, qm = -INFINITY;
    for (int w = 0; w < nslab; ++w) {  // in group order
      ls += sp[0][w];
      qm = fmaxf(qm, sp[1][w]);
    }
    const float loss = __fmul_rn(ls, g.inv_b);
    g.stats[0] = qm;
    g.stats[1] = loss;
    if (mode == 0) {  // mode 1: the data-parallel stats reduction keeps the sums
      g.acc[0] += (double)qm;
      g.acc[1] += (double)loss;
      g.acc[2] += 1.0;
    }
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
