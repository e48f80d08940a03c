// Memory-bound kernels of the learner step (gfx950): replay gather (K8),
// thin-head finalisers (K1/K2/K4 epilogue reductions, K9 TD target), critic
// head backward, split-K / partial-sum reduction, TF ApplyAdam (K6) and the
// tau soft update (K7).  All fp32; rounding mirrors the TF 1.3 CPU kernels
// (no FMA contraction where TF evaluates separate multiplies and adds).
#pragma once
#include "common.h"

namespace ddpg {

// ---------------------------------------------------------------- K8 gather
// replay_buffer.py:41-45 (np.array stacking of the sampled tuples), from a
// device-resident SoA ring.  One wave per row; lanes stride the features.
// A float64 ring (rsd / rs2d / rrd non-null) keeps the states and rewards the
// reference stores; they are rounded to fp32 here, once, like TF's feed_dict.
// Optional scaler (networks.py:65-69, ddpg.py:184-189), applied to replay
// rows only: fp32((double(x) - mean) / scale).
__global__ void gather_rows_kernel(const int* __restrict__ slots, int B,
                                   const float* __restrict__ rs, const float* __restrict__ ra,
                                   const float* __restrict__ rr, const float* __restrict__ rt,
                                   const float* __restrict__ rs2, const double* __restrict__ rsd,
                                   const double* __restrict__ rs2d,
                                   const double* __restrict__ rrd, int S, int A,
                                   float* __restrict__ s, float* __restrict__ s2, int lds,
                                   float* __restrict__ a, int lda, float* __restrict__ r,
                                   float* __restrict__ t, const double* __restrict__ mean,
                                   const double* __restrict__ scale, __bf16* __restrict__ sh,
                                   __bf16* __restrict__ s2h, long long hps, int hnp) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  // fp32 ring with 4-aligned rows: 16-B accesses (4 features per lane)
  const bool v4 = !rsd && (S & 3) == 0 && (lds & 3) == 0 && (hps & 3) == 0;
  for (int b = wave; b < B; b += nwaves) {
    const size_t slot = (size_t)slots[b];
    if (v4) {
      for (int j = 4 * lane; j < S; j += 256) {
        const size_t e = slot * S + j;
        float4 x = *reinterpret_cast<const float4*>(rs + e);
        float4 x2 = *reinterpret_cast<const float4*>(rs2 + e);
        if (mean) {
          float* px = &x.x;
          float* px2 = &x2.x;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            px[q] = (float)(((double)px[q] - mean[j + q]) / scale[j + q]);
            px2[q] = (float)(((double)px2[q] - mean[j + q]) / scale[j + q]);
          }
        }
        *reinterpret_cast<float4*>(s + (size_t)b * lds + j) = x;
        *reinterpret_cast<float4*>(s2 + (size_t)b * lds + j) = x2;
        if (sh) store_twin4(sh + (size_t)b * lds + j, hps, hnp, x);
        if (s2h) store_twin4(s2h + (size_t)b * lds + j, hps, hnp, x2);
      }
    } else
    for (int j = lane; j < S; j += 64) {
      const size_t e = slot * S + j;
      float x, x2;
      if (rsd) {
        const double xd = rsd[e], x2d = rs2d[e];
        x = mean ? (float)((xd - mean[j]) / scale[j]) : (float)xd;
        x2 = mean ? (float)((x2d - mean[j]) / scale[j]) : (float)x2d;
      } else {
        x = rs[e];
        x2 = rs2[e];
        if (mean) {
          x = (float)(((double)x - mean[j]) / scale[j]);
          x2 = (float)(((double)x2 - mean[j]) / scale[j]);
        }
      }
      s[(size_t)b * lds + j] = x;
      s2[(size_t)b * lds + j] = x2;
      if (sh) store_twin1(sh + (size_t)b * lds + j, hps, hnp, x);
      if (s2h) store_twin1(s2h + (size_t)b * lds + j, hps, hnp, x2);
    }
    for (int j = lane; j < A; j += 64) a[(size_t)b * lda + j] = ra[slot * A + j];
    if (lane == 0) {
      r[b] = rrd ? (float)rrd[slot] : rr[slot];
      t[b] = rt[slot];
    }
  }
}

// The same for an fp32 ring with 4-aligned S <= 64 * QI and A <= 64, 16 rows
// per block: the rows' slots (in pinned host memory when read in place) come
// in one coalesced read by 16 lanes and are parked in LDS -- one host read per
// 16 rows instead of one per row -- and each wave copies 4 rows at once (lane:
// row lane >> 4, feature quads lane & 15 + 16 u), every load of its 4 rows in
// flight together.  Same values as gather_rows_kernel.
template <int QI>
__global__ __launch_bounds__(256) void gather_rows16_kernel(
    const int* __restrict__ slots, int B, const float* __restrict__ rs,
    const float* __restrict__ ra, const float* __restrict__ rr, const float* __restrict__ rt,
    const float* __restrict__ rs2, int S, int A, float* __restrict__ s, float* __restrict__ s2,
    int lds, float* __restrict__ a, int lda, float* __restrict__ r, float* __restrict__ t,
    const double* __restrict__ mean, const double* __restrict__ scale, __bf16* __restrict__ sh,
    __bf16* __restrict__ s2h, long long hps, int hnp) {
  __shared__ int sl[16];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int b0 = blockIdx.x * 16;
  if (tid < 16) sl[tid] = b0 + tid < B ? slots[b0 + tid] : 0;
  __syncthreads();
  const int i = 4 * wave + (lane >> 4), q = lane & 15, b = b0 + i;
  if (b >= B) return;
  const size_t slot = (size_t)sl[i];
  float4 x[QI], x2[QI];
#pragma unroll
  for (int u = 0; u < QI; ++u) {
    const int j = 4 * (q + 16 * u);
    x[u] = x2[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (j < S) {
      x[u] = *reinterpret_cast<const float4*>(rs + slot * S + j);
      x2[u] = *reinterpret_cast<const float4*>(rs2 + slot * S + j);
    }
  }
  float av[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) av[u] = q + 16 * u < A ? ra[slot * A + q + 16 * u] : 0.f;
  float rv = 0.f, tv = 0.f;
  if (q == 0) {
    rv = rr[slot];
    tv = rt[slot];
  }
#pragma unroll
  for (int u = 0; u < QI; ++u) {
    const int j = 4 * (q + 16 * u);
    if (j >= S) continue;
    if (mean) {
      float* px = &x[u].x;
      float* px2 = &x2[u].x;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        px[e] = (float)(((double)px[e] - mean[j + e]) / scale[j + e]);
        px2[e] = (float)(((double)px2[e] - mean[j + e]) / scale[j + e]);
      }
    }
    *reinterpret_cast<float4*>(s + (size_t)b * lds + j) = x[u];
    *reinterpret_cast<float4*>(s2 + (size_t)b * lds + j) = x2[u];
    if (sh) store_twin4(sh + (size_t)b * lds + j, hps, hnp, x[u]);
    if (s2h) store_twin4(s2h + (size_t)b * lds + j, hps, hnp, x2[u]);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (q + 16 * u < A) a[(size_t)b * lda + q + 16 * u] = av[u];
  if (q == 0) {
    r[b] = rv;
    t[b] = tv;
  }
}

// ---------------------------------------------------------------- thin heads
// actor output: o = tanh(sum_t part[t][b][a]); mu = o * scale  (networks.py:59-61)
// Sum of NT strided slab values in slab order (z = ((v0 + v1) + v2) + ...),
// with the loads of up to 8 slabs in flight at once: a plain loop over a
// runtime count made hipcc wait for each load before issuing the next, one
// memory round trip per slab.
DDPG_DEV float slab_sum(const float* __restrict__ p, int NT, size_t stride, float z) {
  for (int t0 = 0; t0 < NT; t0 += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = t0 + i < NT ? p[(size_t)(t0 + i) * stride] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (t0 + i < NT) z += v[i];
  }
  return z;
}

__global__ void actor_out_kernel(const float* __restrict__ part, int NT, int B, int A,
                                 float scale, float* __restrict__ o, float* __restrict__ mu,
                                 int ld) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  const int b = i / A, a = i - b * A;
  const float z = slab_sum(part + (size_t)b * A + a, NT, (size_t)B * A, 0.f);
  const float ov = tanhf(z);
  if (o) o[(size_t)b * ld + a] = ov;
  if (mu) mu[(size_t)b * ld + a] = __fmul_rn(ov, scale);
}

// critic output q = sum_t qpart[t][b] + bo, then by mode:
//   mode 0: q only;  mode 1: TD target y = t ? r : r + gamma*q  (ddpg.py:92-100)
__global__ void critic_q_kernel(const float* __restrict__ qpart, int NT, int B,
                                const float* __restrict__ bo, float* __restrict__ q,
                                int mode, const float* __restrict__ r,
                                const float* __restrict__ t, float gamma,
                                float* __restrict__ y) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  float z = slab_sum(qpart + b, NT, (size_t)B, 0.f);
  z = __fadd_rn(z, bo[0]);
  if (q) q[b] = z;
  if (mode == 1) y[b] = (t[b] != 0.f) ? r[b] : __fadd_rn(r[b], __fmul_rn(gamma, z));
}

// Critic train head (networks.py:136, tflearn.mean_square): q = sum + bo,
// L = mean((y - q)^2), dq = -((1/B) * (2 * (y - q))).  One row per thread,
// 256 rows per block; each block leaves its {sum (y-q)^2, max q} partial in
// lpart, and the critic-head kernel that runs next folds them (stats_fold).
// inv_b is 1/B_global; the loss is this rank's share of the mean.
// td (fused learner step): the TD target y = r + gamma (1 - t) Q'(s2, mu') of
// critic_q_kernel mode 1 is formed here from the target critic's partials
// (same sums, same ops) and stored to y, one launch fewer.
struct TdTarget {
  const float* qpart;  // target critic head partials, null: read y
  int NT;
  const float* bo;
  const float* r;
  const float* t;
  float gamma;
};

__global__ __launch_bounds__(256) void critic_loss_kernel(
    const float* __restrict__ qpart, int NT, int B, const float* __restrict__ bo,
    float* __restrict__ y, float inv_b, float* __restrict__ q, float* __restrict__ dq,
    float2* __restrict__ lpart, TdTarget td) {
  __shared__ float s_sum[256];
  __shared__ float s_max[256];
  const int b = blockIdx.x * 256 + threadIdx.x;
  float lsum = 0.f, lmax = -INFINITY;
  if (b < B) {
    float yb;
    if (td.qpart) {
      float zt = slab_sum(td.qpart + b, td.NT, (size_t)B, 0.f);
      zt = __fadd_rn(zt, td.bo[0]);
      yb = (td.t[b] != 0.f) ? td.r[b] : __fadd_rn(td.r[b], __fmul_rn(td.gamma, zt));
      y[b] = yb;
    } else {
      yb = y[b];
    }
    float z = 0.f;  // slab order; loads issued ahead of the adds
#pragma unroll 8
    for (int tt = 0; tt < NT; ++tt) z += qpart[(size_t)tt * B + b];
    z = __fadd_rn(z, bo[0]);
    q[b] = z;
    const float d = __fsub_rn(yb, z);
    dq[b] = -__fmul_rn(inv_b, __fmul_rn(2.f, d));
    lsum = __fmul_rn(d, d);
    lmax = z;
  }
  s_sum[threadIdx.x] = lsum;
  s_max[threadIdx.x] = lmax;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      s_sum[threadIdx.x] += s_sum[threadIdx.x + w];
      s_max[threadIdx.x] = fmaxf(s_max[threadIdx.x], s_max[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) lpart[blockIdx.x] = make_float2(s_sum[0], s_max[0]);
}

// Per-step stats {q_max, loss} from the loss kernel's block partials (fixed
// order), and their running sums (acc may be null).  One thread.
DDPG_DEV void stats_fold(const float2* __restrict__ lpart, int nlp, float inv_b,
                         float* __restrict__ stats, double* __restrict__ acc) {
  float sum = 0.f, mx = -INFINITY;
  for (int i0 = 0; i0 < nlp; i0 += 8) {  // in order, 8 loads in flight
    float2 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i0 + i < nlp ? lpart[i0 + i] : make_float2(0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i0 + i < nlp) {
        sum += v[i].x;
        mx = fmaxf(mx, v[i].y);
      }
  }
  const float loss = __fmul_rn(sum, inv_b);
  stats[0] = mx;
  stats[1] = loss;
  if (acc) {
    acc[0] += (double)mx;
    acc[1] += (double)loss;
    acc[2] += 1.0;
  }
}

// Critic head backward (gradients_1 of networks.py:137):
//   dh[b,j] = dq[b]*Wo[j];  dh_pre = EluGrad(dh, h);  dWo[j] = sum_b h*dq;
//   dbh[j] = sum_b dh_pre;  dbo = sum_b dq.   Partial sums per row chunk.
__global__ void critic_head_bwd_kernel(const float* __restrict__ h, int ldh,
                                       const float* __restrict__ dq,
                                       const float* __restrict__ Wo, int B, int H2,
                                       int rows_per_chunk, float* __restrict__ dh_pre,
                                       int ld_dh, float* __restrict__ part_dWo,
                                       float* __restrict__ part_dbh,
                                       float* __restrict__ part_dbo,
                                       const float2* __restrict__ lpart, int nlp, float inv_b,
                                       float* __restrict__ stats, double* __restrict__ acc) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = blockIdx.y;
  const int b0 = chunk * rows_per_chunk;
  const int b1 = min(B, b0 + rows_per_chunk);
  if (j < H2) {
    const float w = Wo[j];
    float sw = 0.f, sb = 0.f;
    for (int b = b0; b < b1; ++b) {
      const float hv = h[(size_t)b * ldh + j];
      const float d = dq[b];
      const float dp = __fmul_rn(__fmul_rn(d, w), elu_grad_factor(hv));
      dh_pre[(size_t)b * ld_dh + j] = dp;
      sw = fmaf(hv, d, sw);
      sb += dp;
    }
    part_dWo[(size_t)chunk * H2 + j] = sw;
    part_dbh[(size_t)chunk * H2 + j] = sb;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float s = slab_sum(dq + b0, b1 - b0, 1, 0.f);  // in row order, 8 loads in flight
    part_dbo[chunk] = s;
    if (chunk == 0) stats_fold(lpart, nlp, inv_b, stats, acc);
  }
}

// The same on column quads (H2, ldh, ld_dh % 4 == 0): a block covers 64
// column quads x 4 row groups of a chunk (16-B loads / stores, several rows
// in flight per thread), the groups' partial sums combined in LDS in a fixed
// order; also writes dh_pre's bf16 twin (dtw, tnp planes tps apart) for the
// bf16-operand GEMMs that read it (dh_pre may be null: twin only).
__global__ __launch_bounds__(256) void critic_head_bwd4_kernel(
    const float* __restrict__ h, int ldh, const float* __restrict__ dq,
    const float* __restrict__ Wo, int B, int H2, int rows_per_chunk, float* __restrict__ dh_pre,
    int ld_dh, float* __restrict__ part_dWo, float* __restrict__ part_dbh,
    float* __restrict__ part_dbo, __bf16* __restrict__ dtw, long long tps, int tnp,
    const float2* __restrict__ lpart, int nlp, float inv_b, float* __restrict__ stats,
    double* __restrict__ acc) {
  __shared__ float4 red[2][3][64];
  const int cq = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int j = 4 * (blockIdx.x * 64 + cq);
  const int chunk = blockIdx.y;
  const int b0 = chunk * rows_per_chunk;
  const int b1 = min(B, b0 + rows_per_chunk);
  float4 sw = make_float4(0.f, 0.f, 0.f, 0.f), sb = sw;
  if (j < H2) {
    const float4 w = *reinterpret_cast<const float4*>(Wo + j);
    // 16 rows per batch, all loads in flight before the first use (one HBM
    // round trip per batch instead of one per 4 rows)
    constexpr int RB = 16;
    for (int bb = b0 + rg; bb < b1; bb += 4 * RB) {
    float4 hvs[RB];
    float ds[RB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int b = bb + 4 * i;
      hvs[i] = make_float4(0.f, 0.f, 0.f, 0.f);
      ds[i] = 0.f;
      if (b < b1) {
        hvs[i] = *reinterpret_cast<const float4*>(h + (size_t)b * ldh + j);
        ds[i] = dq[b];
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int b = bb + 4 * i;
      if (b >= b1) continue;
      const float4 hv = hvs[i];
      const float d = ds[i];
      float4 dp;
      dp.x = __fmul_rn(__fmul_rn(d, w.x), elu_grad_factor(hv.x));
      dp.y = __fmul_rn(__fmul_rn(d, w.y), elu_grad_factor(hv.y));
      dp.z = __fmul_rn(__fmul_rn(d, w.z), elu_grad_factor(hv.z));
      dp.w = __fmul_rn(__fmul_rn(d, w.w), elu_grad_factor(hv.w));
      if (dh_pre) *reinterpret_cast<float4*>(dh_pre + (size_t)b * ld_dh + j) = dp;
      if (dtw) store_twin4(dtw + (size_t)b * ld_dh + j, tps, tnp, dp);
      sw.x = fmaf(hv.x, d, sw.x);
      sw.y = fmaf(hv.y, d, sw.y);
      sw.z = fmaf(hv.z, d, sw.z);
      sw.w = fmaf(hv.w, d, sw.w);
      sb.x += dp.x;
      sb.y += dp.y;
      sb.z += dp.z;
      sb.w += dp.w;
    }
    }
  }
  if (rg > 0) {
    red[0][rg - 1][cq] = sw;
    red[1][rg - 1][cq] = sb;
  }
  __syncthreads();
  if (rg == 0 && j < H2) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      sw = make_float4(sw.x + red[0][q][cq].x, sw.y + red[0][q][cq].y, sw.z + red[0][q][cq].z,
                       sw.w + red[0][q][cq].w);
      sb = make_float4(sb.x + red[1][q][cq].x, sb.y + red[1][q][cq].y, sb.z + red[1][q][cq].z,
                       sb.w + red[1][q][cq].w);
    }
    *reinterpret_cast<float4*>(part_dWo + (size_t)chunk * H2 + j) = sw;
    *reinterpret_cast<float4*>(part_dbh + (size_t)chunk * H2 + j) = sb;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const float s = slab_sum(dq + b0, b1 - b0, 1, 0.f);  // in row order, 8 loads in flight
    part_dbo[chunk] = s;
    if (chunk == 0) stats_fold(lpart, nlp, inv_b, stats, acc);
  }
}

// dQ/da finaliser (networks.py:143 action half) + actor grad_ys
// (networks.py:44): da = sum_t part[t][b][a];
// dz3 = TanhGrad(o, (-da) * scale) = ((-da)*scale) * (1 - o*o).
__global__ void action_grad_kernel(const float* __restrict__ part, int NT, int B, int A,
                                   int ld_part_b /* rows stride inside a tile slab = B */,
                                   const float* __restrict__ o, int ld, float scale,
                                   float* __restrict__ da, float* __restrict__ dz3) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * A) return;
  const int b = i / A, a = i - b * A;
  const float g = slab_sum(part + (size_t)b * A + a, NT, (size_t)ld_part_b * A, 0.f);
  if (da) da[(size_t)b * ld + a] = g;
  if (dz3) {
    const float ov = o[(size_t)b * ld + a];
    const float dy = __fmul_rn(-g, scale);
    dz3[(size_t)b * ld + a] = __fmul_rn(dy, __fsub_rn(1.f, __fmul_rn(ov, ov)));
  }
}

// ---------------------------------------------------------------- reductions
// dst[i] = sum_k src[k * slab_stride + i], i < count  (deterministic order).
// Split-K weight-gradient slabs, bias column-sum partials and critic-head
// partials all have this shape.  blockIdx.y selects the segment.
struct ReduceSeg {
  const float* src;
  float* dst;
  long long slab_stride;  // floats between slabs
  long long count;
  int nslab;
  int vec4;               // count, stride and pointers allow float4
};
constexpr int MAX_SEGS = 12;
struct ReduceTable {
  ReduceSeg seg[MAX_SEGS];
  int nseg;
};

// Each block reduces EPB = 256 / SG elements (float4 or scalar) of one
// segment with SG slab groups (SG = 4, 2 or 1 by the slab count): thread
// group sg sums slabs sg, sg + SG, ... in order (eight loads in flight), and
// the groups are combined in LDS in a fixed order -- deterministic, and
// segments with few elements and many slabs (bias partials: 32 slabs of
// 1024, fused narrow weight-gradient partials: 32-128 slabs) still put 256
// threads on every 64 elements.  slab_partial / slab_groups are shared with
// the Adam pass that folds the reduction in (adam_reduce_kernel): both give
// the same sum, bit for bit.
template <class T>
DDPG_DEV T rs_add(T a, T b);
template <>
DDPG_DEV float rs_add(float a, float b) { return a + b; }
template <>
DDPG_DEV float4 rs_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__host__ __device__ inline int slab_groups(int nslab) { return nslab >= 4 ? 4 : (nslab >= 2 ? 2 : 1); }

// slabs sg, sg + SG, ... < nslab of element i, summed left to right
template <class T>
DDPG_DEV T slab_partial(const T* __restrict__ src, long long i, long long ss, int nslab, int sg,
                        int SG) {
  int k = sg;
  T acc = src[i + k * ss];
  k += SG;
  for (; k + 7 * SG < nslab; k += 8 * SG) {
    T x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = src[i + (k + u * SG) * ss];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = rs_add(acc, x[u]);
  }
  for (; k + 3 * SG < nslab; k += 4 * SG) {
    const T x0 = src[i + k * ss], x1 = src[i + (k + SG) * ss];
    const T x2 = src[i + (k + 2 * SG) * ss], x3 = src[i + (k + 3 * SG) * ss];
    acc = rs_add(rs_add(rs_add(rs_add(acc, x0), x1), x2), x3);
  }
  for (; k < nslab; k += SG) acc = rs_add(acc, src[i + k * ss]);
  return acc;
}

template <class T>
DDPG_DEV void reduce_seg(const T* __restrict__ src, T* __restrict__ dst, long long n,
                         long long ss, int nslab, T* part) {
  const int SG = slab_groups(nslab);
  const int EPB = 256 / SG;
  const int e = threadIdx.x % EPB, sg = threadIdx.x / EPB;
  for (long long i0 = (long long)blockIdx.x * EPB; i0 < n; i0 += (long long)gridDim.x * EPB) {
    const long long i = i0 + e;
    T acc{};
    if (i < n) acc = slab_partial(src, i, ss, nslab, sg, SG);
    if (sg > 0) part[(sg - 1) * 256 + e] = acc;
    __syncthreads();
    if (sg == 0 && i < n) {
      for (int q = 1; q < SG; ++q) acc = rs_add(acc, part[(q - 1) * 256 + e]);
      dst[i] = acc;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void reduce_slabs_kernel(ReduceTable tab) {
  __shared__ float4 part[3 * 256];
  const ReduceSeg g = tab.seg[blockIdx.y];
  if (g.vec4)
    reduce_seg<float4>(reinterpret_cast<const float4*>(g.src), reinterpret_cast<float4*>(g.dst),
                       g.count >> 2, g.slab_stride >> 2, g.nslab, part);
  else
    reduce_seg<float>(g.src, g.dst, g.count, g.slab_stride, g.nslab,
                      reinterpret_cast<float*>(part));
}

// ---------------------------------------------------------------- K6 Adam
// TF 1.3 ApplyAdam (use_nesterov = false), one flat pass per network:
//   alpha = lr * sqrt(1 - b2p) / (1 - b1p)
//   m += (g - m) * (1 - b1);  v += (g*g - v) * (1 - b2)
//   p -= (m * alpha) / (sqrt(v) + eps)
// The beta powers live on device (pw = {b1p, b2p}); advance_powers_kernel,
// launched after the pass, advances them (b1p *= b1, b2p *= b2), i.e. the
// AdamOptimizer._finish update (folding it into this kernel's last-arriving
// block was slower: profiles/r3/adam_adv_fold_ab.txt).
// tw (optional): the bf16 twin of p (tnp planes, tps elements apart), kept
// current for the bf16-operand GEMMs.
// tt (optional, fused learner step): the network's target parameters, soft-
// updated from the new p in the same pass (networks.py:34-37, the same fp32
// ops as soft_update_kernel; nothing reads the targets between this network's
// Adam step and the end of the step), ttw its twin.
// alpha = lr * sqrt(1 - b2p) / (1 - b1p) from a network's beta powers
DDPG_DEV float adam_alpha(const float* pw, float lr) {
  return __fdiv_rn(__fmul_rn(lr, __fsqrt_rn(__fsub_rn(1.f, pw[1]))), __fsub_rn(1.f, pw[0]));
}

// The fused learner step's beta-power bookkeeping, folded into its two Adam
// passes instead of a launch of its own at the end of the step (AdamHooks):
// the critic's pass (first) computes the actor's step size into a device slot
// and then advances the actor's powers -- nothing reads them until the next
// step; the actor's pass (second) takes its step size from that slot and
// advances the critic's powers, which the critic's pass has consumed.  Same
// values and ops as adam_alpha + advance_powers_kernel after both passes.
struct AdamHooks {
  const float* alpha_in;  // step size from here instead of pw
  float* pre_pw;          // block 0: *pre_alpha = alpha(pre_pw, pre_lr), then advance pre_pw
  float* pre_alpha;
  float pre_lr;
  float* adv_pw;          // block 0: advance adv_pw
};
DDPG_DEV void adam_hooks(const AdamHooks& h, float b1, float b2) {
  if (blockIdx.x || threadIdx.x) return;
  if (h.pre_pw) {
    *h.pre_alpha = adam_alpha(h.pre_pw, h.pre_lr);
    h.pre_pw[0] = __fmul_rn(h.pre_pw[0], b1);
    h.pre_pw[1] = __fmul_rn(h.pre_pw[1], b2);
  }
  if (h.adv_pw) {
    h.adv_pw[0] = __fmul_rn(h.adv_pw[0], b1);
    h.adv_pw[1] = __fmul_rn(h.adv_pw[1], b2);
  }
}

__global__ void adam_kernel(float* __restrict__ p, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ g, long long n,
                            const float* __restrict__ pw, float lr, float b1, float b2,
                            float eps, __bf16* __restrict__ tw, long long tps, int tnp,
                            float* __restrict__ tt, float tau, float omt,
                            __bf16* __restrict__ ttw, AdamHooks hk) {
  const float alpha = hk.alpha_in ? *hk.alpha_in : adam_alpha(pw, lr);
  adam_hooks(hk, b1, b2);
  const float omb1 = __fsub_rn(1.f, b1), omb2 = __fsub_rn(1.f, b2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 P = reinterpret_cast<float4*>(p)[i];
    float4 Mv = reinterpret_cast<float4*>(m)[i];
    float4 V = reinterpret_cast<const float4*>(v)[i];
    const float4 G = reinterpret_cast<const float4*>(g)[i];
    float* pp = &P.x;
    float* pm = &Mv.x;
    float* pv = &V.x;
    const float* pg = &G.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pm[k] = __fadd_rn(pm[k], __fmul_rn(__fsub_rn(pg[k], pm[k]), omb1));
      pv[k] = __fadd_rn(pv[k], __fmul_rn(__fsub_rn(__fmul_rn(pg[k], pg[k]), pv[k]), omb2));
      pp[k] = __fsub_rn(pp[k], __fdiv_rn(__fmul_rn(pm[k], alpha),
                                         __fadd_rn(__fsqrt_rn(pv[k]), eps)));
    }
    reinterpret_cast<float4*>(p)[i] = P;
    reinterpret_cast<float4*>(m)[i] = Mv;
    reinterpret_cast<float4*>(v)[i] = V;
    if (tw) store_twin4(tw + 4 * i, tps, tnp, P);
    if (tt) {
      float4 b = reinterpret_cast<float4*>(tt)[i];
      b.x = __fadd_rn(__fmul_rn(P.x, tau), __fmul_rn(b.x, omt));
      b.y = __fadd_rn(__fmul_rn(P.y, tau), __fmul_rn(b.y, omt));
      b.z = __fadd_rn(__fmul_rn(P.z, tau), __fmul_rn(b.z, omt));
      b.w = __fadd_rn(__fmul_rn(P.w, tau), __fmul_rn(b.w, omt));
      reinterpret_cast<float4*>(tt)[i] = b;
      if (ttw) store_twin4(ttw + 4 * i, tps, tnp, b);
    }
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    m[i] = __fadd_rn(m[i], __fmul_rn(__fsub_rn(g[i], m[i]), omb1));
    v[i] = __fadd_rn(v[i], __fmul_rn(__fsub_rn(__fmul_rn(g[i], g[i]), v[i]), omb2));
    p[i] = __fsub_rn(p[i], __fdiv_rn(__fmul_rn(m[i], alpha), __fadd_rn(__fsqrt_rn(v[i]), eps)));
    if (tw) store_twin1(tw + i, tps, tnp, p[i]);
    if (tt) {
      tt[i] = __fadd_rn(__fmul_rn(p[i], tau), __fmul_rn(tt[i], omt));
      if (ttw) store_twin1(ttw + i, tps, tnp, tt[i]);
    }
  }
}

// Adam with the network's gradient reduction folded in (no exchange between
// them: one rank, or no communicator).  The network's flat region is covered
// by segments: slab segments (the reduce table's, summed exactly as
// reduce_slabs_kernel sums them, the sum also stored to the flat gradient)
// and direct ones (the gradient already in place).  Per element the same
// ApplyAdam / soft-update / twin ops as adam_kernel, so the two forms agree
// bit for bit.  Blocks [blk0, blk0 + nblk) work on a segment.
struct AdamSeg {
  const float* src;
  long long off;    // flat index of the segment's first element
  long long count;
  long long slab_stride;
  int nslab, vec4, wg, blk0, nblk;
};
constexpr int ADAM_MAXSEG = 20;
struct AdamTable {
  AdamSeg seg[ADAM_MAXSEG];
  int nseg;
};
struct AdamArgs {
  float *p, *m, *v, *g;  // flat bases (index = flat element)
  const float* pw;
  float lr, b1, b2, eps;
  __bf16* tw;            // theta's twin (flat base) or null
  long long tps;
  int tnp;
  float* tt;             // targets (fused step) or null
  float tau, omt;
  __bf16* ttw;
  AdamHooks hk;
};

DDPG_DEV void adam_elem(float& p, float& m, float& v, float g, float alpha, float omb1, float omb2,
                        float eps) {
  m = __fadd_rn(m, __fmul_rn(__fsub_rn(g, m), omb1));
  v = __fadd_rn(v, __fmul_rn(__fsub_rn(__fmul_rn(g, g), v), omb2));
  p = __fsub_rn(p, __fdiv_rn(__fmul_rn(m, alpha), __fadd_rn(__fsqrt_rn(v), eps)));
}

// The element's optimizer state, loaded before its gradient is summed (the
// loads are independent of the slab sum: issuing them first keeps both round
// trips in flight instead of one after the other -- the compiler cannot hoist
// them across the gradient store to a.g, which may alias for all it knows)
template <class T>
struct AdamState {
  T p, m, v, t;
};
template <class T>
DDPG_DEV AdamState<T> adam_load(const AdamArgs& a, long long j) {
  AdamState<T> st;
  st.p = *reinterpret_cast<const T*>(a.p + j);
  st.m = *reinterpret_cast<const T*>(a.m + j);
  st.v = *reinterpret_cast<const T*>(a.v + j);
  if (a.tt) st.t = *reinterpret_cast<const T*>(a.tt + j);
  return st;
}

template <class T>
DDPG_DEV void adam_apply(const AdamArgs& a, long long j, T G, AdamState<T> st, float alpha,
                         float omb1, float omb2);
template <>
DDPG_DEV void adam_apply(const AdamArgs& a, long long j, float4 G, AdamState<float4> st,
                         float alpha, float omb1, float omb2) {
  float4 P = st.p, M = st.m, V = st.v;
  adam_elem(P.x, M.x, V.x, G.x, alpha, omb1, omb2, a.eps);
  adam_elem(P.y, M.y, V.y, G.y, alpha, omb1, omb2, a.eps);
  adam_elem(P.z, M.z, V.z, G.z, alpha, omb1, omb2, a.eps);
  adam_elem(P.w, M.w, V.w, G.w, alpha, omb1, omb2, a.eps);
  *reinterpret_cast<float4*>(a.p + j) = P;
  *reinterpret_cast<float4*>(a.m + j) = M;
  *reinterpret_cast<float4*>(a.v + j) = V;
  if (a.tw) store_twin4(a.tw + j, a.tps, a.tnp, P);
  if (a.tt) {
    float4 b = st.t;
    b.x = __fadd_rn(__fmul_rn(P.x, a.tau), __fmul_rn(b.x, a.omt));
    b.y = __fadd_rn(__fmul_rn(P.y, a.tau), __fmul_rn(b.y, a.omt));
    b.z = __fadd_rn(__fmul_rn(P.z, a.tau), __fmul_rn(b.z, a.omt));
    b.w = __fadd_rn(__fmul_rn(P.w, a.tau), __fmul_rn(b.w, a.omt));
    *reinterpret_cast<float4*>(a.tt + j) = b;
    if (a.ttw) store_twin4(a.ttw + j, a.tps, a.tnp, b);
  }
}
template <>
DDPG_DEV void adam_apply(const AdamArgs& a, long long j, float G, AdamState<float> st, float alpha,
                         float omb1, float omb2) {
  float P = st.p, M = st.m, V = st.v;
  adam_elem(P, M, V, G, alpha, omb1, omb2, a.eps);
  a.p[j] = P;
  a.m[j] = M;
  a.v[j] = V;
  if (a.tw) store_twin1(a.tw + j, a.tps, a.tnp, P);
  if (a.tt) {
    const float b = __fadd_rn(__fmul_rn(P, a.tau), __fmul_rn(st.t, a.omt));
    a.tt[j] = b;
    if (a.ttw) store_twin1(a.ttw + j, a.tps, a.tnp, b);
  }
}

template <class T>
DDPG_DEV void adam_seg(const AdamSeg& g, const AdamArgs& a, int lb, T* part, float alpha,
                       float omb1, float omb2) {
  constexpr int W = sizeof(T) / sizeof(float);
  const T* __restrict__ src = reinterpret_cast<const T*>(g.src);
  const long long n = g.count / W, ss = g.slab_stride / W;
  const int SG = slab_groups(g.nslab);
  const int EPB = 256 / SG;
  const int e = threadIdx.x % EPB, sg = threadIdx.x / EPB;
  for (long long i0 = (long long)lb * EPB; i0 < n; i0 += (long long)g.nblk * EPB) {
    const long long i = i0 + e;
    const long long j = g.off + i * W;
    const bool mine = sg == 0 && i < n;  // this thread applies Adam to element i
    AdamState<T> st{};
    if (mine) st = adam_load<T>(a, j);
    T acc{};
    if (i < n) acc = slab_partial(src, i, ss, g.nslab, sg, SG);
    if (SG > 1) {
      if (sg > 0) part[(sg - 1) * 256 + e] = acc;
      __syncthreads();
    }
    if (mine) {
      for (int q = 1; q < SG; ++q) acc = rs_add(acc, part[(q - 1) * 256 + e]);
      if (g.wg) *reinterpret_cast<T*>(a.g + j) = acc;
      adam_apply(a, j, acc, st, alpha, omb1, omb2);
    }
    if (SG > 1) __syncthreads();
  }
}

__global__ __launch_bounds__(256) void adam_reduce_kernel(AdamTable t, AdamArgs a) {
  __shared__ float4 part[3 * 256];
  int s = 0;
  while (s + 1 < t.nseg && (int)blockIdx.x >= t.seg[s + 1].blk0) ++s;
  const AdamSeg g = t.seg[s];
  const float alpha = a.hk.alpha_in ? *a.hk.alpha_in : adam_alpha(a.pw, a.lr);
  adam_hooks(a.hk, a.b1, a.b2);
  const float omb1 = __fsub_rn(1.f, a.b1), omb2 = __fsub_rn(1.f, a.b2);
  const int lb = (int)blockIdx.x - g.blk0;
  if (g.vec4)
    adam_seg<float4>(g, a, lb, part, alpha, omb1, omb2);
  else
    adam_seg<float>(g, a, lb, reinterpret_cast<float*>(part), alpha, omb1, omb2);
}

// AdamOptimizer._finish: beta1_power *= beta1, beta2_power *= beta2 (fp32),
// for each network selected in mask (bit 0 actor, bit 1 critic).
DDPG_DEV void advance_powers(float* pw, int mask, float b1, float b2) {
  for (int net = 0; net < 2; ++net)
    if (mask & (1 << net)) {
      pw[2 * net] = __fmul_rn(pw[2 * net], b1);
      pw[2 * net + 1] = __fmul_rn(pw[2 * net + 1], b2);
    }
}

// A synchronous call's stats (q_max, loss) to pinned coherent host memory,
// then the call's sequence number to its completion word with a system-scope
// release: the host polls the word instead of a copy plus a stream wait.
__global__ void stats_out_kernel(const float* __restrict__ st, float* out, unsigned* word,
                                 unsigned seq) {
  if (threadIdx.x == 0) {
    out[0] = st[0];
    out[1] = st[1];
    __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A small row block [B][cols] (leading dimension ld) to pinned coherent host
// memory, then the call's completion word (system-scope release): the 1:1
// methods' small results without a staged copy into pageable memory.
__global__ __launch_bounds__(256) void rows_out_kernel(const float* __restrict__ src, int ld,
                                                       int B, int cols, float* out,
                                                       unsigned* word, unsigned seq) {
  for (int i = threadIdx.x; i < B * cols; i += 256) {
    const int r = i / cols;
    out[i] = src[(size_t)r * ld + (i - r * cols)];
  }
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A small row block [B][cols] uploaded in the kernel arguments (no staged
// copy from pageable memory): dst rows (leading dimension ld) get the values.
constexpr int kRowsInMax = 256;  // floats
struct RowsIn {
  float v[kRowsInMax];
};
__global__ __launch_bounds__(256) void rows_in_kernel(RowsIn in, float* __restrict__ dst, int ld,
                                                      int B, int cols) {
  for (int i = threadIdx.x; i < B * cols; i += 256) {
    const int r = i / cols;
    dst[(size_t)r * ld + (i - r * cols)] = in.v[i];
  }
}

// ddpg_sync's completion word: everything queued before it has finished
__global__ void word_kernel(unsigned* word, unsigned seq) {
  if (threadIdx.x == 0) __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void advance_powers_kernel(float* pw, int mask, float b1, float b2) {
  advance_powers(pw, mask, b1, b2);
}

// ---------------------------------------------------------------- K7 soft update
// networks.py:34-37: target.assign(theta * tau + target * (1. - tau)), fp32.
__global__ void soft_update_kernel(const float* __restrict__ th, float* __restrict__ tt,
                                   long long n, float tau, float omt, float* pw, int pw_mask,
                                   float b1, float b2, __bf16* __restrict__ tw, long long tps,
                                   int tnp) {
  if (pw_mask && blockIdx.x == 0 && threadIdx.x == 0) advance_powers(pw, pw_mask, b1, b2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(th)[i];
    float4 b = reinterpret_cast<float4*>(tt)[i];
    b.x = __fadd_rn(__fmul_rn(a.x, tau), __fmul_rn(b.x, omt));
    b.y = __fadd_rn(__fmul_rn(a.y, tau), __fmul_rn(b.y, omt));
    b.z = __fadd_rn(__fmul_rn(a.z, tau), __fmul_rn(b.z, omt));
    b.w = __fadd_rn(__fmul_rn(a.w, tau), __fmul_rn(b.w, omt));
    reinterpret_cast<float4*>(tt)[i] = b;
    if (tw) store_twin4(tw + 4 * i, tps, tnp, b);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    tt[i] = __fadd_rn(__fmul_rn(th[i], tau), __fmul_rn(tt[i], omt));
    if (tw) store_twin1(tw + i, tps, tnp, tt[i]);
  }
}

// dst = twin of src[0 .. n) (np planes, ps elements apart): parameter twins
// after a host write, activation twins after an upload.
__global__ void twin_kernel(const float* __restrict__ src, long long n, __bf16* __restrict__ dst,
                            long long ps, int np) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    store_twin1(dst + i, ps, np, src[i]);
}

}  // namespace ddpg
