// Shared device helpers for the DDPG HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DDPG_DEV __device__ __forceinline__

// TF 1.3 Elu: (x < 0).select(exp(x) - 1, x)
// elu: exp(x) - 1 for x < 0 (TF 1.3's Elu, exp then subtract) with exp(x) as
// 2^(x log2 e) on v_exp_f32 (1 ulp).  Rounding x log2 e moves exp(x) by at
// most |x| 2^-24 ln 2 relative, so the absolute error of elu stays below
// ~1.5e-7 for every x < 0 -- within the fp32 subtraction's own rounding of
// the libm form, at 3 instructions instead of ~12 (the epilogues that apply it
// are VALU-bound: thin_k's five-part launch 49.5 -> 44.2 us,
// profiles/r4/thin_k_fast_elu.txt)
DDPG_DEV float elu_f(float x) {
  return x < 0.f ? __fsub_rn(__builtin_amdgcn_exp2f(__fmul_rn(x, 1.44269504f)), 1.f) : x;
}
// TF 1.3 EluGrad from the OUTPUT y: y < 0 ? dy * (y + 1) : dy
DDPG_DEV float elu_grad_factor(float y) { return y < 0.f ? __fadd_rn(y, 1.f) : 1.f; }

// Address-space-qualified pointers for out-of-line helpers: a generic pointer
// argument compiles to FLAT loads, which wait on both the vector-memory and
// the LDS counters (every access serialises behind all outstanding memory).
typedef __attribute__((address_space(3))) float lds_f;
typedef __attribute__((address_space(1))) float glb_f;
typedef __attribute__((address_space(3))) float4 lds_f4;
typedef __attribute__((address_space(1))) float4 glb_f4;
#define LDS(p) ((lds_f*)(p))
#define GLB(p) ((glb_f*)(p))

// ---------------------------------------------------------------- bf16 twins
// bf16 operand types, and the exact three-plane split of an fp32 value used
// by the bf16 "twins" of fp32 tensors (the operands of gemm_h.h).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
// (x0, x1) -> packed (h, m, l) bf16 pairs: three v_cvt_pk_bf16_f32, the
// widening of a bf16 pair is two bit operations, the residuals packed f32 subs.
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
DDPG_DEV f32x2v widen(bf16x2 b) {
  const unsigned u = __builtin_bit_cast(unsigned, b);
  return f32x2v{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xFFFF0000u)};
}
DDPG_DEV void split3_pair(f32x2v x, bf16x2& h, bf16x2& m, bf16x2& l) {
  h = __builtin_convertvector(x, bf16x2);
  const f32x2v r1 = x - widen(h);  // exact
  m = __builtin_convertvector(r1, bf16x2);
  const f32x2v r2 = r1 - widen(m);  // exact
  l = __builtin_convertvector(r2, bf16x2);
}

// Store the twin of 4 (or 1) consecutive fp32 values: np = 1 stores bf16(v);
// np = 3 stores the h / m / l planes, ps elements apart.
DDPG_DEV void store_twin4(__bf16* q, long long ps, int np, float4 v) {
  if (np == 3) {
    bf16x2 h0, m0, l0, h1, m1, l1;
    split3_pair(f32x2v{v.x, v.y}, h0, m0, l0);
    split3_pair(f32x2v{v.z, v.w}, h1, m1, l1);
    *reinterpret_cast<bf16x4*>(q) = bf16x4{h0[0], h0[1], h1[0], h1[1]};
    *reinterpret_cast<bf16x4*>(q + ps) = bf16x4{m0[0], m0[1], m1[0], m1[1]};
    *reinterpret_cast<bf16x4*>(q + 2 * ps) = bf16x4{l0[0], l0[1], l1[0], l1[1]};
  } else {
    const bf16x2 h0 = __builtin_convertvector(f32x2v{v.x, v.y}, bf16x2);
    const bf16x2 h1 = __builtin_convertvector(f32x2v{v.z, v.w}, bf16x2);
    *reinterpret_cast<bf16x4*>(q) = bf16x4{h0[0], h0[1], h1[0], h1[1]};
  }
}
// Twin of 8 consecutive fp32 values (a, b): one 16-B store per plane (q and
// ps multiples of 8 elements).
DDPG_DEV void store_twin8(__bf16* q, long long ps, int np, float4 a, float4 b) {
  bf16x2 h[4], m[4], l[4];
  const f32x2v x[4] = {f32x2v{a.x, a.y}, f32x2v{a.z, a.w}, f32x2v{b.x, b.y}, f32x2v{b.z, b.w}};
  if (np == 3) {
#pragma unroll
    for (int i = 0; i < 4; ++i) split3_pair(x[i], h[i], m[i], l[i]);
    *reinterpret_cast<bf16x8*>(q + ps) =
        bf16x8{m[0][0], m[0][1], m[1][0], m[1][1], m[2][0], m[2][1], m[3][0], m[3][1]};
    *reinterpret_cast<bf16x8*>(q + 2 * ps) =
        bf16x8{l[0][0], l[0][1], l[1][0], l[1][1], l[2][0], l[2][1], l[3][0], l[3][1]};
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) h[i] = __builtin_convertvector(x[i], bf16x2);
  }
  *reinterpret_cast<bf16x8*>(q) =
      bf16x8{h[0][0], h[0][1], h[1][0], h[1][1], h[2][0], h[2][1], h[3][0], h[3][1]};
}
DDPG_DEV void store_twin1(__bf16* q, long long ps, int np, float x) {
  const __bf16 h = (__bf16)x;
  q[0] = h;
  if (np == 3) {
    const float r1 = x - (float)h;
    const __bf16 m = (__bf16)r1;
    q[ps] = m;
    q[2 * ps] = (__bf16)(r1 - (float)m);
  }
}

// Round-up helper
static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
