// Shared device helpers for the DDPG HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DDPG_DEV __device__ __forceinline__

// TF 1.3 Elu: (x < 0).select(exp(x) - 1, x)
DDPG_DEV float elu_f(float x) { return x < 0.f ? __fsub_rn(expf(x), 1.f) : x; }
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

// Round-up helper
static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
