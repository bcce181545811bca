// Shared helpers for the iit_amd gfx950 (MI355X / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define IIT_EXPORT extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }
__device__ __forceinline__ __bf16 f2bf(float v) { return (__bf16)v; }
__device__ __forceinline__ float u16_to_f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// tanh(u) = 1 - 2 / (exp(2u) + 1): one v_exp_f32 + one v_rcp_f32 (the raw 1-ulp reciprocal, not the IEEE
// division sequence __frcp_rn compiles to) instead of libm tanhf's ~40-instruction
// branchy sequence (which made the fused dgelu epilogue VALU-bound); saturates correctly at +-inf
__device__ __forceinline__ float tanh_fast(float u) { return 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f); }

// gelu_new (tanh approximation, as TransformerLens / GPT-2) in its sigmoid form: 0.5 (1 + tanh(u)) = sigmoid(2u),
// u = sqrt(2/pi) (x + 0.044715 x^3), with log2(e) folded into the constants -> one v_exp_f32 + one v_rcp_f32 and
// a handful of FMAs per element (the GEMM epilogues that apply it are VALU-bound)
__device__ __forceinline__ float gelu_sig2u(float x, float x2) {  // sigmoid(2u)
  const float m = x * __builtin_fmaf(0.10294324f, x2, 2.3022082f);  // 2u * log2(e)
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-m));
}
__device__ __forceinline__ float gelu_new_f(float x) { return x * gelu_sig2u(x, x * x); }
__device__ __forceinline__ float gelu_new_grad_f(float x) {
  // d/dx [x s(2u)] = s + x s (1 - s) d(2u)/dx,  d(2u)/dx = 2 sqrt(2/pi) (1 + 3 * 0.044715 x^2)
  const float x2 = x * x;
  const float s = gelu_sig2u(x, x2);
  const float du = __builtin_fmaf(0.21406445f, x2, 1.5957691f);
  return __builtin_fmaf(x * du, __builtin_fmaf(-s, s, s), s);
}

// exact (erf) GELU, as BERT / torch.nn.functional.gelu
__device__ __forceinline__ float gelu_erf_f(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }
__device__ __forceinline__ float gelu_erf_grad_f(float x) {
  return 0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

static inline int cdiv(long a, long b) { return (int)((a + b - 1) / b); }
