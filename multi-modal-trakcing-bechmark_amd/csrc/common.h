// Shared device helpers for the MI355X (gfx950 / CDNA4) tracking engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;                                              // storage type
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));            // MFMA A/B fragment
typedef float f32x4 __attribute__((ext_vector_type(4)));              // 16x16 accumulator

#define WAVE 64

__device__ __forceinline__ bf16_t f2bf(float x) {                    // RNE (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, (__bf16)x);
}
__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(((uint32_t)x) << 16);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Exact-erf GELU (nn.GELU default; vit_ce_prompt.py:122), GELU(x) = x * (1 - erfc(x/sqrt2)/2),
// with erfc from the Chebyshev-fitted form of Numerical Recipes' erfcc (fractional error < 1.2e-7
// everywhere).  For x < 0 it is x * erfc(|x|/sqrt2) / 2 directly, so there is no cancellation.
__device__ __forceinline__ float erfc_pos(float z) {   // z >= 0
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.5f * z);   // v_rcp_f32 (1 ulp); __frcp_rn is a full IEEE divide
  const float p = -1.26551223f + t * (1.00002368f + t * (0.37409196f + t * (0.09678418f + t * (-0.18628806f +
                  t * (0.27886807f + t * (-1.13520398f + t * (1.48851587f + t * (-0.82215223f + t * 0.17087277f))))))));
  return t * __expf(-z * z + p);
}
__device__ __forceinline__ float gelu_erf(float x) {
  const float u = fabsf(x) * 0.70710678118654752440f;
  const float h = 0.5f * erfc_pos(u);
  return x >= 0.f ? x * (1.0f - h) : x * h;
}
