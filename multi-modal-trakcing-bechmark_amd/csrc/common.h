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

// ---- fp32-faithful operands ("f16x3"): a value v, pre-multiplied by its tensor's power-of-two range
// scale s (|v s| <= 2^14 by a host-computed bound, engine.cpp range_scale), travels as two fp16 halves
// hi = f16(v s), lo = f16(v s - hi) -- 22 significant bits -- and a product is hi*hi + lo*hi + hi*lo
// (three fp16 MFMAs at the bf16 rate; the dropped lo*lo is 2^-22 relative).  The GEMM / attention
// epilogues multiply the fp32 accumulator by 1 / (s_a s_w), exact for powers of two.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// a value the compiler cannot prove wave-uniform (e.g. selected from kernel arguments by blockIdx, or CSE'd with
// a per-lane product) moved to SGPRs, so a buffer resource built from it needs no waterfall loop
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, int64_t bytes) {
  // raw buffer: stride 0, num_records = bytes (loads past it return 0), gfx9 dword3; callers pass wave-uniform
  // operands, made SGPR-resident here
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : (int64_t)0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(uniform_ptr(p)), (short)0, n, 0x00020000);
}
constexpr uint32_t kBufOob = 0x80000000u;   // a buffer offset past every resource: the load returns zeros
// the same descriptor as four dwords (for inline-asm buffer instructions, "s" operand)
__device__ __forceinline__ u32x4 make_rsrc_words(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(uniform_ptr(p));
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : (int64_t)0x7fffffff));
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xffffu, n, 0x00020000u};
}
__device__ __forceinline__ uint16_t f2h(float x) { return __builtin_bit_cast(uint16_t, (_Float16)x); }  // RNE
__device__ __forceinline__ float h2f(uint16_t x) { return (float)__builtin_bit_cast(_Float16, x); }
__device__ __forceinline__ void split_h(float v, uint16_t& hi, uint16_t& lo) {
  hi = f2h(v);
  lo = f2h(v - h2f(hi));   // v - hi is exact in fp32
}
// 16x16x32 MFMA on 8-element fragments held as bf16x8 registers: bf16 operands, or fp16 (F16 = true)
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ---- cross-lane butterflies without the LDS.  __shfl_xor lowers to ds_bpermute_b32 (an LDS round trip
// per step, serialised along a reduction); these use v_permlane32_swap / v_permlane16_swap across the
// 32- and 16-lane halves and DPP inside a 16-lane row (row_ror:8 is xor 8; once bit 3 is uniform,
// row_ror:4 reads the xor-4 partner's value; quad_perm gives xor 2 / xor 1).  Every step adds or maxes
// a lane's own value with its xor partner's, in the order 32, 16, 8, 4, 2, 1, so the results are bit for
// bit those of the __shfl_xor butterfly.
__device__ __forceinline__ uint32_t f2u(float v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ float u2f(uint32_t v) { return __builtin_bit_cast(float, v); }
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
enum { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128 };
// (x, y) -> lanes < 32 get x[l] + x[l+32] (or x's partner), lanes >= 32 the same for y: the half-exchange
// of v_permlane32_swap (vdst x: its upper half swaps with the lower half of y)
__device__ __forceinline__ float xsum32(float x, float y) {
  const auto r = __builtin_amdgcn_permlane32_swap(f2u(x), f2u(y), false, false);
  return u2f(r[0]) + u2f(r[1]);
}
// rows of 16 lanes: rows 0 / 2 get x[l] + x[l^16], rows 1 / 3 get y[l] + y[l^16]
__device__ __forceinline__ float xsum16(float x, float y) {
  const auto r = __builtin_amdgcn_permlane16_swap(f2u(x), f2u(y), false, false);
  return u2f(r[0]) + u2f(r[1]);
}
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(f2u(v), f2u(v), false, false);
  return fmaxf(u2f(r[0]), u2f(r[1]));
}
__device__ __forceinline__ float xmax16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(f2u(v), f2u(v), false, false);
  return fmaxf(u2f(r[0]), u2f(r[1]));
}
__device__ __forceinline__ float row16_sum(float v) {   // xor 8, 4, 2, 1 inside each 16-lane row
  v += dpp<DPP_ROR8>(v);
  v += dpp<DPP_ROR4>(v);
  v += dpp<DPP_XOR2>(v);
  v += dpp<DPP_XOR1>(v);
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
  v = xsum32(v, v);
  v = xsum16(v, v);
  return row16_sum(v);
}
__device__ __forceinline__ float wave_max(float v) {
  v = xmax32(v);
  v = xmax16(v);
  v = fmaxf(v, dpp<DPP_ROR8>(v));
  v = fmaxf(v, dpp<DPP_ROR4>(v));
  v = fmaxf(v, dpp<DPP_XOR2>(v));
  return fmaxf(v, dpp<DPP_XOR1>(v));
}

// Exact-erf GELU (nn.GELU default; vit_ce_prompt.py:122), GELU(x) = x * (1 - h) for x >= 0 and x * h for
// x < 0, h = Phi(-|x|) = erfc(|x|/sqrt2) / 2, with erfc from the Chebyshev-fitted form of Numerical
// Recipes' erfcc (fractional error < 1.2e-7 everywhere, no cancellation in the negative tail):
//   h = t * 2^(-u^2 log2(e) + q(t)),  t = 1 / (1 + u/2),  u = |x|/sqrt2,
// with erfcc's polynomial pre-scaled by log2(e) and the 1/2 folded into its constant term, so the
// evaluation is one v_rcp_f32, ten FMAs and one v_exp_f32.
__device__ __forceinline__ float gelu_erf(float x) {
  const float u = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, u, 1.0f));
  float q = 0.246517298f;
  q = fmaf(q, t, -1.18611495f);
  q = fmaf(q, t, 2.14747446f);
  q = fmaf(q, t, -1.63775315f);
  q = fmaf(q, t, 0.402321582f);
  q = fmaf(q, t, -0.26875686f);
  q = fmaf(q, t, 0.139630057f);
  q = fmaf(q, t, 0.539700616f);
  q = fmaf(q, t, 1.4427292f);
  q = fmaf(q, t, -2.82574822f);
  const float h = t * __builtin_amdgcn_exp2f(fmaf(-1.44269504f * u, u, q));
  const float xh = x * h;
  return x >= 0.f ? x - xh : xh;
}

// gelu_erf on a pair, in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of FMA per instruction; the
// reciprocal and exp2 stay per element): the same operations in the same order, element by element, for the
// VALU-bound GELU epilogue of fc1 (half the FMA issue slots)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 u = __builtin_elementwise_abs(x) * (f32x2)0.70710678118654752440f;
  const f32x2 d = __builtin_elementwise_fma((f32x2)0.5f, u, (f32x2)1.0f);
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = (f32x2)0.246517298f;
  q = __builtin_elementwise_fma(q, t, (f32x2)-1.18611495f);
  q = __builtin_elementwise_fma(q, t, (f32x2)2.14747446f);
  q = __builtin_elementwise_fma(q, t, (f32x2)-1.63775315f);
  q = __builtin_elementwise_fma(q, t, (f32x2)0.402321582f);
  q = __builtin_elementwise_fma(q, t, (f32x2)-0.26875686f);
  q = __builtin_elementwise_fma(q, t, (f32x2)0.139630057f);
  q = __builtin_elementwise_fma(q, t, (f32x2)0.539700616f);
  q = __builtin_elementwise_fma(q, t, (f32x2)1.4427292f);
  q = __builtin_elementwise_fma(q, t, (f32x2)-2.82574822f);
  const f32x2 a = __builtin_elementwise_fma((f32x2)-1.44269504f * u, u, q);
  const f32x2 h = t * f32x2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  const f32x2 xh = x * h;
  return f32x2{x.x >= 0.f ? x.x - xh.x : xh.x, x.y >= 0.f ? x.y - xh.y : xh.y};
}

// gelu_erf2 on two pairs.  GELU_INTERLEAVE (tuning build): the two Horner chains interleaved statement by statement
// and fenced in lockstep -- the fc1 epilogue's 256 x 256 tile drops 32.8k -> 30.0k cycles, but the 32-sequence line
// measured 6 327 -> 6 307 frames/s (three alternating rounds, profiles/r05_ab_gelu_interleave_b32_rejected.txt), so the
// default runs the pairs one after the other; same operations per element, same bits either way
__device__ __forceinline__ void gelu_erf4(f32x2& x0, f32x2& x1) {
#ifndef GELU_INTERLEAVE
  x0 = gelu_erf2(x0);
  x1 = gelu_erf2(x1);
  return;
#endif
  const f32x2 u0 = __builtin_elementwise_abs(x0) * (f32x2)0.70710678118654752440f;
  const f32x2 u1 = __builtin_elementwise_abs(x1) * (f32x2)0.70710678118654752440f;
  const f32x2 d0 = __builtin_elementwise_fma((f32x2)0.5f, u0, (f32x2)1.0f);
  const f32x2 d1 = __builtin_elementwise_fma((f32x2)0.5f, u1, (f32x2)1.0f);
  const f32x2 t0 = {__builtin_amdgcn_rcpf(d0.x), __builtin_amdgcn_rcpf(d0.y)};
  const f32x2 t1 = {__builtin_amdgcn_rcpf(d1.x), __builtin_amdgcn_rcpf(d1.y)};
  f32x2 q0 = (f32x2)0.246517298f, q1 = (f32x2)0.246517298f;
  constexpr float C[9] = {-1.18611495f, 2.14747446f, -1.63775315f, 0.402321582f, -0.26875686f,
                          0.139630057f, 0.539700616f, 1.4427292f, -2.82574822f};
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    q0 = __builtin_elementwise_fma(q0, t0, (f32x2)C[k]);
    q1 = __builtin_elementwise_fma(q1, t1, (f32x2)C[k]);
    asm volatile("" : "+v"(q0), "+v"(q1));   // lockstep: the scheduler otherwise serialises the two chains again
  }
  const f32x2 a0 = __builtin_elementwise_fma((f32x2)-1.44269504f * u0, u0, q0);
  const f32x2 a1 = __builtin_elementwise_fma((f32x2)-1.44269504f * u1, u1, q1);
  const f32x2 h0 = t0 * f32x2{__builtin_amdgcn_exp2f(a0.x), __builtin_amdgcn_exp2f(a0.y)};
  const f32x2 h1 = t1 * f32x2{__builtin_amdgcn_exp2f(a1.x), __builtin_amdgcn_exp2f(a1.y)};
  const f32x2 xh0 = x0 * h0, xh1 = x1 * h1;
  x0 = f32x2{x0.x >= 0.f ? x0.x - xh0.x : xh0.x, x0.y >= 0.f ? x0.y - xh0.y : xh0.y};
  x1 = f32x2{x1.x >= 0.f ? x1.x - xh1.x : xh1.x, x1.y >= 0.f ? x1.y - xh1.y : xh1.y};
}

// bf16-output GELU: the same erf GELU with erfc from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7 on
// erf, five coefficients; 1/2 and log2(e) folded as above), written as
//   GELU(x) = relu(x) - |x| * h(|x|),   h(a) = t p(t) 2^(-x^2 log2(e) / 2),  t = 1 / (1 + 0.3275911 a / sqrt2)
// (x >= 0: x - x h; x < 0: x h), so the epilogue spends one v_rcp_f32, one v_exp_f32 and eleven
// single-issue VALU ops per output (|x| and -|x| are source modifiers, no select).
// Against exact erf GELU the result differs by < 5e-7 * max(1, |x|); after rounding to bf16, about
// 0.1 % of outputs move by one bf16 ulp (tests/test_oracle_golden.py).  Used where the GEMM writes
// plain bf16 (the fp32-faithful mode keeps gelu_erf).
__device__ __forceinline__ float gelu_erf_bf16out(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.2316418917f, a, 1.0f));   // 0.3275911 / sqrt2
  float p = 0.5307027145f;
  p = fmaf(p, t, -0.7265760135f);
  p = fmaf(p, t, 0.7107068705f);
  p = fmaf(p, t, -0.142248368f);
  p = fmaf(p, t, 0.127414796f);
  const float e = __builtin_amdgcn_exp2f((x * -0.7213475204f) * x);      // exp(-x^2 / 2)
  return fmaf(-a, (p * t) * e, fmaxf(x, 0.f));
}
