// mfDiMP / DeT-DiMP ResNet-50 convolutions on the fp16 matrix cores at fp32-faithful precision ("f16x3"),
// gfx950.  The same implicit GEMM as dimpnet.hip's conv_f32_kernel (C[m][n] = sum_k A[m][k] W[n][k],
// m = output pixel, n = output channel, k = (ky, kx, c); activations NHWC fp32, weights [Cout][kh][kw][Cin]
// with BN folded on the host), but every product is carried as the fp16 pair of a power-of-two range-scaled
// value (common.h): acc += Wh*Ah + Wl*Ah + Wh*Al on v_mfma_f32_16x16x32_f16 -- 22-bit operands and fp32
// accumulation, the reference's fp32 arithmetic to within 2^-22 per product, at 5.3x the fp32 matrix peak
// (833 vs 157 TF/s of algorithmic FLOPs).
//
// Range scales.  Weights: s_w = 2^(14 - ceil(log2 max|w|)), split on the host.  Activations: each conv's
// epilogue folds max|y| of its output into 64 sharded max words (one per 128-B line, agent-scope atomic max
// of the float bits -- a wave's maximum per atomic), and the consuming conv reads the 64 words, takes
// s_a = 2^(14 - ceil(log2 max)) and splits its input on the fly while staging it into LDS (loads through
// registers); so |v s_a| <= 2^14 for every element, and an element keeps full 22-bit precision down to
// 2^-17 of its tensor's maximum (below that its absolute error is under 2^-38 of the maximum).  Image
// inputs (normalised pixels, |v| <= 2.64) use the static scale 2^12.
//
// Tile: 128 output pixels x BN (64 / 128) output channels, 8 waves (4 x 2, 32 x BN/2 each), K-tiles of 32:
// FAST = 32 channels of one tap (Cin % 32 == 0); STEM = 8 taps x 4 channels (Cin = 3, weights padded to 4
// channels per tap and to whole K-tiles).  Two LDS stages (hi / lo images of A and W, 16-B chunks XOR-swizzled
// as gemm.hip's BK = 32 tiles, so fragment reads are conflict-free ds_read_b128) and two register sets: the
// global loads of K-tile k + 2 are issued before K-tile k is multiplied.  The MFMA is issued W x A, so a lane
// ends with 4 consecutive output channels of one pixel (16-B NHWC stores).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mmtrack.h"
#include "common.h"

namespace mmt {

constexpr int kMaxShards = 64, kShardStride = 32;   // sharded max words: 64 x 128-B lines per tensor

struct ConvF16Args {
  const float* x;                 // [N][H][W][Cin] fp32
  const uint16_t* wh;             // [Cout][Kp] fp16 halves of w * s_w
  const uint16_t* wl;
  const float* bias;              // [Cout] or null
  const float* resid;             // [M][Cout] or null
  float* y;                       // [M][Cout]
  const float* xmax;              // sharded max|x| words of the input, or null: xscale
  float xscale;                   // static input scale (power of two) when xmax is null
  float* ymax;                    // sharded max|y| words of the output (accumulated), or null
  float inv_w;                    // 1 / s_w
  int N, H, W, Cin, Cout, kh, kw, stride, pad, Ho, Wo, Kp, flags;
};

__device__ __forceinline__ int cswz(int r, int c) { return r * 32 + ((c ^ ((r >> 2) & 2)) << 3); }   // gemm.hip swzk<32>

__device__ __forceinline__ float pow2_scale(float m) {   // 2^(14 - ceil(log2 m)), m > 0
  int e;
  const float f = frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
  const int c = f == 0.5f ? e - 1 : e;
  return ldexpf(1.0f, 14 - c);
}

template <int BN, bool STEM>
__global__ __launch_bounds__(512) void conv_f16x3_kernel(const ConvF16Args a) {
  constexpr int BM = 128, BK = 32;
  constexpr int WN = BN / 2, FM = 2, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][2][BM * BK];   // [stage][hi, lo]
  __shared__ __attribute__((aligned(16))) uint16_t sW[2][2][BN * BK];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int M = a.N * a.Ho * a.Wo;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  // input scale: the maximum over the producer's 64 shard words (every wave forms it itself)
  float sa = a.xscale;
  if (a.xmax) {
    const float mx = wave_max(a.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  const float inv = a.inv_w / sa;

  // A load slot: row (pixel) t >> 2, K chunk t & 3 (8 values); W load slot: row t >> 2, chunk t & 3
  const int ar = t >> 2, ac = t & 3;
  const int m = m0 + ar;
  const bool mval = m < M;
  int iy0 = 0, ix0 = 0;
  const float* xb = a.x;
  if (mval) {
    const int nimg = m / (a.Ho * a.Wo);
    const int r = m - nimg * a.Ho * a.Wo;
    const int oy = r / a.Wo, ox = r - oy * a.Wo;
    iy0 = oy * a.stride - a.pad;
    ix0 = ox * a.stride - a.pad;
    xb = a.x + (int64_t)nimg * a.H * a.W * a.Cin;
  }
  const bool wload = ar < BN;
  const uint16_t* wrh = a.wh + (int64_t)(n0 + (wload ? ar : 0)) * a.Kp + ac * 8;
  const uint16_t* wrl = a.wl + (int64_t)(n0 + (wload ? ar : 0)) * a.Kp + ac * 8;
  const int nk = a.Kp / BK;
  const int cpt = STEM ? 1 : a.Cin / BK;   // K-tiles per tap

  float4 ra[2][2];
  uint4 rwh[2], rwl[2];
  auto load = [&](int kt, int set) {
    if constexpr (STEM) {
      // taps 8 kt + 2 ac, + 1: three channels each (the fourth is the weights' zero pad)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = kt * 8 + ac * 2 + h;
        const int ky = tap / a.kw, kx = tap - ky * a.kw;
        const int iy = iy0 + ky, ix = ix0 + kx;
        const bool ok = mval && tap < a.kh * a.kw && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const float* src = xb + ((int64_t)iy * a.W + ix) * 3;
        ra[set][h] = ok ? make_float4(src[0], src[1], src[2], 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
      const int tap = kt / cpt, c0 = (kt - tap * cpt) * BK + ac * 8;
      const int ky = tap / a.kw, kx = tap - ky * a.kw;
      const int iy = iy0 + ky, ix = ix0 + kx;
      const bool ok = mval && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const float4* src = reinterpret_cast<const float4*>(xb + ((int64_t)iy * a.W + ix) * a.Cin + c0);
      ra[set][0] = ok ? src[0] : make_float4(0.f, 0.f, 0.f, 0.f);
      ra[set][1] = ok ? src[1] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (wload) {
      rwh[set] = *reinterpret_cast<const uint4*>(wrh + kt * BK);
      rwl[set] = *reinterpret_cast<const uint4*>(wrl + kt * BK);
    }
  };
  auto stash = [&](int set, int st) {
    const float v[8] = {ra[set][0].x, ra[set][0].y, ra[set][0].z, ra[set][0].w,
                        ra[set][1].x, ra[set][1].y, ra[set][1].z, ra[set][1].w};
    uint16_t h[8], l[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) split_h(v[e] * sa, h[e], l[e]);
    const uint4 hv = make_uint4(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16, h[4] | (uint32_t)h[5] << 16,
                                h[6] | (uint32_t)h[7] << 16);
    const uint4 lv = make_uint4(l[0] | (uint32_t)l[1] << 16, l[2] | (uint32_t)l[3] << 16, l[4] | (uint32_t)l[5] << 16,
                                l[6] | (uint32_t)l[7] << 16);
    *reinterpret_cast<uint4*>(&sA[st][0][cswz(ar, ac)]) = hv;
    *reinterpret_cast<uint4*>(&sA[st][1][cswz(ar, ac)]) = lv;
    if (wload) {
      *reinterpret_cast<uint4*>(&sW[st][0][cswz(ar, ac)]) = rwh[set];
      *reinterpret_cast<uint4*>(&sW[st][1][cswz(ar, ac)]) = rwl[set];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int st) {
    const int c = lane >> 4;
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * 32 + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[st][0][cswz(row, c)]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[st][1][cswz(row, c)]);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      bh[j] = *reinterpret_cast<const bf16x8*>(&sW[st][0][cswz(row, c)]);
      bl[j] = *reinterpret_cast<const bf16x8*>(&sW[st][1][cswz(row, c)]);
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16<true>(bh[j], ah[i], acc[i][j]);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16<true>(bl[j], ah[i], acc[i][j]);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = mfma16<true>(bh[j], al[i], acc[i][j]);
  };

  // K-tile k: loaded into register set k & 1 two tiles ahead, stashed into LDS stage k & 1 one tile ahead.  The
  // loop is unrolled by two so every register set and LDS stage index is a compile-time constant (a runtime
  // index would put the register sets behind selects and make every stash wait for all loads in flight)
  load(0, 0);
  if (nk > 1) load(1, 1);
  stash(0, 0);
  __syncthreads();
  auto step = [&](int kt, auto set_c) {
    constexpr int S = decltype(set_c)::value;   // == kt & 1
    if (kt + 2 < nk) load(kt + 2, S);
    compute(S);
    if (kt + 1 < nk) stash(1 - S, 1 - S);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < nk) step(kt + 1, std::integral_constant<int, 1>{});
  }

  // epilogue: lane holds channels n0 + wn * WN + j * 16 + 4 * (lane >> 4) + (0..3) of pixel m0 + wm * 32 + i * 16 +
  // (lane & 15): acc * inv + bias (+ residual), ReLU, the backbones' running max; max|y| into the shard words
  float ymx = 0.f;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int mo = m0 + wm * 32 + i * 16 + li;
    if (mo >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int no = n0 + wn * WN + j * 16 + 4 * lk;
      f32x4 v = acc[i][j] * inv;
      if (a.bias) {
        const float4 b = *reinterpret_cast<const float4*>(a.bias + no);
        v += f32x4{b.x, b.y, b.z, b.w};
      }
      if (a.resid) {
        const float4 r = *reinterpret_cast<const float4*>(a.resid + (int64_t)mo * a.Cout + no);
        v += f32x4{r.x, r.y, r.z, r.w};
      }
      if (a.flags & MMT_CONV_RELU)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      float4* dst = reinterpret_cast<float4*>(a.y + (int64_t)mo * a.Cout + no);
      if (a.flags & MMT_CONV_MAX) {
        const float4 o = *dst;   // torch.max(color, depth) (dimpnet.py:103)
        v = f32x4{fmaxf(o.x, v[0]), fmaxf(o.y, v[1]), fmaxf(o.z, v[2]), fmaxf(o.w, v[3])};
      }
      *dst = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
    }
  }
  if (a.ymax) {
    ymx = wave_max(ymx);
    if (lane == 0 && ymx > 0.f)
      __hip_atomic_fetch_max(reinterpret_cast<unsigned*>(a.ymax) + ((blockIdx.x * 8 + wave) % kMaxShards) * kShardStride,
                             __float_as_uint(ymx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace mmt

using namespace mmt;

extern "C" {

size_t mmt_conv_max_words(void) { return (size_t)kMaxShards * kShardStride; }

int mmt_conv2d_f16x3(const float* x, int N, int H, int W, int Cin, const uint16_t* w_hi, const uint16_t* w_lo,
                     float w_scale, int Kp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                     const float* resid, float* y, const float* x_max, float x_scale, float* y_max, int flags,
                     void* stream) {
  const bool stem = Cin == 3;
  if (!x || !w_hi || !w_lo || !y || N <= 0 || H <= 0 || W <= 0 || Cout <= 0 || Cout % 64 || kh <= 0 || kw <= 0 ||
      stride <= 0 || pad < 0 || !(w_scale > 0) || (flags & ~(MMT_CONV_RELU | MMT_CONV_MAX)) ||
      (!stem && Cin % 32) || (!x_max && !(x_scale > 0)))
    return MMT_E_ARG;
  const int K = stem ? kh * kw * 4 : kh * kw * Cin;
  if (Kp != (K + 31) / 32 * 32) return MMT_E_ARG;
  ConvF16Args a{x, w_hi, w_lo, bias, resid, y, x_max, x_scale, y_max, 1.0f / w_scale, N, H, W, Cin, Cout, kh, kw,
                stride, pad, 0, 0, Kp, flags};
  a.Ho = (H + 2 * pad - kh) / stride + 1;
  a.Wo = (W + 2 * pad - kw) / stride + 1;
  if (a.Ho <= 0 || a.Wo <= 0) return MMT_E_ARG;
  const int64_t M = (int64_t)N * a.Ho * a.Wo;
  if (M > (int64_t)1 << 30 || (int64_t)Cout * Kp > (int64_t)1 << 30) return MMT_E_ARG;
  const unsigned gm = (unsigned)((M + 127) / 128);
  const hipStream_t s = (hipStream_t)stream;
  if (stem) {
    if (Cout % 64) return MMT_E_ARG;
    hipLaunchKernelGGL((conv_f16x3_kernel<64, true>), dim3(gm, Cout / 64), dim3(512), 0, s, a);
  } else if (Cout % 128 == 0) {
    hipLaunchKernelGGL((conv_f16x3_kernel<128, false>), dim3(gm, Cout / 128), dim3(512), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv_f16x3_kernel<64, false>), dim3(gm, Cout / 64), dim3(512), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

}  // extern "C"
