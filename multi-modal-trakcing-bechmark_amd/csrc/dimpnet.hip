// mfDiMP / DeT-DiMP feature path on gfx950 (fp32): the per-frame image -> classification-feature chain
// of DiMPnet_DeT (RGBD/models/DeT/ltr/models/tracking/dimpnet.py:15-156, merge_type 'max') and its
// classifier initialiser, plus pytracking's patch sampling.
//
//   sample_patch          pytracking/features/preprocessing.py:49-125 (pre-downsample, replicate pad, bilinear)
//   patch transforms      pytracking/features/augmentation.py (Identity / Translation / FlipHorizontal / Blur /
//                         Rotate, each cropped to the output with replicate padding, crop_to_output)
//   preprocess_image      pytracking/features/net_wrappers.py:55-79 (/255, -mean, /std per 3-channel half)
//   ResNet-50 conv/BN     ltr/models/backbone/resnet.py (convs as implicit GEMMs, BN folded on the host)
//   maxpool 3x3 s2 p1     resnet.py (ResNet stem)
//   InstanceL2Norm        ltr/models/layers/normalization.py:6-21
//   PrRoIPool2D           ltr/external/PreciseRoIPooling (exact integral of the bilinear surface per bin)
//
// Arithmetic: fp32 throughout, the convolutions on v_mfma_f32_16x16x4_f32 (fp32 products, fp32 accumulate --
// the feature net feeds a Gauss-Newton optimiser and a 19 x 19 argmax, so it runs at the reference's own
// precision; 157 TF/s dense fp32 matrix peak).  Activations NHWC, weights [Cout][kh][kw][Cin].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mmtrack.h"

// no FMA contraction: the elementwise float ops restate the reference's separate multiplies and adds
#pragma clang fp contract(off)

namespace mmt {

typedef float f32x4v __attribute__((ext_vector_type(4)));

struct ConvArgs {
  const float* x;       // [N][H][W][Cin]
  const float* w;       // [Cout][kh][kw][Cin]
  const float* bias;    // [Cout] or null
  const float* resid;   // [M][Cout] or null
  float* y;             // [M][Cout], M = N * Ho * Wo
  int N, H, W, Cin, Cout, kh, kw, stride, pad, Ho, Wo, flags;
  int ldx, ldy;         // channel pitch of x / of y and resid (Cin / Cout; wider for one group of a grouped conv)
};

// ---------------------------------------------------------------------------------------------------
// Implicit-GEMM convolution: C[m][n] = sum_k A[m][k] W[n][k], m = output pixel, n = output channel,
// k = (ky, kx, c).  64 x 64 output tile, 4 waves (2 x 2, each 32 pixels x 32 channels = 2 x 2 MFMA blocks),
// K-tiles of 32 (16 when Cin % 32 != 0) staged through LDS k-major ([k][64 + 4], conflict-free fragment
// reads), the next K-tile's
// global loads held in registers while the current one is multiplied.  The MFMA is issued W x A so a lane
// ends with 4 consecutive output channels of one pixel: 16-B NHWC stores with bias / residual / ReLU /
// running-max epilogues.  FAST: a K-tile is BK channels of one tap (float4 loads);
// otherwise (the 3-channel stem) each k is decoded separately.
// W4 (the 3-channel stem, MMT_CONV_W4): weights padded to 4 channels per tap, a K-tile is 4 taps and a
// thread loads one tap (3 pixel values + 0, one float4 of weights) -- no per-element index decode
#ifndef CONV_F32_NACC
#define CONV_F32_NACC 4
#endif
template <bool FAST, int BK, bool W4 = false, int NACC = CONV_F32_NACC>
__global__ __launch_bounds__(256) void conv_f32_kernel(const ConvArgs a) {
  static_assert(!W4 || (!FAST && BK == 16), "W4: BK 16");
  constexpr int VPT = BK / 4;   // K values per thread per K-tile (A and W each)
  // KV (FAST or W4): the tile is stored row-major with K contiguous and lane group lk of the MFMA owns
  // K-range [VPT lk, VPT lk + VPT) -- step k4 multiplies k = VPT lk + k4 -- so a lane's fragments come in
  // 16-B reads and the stash is 16-B writes (k-major tiles took a 4-B LDS op per value): +5 % mfDiMP
  constexpr bool KV = FAST || W4;
  __shared__ float sA[KV ? 64 : BK][KV ? BK + 4 : 68];
  __shared__ float sB[KV ? 64 : BK][KV ? BK + 4 : 68];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int wr = wv >> 1, wc = wv & 1;
  const int M = a.N * a.Ho * a.Wo, K = a.kh * a.kw * (W4 ? 4 : a.Cin);
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  // this thread's load slot: row (pixel / channel) t >> 2, K offset (t & 3) * VPT
  const int lr = t >> 2, kq = (t & 3) * VPT;
  const int m = m0 + lr;
  const bool mval = m < M;
  int nimg = 0, oy = 0, ox = 0;
  if (mval) {
    nimg = m / (a.Ho * a.Wo);
    const int r = m - nimg * a.Ho * a.Wo;
    oy = r / a.Wo;
    ox = r - oy * a.Wo;
  }
  const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
  const float* xb = a.x + (int64_t)nimg * a.H * a.W * a.ldx;
  const float* wrow = a.w + (int64_t)(n0 + lr) * K;
  const int nk = (K + BK - 1) / BK;
  const int cpt = FAST ? a.Cin / BK : 1;   // K-tiles per tap

  f32x4v ra[VPT / 4], rb[VPT / 4];
  auto load = [&](int kt) {
    if constexpr (FAST) {
      const int tap = kt / cpt, c0 = (kt - tap * cpt) * BK + kq;
      const int ky = tap / a.kw, kx = tap - ky * a.kw;
      const int iy = iy0 + ky, ix = ix0 + kx;
      const bool ok = mval && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const float* src = xb + ((int64_t)iy * a.W + ix) * a.ldx + c0;
#pragma unroll
      for (int v = 0; v < VPT / 4; ++v) {
        ra[v] = ok ? *reinterpret_cast<const f32x4v*>(src + 4 * v) : f32x4v{0.f, 0.f, 0.f, 0.f};
        rb[v] = *reinterpret_cast<const f32x4v*>(wrow + kt * BK + kq + 4 * v);
      }
    } else if constexpr (W4) {
      const int tap = kt * 4 + (t & 3);
      const bool tv = tap < a.kh * a.kw;
      const int ky = tap / a.kw, kx = tap - ky * a.kw;
      const int iy = iy0 + ky, ix = ix0 + kx;
      const bool ok = tv && mval && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const float* src = xb + ((int64_t)iy * a.W + ix) * a.ldx;
      ra[0] = ok ? f32x4v{src[0], src[1], src[2], 0.f} : f32x4v{0.f, 0.f, 0.f, 0.f};
      rb[0] = tv ? *reinterpret_cast<const f32x4v*>(wrow + tap * 4) : f32x4v{0.f, 0.f, 0.f, 0.f};
    } else {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        const int k = kt * BK + kq + j;
        float va = 0.f, vb = 0.f;
        if (k < K) {
          const int tap = k / a.Cin, c = k - tap * a.Cin;
          const int ky = tap / a.kw, kx = tap - ky * a.kw;
          const int iy = iy0 + ky, ix = ix0 + kx;
          if (mval && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W) va = xb[((int64_t)iy * a.W + ix) * a.ldx + c];
          vb = wrow[k];
        }
        ra[j / 4][j % 4] = va;
        rb[j / 4][j % 4] = vb;
      }
    }
  };
  auto stash = [&]() {
    if constexpr (KV) {
#pragma unroll
      for (int v = 0; v < VPT / 4; ++v) {
        *reinterpret_cast<f32x4v*>(&sA[lr][kq + 4 * v]) = ra[v];
        *reinterpret_cast<f32x4v*>(&sB[lr][kq + 4 * v]) = rb[v];
      }
    } else {
#pragma unroll
      for (int j = 0; j < VPT; ++j) {
        sA[kq + j][lr] = ra[j / 4][j % 4];
        sB[kq + j][lr] = rb[j / 4][j % 4];
      }
    }
  };

  // NACC accumulator sets, K-tile kt into set kt % NACC, summed pairwise after the loop: each MFMA adds its 4
  // products to the accumulator one rounding at a time (an fmaf chain), so one set is a K-long sequential fp32 sum
  f32x4v acc[NACC][2][2];
#pragma unroll
  for (int s = 0; s < NACC; ++s)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[s][i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};

  load(0);
  stash();
  __syncthreads();
  const int li = lane & 15, lk = lane >> 4;
  auto ktile = [&](int kt, f32x4v (&A)[2][2]) {
    if (kt + 1 < nk) load(kt + 1);
    if constexpr (KV) {
      f32x4v av[2][VPT / 4], bv[2][VPT / 4];
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int h = 0; h < VPT / 4; ++h)
          av[p][h] = *reinterpret_cast<const f32x4v*>(&sA[wr * 32 + p * 16 + li][lk * VPT + 4 * h]);
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < VPT / 4; ++h)
          bv[c][h] = *reinterpret_cast<const f32x4v*>(&sB[wc * 32 + c * 16 + li][lk * VPT + 4 * h]);
#pragma unroll
      for (int k4 = 0; k4 < VPT; ++k4)
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            A[p][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(bv[c][k4 / 4][k4 % 4], av[p][k4 / 4][k4 % 4], A[p][c], 0, 0, 0);
    } else {
#pragma unroll
      for (int k4 = 0; k4 < BK / 4; ++k4) {
        const int kk = k4 * 4 + lk;
        float fa[2], fb[2];
#pragma unroll
        for (int p = 0; p < 2; ++p) fa[p] = sA[kk][wr * 32 + p * 16 + li];
#pragma unroll
        for (int c = 0; c < 2; ++c) fb[c] = sB[kk][wc * 32 + c * 16 + li];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int c = 0; c < 2; ++c) A[p][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[c], fa[p], A[p][c], 0, 0, 0);
      }
    }
    __syncthreads();
    if (kt + 1 < nk) {
      stash();
      __syncthreads();
    }
  };
  for (int kt = 0; kt < nk; kt += NACC) {
#pragma unroll
    for (int s = 0; s < NACC; ++s)
      if (kt + s < nk) ktile(kt + s, acc[s]);
  }
#pragma unroll
  for (int w = 1; w < NACC; w *= 2)   // pairwise: (s0 + s1) + (s2 + s3)
#pragma unroll
    for (int s = 0; s + w < NACC; s += 2 * w)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[s][p][c] += acc[s + w][p][c];
  // lane holds channels n0 + wc*32 + c*16 + 4*lk + (0..3) of pixel m0 + wr*32 + p*16 + li
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int mo = m0 + wr * 32 + p * 16 + li;
    if (mo >= M) continue;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int no = n0 + wc * 32 + c * 16 + 4 * lk;
      f32x4v v = acc[0][p][c];
      if (a.bias) v += *reinterpret_cast<const f32x4v*>(a.bias + no);
      if (a.resid) v += *reinterpret_cast<const f32x4v*>(a.resid + (int64_t)mo * a.ldy + no);
      if (a.flags & MMT_CONV_RELU)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.f);
      f32x4v* dst = reinterpret_cast<f32x4v*>(a.y + (int64_t)mo * a.ldy + no);
      if (a.flags & MMT_CONV_MAX) {
        const f32x4v o = *dst;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = fmaxf(o[j], v[j]);   // torch.max(color, depth) (dimpnet.py:103)
      }
      *dst = v;
    }
  }
}

// max over a k x k window, stride s, zero-free padding (padded taps never win: -inf), NHWC
__global__ __launch_bounds__(256) void maxpool_kernel(const float* __restrict__ x, int N, int H, int W, int C, int k,
                                                      int s, int pad, int Ho, int Wo, float* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * Wo * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  int64_t r = i / C;
  const int ox = (int)(r % Wo);
  r /= Wo;
  const int oy = (int)(r % Ho);
  const int n = (int)(r / Ho);
  float m = -INFINITY;
  for (int dy = 0; dy < k; ++dy) {
    const int iy = oy * s - pad + dy;
    if (iy < 0 || iy >= H) continue;
    for (int dx = 0; dx < k; ++dx) {
      const int ix = ox * s - pad + dx;
      if (ix < 0 || ix >= W) continue;
      m = fmaxf(m, x[(((int64_t)n * H + iy) * W + ix) * C + c]);
    }
  }
  y[i] = m;
}

// the same over 4 channels per thread (C % 4 == 0): float4 loads and stores
__global__ __launch_bounds__(256) void maxpool4_kernel(const float4* __restrict__ x, int N, int H, int W, int C4, int k,
                                                       int s, int pad, int Ho, int Wo, float4* __restrict__ y) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)N * Ho * Wo * C4;
  if (i >= total) return;
  const int c = (int)(i % C4);
  int64_t r = i / C4;
  const int ox = (int)(r % Wo);
  r /= Wo;
  const int oy = (int)(r % Ho);
  const int n = (int)(r / Ho);
  float4 m = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  for (int dy = 0; dy < k; ++dy) {
    const int iy = oy * s - pad + dy;
    if (iy < 0 || iy >= H) continue;
    for (int dx = 0; dx < k; ++dx) {
      const int ix = ox * s - pad + dx;
      if (ix < 0 || ix >= W) continue;
      const float4 v = x[(((int64_t)n * H + iy) * W + ix) * C4 + c];
      m = make_float4(fmaxf(m.x, v.x), fmaxf(m.y, v.y), fmaxf(m.z, v.z), fmaxf(m.w, v.w));
    }
  }
  y[i] = m;
}

// NCHW [N][C][H][W] pixel values (0..255) -> per 3-channel half NHWC ((v / 255) - mean) / std
// (net_wrappers.py:62-72: color and depth halves normalised with the same ImageNet constants)
__global__ __launch_bounds__(256) void normalize_kernel(const float* __restrict__ im, int N, int C, int H, int W,
                                                        float m0, float m1, float m2, float s0, float s1, float s2,
                                                        float* __restrict__ outa, float* __restrict__ outb, int oc) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t HW = (int64_t)H * W;
  if (i >= (int64_t)N * HW) return;
  const int n = (int)(i / HW);
  const int64_t p = i - n * HW;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    if (c >= C) break;
    float v = im[((int64_t)n * C + c) * HW + p] / 255.f;
    v = v - mean[c % 3];
    v = v / sd[c % 3];
    float* o = c < 3 ? outa : outb;
    o[(n * HW + p) * oc + (c % 3)] = v;
  }
  if (oc == 4) {   // the zero fourth channel of a padded pixel
    outa[(n * HW + p) * 4 + 3] = 0.f;
    if (C == 6) outb[(n * HW + p) * 4 + 3] = 0.f;
  }
}

// InstanceL2Norm (size_average): y = x * (scale * sqrt((1 / (sum x^2 + eps)) * C*H*W)).  Two passes over
// workgroups of kL2Pix pixels x C channels of one sample: the squares summed per workgroup (fixed order) into
// ws[n][chunk]; then every workgroup sums its sample's chunk sums in chunk order and scales its pixels, writing
// NHWC (float4) and / or NCHW (transposed through the LDS: runs of kL2Pix pixels per channel)
constexpr int kL2Pix = 16, kL2MaxC = 1024;

__device__ __forceinline__ float block_sum_256(float v, float* red) {   // fixed-order workgroup sum (256 threads)
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  return red[0];
}

__global__ __launch_bounds__(256) void l2norm_sumsq_kernel(const float* __restrict__ x, int HW, int C,
                                                           float* __restrict__ ws) {
  __shared__ float red[256];
  const int n = blockIdx.y, p0 = blockIdx.x * kL2Pix, np = min(kL2Pix, HW - p0);
  const float4* xs = reinterpret_cast<const float4*>(x + ((int64_t)n * HW + p0) * C);
  const int q = np * C / 4;
  float s = 0.f;
  for (int i = threadIdx.x; i < q; i += 256) {
    const float4 v = xs[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) ws[(int64_t)n * gridDim.x + blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void l2norm_scale_kernel(const float* __restrict__ x, int HW, int C, float scale,
                                                           float eps, const float* __restrict__ ws,
                                                           float* __restrict__ y_nhwc, float* __restrict__ y_nchw) {
  // pixel rows padded by 4 floats: the transposed read (16 pixels of one channel per 16 lanes) strides C + 4 words, so
  // a 32-lane group covers 32 distinct banks (unpadded, C % 64 == 0 put all 16 pixels on one bank: 88 % of the
  // kernel's LDS cycles were conflicts, r05_pmc_mfma_dimp_b1.txt); the float4 stores stay 16-B aligned
  constexpr int kPad = 4;
  __shared__ __attribute__((aligned(16))) float tile[kL2Pix * (kL2MaxC + kPad)];
  __shared__ float fsh;
  const int n = blockIdx.y, p0 = blockIdx.x * kL2Pix, np = min(kL2Pix, HW - p0);
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < (int)gridDim.x; ++k) t += ws[(int64_t)n * gridDim.x + k];
    fsh = sqrtf((1.0f / (t + eps)) * ((float)HW * (float)C)) * scale;
  }
  __syncthreads();
  const float f = fsh;
  const int64_t base = ((int64_t)n * HW + p0) * C;
  const float4* xs = reinterpret_cast<const float4*>(x + base);
  const int q = np * C / 4;
  for (int i = threadIdx.x; i < q; i += 256) {
    float4 v = xs[i];
    v.x *= f; v.y *= f; v.z *= f; v.w *= f;
    if (y_nhwc) reinterpret_cast<float4*>(y_nhwc + base)[i] = v;
    if (y_nchw) {
      const int p = (i * 4) / C, c = i * 4 - p * C;
      *reinterpret_cast<float4*>(&tile[p * (C + kPad) + c]) = v;
    }
  }
  if (!y_nchw) return;
  __syncthreads();
  float* yo = y_nchw + (int64_t)n * C * HW + p0;
  for (int i = threadIdx.x; i < kL2Pix * C; i += 256) {
    const int c = i / kL2Pix, p = i - c * kL2Pix;
    if (p < np) yo[(int64_t)c * HW + p] = tile[p * (C + kPad) + c];
  }
}

// ---- PrRoIPool2D (prroi_pooling_gpu_impl.cu forward, restated): the integral of the bilinear surface
// through the feature cells over each bin, / bin area; cells outside the map read as 0
__device__ __forceinline__ float prroi_get(const float* d, int h, int w, int H, int W, int C) {
  return (h < 0 || w < 0 || h >= H || w >= W) ? 0.f : d[((int64_t)h * W + w) * C];
}
__device__ __forceinline__ float prroi_cell(const float* d, int sh, int sw, int eh, int ew, float y0, float x0,
                                            float y1, float x1, int H, int W, int C) {
  float alpha = x0 - (float)sw, beta = y0 - (float)sh;
  float la = x1 - (float)sw, lb = y1 - (float)sh;
  float sum = 0.f, tmp;
  tmp = (la - 0.5f * la * la - alpha + 0.5f * alpha * alpha) * (lb - 0.5f * lb * lb - beta + 0.5f * beta * beta);
  sum += prroi_get(d, sh, sw, H, W, C) * tmp;
  alpha = (float)ew - x1;
  la = (float)ew - x0;
  tmp = (la - 0.5f * la * la - alpha + 0.5f * alpha * alpha) * (lb - 0.5f * lb * lb - beta + 0.5f * beta * beta);
  sum += prroi_get(d, sh, ew, H, W, C) * tmp;
  alpha = x0 - (float)sw;
  beta = (float)eh - y1;
  la = x1 - (float)sw;
  lb = (float)eh - y0;
  tmp = (la - 0.5f * la * la - alpha + 0.5f * alpha * alpha) * (lb - 0.5f * lb * lb - beta + 0.5f * beta * beta);
  sum += prroi_get(d, eh, sw, H, W, C) * tmp;
  alpha = (float)ew - x1;
  la = (float)ew - x0;
  tmp = (la - 0.5f * la * la - alpha + 0.5f * alpha * alpha) * (lb - 0.5f * lb * lb - beta + 0.5f * beta * beta);
  sum += prroi_get(d, eh, ew, H, W, C) * tmp;
  return sum;
}

// feat NHWC [N][H][W][C]; rois [N][4] (x0, y0, x1, y1) image coordinates; out [N][C][PH][PW]
__global__ __launch_bounds__(256) void prroi_kernel(const float* __restrict__ feat, int N, int H, int W, int C,
                                                    const float* __restrict__ rois, float scale, int PH, int PW,
                                                    float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)N * C * PH * PW) return;
  const int pw = (int)(i % PW), ph = (int)((i / PW) % PH), c = (int)((i / PW / PH) % C), n = (int)(i / PW / PH / C);
  const float* r = rois + n * 4;
  const float rsw = r[0] * scale, rsh = r[1] * scale, rew = r[2] * scale, reh = r[3] * scale;
  const float rw = fmaxf(rew - rsw, 0.f), rh = fmaxf(reh - rsh, 0.f);
  const float bh = rh / (float)PH, bw = rw / (float)PW;
  const float ws = rsw + bw * pw, hs = rsh + bh * ph;
  const float we = ws + bw, he = hs + bh;
  const float area = fmaxf(0.f, bw * bh);
  if (area == 0.f) {
    out[i] = 0.f;
    return;
  }
  const float* d = feat + (int64_t)n * H * W * C + c;
  float sum = 0.f;
  const int sw = (int)floorf(ws), ew = (int)ceilf(we), sh = (int)floorf(hs), eh = (int)ceilf(he);
  for (int wi = sw; wi < ew; ++wi)
    for (int hi = sh; hi < eh; ++hi)
      sum += prroi_cell(d, hi, wi, hi + 1, wi + 1, fmaxf(hs, (float)hi), fmaxf(ws, (float)wi), fminf(he, (float)hi + 1.0f),
                        fminf(we, (float)(wi + 1)), H, W, C);
  out[i] = sum / area;
}

// ---- sample_patch: crop rows [tl_y, tl_y + sz_h) x cols [tl_x, tl_x + sz_w) of the df-strided image
// (im[..., os::df, os::df]) with replicate padding, resized to out_h x out_w by F.interpolate(bilinear,
// align_corners=False); float NCHW out [C][out_h][out_w].  The float ops follow ATen's CPU upsample
// (scale = in / out in float, src = max(scale * (dst + 0.5) - 0.5, 0), (x00*w0 + x01*w1)*h0 + (...)*h1).
struct PatchGeom {
  int df, os_y, os_x, tl_y, tl_x, sz_h, sz_w, H2, W2;
};
__device__ __forceinline__ float frame_px(const uint8_t* f, int64_t rs, int C, const PatchGeom& g, int cy, int cx, int c) {
  int r = g.tl_y + cy, q = g.tl_x + cx;
  r = min(max(r, 0), g.H2 - 1);
  q = min(max(q, 0), g.W2 - 1);
  return (float)f[(int64_t)(g.os_y + r * g.df) * rs + (int64_t)(g.os_x + q * g.df) * C + c];
}
__global__ __launch_bounds__(256) void sample_patch_kernel(const uint8_t* __restrict__ f, int64_t rs, int C, PatchGeom g,
                                                           int oh, int ow, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)oh * ow) return;
  const int oy = (int)(i / ow), ox = (int)(i - (int64_t)oy * ow);
  if (g.sz_h == oh && g.sz_w == ow) {
    for (int c = 0; c < C; ++c) out[(int64_t)c * oh * ow + i] = frame_px(f, rs, C, g, oy, ox, c);
    return;
  }
  // ATen's CPU kernel (UpSampleKernel.cpp, built with FMA contraction): src = scale * (dst + 0.5) - 0.5 as
  // one fma, t = x0 * w0 then += x1 * w1 as an fma, likewise across rows
  const float sy = (float)g.sz_h / (float)oh, sx = (float)g.sz_w / (float)ow;
  float fy = __builtin_fmaf(sy, (float)oy + 0.5f, -0.5f), fx = __builtin_fmaf(sx, (float)ox + 0.5f, -0.5f);
  fy = fy < 0.f ? 0.f : fy;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < g.sz_h - 1 ? 1 : 0), x1 = x0 + (x0 < g.sz_w - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  for (int c = 0; c < C; ++c) {
    const float t0 = __builtin_fmaf(frame_px(f, rs, C, g, y0, x1, c), lx1, frame_px(f, rs, C, g, y0, x0, c) * lx0);
    const float t1 = __builtin_fmaf(frame_px(f, rs, C, g, y1, x1, c), lx1, frame_px(f, rs, C, g, y1, x0, c) * lx0);
    out[(int64_t)c * oh * ow + i] = __builtin_fmaf(t1, ly1, t0 * ly0);
  }
}

// ---- init-sample transforms (augmentation.py): out[c][oy][ox] = T(img)[clamp(oy - top)][clamp(ox - left)]
// (crop_to_output: replicate pad / crop by floor / ceil of (out - in) / 2 plus the transform's shift)
struct PatchTf {
  int kind;            // MMT_TF_*
  int top, left;       // crop_to_output offsets (pad_top, pad_left)
  int ry, rx;          // blur radii
  float fy[33], fx[33];
  double m[6];         // rotate: OpenCV warpAffine matrix (dst -> src, inverted on the host), row-major 2 x 3
};
__device__ __forceinline__ float img_at(const float* im, int E_h, int E_w, int y, int x) {
  return im[(int64_t)y * E_w + x];
}
__global__ __launch_bounds__(256) void patch_tf_kernel(const float* __restrict__ img, int C, int E_h, int E_w, PatchTf t,
                                                       int oh, int ow, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)C * oh * ow) return;
  const int c = (int)(i / ((int64_t)oh * ow));
  const int64_t p = i - (int64_t)c * oh * ow;
  const int oy = (int)(p / ow), ox = (int)(p - (int64_t)oy * ow);
  const int y = min(max(oy - t.top, 0), E_h - 1), x = min(max(ox - t.left, 0), E_w - 1);
  const float* im = img + (int64_t)c * E_h * E_w;
  float v;
  if (t.kind == MMT_TF_FLIP) {
    v = img_at(im, E_h, E_w, y, E_w - 1 - x);
  } else if (t.kind == MMT_TF_BLUR) {
    // vertical pass then horizontal (F.conv2d with zero padding, augmentation.py Blur)
    v = 0.f;
    for (int kx = -t.rx; kx <= t.rx; ++kx) {
      const int xx = x + kx;
      if (xx < 0 || xx >= E_w) continue;
      float col = 0.f;
      for (int ky = -t.ry; ky <= t.ry; ++ky) {
        const int yy = y + ky;
        if (yy < 0 || yy >= E_h) continue;
        col += img_at(im, E_h, E_w, yy, xx) * t.fy[ky + t.ry];
      }
      v += col * t.fx[kx + t.rx];
    }
  } else if (t.kind == MMT_TF_ROTATE) {
    // cv2.warpAffine(INTER_LINEAR, BORDER_REPLICATE) on a float image: source coordinates in 1/32 pixel
    // fixed point (AB_BITS 10, INTER_BITS 5, round_delta 16), bilinear weights from the 32 x 32 table
    const int X0 = __double2int_rn((t.m[1] * y + t.m[2]) * 1024.0) + 16;
    const int Y0 = __double2int_rn((t.m[4] * y + t.m[5]) * 1024.0) + 16;
    const int X = (X0 + __double2int_rn(t.m[0] * x * 1024.0)) >> 5;
    const int Y = (Y0 + __double2int_rn(t.m[3] * x * 1024.0)) >> 5;
    const int sx = X >> 5, sy = Y >> 5;
    const float ax = (float)(X & 31) * (1.0f / 32), ay = (float)(Y & 31) * (1.0f / 32);
    const float w00 = (1.f - ay) * (1.f - ax), w01 = (1.f - ay) * ax, w10 = ay * (1.f - ax), w11 = ay * ax;
    const int x0 = min(max(sx, 0), E_w - 1), x1 = min(max(sx + 1, 0), E_w - 1);
    const int y0 = min(max(sy, 0), E_h - 1), y1 = min(max(sy + 1, 0), E_h - 1);
    v = img_at(im, E_h, E_w, y0, x0) * w00 + img_at(im, E_h, E_w, y0, x1) * w01 + img_at(im, E_h, E_w, y1, x0) * w10 +
        img_at(im, E_h, E_w, y1, x1) * w11;
  } else {
    v = img_at(im, E_h, E_w, y, x);
  }
  out[i] = v;
}

}  // namespace mmt

using namespace mmt;

static inline unsigned blocks_for(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }
static inline int last_err() { return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP; }

extern "C" {

int mmt_conv2d_f32_ld(const float* x, int N, int H, int W, int Cin, int ldx, const float* w, const float* bias, int Cout,
                      int kh, int kw, int stride, int pad, const float* resid, float* y, int ldy, int flags, void* stream) {
  if (!x || !w || !y || N <= 0 || H <= 0 || W <= 0 || Cin <= 0 || ldx < Cin || Cout <= 0 || Cout % 64 || ldy < Cout ||
      ldy % 4 || (reinterpret_cast<uintptr_t>(y) & 15) || (resid && (reinterpret_cast<uintptr_t>(resid) & 15)) ||
      (bias && (reinterpret_cast<uintptr_t>(bias) & 15)) || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0 ||
      (flags & ~(MMT_CONV_RELU | MMT_CONV_MAX | MMT_CONV_W4)) || ((flags & MMT_CONV_W4) && Cin != 3))
    return MMT_E_ARG;
  ConvArgs a{x, w, bias, resid, y, N, H, W, Cin, Cout, kh, kw, stride, pad, 0, 0, flags, ldx, ldy};
  a.Ho = (H + 2 * pad - kh) / stride + 1;
  a.Wo = (W + 2 * pad - kw) / stride + 1;
  if (a.Ho <= 0 || a.Wo <= 0) return MMT_E_ARG;
  const int64_t M = (int64_t)N * a.Ho * a.Wo;
  if (M > (int64_t)1 << 30 || (int64_t)Cout * kh * kw * Cin > (int64_t)1 << 30) return MMT_E_ARG;
  const dim3 grid(blocks_for(M, 64), Cout / 64);
  // the float4 operand loads of the FAST kernels need 16-B aligned pixel rows (a group's channel offset included)
  const bool vec = ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  // 32-deep K-tiles (half the barriers per MFMA) where a tile stays inside one tap; 16 for Cin = 48 / 16
  static const int bk = getenv("MMT_CONV_BK") ? atoi(getenv("MMT_CONV_BK")) : 32;
  if (flags & MMT_CONV_W4)
    hipLaunchKernelGGL((conv_f32_kernel<false, 16, true>), grid, dim3(256), 0, (hipStream_t)stream, a);
  else if (vec && Cin % 32 == 0 && bk == 32)
    hipLaunchKernelGGL((conv_f32_kernel<true, 32>), grid, dim3(256), 0, (hipStream_t)stream, a);
  else if (vec && Cin % 16 == 0)
    hipLaunchKernelGGL((conv_f32_kernel<true, 16>), grid, dim3(256), 0, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL((conv_f32_kernel<false, 16>), grid, dim3(256), 0, (hipStream_t)stream, a);
  return last_err();
}

int mmt_conv2d_f32(const float* x, int N, int H, int W, int Cin, const float* w, const float* bias, int Cout, int kh,
                   int kw, int stride, int pad, const float* resid, float* y, int flags, void* stream) {
  return mmt_conv2d_f32_ld(x, N, H, W, Cin, Cin, w, bias, Cout, kh, kw, stride, pad, resid, y, Cout, flags, stream);
}

int mmt_maxpool2d_f32(const float* x, int N, int H, int W, int C, int k, int stride, int pad, float* y, void* stream) {
  if (!x || !y || N <= 0 || H <= 0 || W <= 0 || C <= 0 || k <= 0 || stride <= 0 || pad < 0 || 2 * pad > k)
    return MMT_E_ARG;
  const int Ho = (H + 2 * pad - k) / stride + 1, Wo = (W + 2 * pad - k) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return MMT_E_ARG;
  if (C % 4 == 0)
    hipLaunchKernelGGL(maxpool4_kernel, dim3(blocks_for((int64_t)N * Ho * Wo * C / 4)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(x), N, H, W, C / 4, k, stride, pad, Ho, Wo,
                       reinterpret_cast<float4*>(y));
  else
    hipLaunchKernelGGL(maxpool_kernel, dim3(blocks_for((int64_t)N * Ho * Wo * C)), dim3(256), 0, (hipStream_t)stream, x,
                       N, H, W, C, k, stride, pad, Ho, Wo, y);
  return last_err();
}

int mmt_image_normalize(const float* im, int N, int C, int H, int W, const float mean[3], const float std_[3],
                        float* out_a, float* out_b, void* stream) {
  if (!im || !mean || !std_ || !out_a || N <= 0 || H <= 0 || W <= 0 || (C != 3 && C != 6) || (C == 6 && !out_b))
    return MMT_E_ARG;
  hipLaunchKernelGGL(normalize_kernel, dim3(blocks_for((int64_t)N * H * W)), dim3(256), 0, (hipStream_t)stream, im, N, C,
                     H, W, mean[0], mean[1], mean[2], std_[0], std_[1], std_[2], out_a, out_b, 3);
  return last_err();
}

int mmt_image_normalize4(const float* im, int N, int C, int H, int W, const float mean[3], const float std_[3],
                         float* out_a, float* out_b, void* stream) {
  if (!im || !mean || !std_ || !out_a || N <= 0 || H <= 0 || W <= 0 || (C != 3 && C != 6) || (C == 6 && !out_b))
    return MMT_E_ARG;
  hipLaunchKernelGGL(normalize_kernel, dim3(blocks_for((int64_t)N * H * W)), dim3(256), 0, (hipStream_t)stream, im, N, C,
                     H, W, mean[0], mean[1], mean[2], std_[0], std_[1], std_[2], out_a, out_b, 4);
  return last_err();
}

size_t mmt_instance_l2norm_ws_bytes(int N, int H, int W) {
  if (N <= 0 || H <= 0 || W <= 0) return 0;
  return (size_t)N * ((H * W + kL2Pix - 1) / kL2Pix) * sizeof(float);
}

int mmt_instance_l2norm(const float* x, int N, int H, int W, int C, float scale, float eps, float* y_nhwc, float* y_nchw,
                        float* ws, void* stream) {
  if (!x || !ws || (!y_nhwc && !y_nchw) || N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 4 || C > kL2MaxC)
    return MMT_E_ARG;
  const int HW = H * W;
  const dim3 grid((HW + kL2Pix - 1) / kL2Pix, N);
  hipLaunchKernelGGL(l2norm_sumsq_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, HW, C, ws);
  hipLaunchKernelGGL(l2norm_scale_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, HW, C, scale, eps, ws, y_nhwc,
                     y_nchw);
  return last_err();
}

int mmt_prroi_pool(const float* feat, int N, int H, int W, int C, const float* rois, float spatial_scale, int PH, int PW,
                   float* out, void* stream) {
  if (!feat || !rois || !out || N <= 0 || H <= 0 || W <= 0 || C <= 0 || PH <= 0 || PW <= 0) return MMT_E_ARG;
  hipLaunchKernelGGL(prroi_kernel, dim3(blocks_for((int64_t)N * C * PH * PW)), dim3(256), 0, (hipStream_t)stream, feat, N,
                     H, W, C, rois, spatial_scale, PH, PW, out);
  return last_err();
}

int mmt_sample_patch(const uint8_t* frame, int H, int W, int C, int64_t row_stride, const int geom[7], int out_h,
                     int out_w, float* out, void* stream) {
  if (!frame || !geom || !out || H <= 0 || W <= 0 || C <= 0 || row_stride < (int64_t)W * C || out_h <= 0 || out_w <= 0)
    return MMT_E_ARG;
  PatchGeom g{geom[0], geom[1], geom[2], geom[3], geom[4], geom[5], geom[6], 0, 0};
  if (g.df < 1 || g.os_y < 0 || g.os_x < 0 || g.os_y >= g.df || g.os_x >= g.df || g.sz_h < 1 || g.sz_w < 1)
    return MMT_E_ARG;
  g.H2 = (H - g.os_y + g.df - 1) / g.df;
  g.W2 = (W - g.os_x + g.df - 1) / g.df;
  if (g.H2 <= 0 || g.W2 <= 0) return MMT_E_ARG;
  hipLaunchKernelGGL(sample_patch_kernel, dim3(blocks_for((int64_t)out_h * out_w)), dim3(256), 0, (hipStream_t)stream,
                     frame, row_stride, C, g, out_h, out_w, out);
  return last_err();
}

int mmt_patch_transform(const float* img, int C, int E_h, int E_w, const mmt_patch_tf* tf, int out_h, int out_w,
                        float* out, void* stream) {
  if (!img || !tf || !out || C <= 0 || E_h <= 0 || E_w <= 0 || out_h <= 0 || out_w <= 0) return MMT_E_ARG;
  PatchTf t{};
  t.kind = tf->kind;
  t.top = tf->top;
  t.left = tf->left;
  if (t.kind == MMT_TF_BLUR) {
    if (tf->blur_ry < 0 || tf->blur_ry > 16 || tf->blur_rx < 0 || tf->blur_rx > 16) return MMT_E_ARG;
    t.ry = tf->blur_ry;
    t.rx = tf->blur_rx;
    for (int k = 0; k < 33; ++k) {
      t.fy[k] = tf->blur_fy[k];
      t.fx[k] = tf->blur_fx[k];
    }
  } else if (t.kind == MMT_TF_ROTATE) {
    for (int k = 0; k < 6; ++k) t.m[k] = tf->affine[k];
  } else if (t.kind != MMT_TF_IDENTITY && t.kind != MMT_TF_FLIP) {
    return MMT_E_ARG;
  }
  hipLaunchKernelGGL(patch_tf_kernel, dim3(blocks_for((int64_t)C * out_h * out_w)), dim3(256), 0, (hipStream_t)stream, img,
                     C, E_h, E_w, t, out_h, out_w, out);
  return last_err();
}

}  // extern "C"
