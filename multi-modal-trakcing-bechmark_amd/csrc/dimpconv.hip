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
#include <stdlib.h>

#include <algorithm>
#include <type_traits>
#include <vector>
#include <cstdio>

#include "../../include/mmtrack.h"
#include "common.h"

namespace mmt {

constexpr int kMaxShards = 64, kShardStride = 32;   // sharded max words: 64 x 128-B lines per tensor

#if defined(CONV_STAMPS)   // tuning builds only: per-workgroup phase cycles of conv_f16x3_deep_kernel
__device__ unsigned long long* g_conv_stamps = nullptr;   // [block][8]
#define CSTAMP_T() (threadIdx.x == 0 ? __builtin_amdgcn_s_memtime() : 0ull)
#else
#define CSTAMP_T() 0ull
#endif
constexpr int kMaxGroups = 2, kMaxSplitK = 8;

struct ConvGroupArgs {            // one convolution of a grouped launch (the RGB / aux backbones' twin layers)
  const float* x;                 // [N][H][W][Cin] fp32
  const uint16_t* wh;             // [Cout][Kp] fp16 halves of w * s_w
  const uint16_t* wl;
  const float* bias;              // [Cout] or null
  const float* resid;             // [M][Cout] or null
  float* y;                       // [M][Cout]
  const float* xmax;              // sharded max|x| words of the input, or null: xscale
  float* ymax;                    // sharded max|y| words of the output (accumulated), or null
  float xscale;                   // static input scale (power of two) when xmax is null
  float inv_w;                    // 1 / s_w
  int flags;
  const float* x2;                // Cin2 > 0: the block input the fused downsample reads ([N][H2][W2][Cin2])
  const float* x2max;             // its sharded max words, or null: x2scale
  float x2scale;
};

struct ConvF16Args {
  ConvGroupArgs g[kMaxGroups];
  float* part;                    // split-K partials [ks][G][M][Cout] (ks > 1)
  int N, H, W, Cin, Cout, kh, kw, stride, pad, Ho, Wo, Kp, ks;
  int xcd_order;                  // conv_f16x3_deep_kernel: XCD-aware tile order (else M tiles fastest)
  // a downsample fused into a 1 x 1 conv3 (conv_f16x3_deep_kernel only): K-tiles from Cin / 32 on read x2 at
  // output pixel (oy, ox) * stride2; 0: none
  int Cin2, H2, W2, stride2;
  int staged_epi;                 // conv_f16x3_deep_kernel (BM 128): the LDS-staged epilogue
};

__device__ __forceinline__ int cswz(int r, int c) { return r * 32 + ((c ^ ((r >> 2) & 2)) << 3); }   // gemm.hip swzk<32>

__device__ __forceinline__ float pow2_scale(float m) {   // 2^(14 - ceil(log2 m)), m > 0
  int e;
  const float f = frexpf(m, &e);   // m = f 2^e, f in [0.5, 1)
  const int c = f == 0.5f ? e - 1 : e;
  return ldexpf(1.0f, 14 - c);
}

__device__ __forceinline__ ConvGroupArgs pick_group(const ConvF16Args& a, int grp) {
  return grp ? a.g[1] : a.g[0];   // a select, not a dynamic index (which would copy the arguments to scratch)
}

// the epilogue arithmetic shared by every conv kernel, spelled out (contraction off, the bias added by an explicit
// fused multiply-add) so that each kernel rounds the same way whatever the compiler would contract:
// conv_lin = acc / (s_w s_a) + bias; conv_tail = + residual, ReLU, the backbones' running max, store
__device__ __forceinline__ f32x4 conv_lin(const ConvGroupArgs& g, const f32x4& acc, float inv, int no) {
#pragma clang fp contract(off)
  if (!g.bias) return acc * inv;
  const float4 b = *reinterpret_cast<const float4*>(g.bias + no);
  return f32x4{__builtin_fmaf(acc[0], inv, b.x), __builtin_fmaf(acc[1], inv, b.y), __builtin_fmaf(acc[2], inv, b.z),
               __builtin_fmaf(acc[3], inv, b.w)};
}
__device__ __forceinline__ f32x4 conv_tail(const ConvGroupArgs& g, f32x4 v, int64_t mo, int no, int Cout) {
#pragma clang fp contract(off)
  if (g.resid) {
    const float4 r = *reinterpret_cast<const float4*>(g.resid + mo * Cout + no);
    v += f32x4{r.x, r.y, r.z, r.w};
  }
  if (g.flags & MMT_CONV_RELU)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  float4* dst = reinterpret_cast<float4*>(g.y + mo * Cout + no);
  if (g.flags & MMT_CONV_MAX) {
    const float4 o = *dst;   // torch.max(color, depth) (dimpnet.py:103)
    v = f32x4{fmaxf(o.x, v[0]), fmaxf(o.y, v[1]), fmaxf(o.z, v[2]), fmaxf(o.w, v[3])};
  }
  *dst = make_float4(v[0], v[1], v[2], v[3]);
  return v;
}
// the split-K path: v = the slices' sum (each slice already scaled) + bias, then the tail
__device__ __forceinline__ f32x4 conv_out(const ConvGroupArgs& g, f32x4 v, int64_t mo, int no, int Cout) {
#pragma clang fp contract(off)
  if (g.bias) {
    const float4 b = *reinterpret_cast<const float4*>(g.bias + no);
    v += f32x4{b.x, b.y, b.z, b.w};
  }
  return conv_tail(g, v, mo, no, Cout);
}

// a wave's FM x FN output fragments (rows mo[i] where mv[i], columns nb + 16 j .. + 3) through conv_out's arithmetic
// in its order, the operands requested together before any is used (the FN bias groups, every fragment's residual)
// through raw buffer loads -- an absent operand is a zero-sized buffer, a row past the map an out-of-range offset, both
// read zeros -- so the FM x FN residual round trips overlap instead of each waiting in place (the K loop's registers
// are dead by now: no register cost); returns the lane's max |y|.  rows = the launch's output rows (M)
template <int FM, int FN>
__device__ __forceinline__ float conv_store_tile(const ConvGroupArgs& g, const f32x4 (&acc)[FM][FN], float inv,
                                                 const int64_t (&mo)[FM], const bool (&mv)[FM], int nb, int Cout,
                                                 int64_t rows) {
#pragma clang fp contract(off)
  if (rows * Cout * 4 >= ((int64_t)1 << 31)) {   // past a 32-bit buffer offset: conv_tail's plain loads
    float ymx = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      if (!mv[i]) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const f32x4 v = conv_tail(g, conv_lin(g, acc[i][j], inv, nb + 16 * j), mo[i], nb + 16 * j, Cout);
#pragma unroll
        for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
      }
    }
    return ymx;
  }
  const rsrc_t rR = make_rsrc(g.resid, g.resid ? rows * Cout * 4 : 0);
  const rsrc_t rB = make_rsrc(g.bias, g.bias ? (int64_t)Cout * 4 : 0);
  f32x4 bv[FN], rv[FM][FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    bv[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, (uint32_t)((nb + 16 * j) * 4), 0, 0));
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const uint32_t vo = mv[i] ? (uint32_t)((mo[i] * Cout + nb + 16 * j) * 4) : kBufOob;
      rv[i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rR, vo, 0, 0));
    }
  float ymx = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    if (!mv[i]) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      f32x4 v = acc[i][j] * inv;
      if (g.bias)
        v = f32x4{__builtin_fmaf(acc[i][j][0], inv, bv[j][0]), __builtin_fmaf(acc[i][j][1], inv, bv[j][1]),
                  __builtin_fmaf(acc[i][j][2], inv, bv[j][2]), __builtin_fmaf(acc[i][j][3], inv, bv[j][3])};
      if (g.resid) v += rv[i][j];
      if (g.flags & MMT_CONV_RELU)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      float4* dst = reinterpret_cast<float4*>(g.y + mo[i] * Cout + nb + 16 * j);
      if (g.flags & MMT_CONV_MAX) {
        const float4 o = *dst;   // torch.max(color, depth) (dimpnet.py:103)
        v = f32x4{fmaxf(o.x, v[0]), fmaxf(o.y, v[1]), fmaxf(o.z, v[2]), fmaxf(o.w, v[3])};
      }
      *dst = make_float4(v[0], v[1], v[2], v[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
    }
  }
  return ymx;
}

// conv_store_tile through the LDS: the workgroup's 128-pixel x BN tile (8 waves: 4 row quarters x 2 column halves,
// FM = 2) goes to `lds` (>= 128 x BN floats; 16-B chunk q of row r at q ^ (r & 7)) as conv_lin's values, then every
// thread takes whole 16-B row chunks -- 32 lanes cover a pixel's 512 B of a 128-wide tile -- adds the residual,
// ReLU and the merge and stores them: full 128-B lines for the output and the residual instead of a fragment's 16
// rows x 16 B per wave instruction (the HBM-bound 1 x 1 convs of layers 1 / 2 spend most of their time here).  Same
// arithmetic, same order as conv_store_tile, so the same bits.  Rows r valid below row_end (row0 + r = the pixel).
template <int FN, int BN>
__device__ __forceinline__ float conv_store_tile_staged(const ConvGroupArgs& g, const f32x4 (&acc)[2][FN], float inv,
                                                        float* lds, int wm, int wn, int lane, int64_t row0,
                                                        int64_t row_end, int n0, int Cout, int64_t rows) {
#pragma clang fp contract(off)
  constexpr int WN = BN / 2, NCH = BN / 4, PER = 128 * NCH / 512;
  const int li = lane & 15, lk = lane >> 4, t = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every LDS-DMA of the K loop has landed
  __syncthreads();                                   // and every wave is past its last fragment read
  const rsrc_t rB = make_rsrc(g.bias, g.bias ? (int64_t)Cout * 4 : 0);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int c = wn * WN + j * 16 + 4 * lk;
    const f32x4 bv = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rB, (uint32_t)((n0 + c) * 4), 0, 0));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = wm * 32 + i * 16 + li;
      f32x4 v = acc[i][j] * inv;
      if (g.bias)
        v = f32x4{__builtin_fmaf(acc[i][j][0], inv, bv[0]), __builtin_fmaf(acc[i][j][1], inv, bv[1]),
                  __builtin_fmaf(acc[i][j][2], inv, bv[2]), __builtin_fmaf(acc[i][j][3], inv, bv[3])};
      *reinterpret_cast<f32x4*>(lds + r * BN + (((c >> 2) ^ (r & 7)) << 2)) = v;
    }
  }
  __syncthreads();
  const rsrc_t rR = make_rsrc(g.resid, g.resid ? rows * Cout * 4 : 0);
  const rsrc_t rY = make_rsrc(g.y, rows * Cout * 4);
  const bool mx = g.flags & MMT_CONV_MAX;
  constexpr int GRP = PER < 4 ? PER : 4;   // residual chunks requested together (registers: 4 x 4 per thread)
  float ymx = 0.f;
#pragma unroll
  for (int k0 = 0; k0 < PER; k0 += GRP) {
    f32x4 res[GRP];
#pragma unroll
    for (int k = 0; k < GRP; ++k) {
      const int idx = t + 512 * (k0 + k), r = idx / NCH, q = idx - r * NCH;
      const uint32_t off = row0 + r < row_end ? (uint32_t)(((row0 + r) * Cout + n0 + 4 * q) * 4) : kBufOob;
      res[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rR, off, 0, 0));
    }
#pragma unroll
    for (int k = 0; k < GRP; ++k) {
      const int idx = t + 512 * (k0 + k), r = idx / NCH, q = idx - r * NCH;
      if (row0 + r >= row_end) continue;
      const uint32_t off = (uint32_t)(((row0 + r) * Cout + n0 + 4 * q) * 4);
      f32x4 v = *reinterpret_cast<const f32x4*>(lds + r * BN + ((q ^ (r & 7)) << 2));
      if (g.resid) v += res[k];
      if (g.flags & MMT_CONV_RELU)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      if (mx) {   // torch.max(color, depth) (dimpnet.py:103): the RGB map already in y
        const f32x4 o = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rY, off, 0, 0));
        v = f32x4{fmaxf(o[0], v[0]), fmaxf(o[1], v[1]), fmaxf(o[2], v[2]), fmaxf(o[3], v[3])};
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rY, off, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
    }
  }
  __syncthreads();   // the LDS is free again (the caller's max fold uses it)
  return ymx;
}

// the workgroup's max|y| into shard word blockIdx-derived: one agent-scope atomic max per workgroup (a per-wave
// atomic put ~1 300 atomics on each of the 64 words for the stem's 10 368 workgroups); every thread calls it
template <int NWAVES>
__device__ __forceinline__ void fold_max(float* ymax, float ymx, int shard, float* wmax /* LDS, NWAVES floats */) {
  ymx = wave_max(ymx);
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = ymx;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = wmax[0];
#pragma unroll
    for (int w = 1; w < NWAVES; ++w) m = fmaxf(m, wmax[w]);
    if (m > 0.f)
      __hip_atomic_fetch_max(reinterpret_cast<unsigned*>(ymax) + (shard % kMaxShards) * kShardStride,
                             __float_as_uint(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

typedef __attribute__((address_space(3))) void* lptr_t;

// one K-tile's activations in flight: 8 fp32 values of one output pixel (split into fp16 hi / lo on the way
// into the LDS); two named sets (no array, so nothing is indexed at run time and nothing goes to scratch)
struct ConvRegs {
  float4 a0, a1;
};

// grid (ceil(M / 128), Cout / BN, G * ks): blockIdx.z = group * ks + K slice
template <int BN, bool STEM>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void conv_f16x3_kernel(const ConvF16Args a) {
  constexpr int BM = 128, BK = 32, NWS = 3;   // W ring depth
  constexpr int WN = BN / 2, FM = 2, FN = WN / 16;
  constexpr int NW = BN / 64;                  // W LDS-DMA pieces (16 rows x 64 B) per wave per K-tile
  constexpr int NA = STEM ? 6 : 2;             // A loads per thread per K-tile
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][2][BM * BK];     // [stage][hi, lo]
  __shared__ __attribute__((aligned(16))) uint16_t sW[NWS][2][BN * BK];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int grp = blockIdx.z / a.ks, slice = blockIdx.z - grp * a.ks;
  const ConvGroupArgs g = pick_group(a, grp);
  const int M = a.N * a.Ho * a.Wo;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  // input scale: the maximum over the producer's 64 shard words (every wave forms it itself)
  float sa = g.xscale;
  if (g.xmax) {
    const float mx = wave_max(g.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  const float inv = g.inv_w / sa;

  // A load slot: row (pixel) t >> 2, K chunk t & 3 (8 values)
  const int ar = t >> 2, ac = t & 3;
  const int m = m0 + ar;
  const bool mval = m < M;
  int iy0 = 0, ix0 = 0;
  uint32_t xrow = 0;   // the pixel's image base (elements)
  if (mval) {
    const int nimg = m / (a.Ho * a.Wo);
    const int r = m - nimg * a.Ho * a.Wo;
    const int oy = r / a.Wo, ox = r - oy * a.Wo;
    iy0 = oy * a.stride - a.pad;
    ix0 = ox * a.stride - a.pad;
    xrow = (uint32_t)(nimg * a.H * a.W * a.Cin);
  }
  // operands through raw buffer loads: a tap outside the image, a row past M or a K-tile past the slice takes
  // an offset past the resource and reads zeros, so every load is issued unconditionally (a branch around a
  // load makes the compiler wait for it in place)
  const rsrc_t rX = make_rsrc(g.x, (int64_t)a.N * a.H * a.W * a.Cin * 4);
  const int nk = a.Kp / BK;
  const int kt0 = (int)((int64_t)slice * nk / a.ks), nt = (int)((int64_t)(slice + 1) * nk / a.ks) - kt0;
  const int cpt = STEM ? 1 : a.Cin / BK;   // K-tiles per tap

  auto load_a = [&](int kt, bool kv, ConvRegs& r) {   // kv false: zeros (a tile past the slice, no traffic)
    if constexpr (STEM) {
      // taps 8 kt + 2 ac, + 1: three channels each (the fourth is the weights' zero pad); a 4-channel input
      // (Cin 4: pixels padded with a zero fourth channel, mmt_image_normalize4) loads a tap as one float4
      if (a.Cin == 4) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tap = kt * 8 + ac * 2 + h;
          const int ky = tap / a.kw, kx = tap - ky * a.kw;
          const int iy = iy0 + ky, ix = ix0 + kx;
          const bool ok = kv && mval && tap < a.kh * a.kw && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
          const uint32_t vo = ok ? (xrow + (uint32_t)((iy * a.W + ix) * 4)) * 4 : kBufOob;
          (h ? r.a1 : r.a0) = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo, 0, 0));
        }
        return;
      }
      float v[2][3];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = kt * 8 + ac * 2 + h;
        const int ky = tap / a.kw, kx = tap - ky * a.kw;
        const int iy = iy0 + ky, ix = ix0 + kx;
        const bool ok = kv && mval && tap < a.kh * a.kw && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
        const uint32_t vo = ok ? (xrow + (uint32_t)((iy * a.W + ix) * 3)) * 4 : kBufOob;
#pragma unroll
        for (int e = 0; e < 3; ++e)
          v[h][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rX, vo + 4 * e, 0, 0));
      }
      r.a0 = make_float4(v[0][0], v[0][1], v[0][2], 0.f);
      r.a1 = make_float4(v[1][0], v[1][1], v[1][2], 0.f);
    } else {
      const int tap = kt / cpt, c0 = (kt - tap * cpt) * BK + ac * 8;
      const int ky = tap / a.kw, kx = tap - ky * a.kw;
      const int iy = iy0 + ky, ix = ix0 + kx;
      const bool ok = kv && mval && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
      const uint32_t vo = ok ? (xrow + (uint32_t)((iy * a.W + ix) * a.Cin + c0)) * 4 : kBufOob;
      r.a0 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo, 0, 0));
      r.a1 = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo + 16, 0, 0));
    }
  };
  // W by LDS-DMA (buffer_load ... lds, no VGPRs): piece p = wave * NW + j holds rows 16 (p % (BN / 16)) .. + 15
  // of image p / (BN / 16); lane writes LDS chunk lane & 3 of row lane >> 2 and loads the source chunk that the
  // cswz swizzle puts there
  // the W pieces are issued as inline asm: the compiler neither orders LDS reads behind them (it cannot tell the
  // ring stages apart and would wait for every DMA before each fragment read) nor counts them; the K loop waits
  // for them itself, and the compiler's own vmcnt waits for the A registers only ever wait longer because of them
  const u32x4 qWh = make_rsrc_words(g.wh, (int64_t)a.Cout * a.Kp * 2);
  const u32x4 qWl = make_rsrc_words(g.wl, (int64_t)a.Cout * a.Kp * 2);
  auto load_w = [&](int kt, bool kv, int st) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int p = wave * NW + j, img = p / (BN / 16), rb = p % (BN / 16);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lptr_t)(&sW[st][img][rb * 16 * BK]));
      const int row = rb * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 2);
      const uint32_t vo = kv ? (uint32_t)(((n0 + row) * a.Kp + c * 8) * 2) : kBufOob;
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
      if (img)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWl), "s"(so), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWh), "s"(so), "{m0}"(dst) : "memory");
    }
  };
  auto pack2 = [&](float x, float y, uint32_t& h, uint32_t& l) {
    uint16_t hx, lx, hy, ly;
    split_h(x * sa, hx, lx);
    split_h(y * sa, hy, ly);
    h = hx | (uint32_t)hy << 16;
    l = lx | (uint32_t)ly << 16;
  };
  auto stash = [&](const ConvRegs& r, int st) {
#if defined(CONV_EXP_NOSTASH)   // tuning experiment only: no A split / LDS write (wrong results)
    if (r.a0.x == 12345.f) *reinterpret_cast<float*>(&sA[st][0][0]) = r.a0.y + r.a1.z;
    return;
#endif
    uint4 hv, lv;
#if defined(CONV_EXP_HIONLY)    // tuning experiment only: hi halves, lo = 0 (wrong results)
    hv.x = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.a0.x * sa, r.a0.y * sa));
    hv.y = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.a0.z * sa, r.a0.w * sa));
    hv.z = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.a1.x * sa, r.a1.y * sa));
    hv.w = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(r.a1.z * sa, r.a1.w * sa));
    lv = make_uint4(0, 0, 0, 0);
#else
    pack2(r.a0.x, r.a0.y, hv.x, lv.x);
    pack2(r.a0.z, r.a0.w, hv.y, lv.y);
    pack2(r.a1.x, r.a1.y, hv.z, lv.z);
    pack2(r.a1.z, r.a1.w, hv.w, lv.w);
#endif
    *reinterpret_cast<uint4*>(&sA[st][0][cswz(ar, ac)]) = hv;
    *reinterpret_cast<uint4*>(&sA[st][1][cswz(ar, ac)]) = lv;
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int sta, int stw) {
    const int c = lane >> 4;
    bf16x8 ah[FM], al[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * 32 + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][0][cswz(row, c)]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][1][cswz(row, c)]);
    }
    // weight fragments one column block at a time (fewer live registers: two workgroups per CU; a dependent
    // 16x16x32 MFMA chain issues at the full rate, MI355X_MICROARCH.md); each accumulator takes Wh*Ah, Wl*Ah,
    // Wh*Al in that order
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&sW[stw][0][cswz(row, c)]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sW[stw][1][cswz(row, c)]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc[i][j] = mfma16<true>(bh, ah[i], acc[i][j]);
#if !defined(CONV_EXP_ONEMFMA)  // tuning experiment only: one MFMA per product (wrong results)
        acc[i][j] = mfma16<true>(bl, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh, al[i], acc[i][j]);
#endif
      }
    }
  };

  // K-tile kt0 + i: A loaded into register set i & 1 two tiles ahead and stashed (split) into LDS stage i & 1
  // one tile ahead; W DMA'd into ring stage i % 3 right after the stash of the tile before (one tile ahead).
  // Issue order per tile: A(i + 2), multiply i, stash A(i + 1) (the compiler's wait for its registers leaves
  // A(i + 2) in flight and retires W(i + 1), issued before it), W(i + 2), then the wait that leaves exactly
  // A(i + 2) and W(i + 2) in flight, and a raw s_barrier (__syncthreads() would wait for every load).  Loads
  // past the slice are zeros into stages nobody reads, so every load and stash is unconditional.
  auto tile_wait = [&]() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NA + NW) : "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  ConvRegs r0, r1;
  load_a(kt0, true, r0);
  load_w(kt0, true, 0);
  load_a(kt0 + 1, nt > 1, r1);
  stash(r0, 0);
  load_w(kt0 + 1, nt > 1, 1);
  tile_wait();
  int sw = 0;   // i % 3
  for (int i = 0; i < nt; i += 2) {
    const int sw2 = sw == 0 ? 2 : sw - 1;   // (i + 2) % 3
    load_a(kt0 + i + 2, i + 2 < nt, r0);
    compute(0, sw);
    stash(r1, 1);
    load_w(kt0 + i + 2, i + 2 < nt, sw2);
    tile_wait();
    sw = sw == 2 ? 0 : sw + 1;
    if (i + 1 >= nt) break;
    const int sw3 = sw == 0 ? 2 : sw - 1;   // (i + 3) % 3
    load_a(kt0 + i + 3, i + 3 < nt, r1);
    compute(1, sw);
    stash(r0, 0);
    load_w(kt0 + i + 3, i + 3 < nt, sw3);
    tile_wait();
    sw = sw == 2 ? 0 : sw + 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the zero-loads past the slice, before the LDS is left

  // lane holds channels n0 + wn * WN + j * 16 + 4 * (lane >> 4) + (0..3) of pixel m0 + wm * 32 + i * 16 + (lane & 15)
  const int li = lane & 15, lk = lane >> 4;
  if (a.ks > 1) {   // a K slice: its share of acc / (s_w s_a), summed in slice order by conv_splitk_reduce
    const int G = gridDim.z / a.ks;
    float* pb = a.part + ((int64_t)slice * G + grp) * M * a.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int mo = m0 + wm * 32 + i * 16 + li;
      if (mo >= M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int no = n0 + wn * WN + j * 16 + 4 * lk;
        const f32x4 v = acc[i][j] * inv;
        *reinterpret_cast<float4*>(pb + (int64_t)mo * a.Cout + no) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }
  float ymx = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int mo = m0 + wm * 32 + i * 16 + li;
    if (mo >= M) continue;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int no = n0 + wn * WN + j * 16 + 4 * lk;
      const f32x4 v = conv_tail(g, conv_lin(g, acc[i][j], inv, no), mo, no, a.Cout);
#pragma unroll
      for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
    }
  }
  // (the operand stages are free: the K loop ended on a barrier after the last multiply)
  if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.y * 7 + blockIdx.z * 13, reinterpret_cast<float*>(&sA[0][0][0]));
}

// The stem (kh x kw / stride on a 4-channel image -- 3 channels padded with a zero one, mmt_image_normalize4 --
// and 64 output channels) as 2-D tiles of 8 x 16 output pixels: the tile's input patch ((8 - 1) s + kh rows x
// (16 - 1) s + kw columns, zeros outside the image) is loaded ONCE, split into fp16 hi / lo into LDS, and every
// K-tile's A fragments are read from it (a tap is 4 channels, 8 B per half); the weights of all K-tiles arrive
// by LDS-DMA alongside.  One dependent round trip per workgroup instead of one per K-tile
// (conv_f16x3_kernel<64, true>: 7 K-tiles of register-staged gathers), with the same products in the same
// order, so the output is that kernel's bit for bit.
// TH: tile rows (8 or 16; 16 halves the weight re-fetch per output pixel, 79 KB of LDS: still two workgroups per CU)
constexpr int kStemTW = 16, kStemMaxKt = 7;
template <int TH>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void conv_stem_f16x3_kernel(const ConvF16Args a) {
  constexpr int kStemTH = TH, kStemMaxP = ((TH - 1) * 2 + 7) * ((kStemTW - 1) * 2 + 7), NPL = (kStemMaxP + 511) / 512;
  constexpr int BN = 64, BK = 32, WN = BN / 2, FM = TH / 4, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) uint16_t sP[2][(kStemMaxP + 1) * 4];   // [hi, lo][pixel][4 ch]; + a zero pixel
  __shared__ __attribute__((aligned(16))) uint16_t sW[kStemMaxKt][2][BN * BK];
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int grp = blockIdx.z;
  const ConvGroupArgs g = pick_group(a, grp);
  const int tiles_x = (a.Wo + kStemTW - 1) / kStemTW, tiles_y = (a.Ho + kStemTH - 1) / kStemTH;
  const int img = blockIdx.x / (tiles_x * tiles_y), trem = blockIdx.x - img * (tiles_x * tiles_y);
  const int ty = trem / tiles_x, tx = trem - ty * tiles_x;
  const int oy0 = ty * kStemTH, ox0 = tx * kStemTW;
  const int PW = (kStemTW - 1) * a.stride + a.kw, NP = ((kStemTH - 1) * a.stride + a.kh) * PW;
  const int iy0 = oy0 * a.stride - a.pad, ix0 = ox0 * a.stride - a.pad;
  const int nk = a.Kp / BK, taps = a.kh * a.kw;

  float sa = g.xscale;
  if (g.xmax) {
    const float mx = wave_max(g.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  const float inv = g.inv_w / sa;

  // the weights of every K-tile: one 16-row x 64-B piece per wave and K-tile (conv_f16x3_kernel's load_w, BN = 64)
  const u32x4 qWh = make_rsrc_words(g.wh, (int64_t)a.Cout * a.Kp * 2);
  const u32x4 qWl = make_rsrc_words(g.wl, (int64_t)a.Cout * a.Kp * 2);
  {
    const int wimg = wave / (BN / 16), rb = wave % (BN / 16);
    const int row = rb * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 2);
    const uint32_t vo = (uint32_t)((row * a.Kp + c * 8) * 2);
    for (int kt = 0; kt < nk; ++kt) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lptr_t)(&sW[kt][wimg][rb * 16 * BK]));
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
      if (wimg)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWl), "s"(so), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWh), "s"(so), "{m0}"(dst) : "memory");
    }
  }
  // the input patch: pixel q = t + 512 k of the patch, one float4 (4 channels) each
  const rsrc_t rX = make_rsrc(g.x, (int64_t)a.N * a.H * a.W * 16);
  float4 pv[NPL];
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int q = t + 512 * k, py = q / PW, px = q - py * PW;
    const int iy = iy0 + py, ix = ix0 + px;
    const bool ok = q < NP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    const uint32_t vo = ok ? (uint32_t)(((img * a.H + iy) * a.W + ix) * 16) : kBufOob;
    pv[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo, 0, 0));
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int q = t + 512 * k;
    if (q < NP) {
      uint16_t h[4], l[4];
      split_h(pv[k].x * sa, h[0], l[0]);
      split_h(pv[k].y * sa, h[1], l[1]);
      split_h(pv[k].z * sa, h[2], l[2]);
      split_h(pv[k].w * sa, h[3], l[3]);
      *reinterpret_cast<uint2*>(&sP[0][q * 4]) = make_uint2(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16);
      *reinterpret_cast<uint2*>(&sP[1][q * 4]) = make_uint2(l[0] | (uint32_t)l[1] << 16, l[2] | (uint32_t)l[3] << 16);
    }
  }
  if (t < 2) *reinterpret_cast<uint2*>(&sP[t][kStemMaxP * 4]) = make_uint2(0u, 0u);   // the zero taps' pixel
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment row = local pixel wm * 16 FM + i * 16 + (lane & 15): tile row wm * FM + i, column lane & 15; K chunk
  // lane >> 4 = taps 8 kt + 2 (lane >> 4) + (0, 1), 4 channels each (conv_f16x3_kernel's STEM K order)
  const int c = lane >> 4, col = lane & 15;
  for (int kt = 0; kt < nk; ++kt) {
    bf16x8 ah[FM], al[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int r = wm * FM + i;
      uint2 hv[2], lv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = kt * 8 + 2 * c + h, ky = tap / a.kw, kx = tap - ky * a.kw;
        const int pix = tap < taps ? (r * a.stride + ky) * PW + col * a.stride + kx : kStemMaxP;
        hv[h] = *reinterpret_cast<const uint2*>(&sP[0][pix * 4]);
        lv[h] = *reinterpret_cast<const uint2*>(&sP[1][pix * 4]);
      }
      ah[i] = __builtin_bit_cast(bf16x8, make_uint4(hv[0].x, hv[0].y, hv[1].x, hv[1].y));
      al[i] = __builtin_bit_cast(bf16x8, make_uint4(lv[0].x, lv[0].y, lv[1].x, lv[1].y));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&sW[kt][0][cswz(row, c)]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sW[kt][1][cswz(row, c)]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc[i][j] = mfma16<true>(bh, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bl, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh, al[i], acc[i][j]);
      }
    }
  }

  const int lk = lane >> 4;
  float ymx = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int oy = oy0 + wm * FM + i, ox = ox0 + col;
    if (oy >= a.Ho || ox >= a.Wo) continue;
    const int64_t mo = ((int64_t)img * a.Ho + oy) * a.Wo + ox;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int no = wn * WN + j * 16 + 4 * lk;
      const f32x4 v = conv_tail(g, conv_lin(g, acc[i][j], inv, no), mo, no, a.Cout);
#pragma unroll
      for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
    }
  }
  __syncthreads();   // the patch is free for the max fold
  if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.z * 13, reinterpret_cast<float*>(&sP[0][0]));
}

// The stem with ResNet's max-pool (3 x 3 / stride 2 / pad 1, dimpnet.py's backbone conv1 -> bn1 -> relu -> maxpool)
// fused in (MMT_CONV_POOL): a workgroup owns an 8 x 8 tile of POOLED outputs, computes the 17 x 17 stem outputs
// their windows read (rows 16 ty - 1 .. 16 ty + 15; the shared edge row / column is computed by both neighbours), max-
// pools them from the LDS and writes only the pooled map -- the full-resolution stem map (4x the pooled bytes) is never
// written or read back, and the separate max-pool launch goes.  The 289 stem pixels run as 19 MFMA row fragments
// (five per wave row, the twentieth idle) over the conv_stem_f16x3_kernel K order; same products, same order, and the
// window max in maxpool4_kernel's order over the valid pixels (-inf elsewhere): the pooled map is the two kernels'
// bit for bit.  7 x 7 / stride 2 / 4 channels / 64 outputs only: K = 49 taps x 4 = 196, so the last of the seven
// 32-deep K-tiles holds one tap and only its first 16-B chunk of each weight row is staged (the other three lanes'
// fragments read the same finite weights against the zero pixel).
constexpr int kPoolT = 8, kPoolS = 2 * kPoolT + 1, kPoolPx = kPoolS * kPoolS;   // 8 x 8 pooled, 17 x 17 stem
constexpr int kPoolPW = (kPoolS - 1) * 2 + 7, kPoolMaxP = kPoolPW * kPoolPW;      // 39 x 39 input pixels
constexpr int kPoolHalf = (kPoolPW + 1) / 2;                                         // a row's even columns
constexpr int kPoolLdsP = 2 * (kPoolMaxP + 1) * 4 * 2;                               // patch hi / lo (+ zero pixel)
constexpr int kPoolLdsW = 6 * 2 * 64 * 32 * 2 + 2 * 64 * 8 * 2;                     // K-tiles 0-5, chunk 0 of 6
constexpr int kPoolLds = kPoolLdsP + kPoolLdsW > kPoolPx * 64 * 4 ? kPoolLdsP + kPoolLdsW : kPoolPx * 64 * 4;
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void conv_stem_pool_f16x3_kernel(
    const ConvF16Args a, int PHo, int PWo) {
  constexpr int BN = 64, BK = 32, WN = BN / 2, FM = 5, FN = WN / 16, NPL = (kPoolMaxP + 511) / 512;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kPoolLds];
  uint16_t* sPh = reinterpret_cast<uint16_t*>(lds);
  uint16_t* sPl = sPh + (kPoolMaxP + 1) * 4;
  uint16_t* sW = reinterpret_cast<uint16_t*>(lds + kPoolLdsP);          // [6][2][64 x 32], cswz rows
  uint16_t* sW6 = sW + 6 * 2 * BN * BK;                                  // [2][64][8]: K-tile 6, chunk 0
  float* sOut = reinterpret_cast<float*>(lds);                           // [289][64] after the K loop
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const ConvGroupArgs g = pick_group(a, blockIdx.z);
  const int tiles_x = (PWo + kPoolT - 1) / kPoolT, tiles_y = (PHo + kPoolT - 1) / kPoolT;
  const int img = blockIdx.x / (tiles_x * tiles_y), trem = blockIdx.x - img * (tiles_x * tiles_y);
  const int ty = trem / tiles_x, tx = trem - ty * tiles_x;
  const int sy0 = 2 * kPoolT * ty - 1, sx0 = 2 * kPoolT * tx - 1;       // the stem tile's first output row / col
  const int iy0 = sy0 * 2 - a.pad, ix0 = sx0 * 2 - a.pad;

  float sa = g.xscale;
  if (g.xmax) {
    const float mx = wave_max(g.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  const float inv = g.inv_w / sa;

  const u32x4 qWh = make_rsrc_words(g.wh, (int64_t)a.Cout * a.Kp * 2);
  const u32x4 qWl = make_rsrc_words(g.wl, (int64_t)a.Cout * a.Kp * 2);
  {
    const int wimg = wave / (BN / 16), rb = wave % (BN / 16);
    const int row = rb * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 2);
    const uint32_t vo = (uint32_t)((row * a.Kp + c * 8) * 2);
    for (int kt = 0; kt < 6; ++kt) {
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lptr_t)(&sW[(kt * 2 + wimg) * BN * BK + rb * 16 * BK]));
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
      if (wimg)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWl), "s"(so), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWh), "s"(so), "{m0}"(dst) : "memory");
    }
    if (wave < 2) {   // K-tile 6, chunk 0 (K 192-199) of row = lane: 16 B per lane, rows contiguous
      const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lptr_t)(&sW6[wave * BN * 8]));
      const uint32_t vo6 = (uint32_t)((lane * a.Kp + 6 * BK) * 2);
      if (wave)
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(vo6), "s"(qWl), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(vo6), "s"(qWh), "{m0}"(dst) : "memory");
    }
  }
  const rsrc_t rX = make_rsrc(g.x, (int64_t)a.N * a.H * a.W * 16);
  float4 pv[NPL];
  int lq[NPL];   // the pixel's LDS slot: each patch row stores its even columns, then its odd ones (see below)
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int q = t + 512 * k, py = q / kPoolPW, px = q - py * kPoolPW;
    lq[k] = py * kPoolPW + (px & 1) * kPoolHalf + (px >> 1);
    const int iy = iy0 + py, ix = ix0 + px;
    const bool ok = q < kPoolMaxP && iy >= 0 && iy < a.H && ix >= 0 && ix < a.W;
    const uint32_t vo = ok ? (uint32_t)(((img * a.H + iy) * a.W + ix) * 16) : kBufOob;
    pv[k] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo, 0, 0));
  }
#pragma unroll
  for (int k = 0; k < NPL; ++k) {
    const int q = t + 512 * k;
    if (q < kPoolMaxP) {
      uint16_t h[4], l[4];
      split_h(pv[k].x * sa, h[0], l[0]);
      split_h(pv[k].y * sa, h[1], l[1]);
      split_h(pv[k].z * sa, h[2], l[2]);
      split_h(pv[k].w * sa, h[3], l[3]);
      *reinterpret_cast<uint2*>(&sPh[lq[k] * 4]) = make_uint2(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16);
      *reinterpret_cast<uint2*>(&sPl[lq[k] * 4]) = make_uint2(l[0] | (uint32_t)l[1] << 16, l[2] | (uint32_t)l[3] << 16);
    }
  }
  if (t < 2) *reinterpret_cast<uint2*>(&(t ? sPl : sPh)[kPoolMaxP * 4]) = make_uint2(0u, 0u);   // the zero pixel
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // fragment i of wave row wm: stem pixels p = (wm + 4 i) * 16 + (lane & 15) of the 17 x 17 tile (p >= 289: idle).
  // The stride-2 stem reads input columns 2 sc + kx: with each patch row stored as its even columns then its odd ones,
  // the 16 lanes of a fragment column read 16 consecutive 8-B slots (32 banks) for any tap, and the next lane group's
  // tap (kx + 2, same parity) the slots one further -- the same addresses but for its last lane, whose banks are free.
  // Interleaved, the slots were 16 B apart and that last lane met lane 0's banks: 38 % of the kernel's LDS cycles
  // were bank conflicts (r05_pmc_mfma_dimp_b1.txt)
  const int c = lane >> 4, col = lane & 15;
  int pbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int p = (wm + 4 * i) * 16 + col, sr = p / kPoolS, sc = p - sr * kPoolS;
    pbase[i] = p < kPoolPx ? (sr * 2) * kPoolPW + sc : -1;
  }
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool last_idle = wm == 3;   // fragment 19 (wave row 3, i = 4) holds no pixel
#pragma unroll
  for (int kt = 0; kt < 7; ++kt) {
    bf16x8 ah[FM], al[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      uint2 hv[2], lv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int tap = kt * 8 + 2 * c + h, ky = tap / 7, kx = tap - ky * 7;
        const int pix = tap < 49 && pbase[i] >= 0 ? pbase[i] + ky * kPoolPW + (kx & 1) * kPoolHalf + (kx >> 1)
                                                  : kPoolMaxP;
        hv[h] = *reinterpret_cast<const uint2*>(&sPh[pix * 4]);
        lv[h] = *reinterpret_cast<const uint2*>(&sPl[pix * 4]);
      }
      ah[i] = __builtin_bit_cast(bf16x8, make_uint4(hv[0].x, hv[0].y, hv[1].x, hv[1].y));
      al[i] = __builtin_bit_cast(bf16x8, make_uint4(lv[0].x, lv[0].y, lv[1].x, lv[1].y));
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      bf16x8 bh, bl;
      if (kt < 6) {
        bh = *reinterpret_cast<const bf16x8*>(&sW[(kt * 2 + 0) * BN * BK + cswz(row, c)]);
        bl = *reinterpret_cast<const bf16x8*>(&sW[(kt * 2 + 1) * BN * BK + cswz(row, c)]);
      } else {
        bh = *reinterpret_cast<const bf16x8*>(&sW6[row * 8]);
        bl = *reinterpret_cast<const bf16x8*>(&sW6[BN * 8 + row * 8]);
      }
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        if (i == FM - 1 && last_idle) continue;
        acc[i][j] = mfma16<true>(bh, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bl, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh, al[i], acc[i][j]);
      }
    }
  }
  __syncthreads();   // the patch and weights are free: the stem tile goes to sOut

  // bias + ReLU per stem pixel (-inf outside the stem map: the pool's padding); 16-B chunk q of pixel p at
  // q ^ (p & 15) (the 16 lanes of one fragment column write 16 distinct chunks: no bank conflict)
  const int lk = lane >> 4;
  float ymx = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int p = (wm + 4 * i) * 16 + col;
    if (p >= kPoolPx) continue;
    const int sr = p / kPoolS, sc = p - sr * kPoolS, oy = sy0 + sr, ox = sx0 + sc;
    const bool valid = oy >= 0 && oy < a.Ho && ox >= 0 && ox < a.Wo;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int no = wn * WN + j * 16 + 4 * lk;
      f32x4 v = conv_lin(g, acc[i][j], inv, no);   // (the stem kernel's arithmetic: bit-identical to stem + pool)
      if (g.flags & MMT_CONV_RELU)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      if (valid) {
#pragma unroll
        for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
      } else {
        v = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      }
      *reinterpret_cast<f32x4*>(&sOut[p * 64 + (((no >> 2) ^ (p & 15)) << 2)]) = v;
    }
  }
  __syncthreads();
  // the pooled 8 x 8 tile: thread t takes 4 channels (chunk t & 15) of pooled pixels t >> 4 and (t >> 4) + 32
  {
    const int q = t & 15;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pq = (t >> 4) + 32 * h, pr = pq >> 3, pc = pq & 7;
      const int py = kPoolT * ty + pr, px = kPoolT * tx + pc;
      if (py >= PHo || px >= PWo) continue;
      f32x4 m = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
      for (int dy = 0; dy < 3; ++dy)
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
          const int p = (2 * pr + dy) * kPoolS + 2 * pc + dx;
          const f32x4 v = *reinterpret_cast<const f32x4*>(&sOut[p * 64 + ((q ^ (p & 15)) << 2)]);
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], v[e]);
        }
      *reinterpret_cast<float4*>(g.y + (((int64_t)img * PHo + py) * PWo + px) * 64 + 4 * q) =
          make_float4(m[0], m[1], m[2], m[3]);
    }
  }
  __syncthreads();   // sOut is free for the max fold
  if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.z * 13, reinterpret_cast<float*>(lds));
}

// The generic conv with a deeper operand pipeline.  conv_f16x3_kernel keeps one K-tile of weights and two of
// activations in flight per workgroup (about 48 KB), which, at the several-microsecond latency of a loaded memory
// system, caps a workgroup near 20 GB/s and the K loop at about 1.5 us per 32-deep K-tile -- measured: removing two
// of the three MFMAs and the whole activation split / stash together saves only a third of the kernel's time.  Here
// the activation loads are inline-asm buffer loads (the compiler neither counts nor waits for them; every wait is
// written out, naming the registers it guards), so the weights can go two K-tiles ahead into the three-stage ring and
// the activations NR K-tiles ahead into NR register sets without the compiler draining one queue to reach the other.
// Step j issues W(j + 2) then A(j + NR), multiplies K-tile j, waits for A(j + 1) -- 2 (NW + NA) younger operations
// (for NR = 3) -- and stashes it, then waits for W(j + 1) and passes the barrier.  Same products, same summation
// order as conv_f16x3_kernel (bit-identical).
// BM = 256 (tuning, MMT_CONV_BM=256): 64 x 64 per wave -- 16 fragment reads per 48 MFMAs instead of 12 per 24, one
// barrier per 48 -- at one workgroup per CU (112 KB of LDS)
// OVL: K-tile j + 1's activations are waited for BEFORE K-tile j is multiplied, and split and stashed in the same
// scheduling region as its MFMAs (no inline asm between them), so the split's VALU work and the LDS stores issue
// between the MFMAs instead of after them while every wave of the CU sits in the same phase between two barriers.
template <int BN, int NR, int BM = 128, bool OVL = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(BM == 128 ? 4 : 2))) void conv_f16x3_deep_kernel(
    const ConvF16Args a) {
  constexpr int BK = 32, NWS = 3;
  constexpr int WN = BN / 2, FM = BM / 64, FN = WN / 16;
  constexpr int SL = BM / 128;                 // activation slots (a row's 8 K values) per thread
  constexpr int NW = BN / 64;                  // W LDS-DMA pieces per wave per K-tile
  constexpr int NA = 2 * SL;                   // A loads per thread per K-tile
  constexpr int WAIT_A = (NR - 1) * (NW + NA); // younger operations when A(j + 1) is waited for
  constexpr int WAIT_W = 2 * NA + NW;          // ... when W(j + 1) is (A(j + NR - 1), W(j + 2), A(j + NR))
  constexpr int WAIT_AE = (NR - 2) * (NW + NA); // OVL: ... when A(j + 1) is, before step j's loads
  static_assert(NR == 2 || NR == 3, "register sets");
  // one LDS array (the operand rings, then the epilogue's staged tile: 128 x BN floats <= its size)
  __shared__ __attribute__((aligned(16))) uint16_t smem_dk[2 * 2 * BM * BK + NWS * 2 * BN * BK];
  auto& sA = *reinterpret_cast<uint16_t(*)[2][2][BM * BK]>(smem_dk);
  auto& sW = *reinterpret_cast<uint16_t(*)[NWS][2][BN * BK]>(smem_dk + 2 * 2 * BM * BK);
  static_assert(BM != 128 || 128 * BN * 4 <= (int)sizeof(smem_dk), "staged epilogue tile");
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int grp = blockIdx.z / a.ks, slice = blockIdx.z - grp * a.ks;
  const ConvGroupArgs g = pick_group(a, grp);
  const int M = a.N * a.Ho * a.Wo;
  // XCD-aware tile order (grid.x = M tiles x N tiles): the workgroups of XCD x (= b % 8) take a contiguous range of
  // tile ids, N fastest, so the column-tile siblings of an activation tile run on one XCD and share its L2 (the
  // activation tile is fetched from beyond the L2 once per XCD instead of once per column tile)
  // (the default: mfDiMP 6 350 -> 6 394 frames/s in two rounds; applied only to wide outputs and short launches it
  // measured level, although layer1 conv3 alone, without its residual, runs 128 -> 150 us in this order;
  // MMT_CONV_XCD=0: M tiles fastest over the whole chip, profiles/r04_ab_conv_xcd_order.txt)
  int m0, n0;
  {
    const int gn = a.Cout / BN, ntl = gridDim.x, b = blockIdx.x;
    if (a.xcd_order) {
      const int x = b & 7, j = b >> 3, q = ntl >> 3, r8 = ntl & 7;
      const int id = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + j;
      m0 = (id / gn) * BM;
      n0 = (id - (id / gn) * gn) * BN;
    } else {
      const int gm = ntl / gn;
      m0 = (b % gm) * BM;
      n0 = (b / gm) * BN;
    }
  }

  float sa = g.xscale;
  if (g.xmax) {
    const float mx = wave_max(g.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  // fused downsample: both sources split at the smaller scale, so one accumulator holds both sums
  const bool ds = a.Cin2 > 0;
  if (ds) {
    float sb = g.x2scale;
    if (g.x2max) {
      const float mx = wave_max(g.x2max[lane * kShardStride]);
      sb = mx > 0.f ? pow2_scale(mx) : 1.0f;
    }
    sa = fminf(sa, sb);
  }
  const float inv = g.inv_w / sa;

  const int ac = t & 3;   // slot s: row (t >> 2) + 128 s, K chunk ac (8 values)
  bool mval[SL];
  int iy0[SL], ix0[SL];
  uint32_t xrow[SL], xrow2[SL];
#pragma unroll
  for (int sl = 0; sl < SL; ++sl) {
    const int m = m0 + (t >> 2) + 128 * sl;
    mval[sl] = m < M;
    iy0[sl] = ix0[sl] = 0;
    xrow[sl] = xrow2[sl] = 0;
    if (mval[sl]) {
      const int nimg = m / (a.Ho * a.Wo);
      const int r = m - nimg * a.Ho * a.Wo;
      const int oy = r / a.Wo, ox = r - oy * a.Wo;
      iy0[sl] = oy * a.stride - a.pad;
      ix0[sl] = ox * a.stride - a.pad;
      xrow[sl] = (uint32_t)(nimg * a.H * a.W * a.Cin);
      // the downsample's input pixel (1 x 1, no padding): its float offset, channel 0
      if (ds) xrow2[sl] = (uint32_t)(((nimg * a.H2 + oy * a.stride2) * a.W2 + ox * a.stride2) * a.Cin2);
    }
  }
  const u32x4 qX = make_rsrc_words(g.x, (int64_t)a.N * a.H * a.W * a.Cin * 4);
  const u32x4 qX2 = make_rsrc_words(ds ? g.x2 : g.x, ds ? (int64_t)a.N * a.H2 * a.W2 * a.Cin2 * 4 : 0);
  const int nk1 = ds ? a.Cin / BK : 1 << 30;   // K-tiles of the first source (1 x 1 conv3: its Cin)
  const int nk = a.Kp / BK;
  const int kt0 = (int)((int64_t)slice * nk / a.ks), nt = (int)((int64_t)(slice + 1) * nk / a.ks) - kt0;
  const int cpt = a.Cin / BK;

  struct DeepRegs {   // native vectors: an inline-asm register operand, not a struct in memory
    f32x4 a[2 * SL];
  };
  DeepRegs r[NR];
  // K-tile i of the slice (zeros past it: an out-of-range offset, no traffic) into register set `set`.  The calls
  // come in order i = 0, 1, 2, ...: the (tap, chunk) position advances by one chunk per call (wave-uniform
  // counters instead of two integer divisions per K-tile)
  int a_ch, a_ky, a_kx;
  {
    const int tap = kt0 / cpt;
    a_ch = kt0 - tap * cpt;
    a_ky = tap / a.kw;
    a_kx = tap - a_ky * a.kw;
  }
  auto load_a = [&](int i, DeepRegs& set) {
    const int c0 = a_ch * BK + ac * 8, ky = a_ky, kx = a_kx;
    if (++a_ch == cpt) {
      a_ch = 0;
      if (++a_kx == a.kw) {
        a_kx = 0;
        ++a_ky;
      }
    }
    // the fused downsample's K-tiles (wave-uniform; selects, not a branch, so the loads stay straight-line code for
    // tools/isa_audit.py): x2 at the output pixel's stride2 position
    const bool second = kt0 + i >= nk1;
    const int c2 = (kt0 + i - nk1) * BK + ac * 8;
    const u32x4 qA = second ? qX2 : qX;
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      const int iy = iy0[sl] + ky, ix = ix0[sl] + kx;
      // (bitwise, not short-circuit: no control flow around the loads)
      const bool inb = (iy >= 0) & (iy < a.H) & (ix >= 0) & (ix < a.W);
      const bool ok = (i < nt) & mval[sl] & (second | inb);
      const uint32_t off1 = xrow[sl] + (uint32_t)((iy * a.W + ix) * a.Cin + c0), off2 = xrow2[sl] + (uint32_t)c2;
      const uint32_t vo = ok ? (second ? off2 : off1) * 4 : kBufOob;
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(set.a[2 * sl]) : "v"(vo), "s"(qA) : "memory");
      asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:16" : "=v"(set.a[2 * sl + 1]) : "v"(vo), "s"(qA)
                   : "memory");
    }
  };
  const u32x4 qWh = make_rsrc_words(g.wh, (int64_t)a.Cout * a.Kp * 2);
  const u32x4 qWl = make_rsrc_words(g.wl, (int64_t)a.Cout * a.Kp * 2);
  auto load_w = [&](int i, int st) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int p = wave * NW + j, img = p / (BN / 16), rb = p % (BN / 16);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lptr_t)(&sW[st][img][rb * 16 * BK]));
      const int row = rb * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 2);
      const uint32_t vo = i < nt ? (uint32_t)(((n0 + row) * a.Kp + c * 8) * 2) : kBufOob;
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)((kt0 + i) * BK * 2));
      if (img)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWl), "s"(so), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWh), "s"(so), "{m0}"(dst) : "memory");
    }
  };
  // the register set's loads done: all but the CNT youngest vector-memory operations (the set named as read-write,
  // so nothing reads it above this point)
  auto wait_set = [&](DeepRegs& set, auto cnt) {
    if constexpr (SL == 1)
      asm volatile("s_waitcnt vmcnt(%2)" : "+v"(set.a[0]), "+v"(set.a[1]) : "n"(decltype(cnt)::value) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(%4)" : "+v"(set.a[0]), "+v"(set.a[1]), "+v"(set.a[2]), "+v"(set.a[3])
                   : "n"(decltype(cnt)::value) : "memory");
  };
  auto keep_set = [&](DeepRegs& set) {   // the set's registers live up to here (no code, no wait)
    if constexpr (SL == 1)
      asm volatile("" : "+v"(set.a[0]), "+v"(set.a[1]));
    else
      asm volatile("" : "+v"(set.a[0]), "+v"(set.a[1]), "+v"(set.a[2]), "+v"(set.a[3]));
  };
  auto pack2 = [&](float x, float y, uint32_t& h, uint32_t& l) {
    uint16_t hx, lx, hy, ly;
    split_h(x * sa, hx, lx);
    split_h(y * sa, hy, ly);
    h = hx | (uint32_t)hy << 16;
    l = lx | (uint32_t)ly << 16;
  };
  auto stash = [&](const DeepRegs& rr, int st) {
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      const f32x4 &x0 = rr.a[2 * sl], &x1 = rr.a[2 * sl + 1];
      uint4 hv, lv;
      pack2(x0[0], x0[1], hv.x, lv.x);
      pack2(x0[2], x0[3], hv.y, lv.y);
      pack2(x1[0], x1[1], hv.z, lv.z);
      pack2(x1[2], x1[3], hv.w, lv.w);
      const int ar = (t >> 2) + 128 * sl;
      *reinterpret_cast<uint4*>(&sA[st][0][cswz(ar, ac)]) = hv;
      *reinterpret_cast<uint4*>(&sA[st][1][cswz(ar, ac)]) = lv;
    }
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int sta, int stw) {
    const int c = lane >> 4;
    bf16x8 ah[FM], al[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * (BM / 4) + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][0][cswz(row, c)]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][1][cswz(row, c)]);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(&sW[stw][0][cswz(row, c)]);
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(&sW[stw][1][cswz(row, c)]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc[i][j] = mfma16<true>(bh, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bl, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh, al[i], acc[i][j]);
      }
    }
  };
  // OVL: K-tile (sta, stw) multiplied with the next K-tile's split woven in: all fragment reads first, then after
  // every other MFMA triple one pack2 (two values) of the split -- fenced (sched_barrier) so the compiler keeps the
  // weave instead of clustering the MFMAs -- and the stash's LDS stores last
  auto compute_split = [&](int sta, int stw, const DeepRegs& rr, int st) {
    const int c = lane >> 4;
    bf16x8 ah[FM], al[FM], bh[FN], bl[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * (BM / 4) + i * 16 + (lane & 15);
      ah[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][0][cswz(row, c)]);
      al[i] = *reinterpret_cast<const bf16x8*>(&sA[sta][1][cswz(row, c)]);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      bh[j] = *reinterpret_cast<const bf16x8*>(&sW[stw][0][cswz(row, c)]);
      bl[j] = *reinterpret_cast<const bf16x8*>(&sW[stw][1][cswz(row, c)]);
    }
    uint32_t hw[4 * SL], lw[4 * SL];
    constexpr int NP = 4 * SL, NT = FM * FN, EVERY = NT / NP > 0 ? NT / NP : 1;
    int p = 0;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        // empty asm on the operands pins the order (instruction selection moves pure operations across fences)
        asm volatile("" : "+v"(acc[i][j]));
        acc[i][j] = mfma16<true>(bh[j], ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bl[j], ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh[j], al[i], acc[i][j]);
        asm volatile("" : "+v"(acc[i][j]));
        __builtin_amdgcn_sched_barrier(0);
        if ((j * FM + i) % EVERY == EVERY - 1 && p < NP) {
          const f32x4& x = rr.a[p >> 1];
          float x0 = x[(p & 1) * 2], x1 = x[(p & 1) * 2 + 1];
          asm volatile("" : "+v"(x0), "+v"(x1));
          pack2(x0, x1, hw[p], lw[p]);
          asm volatile("" : "+v"(hw[p]), "+v"(lw[p]));
          ++p;
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
    for (; p < NP; ++p) {
      const f32x4& x = rr.a[p >> 1];
      pack2(x[(p & 1) * 2], x[(p & 1) * 2 + 1], hw[p], lw[p]);
    }
#pragma unroll
    for (int sl = 0; sl < SL; ++sl) {
      const int ar = (t >> 2) + 128 * sl;
      *reinterpret_cast<uint4*>(&sA[st][0][cswz(ar, ac)]) =
          make_uint4(hw[4 * sl], hw[4 * sl + 1], hw[4 * sl + 2], hw[4 * sl + 3]);
      *reinterpret_cast<uint4*>(&sA[st][1][cswz(ar, ac)]) =
          make_uint4(lw[4 * sl], lw[4 * sl + 1], lw[4 * sl + 2], lw[4 * sl + 3]);
    }
  };
  using CA = std::integral_constant<int, WAIT_A>;

  // prologue: the loads of steps -NR .. -1 (W(j + 2) where j + 2 >= 0, A(j + NR)), so the steady-state counts hold
  // from step 0 on
#pragma unroll
  for (int j = -NR; j < 0; ++j) {
    if (j + 2 >= 0) load_w(j + 2, j + 2);
    load_a(j + NR, r[j + NR]);
  }
  const unsigned long long ts0 = CSTAMP_T();
  wait_set(r[0], CA{});
  stash(r[0], 0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT_W) : "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  unsigned long long tsl = CSTAMP_T(), sum_issue = 0, sum_mma = 0, sum_awt = 0, sum_stash = 0, sum_bar = 0;
  const unsigned long long ts1 = tsl;
  for (int i0 = 0; i0 < nt; i0 += 6) {
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int j = i0 + u;
      if (j >= nt) break;
      unsigned long long tq, tc;
      if constexpr (OVL) {
        wait_set(r[(u + 1) % NR], std::integral_constant<int, WAIT_AE>{});
        tq = CSTAMP_T();
        sum_awt += tq - tsl;
        load_w(j + 2, (u + 2) % 3);
        load_a(j + NR, r[u % NR]);
        tc = CSTAMP_T();
        sum_issue += tc - tq;
        compute_split(u & 1, u % 3, r[(u + 1) % NR], (u + 1) & 1);
#if defined(CONV_STAMPS)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        tq = CSTAMP_T();
        sum_mma += tq - tc;
        tc = tq;
      } else {
        load_w(j + 2, (u + 2) % 3);
        load_a(j + NR, r[u % NR]);
        tq = CSTAMP_T();
        sum_issue += tq - tsl;
        compute(u & 1, u % 3);
#if defined(CONV_STAMPS)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
        tc = CSTAMP_T();
        sum_mma += tc - tq;
        wait_set(r[(u + 1) % NR], CA{});
        tq = CSTAMP_T();
        sum_awt += tq - tc;
        stash(r[(u + 1) % NR], (u + 1) & 1);
        tc = CSTAMP_T();
        sum_stash += tc - tq;
      }
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WAIT_W) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      tsl = CSTAMP_T();
      sum_bar += tsl - tc;
    }
  }
  // the zero-loads past the slice land before the LDS is left -- and before their registers are reused: the last
  // sets' loads are dead to the compiler, which would otherwise hand their registers to the epilogue while the
  // loads are still in flight (the landing zeros then overwrite epilogue values), so every set is named live across
  // the wait
  wait_set(r[0], std::integral_constant<int, 0>{});
#pragma unroll
  for (int k = 1; k < NR; ++k) keep_set(r[k]);
#if defined(CONV_STAMPS)
  if (threadIdx.x == 0 && g_conv_stamps) {
    const size_t bid = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    unsigned long long* o = g_conv_stamps + bid * 8;
    o[0] = ts1 - ts0; o[1] = sum_issue; o[2] = sum_mma; o[3] = sum_awt; o[4] = sum_stash; o[5] = sum_bar;
    o[6] = (unsigned long long)nt; o[7] = tsl - ts0;
  }
#else
  (void)ts0; (void)ts1; (void)sum_issue; (void)sum_mma; (void)sum_awt; (void)sum_stash; (void)sum_bar;
#endif

  const int li = lane & 15, lk = lane >> 4;
  if (a.ks > 1) {
    const int G = gridDim.z / a.ks;
    float* pb = a.part + ((int64_t)slice * G + grp) * M * a.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int mo = m0 + wm * (BM / 4) + i * 16 + li;
      if (mo >= M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int no = n0 + wn * WN + j * 16 + 4 * lk;
        const f32x4 v = acc[i][j] * inv;
        *reinterpret_cast<float4*>(pb + (int64_t)mo * a.Cout + no) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }
  float ymx;
  if constexpr (BM == 128) {
    if (a.staged_epi && (int64_t)M * a.Cout * 4 < ((int64_t)1 << 31)) {
      ymx = conv_store_tile_staged<FN, BN>(g, acc, inv, reinterpret_cast<float*>(smem_dk), wm, wn, lane, m0, M, n0,
                                           a.Cout, M);
      if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.y * 7 + blockIdx.z * 13, reinterpret_cast<float*>(smem_dk));
      return;
    }
  }
  int64_t mo[FM];
  bool mv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    mo[i] = m0 + wm * (BM / 4) + i * 16 + li;
    mv[i] = mo[i] < M;
  }
  ymx = conv_store_tile<FM, FN>(g, acc, inv, mo, mv, n0 + wn * WN + 4 * lk, a.Cout, M);
  if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.y * 7 + blockIdx.z * 13, reinterpret_cast<float*>(&sA[0][0][0]));
}

// 3 x 3 / stride 1 / pad 1 convolutions with the input PATCH staged once per 32-channel chunk.  The generic kernel
// above gathers, splits and stashes a K-tile of activations for every (tap, chunk) K-tile, so each input element is
// loaded, split into fp16 hi / lo and written to the LDS nine times.  Here a workgroup's tile is 128 consecutive output
// pixels of one image (raster order) and, per chunk of 32 input channels, the rows of the input those pixels' nine taps
// read -- (rows + 2) x (W + 2) pixels, zeros outside the image -- are loaded and split ONCE into an LDS patch; the nine
// taps then read their A fragments from it at pixel offsets (dy, dx), and only the weights (one 32-deep K-tile per tap,
// LDS-DMA into a two-stage ring) move per tap.  Patch layout: pixel P = 64 B per half (32 channels), 16-B chunk q of
// P at q ^ (((P >> 2) & 1) << 1): the fragment reads (16 consecutive pixels x 4 chunks per ds_read_b128 lane group)
// are bank-conflict-free for any start pixel (exhaustive check over start offsets; a tile row that wraps to the next
// image row costs at most one 2-way conflict).  K order: chunk-major, tap-minor (the weights' K-tile tap * Cin / 32 +
// chunk); split-K slices take ranges of chunks.  Same products as conv_f16x3_kernel, summed in a different fp32 order.
constexpr int kPatchMaxPx = 384, kPatchNPL = 6;   // patch pixels (48 KB of fp16 halves), float4 loads per thread
template <int BN>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void conv3x3_patch_f16x3_kernel(
    const ConvF16Args a, int tiles_per_img, int patch_px) {
  constexpr int BM = 128, BK = 32;
  constexpr int WN = BN / 2, FM = 2, FN = WN / 16, NW = BN / 64;
  extern __shared__ __attribute__((aligned(16))) uint16_t dynlds[];
  // fixed offsets (immediate fields of the LDS instructions), sized for the largest patch
  uint16_t* const sPh = dynlds;                          // [kPatchMaxPx][32] hi
  uint16_t* const sPl = dynlds + kPatchMaxPx * 32;       // lo
  uint16_t* const sWb = dynlds + 2 * kPatchMaxPx * 32;   // [2 stages][hi, lo][BN * BK]
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int grp = blockIdx.z / a.ks, slice = blockIdx.z - grp * a.ks;
  const ConvGroupArgs g = pick_group(a, grp);
  const int HW = a.Ho * a.Wo, Wd = a.W, PW = a.W + 2;
  // the tile: global output pixels [g0, gend) -- per image (tiles_per_img > 0: 128 raster pixels of one image) or
  // over the flattened batch (tiles_per_img == 0: no partial tile at each image's end; a tile then spans at most two
  // images, HW >= 128): segment A = image nA's output rows yA0.. (patch rows 0 .. rowsA - 1 with their halo rows),
  // segment B = the next image's first rows (patch rows rowsA .., its own halo above and below)
  int g0, gend, nA, yA0, rowsA, rowsB = 0;
  if (tiles_per_img > 0) {
    const int img = blockIdx.x / tiles_per_img, o0 = (blockIdx.x - img * tiles_per_img) * BM;
    g0 = img * HW + o0;
    gend = img * HW + min(o0 + BM, HW);
  } else {
    g0 = blockIdx.x * BM;
    gend = min(g0 + BM, a.N * HW);
  }
  nA = g0 / HW;
  yA0 = (g0 - nA * HW) / Wd;
  rowsA = (min(gend, (nA + 1) * HW) - nA * HW - 1) / Wd - yA0 + 3;
  if (gend > (nA + 1) * HW) rowsB = (gend - (nA + 1) * HW - 1) / Wd + 3;
  const int npx = (rowsA + rowsB) * PW;   // patch pixels of this tile
  const int n0 = blockIdx.y * BN;

  float sa = g.xscale;
  if (g.xmax) {
    const float mx = wave_max(g.xmax[lane * kShardStride]);
    sa = mx > 0.f ? pow2_scale(mx) : 1.0f;
  }
  const float inv = g.inv_w / sa;

  const int nc = a.Cin / BK;                              // 32-channel chunks
  const int c0 = (int)((int64_t)slice * nc / a.ks), c1 = (int)((int64_t)(slice + 1) * nc / a.ks);

  // the patch: float4 f = t + 512 j is channels 4 (f & 7) .. + 3 of patch pixel f >> 3
  const rsrc_t rX = make_rsrc(g.x, (int64_t)a.N * a.H * a.W * a.Cin * 4);
  float4 pv[kPatchNPL];
  auto load_patch = [&](int c) {
#pragma unroll
    for (int j = 0; j < kPatchNPL; ++j) {
      const int f = t + 512 * j, px = f >> 3, part = f & 7;
      const int pr = px / PW, pc = px - pr * PW;
      const bool segb = pr >= rowsA;
      const int im = segb ? nA + 1 : nA, iy = segb ? pr - rowsA - 1 : yA0 - 1 + pr, ix = pc - 1;
      const bool ok = px < npx && iy >= 0 && iy < a.H && ix >= 0 && ix < Wd;
      const uint32_t vo = ok ? (uint32_t)((((im * a.H + iy) * Wd + ix) * a.Cin + c * BK + 4 * part) * 4) : kBufOob;
      pv[j] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rX, vo, 0, 0));
    }
  };
  auto stash_patch = [&]() {
    // the thread id made opaque here, so the stash addresses are formed at each stash rather than hoisted out of
    // the chunk loop (they would take 12 VGPRs across it, and spill)
    int tt = t;
    asm volatile("" : "+v"(tt));
#pragma unroll
    for (int j = 0; j < kPatchNPL; ++j) {
      const int f = tt + 512 * j, px = f >> 3, part = f & 7;
      if (px < npx) {
        uint16_t h[4], l[4];
        split_h(pv[j].x * sa, h[0], l[0]);
        split_h(pv[j].y * sa, h[1], l[1]);
        split_h(pv[j].z * sa, h[2], l[2]);
        split_h(pv[j].w * sa, h[3], l[3]);
        const int off = px * 32 + (((part >> 1) ^ (((px >> 2) & 1) << 1)) << 3) + ((part & 1) << 2);
        *reinterpret_cast<uint2*>(sPh + off) = make_uint2(h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16);
        *reinterpret_cast<uint2*>(sPl + off) = make_uint2(l[0] | (uint32_t)l[1] << 16, l[2] | (uint32_t)l[3] << 16);
      }
    }
  };
  // weights: conv_f16x3_kernel's LDS-DMA pieces, K-tile (tap, chunk) = tap * nc + chunk
  const u32x4 qWh = make_rsrc_words(g.wh, (int64_t)a.Cout * a.Kp * 2);
  const u32x4 qWl = make_rsrc_words(g.wl, (int64_t)a.Cout * a.Kp * 2);
  auto load_w = [&](int kt, bool kv, int st) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      const int p = wave * NW + j, im = p / (BN / 16), rb = p % (BN / 16);
      const uint32_t dst = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(lptr_t)(sWb + (st * 2 + im) * BN * BK + rb * 16 * BK));
      const int row = rb * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 2);
      const uint32_t vo = kv ? (uint32_t)(((n0 + row) * a.Kp + c * 8) * 2) : kBufOob;
      const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(kt * BK * 2));
      if (im)
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWl), "s"(so), "{m0}"(dst) : "memory");
      else
        asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(vo), "s"(qWh), "s"(so), "{m0}"(dst) : "memory");
    }
  };

  // this lane's fragment rows: patch pixel of tap (0, 0) for output pixel g0 + 32 wm + 16 i + (lane & 15) (rows past
  // the tile's end read the tile's last pixel; their outputs are dropped)
  int pbase[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int o = min(g0 + wm * 32 + i * 16 + (lane & 15), gend - 1);
    const int n = o / HW, r = o - n * HW, y = r / Wd, x = r - y * Wd;
    pbase[i] = (n == nA ? y - yA0 : rowsA + y) * PW + x;
  }
  const int q = lane >> 4;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int tap, int st) {
    const int dy = tap / 3, dx = tap - dy * 3;
    bf16x8 ah[FM], al[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int P = pbase[i] + dy * PW + dx;
      const int off = P * 32 + ((q ^ (((P >> 2) & 1) << 1)) << 3);
      ah[i] = *reinterpret_cast<const bf16x8*>(sPh + off);
      al[i] = *reinterpret_cast<const bf16x8*>(sPl + off);
    }
    const uint16_t* wh = sWb + (st * 2) * BN * BK;
    const uint16_t* wl = sWb + (st * 2 + 1) * BN * BK;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int row = wn * WN + j * 16 + (lane & 15);
      const bf16x8 bh = *reinterpret_cast<const bf16x8*>(wh + cswz(row, q));
      const bf16x8 bl = *reinterpret_cast<const bf16x8*>(wl + cswz(row, q));
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        acc[i][j] = mfma16<true>(bh, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bl, ah[i], acc[i][j]);
        acc[i][j] = mfma16<true>(bh, al[i], acc[i][j]);
      }
    }
  };

  // prologue: the first chunk's patch and tap-0 weights
  load_patch(c0);
  load_w(c0, true, 0);
  stash_patch();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int st = 0;
  for (int c = c0; c < c1; ++c) {
    const bool more = c + 1 < c1;
    // tap 0 (its weights and patch were waited for at the chunk boundary): the next tap's weights, then the next
    // chunk's patch behind them
    load_w(nc + c, true, st ^ 1);
    if (more) load_patch(c + 1);
    compute(0, st);
    st ^= 1;
    for (int tap = 1; tap < 9; ++tap) {
      // tap's weights landed (issued one tap ago; at tap 1 the next chunk's patch loads, issued after them, may stay
      // in flight) and every wave is past the previous tap, whose stage takes the next weights
      if (tap == 1 && more) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPatchNPL) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // the next tap's weights, or the next chunk's tap 0 (zeros past the slice: nobody reads them)
      load_w(tap < 8 ? (tap + 1) * nc + c : c + 1, tap < 8 || more, st ^ 1);
      compute(tap, st);
      st ^= 1;
    }
    if (more) {
      // every wave is past its last read of this chunk's patch before it is overwritten
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      stash_patch();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  const int li = lane & 15, lk = lane >> 4;
  if (a.ks > 1) {
    const int G = gridDim.z / a.ks;
    const int M = a.N * HW;
    float* pb = a.part + ((int64_t)slice * G + grp) * M * a.Cout;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int64_t mo = g0 + wm * 32 + i * 16 + li;
      if (mo >= gend) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int no = n0 + wn * WN + j * 16 + 4 * lk;
        const f32x4 v = acc[i][j] * inv;
        *reinterpret_cast<float4*>(pb + mo * a.Cout + no) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    return;
  }
  // (fragment-shaped stores: the LDS-staged epilogue of the deep kernel pushed this kernel past 128 VGPRs into
  // scratch; the 3 x 3 layers are MFMA-bound, not store-bound)
  int64_t mo[FM];
  bool mv[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    mo[i] = g0 + wm * 32 + i * 16 + li;
    mv[i] = mo[i] < gend;
  }
  const float ymx = conv_store_tile<FM, FN>(g, acc, inv, mo, mv, n0 + wn * WN + 4 * lk, a.Cout, (int64_t)a.N * HW);
  __syncthreads();   // the LDS is free for the max fold
  if (g.ymax) fold_max<8>(g.ymax, ymx, blockIdx.x + blockIdx.y * 7 + blockIdx.z * 13, reinterpret_cast<float*>(dynlds));
}

// split-K: y = sum over the ks slices (in slice order) + bias (+ residual), ReLU, merge; grid (blocks, G), 4 channels
// per thread
__global__ __launch_bounds__(256) void conv_splitk_reduce_kernel(const ConvF16Args a) {
  const int grp = blockIdx.y, G = gridDim.y;
  const ConvGroupArgs g = pick_group(a, grp);
  const int64_t M = (int64_t)a.N * a.Ho * a.Wo, q = M * a.Cout / 4;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  float ymx = 0.f;
  if (i < q) {
    const int64_t mo = i * 4 / a.Cout;
    const int no = (int)(i * 4 - mo * a.Cout);
    float4 p[kMaxSplitK];
#pragma unroll
    for (int s = 0; s < kMaxSplitK; ++s)
      if (s < a.ks) p[s] = reinterpret_cast<const float4*>(a.part + ((int64_t)s * G + grp) * M * a.Cout)[i];
    f32x4 v{p[0].x, p[0].y, p[0].z, p[0].w};
#pragma unroll
    for (int s = 1; s < kMaxSplitK; ++s)
      if (s < a.ks) v += f32x4{p[s].x, p[s].y, p[s].z, p[s].w};
    v = conv_out(g, v, mo, no, a.Cout);
#pragma unroll
    for (int e = 0; e < 4; ++e) ymx = fmaxf(ymx, fabsf(v[e]));
  }
  __shared__ float wmax[4];
  if (g.ymax) fold_max<4>(g.ymax, ymx, blockIdx.x, wmax);
}

// K slices for a launch of `tiles` output tiles over nk K-tiles, when the tiles alone leave the GPU's 256 CUs
// under-filled: the split whose last round of workgroups (over kSlots slots) is fullest (ties: the fewest
// slices), at least 8 K-tiles per slice.  256 slots (one workgroup per CU) measured +1 % over 512 and level
// with no split at all once the two backbones share a launch (profiles/r03_ab_conv_slots.txt)
int conv_pick_ks(int64_t tiles, int nk) {
  // slots: 256 (one workgroup per CU): a launch with a workgroup for every CU is not split.  (Round 3 counted the
  // long-K layers -- >= 72 K-tiles: layer3's 3 x 3 convs and the clf conv -- two per CU, splitting them 4 ways at 32
  // images; with the patch kernel's tiles over the flattened batch, 324 tiles, no split measured +0.3 % on the mfDiMP
  // line and drops the 7 slice-reduce launches of a step, tools/runs_r4/r4_run19.sh.  Small batches still split.)
  // The clf conv's K (288 K-tiles) is long enough that two slices per CU still pay: 512 slots from 144 K-tiles
  // (unsplit 324 us against 254 + 14 us, r4_run20).
  static const int64_t kSlotsEnv = getenv("MMT_CONV_SLOTS") ? atoi(getenv("MMT_CONV_SLOTS")) : 0;   // tuning
  const int64_t kSlots = kSlotsEnv > 0 ? kSlotsEnv : (nk >= 144 ? 512 : 256);
  static const bool nosplit = getenv("MMT_CONV_NOSPLIT") != nullptr;   // batch-invariant summation order
  if (tiles >= kSlots || nosplit) return 1;
  int best = 1;
  double best_eff = 0.0;
  for (int ks = 1; ks <= kMaxSplitK && nk / ks >= 8; ++ks) {
    const int64_t w = tiles * ks, rounds = (w + kSlots - 1) / kSlots;
    const double eff = (double)w / (double)(rounds * kSlots);
    if (eff > best_eff + 0.02) {
      best_eff = eff;
      best = ks;
    }
  }
  return best;
}

}  // namespace mmt

using namespace mmt;

namespace {

int conv_shape(int N, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pad, int& Ho, int& Wo, int& K) {
  const bool stem = Cin == 3 || Cin == 4;   // 4: a 3-channel image padded with a zero channel
  if (N <= 0 || H <= 0 || W <= 0 || Cout <= 0 || Cout % 64 || kh <= 0 || kw <= 0 || stride <= 0 || pad < 0 ||
      (!stem && Cin % 32))
    return MMT_E_ARG;
  K = stem ? kh * kw * 4 : kh * kw * Cin;
  Ho = (H + 2 * pad - kh) / stride + 1;
  Wo = (W + 2 * pad - kw) / stride + 1;
  if (Ho <= 0 || Wo <= 0) return MMT_E_ARG;
  const int64_t M = (int64_t)N * Ho * Wo;
  if (M > (int64_t)1 << 30 || (int64_t)Cout * K > (int64_t)1 << 30) return MMT_E_ARG;
  return MMT_OK;
}

// output channels per tile: 128 where the 128-wide tiles fill the GPU (or everywhere but the stem by default);
// MMT_CONV_PREFER64 (tuning): 64-wide tiles instead of splitting K when the 128-wide ones leave it under-filled
int conv_bn(int64_t gm, int Cin, int Cout, int G) {
  static const bool prefer64 = getenv("MMT_CONV_PREFER64") != nullptr;
  if (Cin <= 4 || Cout % 128) return 64;
  if (prefer64 && gm * (Cout / 128) * G < 512) return 64;
  return 128;
}

// the 3 x 3 / stride-1 patch kernel's geometry: *tiles = the launch's tiles, *tiles_per_img = tiles per image (128
// raster pixels each) or 0 for tiles over the flattened batch (chosen when the images' partial last tiles would waste
// more than 4 % of the rows and every batch tile's patch fits -- HW >= 128, so a tile spans at most two images);
// returns the largest tile's patch (pixels), 0 when the shape is not one it runs
int patch_plan(int N, int H, int W, int Cin, int kh, int kw, int stride, int pad, int* tiles, int* tiles_per_img) {
  static const bool off = getenv("MMT_CONV_NOPATCH") != nullptr;   // tuning A/B: the generic kernel
  static const bool per_img = getenv("MMT_CONV_PATCH_PERIMG") != nullptr;   // tuning A/B: per-image tiles only
  if (off || kh != 3 || kw != 3 || stride != 1 || pad != 1 || Cin % 32 || Cin < 32) return 0;
  const int HW = H * W, tpi = (HW + 127) / 128, PW = W + 2;
  int px = 0;
  for (int tl = 0; tl < tpi; ++tl) {
    const int o0 = tl * 128, o1 = std::min(o0 + 128, HW);
    px = std::max(px, ((o1 - 1) / W - o0 / W + 3) * PW);
  }
  const int64_t total = (int64_t)N * HW, gtiles = (total + 127) / 128;
  if (!per_img && HW >= 128 && (int64_t)N * tpi * 128 > total * 104 / 100 && N > 1) {
    int gpx = 0;
    for (int64_t tl = 0; tl < gtiles; ++tl) {
      const int64_t g0 = tl * 128, gend = std::min(g0 + 128, total);
      const int64_t nA = g0 / HW, y0 = (g0 - nA * HW) / W;
      const int64_t aend = std::min(gend, (nA + 1) * HW) - nA * HW;
      int rows = (int)((aend - 1) / W - y0 + 3);
      if (gend > (nA + 1) * HW) rows += (int)((gend - (nA + 1) * HW - 1) / W + 3);
      gpx = std::max(gpx, rows * PW);
    }
    if (gpx <= kPatchMaxPx) {
      *tiles = (int)gtiles;
      *tiles_per_img = 0;
      return gpx;
    }
  }
  if (px > kPatchMaxPx) return 0;
  *tiles = N * tpi;
  *tiles_per_img = tpi;
  return px;
}

// output pixels per tile of the generic kernel: 128, or 256 with MMT_CONV_BM=256 (tuning) for 128-wide tiles
int conv_bm_for(int Cin, int bn) {
  static const bool old = getenv("MMT_CONV_OLD") != nullptr;
  static const int bm = getenv("MMT_CONV_BM") ? atoi(getenv("MMT_CONV_BM")) : 128;
  return bm == 256 && !old && Cin > 4 && bn == 128 ? 256 : 128;
}

// M tiles of a launch (the patch kernel tiles each image separately) and its K split
int64_t conv_ks_for(int N, int H, int W, int Ho, int Wo, int Cin, int Cout, int kh, int kw, int stride, int pad, int Kp,
                    int G) {
  const int64_t M = (int64_t)N * Ho * Wo;
  const int bn = conv_bn((M + 127) / 128, Cin, Cout, G);
  int ptiles = 0, tpi = 0;
  if (patch_plan(N, H, W, Cin, kh, kw, stride, pad, &ptiles, &tpi))
    return std::min<int64_t>(conv_pick_ks((int64_t)ptiles * (Cout / bn) * G, Kp / 32), Cin / 32);
  const int bm = conv_bm_for(Cin, bn);
  return conv_pick_ks((M + bm - 1) / bm * (Cout / bn) * G, Kp / 32);
}

}  // namespace

extern "C" {

size_t mmt_conv_max_words(void) { return (size_t)kMaxShards * kShardStride; }

size_t mmt_conv2d_f16x3_ws_bytes(int N, int H, int W, int Cin, int Cout, int kh, int kw, int stride, int pad,
                                 int groups) {
  int Ho, Wo, K;
  if (groups < 1 || groups > kMaxGroups || conv_shape(N, H, W, Cin, Cout, kh, kw, stride, pad, Ho, Wo, K) != MMT_OK)
    return 0;
  const int Kp = (K + 31) / 32 * 32;
  const int64_t ks = conv_ks_for(N, H, W, Ho, Wo, Cin, Cout, kh, kw, stride, pad, Kp, groups);
  return ks > 1 ? (size_t)(ks * groups * N * Ho * Wo * (int64_t)Cout * 4) : 0;
}

int mmt_conv2d_f16x3_groups(const mmt_conv_group* groups, int G, int N, int H, int W, int Cin, int Kp, int Cout,
                            int kh, int kw, int stride, int pad, void* ws, size_t ws_bytes, void* stream) {
  int Ho, Wo, K;
  if (!groups || G < 1 || G > kMaxGroups || conv_shape(N, H, W, Cin, Cout, kh, kw, stride, pad, Ho, Wo, K) != MMT_OK ||
      Kp != (K + 31) / 32 * 32)
    return MMT_E_ARG;
  ConvF16Args a{};
  for (int i = 0; i < G; ++i) {
    const mmt_conv_group& c = groups[i];
    if (!c.x || !c.w_hi || !c.w_lo || !c.y || !(c.w_scale > 0) ||
        (c.flags & ~(MMT_CONV_RELU | MMT_CONV_MAX | MMT_CONV_POOL)) || (!c.x_max && !(c.x_scale > 0)) ||
        (c.flags & MMT_CONV_POOL) != (groups[0].flags & MMT_CONV_POOL) ||
        // the pooled stem kernel neither max-merges nor adds a residual: refuse operands it would drop
        ((c.flags & MMT_CONV_POOL) && ((c.flags & MMT_CONV_MAX) || c.resid)))
      return MMT_E_ARG;
    a.g[i] = ConvGroupArgs{c.x, c.w_hi, c.w_lo, c.bias, c.resid, c.y, c.x_max, c.y_max, c.x_scale, 1.0f / c.w_scale,
                           c.flags, nullptr, nullptr, 0.f};
  }
  // the twin layers of a grouped launch write disjoint outputs unless they merge (a MAX layer reads y)
  if (G == 2 && (a.g[0].y == a.g[1].y || (a.g[0].flags | a.g[1].flags) & MMT_CONV_MAX)) return MMT_E_ARG;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.kh = kh; a.kw = kw; a.stride = stride; a.pad = pad;
  a.Ho = Ho; a.Wo = Wo; a.Kp = Kp;
  const int64_t M = (int64_t)N * Ho * Wo;
  const hipStream_t s = (hipStream_t)stream;
  if (groups[0].flags & MMT_CONV_POOL) {
    // the 7 x 7 / stride-2 stem with the 3 x 3 / stride-2 / pad-1 max-pool fused; y is the pooled map
    if (Cin != 4 || Cout != 64 || kh != 7 || kw != 7 || stride != 2 || Kp != 224)
      return MMT_E_ARG;
    const int PHo = (Ho - 1) / 2 + 1, PWo = (Wo - 1) / 2 + 1;
    const unsigned tiles = (unsigned)(N * ((PHo + kPoolT - 1) / kPoolT) * ((PWo + kPoolT - 1) / kPoolT));
    a.ks = 1;
    hipLaunchKernelGGL(conv_stem_pool_f16x3_kernel, dim3(tiles, 1, G), dim3(512), 0, s, a, PHo, PWo);
    return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
  }
  int ks = (int)conv_ks_for(N, H, W, Ho, Wo, Cin, Cout, kh, kw, stride, pad, Kp, G);
  if (ks > 1 && (!ws || ws_bytes < (size_t)(ks * G * M * (int64_t)Cout * 4))) ks = 1;
  a.ks = ks;
  a.part = static_cast<float*>(ws);
  const int bn = conv_bn((M + 127) / 128, Cin, Cout, G);
  const int conv_bm = conv_bm_for(Cin, bn);
  const unsigned gm = (unsigned)((M + conv_bm - 1) / conv_bm);
  const dim3 grid(gm, Cout / bn, G * ks);
  const dim3 dgrid(gm * (Cout / bn), 1, G * ks);   // the deep kernel: M x N tiles flattened
  static const int xcd_env = getenv("MMT_CONV_XCD") ? atoi(getenv("MMT_CONV_XCD")) : -1;   // tuning: 0 / 1 force
  a.xcd_order = xcd_env != 0;
  // the LDS-staged conv epilogue (mfDiMP 7 396 -> 7 531 frames/s, profiles/r05_ab_conv_staged_epilogue.txt;
  // MMT_CONV_STAGED=0, tuning: fragment-shaped stores)
  static const bool staged_env = !getenv("MMT_CONV_STAGED") || atoi(getenv("MMT_CONV_STAGED")) != 0;
  a.staged_epi = staged_env ? 1 : 0;
  // the stem on a 4-channel image: 2-D tiles from an LDS input patch (MMT_CONV_STEM_OLD: the gather kernel, tuning)
  static const bool stem_old = getenv("MMT_CONV_STEM_OLD") != nullptr;
  static const int stem_th = getenv("MMT_CONV_STEM_TH") ? atoi(getenv("MMT_CONV_STEM_TH")) : 16;   // tuning: 8
  static const bool conv_old = getenv("MMT_CONV_OLD") != nullptr;   // tuning: conv_f16x3_kernel (two-deep)
  static const int conv_nr = getenv("MMT_CONV_NR") ? atoi(getenv("MMT_CONV_NR")) : 2;   // tuning: 3
  // the next K-tile's split woven into the MFMAs (+1 % on the mfDiMP line, tools/runs_r4/r4_run8.sh); MMT_CONV_OVL=0
  // (tuning): the split after them
  static const bool conv_ovl = !getenv("MMT_CONV_OVL") || atoi(getenv("MMT_CONV_OVL")) != 0;
  int ptiles = 0, tpi = 0;
  const int ppx = patch_plan(N, H, W, Cin, kh, kw, stride, pad, &ptiles, &tpi);
  if (ppx) {
    const dim3 pgrid((unsigned)ptiles, Cout / bn, G * ks);
    const size_t lds = (size_t)(2 * kPatchMaxPx * 32 + 2 * 2 * bn * 32) * 2;   // 80 KB (BN 128): two per CU
    if (bn == 128)
      hipLaunchKernelGGL(conv3x3_patch_f16x3_kernel<128>, pgrid, dim3(512), lds, s, a, tpi, ppx);
    else
      hipLaunchKernelGGL(conv3x3_patch_f16x3_kernel<64>, pgrid, dim3(512), lds, s, a, tpi, ppx);
  } else if (!stem_old && Cin == 4 && Cout == 64 && ks == 1 && kh <= 7 && kw <= 7 && stride <= 2 && Kp / 32 <= kStemMaxKt) {
    const int th = stem_th == 8 ? 8 : 16;
    const unsigned tiles = (unsigned)(((Ho + th - 1) / th) * ((Wo + kStemTW - 1) / kStemTW) * N);
    if (th == 8)
      hipLaunchKernelGGL(conv_stem_f16x3_kernel<8>, dim3(tiles, 1, G), dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL(conv_stem_f16x3_kernel<16>, dim3(tiles, 1, G), dim3(512), 0, s, a);
  } else if (Cin <= 4)
    hipLaunchKernelGGL((conv_f16x3_kernel<64, true>), grid, dim3(512), 0, s, a);
  else if (conv_old) {   // tuning A/B: the two-deep pipeline
    if (bn == 128)
      hipLaunchKernelGGL((conv_f16x3_kernel<128, false>), grid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_f16x3_kernel<64, false>), grid, dim3(512), 0, s, a);
  } else if (conv_bm == 256) {
    hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 2, 256>), dgrid, dim3(512), 0, s, a);
  } else if (conv_ovl) {
    if (bn == 128)
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 3, 128, true>), dgrid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<64, 3, 128, true>), dgrid, dim3(512), 0, s, a);
  } else if (conv_nr == 2) {
    if (bn == 128)
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 2>), dgrid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<64, 2>), dgrid, dim3(512), 0, s, a);
  } else {
    if (bn == 128)
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 3>), dgrid, dim3(512), 0, s, a);
    else
      hipLaunchKernelGGL((conv_f16x3_deep_kernel<64, 3>), dgrid, dim3(512), 0, s, a);
  }
#if defined(CONV_STAMPS)
  if (!ppx && !conv_old && Cin > 4 && conv_bm == 128) {   // the deep kernel ran: per-phase cycles averaged over its workgroups
    const size_t nb = (size_t)dgrid.x * dgrid.y * dgrid.z;
    unsigned long long* buf = nullptr;
    if (hipMalloc(&buf, nb * 64) == hipSuccess) {
      hipMemsetAsync(buf, 0, nb * 64, s);
      hipMemcpyToSymbolAsync(HIP_SYMBOL(g_conv_stamps), &buf, sizeof(buf), 0, hipMemcpyHostToDevice, s);
      if (conv_ovl)
        hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 3, 128, true>), dgrid, dim3(512), 0, s, a);
      else if (conv_nr == 2)
        hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 2>), dgrid, dim3(512), 0, s, a);
      hipStreamSynchronize(s);
      std::vector<unsigned long long> h(nb * 8);
      hipMemcpy(h.data(), buf, nb * 64, hipMemcpyDeviceToHost);
      double acc[8] = {0};
      for (size_t b = 0; b < nb; ++b)
        for (int k = 0; k < 8; ++k) acc[k] += (double)h[b * 8 + k];
      const double kt = acc[6] > 0 ? acc[6] : 1;
      fprintf(stderr, "conv stamps M=%lld Cin=%d Cout=%d k=%d: per K-tile cycles issue %.0f mfma %.0f a-wait %.0f stash %.0f "
              "w-wait+barrier %.0f | prologue %.0f, total/K-tile %.0f (%zu blocks)\n", (long long)M, Cin, Cout, kh,
              acc[1] / kt, acc[2] / kt, acc[3] / kt, acc[4] / kt, acc[5] / kt, acc[0] / nb, acc[7] / kt, nb);
      const unsigned long long* z = nullptr;
      hipMemcpyToSymbol(HIP_SYMBOL(g_conv_stamps), &z, sizeof(z));
      hipFree(buf);
    }
  }
#endif
  if (ks > 1) {
    const int64_t q = M * Cout / 4;
    hipLaunchKernelGGL(conv_splitk_reduce_kernel, dim3((unsigned)((q + 255) / 256), G), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_conv2d_f16x3_ds_groups(const mmt_conv_group* groups, const mmt_conv_ds* ds, int G, int N, int H, int W,
                               int Cin, int H2, int W2, int Cin2, int stride2, int Kp, int Cout, void* ws,
                               size_t ws_bytes, void* stream) {
  int Ho, Wo, K;
  // conv3 is 1 x 1 / stride 1 over [N][H][W][Cin]; the downsample 1 x 1 / stride2 over [N][H2][W2][Cin2] lands on
  // the same H x W grid; the weights hold both K ranges
  if (!groups || !ds || G < 1 || G > kMaxGroups || Cin < 32 || Cin % 32 || Cin2 < 32 || Cin2 % 32 || stride2 < 1 ||
      H2 <= 0 || W2 <= 0 || (H2 - 1) / stride2 + 1 != H || (W2 - 1) / stride2 + 1 != W || Kp != Cin + Cin2 ||
      conv_shape(N, H, W, Kp, Cout, 1, 1, 1, 0, Ho, Wo, K) != MMT_OK ||
      (int64_t)N * H2 * W2 * Cin2 > ((int64_t)1 << 29))   // 32-bit buffer offsets into x2
    return MMT_E_ARG;
  ConvF16Args a{};
  for (int i = 0; i < G; ++i) {
    const mmt_conv_group& c = groups[i];
    if (!c.x || !c.w_hi || !c.w_lo || !c.y || !(c.w_scale > 0) || c.resid ||
        (c.flags & ~(MMT_CONV_RELU | MMT_CONV_MAX)) || (!c.x_max && !(c.x_scale > 0)) || !ds[i].x2 ||
        (!ds[i].x2_max && !(ds[i].x2_scale > 0)))
      return MMT_E_ARG;
    a.g[i] = ConvGroupArgs{c.x, c.w_hi, c.w_lo, c.bias, nullptr, c.y, c.x_max, c.y_max, c.x_scale, 1.0f / c.w_scale,
                           c.flags, ds[i].x2, ds[i].x2_max, ds[i].x2_scale};
  }
  if (G == 2 && (a.g[0].y == a.g[1].y || (a.g[0].flags | a.g[1].flags) & MMT_CONV_MAX)) return MMT_E_ARG;
  a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.kh = 1; a.kw = 1; a.stride = 1; a.pad = 0;
  a.Ho = H; a.Wo = W; a.Kp = Kp;
  a.Cin2 = Cin2; a.H2 = H2; a.W2 = W2; a.stride2 = stride2;
  const int64_t M = (int64_t)N * H * W;
  int ks = (int)conv_ks_for(N, H, W, H, W, Kp, Cout, 1, 1, 1, 0, Kp, G);
  if (ks > 1 && (!ws || ws_bytes < (size_t)(ks * G * M * (int64_t)Cout * 4))) ks = 1;
  a.ks = ks;
  a.part = static_cast<float*>(ws);
  static const int xcd_env = getenv("MMT_CONV_XCD") ? atoi(getenv("MMT_CONV_XCD")) : -1;
  a.xcd_order = xcd_env != 0;
  // the LDS-staged conv epilogue (mfDiMP 7 396 -> 7 531 frames/s, profiles/r05_ab_conv_staged_epilogue.txt;
  // MMT_CONV_STAGED=0, tuning: fragment-shaped stores)
  static const bool staged_env = !getenv("MMT_CONV_STAGED") || atoi(getenv("MMT_CONV_STAGED")) != 0;
  a.staged_epi = staged_env ? 1 : 0;
  const int bn = conv_bn((M + 127) / 128, Kp, Cout, G);
  const dim3 dgrid((unsigned)((M + 127) / 128 * (Cout / bn)), 1, G * ks);
  const hipStream_t s = (hipStream_t)stream;
  if (bn == 128)
    hipLaunchKernelGGL((conv_f16x3_deep_kernel<128, 3, 128, true>), dgrid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_f16x3_deep_kernel<64, 3, 128, true>), dgrid, dim3(512), 0, s, a);
  if (ks > 1) {
    const int64_t q = M * Cout / 4;
    hipLaunchKernelGGL(conv_splitk_reduce_kernel, dim3((unsigned)((q + 255) / 256), G), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_conv2d_f16x3(const float* x, int N, int H, int W, int Cin, const uint16_t* w_hi, const uint16_t* w_lo,
                     float w_scale, int Kp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                     const float* resid, float* y, const float* x_max, float x_scale, float* y_max, int flags,
                     void* stream) {
  const mmt_conv_group g{x, w_hi, w_lo, w_scale, bias, resid, y, x_max, x_scale, y_max, flags};
  return mmt_conv2d_f16x3_groups(&g, 1, N, H, W, Cin, Kp, Cout, kh, kw, stride, pad, nullptr, 0, stream);
}

}  // extern "C"
