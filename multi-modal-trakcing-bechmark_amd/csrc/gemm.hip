// MFMA bf16 GEMM with fused epilogues, gfx950 (CDNA4).
//
//   C[m][n] = epi( sum_k A[m][k] * W[n][k] + bias[n] )
//
// The ViT-B dense contractions of the tracking path (attn.py:17-19 qkv/proj,
// timm Mlp fc1/fc2, patch_embed.py:20 as a k16s16 conv, head.py:8-21 3x3 convs
// as implicit GEMMs over the NHWC token map) all have this shape: activations
// [tokens x K] and nn.Linear / conv weights [out x K], both K-contiguous.
//
// Tile: BM x BN x 64, 256 threads = 4 waves, v_mfma_f32_16x16x32_bf16.
// LDS: two buffers of (BM+BN) x 64 bf16, 16-B chunks XOR-swizzled by row
// (chunk ^ (row & 7)) so both the 8-lane ds_write_b128 groups and the
// 16-lane ds_read_b128 fragment groups are conflict-free.  Global->register
// staging of tile k+1 overlaps the MFMAs of tile k; one barrier per K-tile.
// The MFMA is issued as W-fragment x A-fragment so each lane ends with four
// consecutive output columns of one row: 8-B (bf16) / 16-B (fp32) stores.
#include "kernels.h"

namespace mmt {

template <int BM, int BN, int WM, int WN>
struct TileCfg {
  static constexpr int WN_WAVES = BN / WN;
  static constexpr int WM_WAVES = BM / WM;
  static_assert(WM_WAVES * WN_WAVES == 4, "tile must map onto 4 waves");
  static constexpr int FM = WM / 16;
  static constexpr int FN = WN / 16;
  static constexpr int ACH = BM * 8 / 256;  // 16-B chunks per thread per A tile
  static constexpr int BCH = BN * 8 / 256;
  static_assert(ACH >= 1 && BCH >= 1, "tile too small");
};

__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((c ^ (r & 7)) << 3); }

template <int BM, int BN, int WM, int WN, int EPI, int AM>
__global__ __launch_bounds__(256) void gemm_kernel(const GemmArgs args) {
  using T = TileCfg<BM, BN, WM, WN>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * (BM + BN) * 64];

  const GemmGroup g = args.g[blockIdx.z];
  const int M = args.M, N = args.N, K = args.K;
  const int tiles_n = N / BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / T::WN_WAVES, wn = wave % T::WN_WAVES;

  uint4 ra[T::ACH], rb[T::BCH];

  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < T::ACH; ++i) {
      const int q = tid + 256 * i, r = q >> 3, c = q & 7;
      const int m = m0 + r;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (AM == A_DENSE) {
        if (m < M) v = *reinterpret_cast<const uint4*>(g.A + (int64_t)m * g.lda + k0 + c * 8);
      } else {
        // implicit 3x3 conv, pad 1, NHWC: k = tap * cin + ch (cin % 64 == 0 -> one tap per K-tile)
        const int hw = args.conv_hw, cin = args.conv_cin;
        const int tap = k0 / cin, ch = k0 - tap * cin;
        const int ky = tap / 3, kx = tap - ky * 3;
        const int plane = hw * hw;
        const int bimg = m / plane, p = m - bimg * plane;
        const int y = p / hw + ky - 1, x = p - (p / hw) * hw + kx - 1;
        if (m < M && y >= 0 && y < hw && x >= 0 && x < hw)
          v = *reinterpret_cast<const uint4*>(g.A + ((int64_t)bimg * plane + y * hw + x) * g.lda + ch + c * 8);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < T::BCH; ++i) {
      const int q = tid + 256 * i, r = q >> 3, c = q & 7;
      rb[i] = *reinterpret_cast<const uint4*>(g.W + (int64_t)(n0 + r) * g.ldw + k0 + c * 8);
    }
  };
  auto store = [&](int buf) {
    bf16_t* As = smem + buf * (BM + BN) * 64;
    bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int i = 0; i < T::ACH; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<uint4*>(As + swz(q >> 3, q & 7)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::BCH; ++i) {
      const int q = tid + 256 * i;
      *reinterpret_cast<uint4*>(Bs + swz(q >> 3, q & 7)) = rb[i];
    }
  };

  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int j = 0; j < T::FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16_t* As = smem + buf * (BM + BN) * 64;
    const bf16_t* Bs = As + BM * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      bf16x8 af[T::FM], bw[T::FN];
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
        af[i] = *reinterpret_cast<const bf16x8*>(As + swz(wm * WM + i * 16 + (lane & 15), c));
#pragma unroll
      for (int j = 0; j < T::FN; ++j)
        bw[j] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * WN + j * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int j = 0; j < T::FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af[i], acc[i][j], 0, 0, 0);
    }
  };

  const int nk = K / 64;
  load(0);
  store(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * 64);
    compute(cur);
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane owns C[m][n..n+3]
#pragma unroll
  for (int i = 0; i < T::FM; ++i) {
    const int m = m0 + wm * WM + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < T::FN; ++j) {
      const int n = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
      float4 bv = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
      float v0 = acc[i][j][0] + bv.x, v1 = acc[i][j][1] + bv.y, v2 = acc[i][j][2] + bv.z, v3 = acc[i][j][3] + bv.w;
      if (EPI == EPI_GELU_BF16) {
        v0 = gelu_erf(v0); v1 = gelu_erf(v1); v2 = gelu_erf(v2); v3 = gelu_erf(v3);
      }
      if (EPI == EPI_RELU_BF16 || EPI == EPI_RELU_F32) {
        v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f);
      }
      if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
        uint2 o;
        o.x = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
        o.y = (uint32_t)f2bf(v2) | ((uint32_t)f2bf(v3) << 16);
        *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.C) + (int64_t)m * g.ldc + n) = o;
      } else {
        float4 o = make_float4(v0, v1, v2, v3);
        if (EPI == EPI_RESID_F32) {
          const float4 r = *reinterpret_cast<const float4*>(g.R + (int64_t)m * g.ldr + n);
          o = make_float4(r.x + v0, r.y + v1, r.z + v2, r.w + v3);
        } else if (EPI == EPI_POS_F32) {
          const float4 r = *reinterpret_cast<const float4*>(g.R + (int64_t)(m % args.pos_rows) * g.ldr + n);
          o = make_float4(v0 + r.x, v1 + r.y, v2 + r.z, v3 + r.w);
        }
        *reinterpret_cast<float4*>(static_cast<float*>(g.C) + (int64_t)m * g.ldc + n) = o;
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int EPI, int AM>
static void launch_one(const GemmArgs& a, hipStream_t s) {
  dim3 grid(((a.M + BM - 1) / BM) * (a.N / BN), 1, a.groups);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, EPI, AM>), grid, dim3(256), 0, s, a);
}

template <int BM, int BN, int WM, int WN>
static void launch_cfg(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.amode == A_CONV3) {
    switch (epi) {
      case EPI_RELU_BF16: return launch_one<BM, BN, WM, WN, EPI_RELU_BF16, A_CONV3>(a, s);
      case EPI_RELU_F32: return launch_one<BM, BN, WM, WN, EPI_RELU_F32, A_CONV3>(a, s);
      default: break;
    }
    return;
  }
  switch (epi) {
    case EPI_BF16: return launch_one<BM, BN, WM, WN, EPI_BF16, A_DENSE>(a, s);
    case EPI_GELU_BF16: return launch_one<BM, BN, WM, WN, EPI_GELU_BF16, A_DENSE>(a, s);
    case EPI_RESID_F32: return launch_one<BM, BN, WM, WN, EPI_RESID_F32, A_DENSE>(a, s);
    case EPI_F32: return launch_one<BM, BN, WM, WN, EPI_F32, A_DENSE>(a, s);
    case EPI_POS_F32: return launch_one<BM, BN, WM, WN, EPI_POS_F32, A_DENSE>(a, s);
    default: break;
  }
}

void gemm(const GemmArgs& a, int epi, hipStream_t s) {
  const int mt128 = (a.M + 127) / 128, mt64 = (a.M + 63) / 64;
  const int target = 240;  // >= ~1 tile per CU of the 256
  if (a.N % 128 == 0 && mt128 * (a.N / 128) * a.groups >= target)
    return launch_cfg<128, 128, 64, 64>(a, epi, s);
  if (a.N % 128 == 0 && mt64 * (a.N / 128) * a.groups >= target)
    return launch_cfg<64, 128, 32, 64>(a, epi, s);
  if (a.N % 64 == 0)
    return launch_cfg<64, 64, 32, 32>(a, epi, s);
  return launch_cfg<64, 32, 16, 32>(a, epi, s);
}

}  // namespace mmt
