// Joint template-search self-attention (attn.py:33-59) with the candidate-
// elimination side output (attn_blocks.py:44-53), gfx950.
//
// One workgroup = WAVES waves, each wave 16 query rows of one (sequence, head).
// K/V tiles of 64 keys are staged in LDS (K row-major, XOR-swizzled; V
// transposed, rows padded to 136 B so the 8-B fragment reads are
// conflict-free).  Scores are computed swapped, S^T = K Q^T, with
// v_mfma_f32_16x16x32_bf16: a lane holds 16 keys of ONE query, so the online
// softmax needs only two cross-lane shuffles per row statistic, and the
// accumulator is already the B operand (P^T) of O^T = V^T P^T.
//
// CE side output: the wave that owns the CTR_POINT template query keeps that
// row's raw logits in LDS and, after the last tile, exports its exact
// probability row p = exp(s - m) / l over the search keys (fp32), which the
// CE kernel averages over heads.
#include "kernels.h"

namespace mmt {

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int KB = 64;         // keys per LDS tile
constexpr int VT_PITCH = 68;   // bf16 per transposed-V row (136 B)
constexpr int CE_MAX = 1024;   // max tokens for the exported CE row

template <int WAVES>
__global__ __launch_bounds__(WAVES * 64) void attn_kernel(const AttnArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[KB * 64];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[64 * VT_PITCH];
  __shared__ float ce_row[CE_MAX];

  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = a.N, Cd = 64 * a.heads, C3 = 3 * Cd;
  const bf16_t* base = a.qkv + (int64_t)b * N * C3;
  const int q0 = blockIdx.x * (16 * WAVES) + wave * 16;
  const int qi = q0 + (lane & 15);
  const int g = lane >> 4;

  bf16x8 qf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (qi < N)
      qf[s] = *reinterpret_cast<const bf16x8*>(base + (int64_t)qi * C3 + h * 64 + 32 * s + 8 * g);
    else
      qf[s] = bf16x8{};
  }

  f32x4 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const bool ce_wave = a.ce_query >= q0 && a.ce_query < q0 + 16;
  const bool ce_lane = ce_wave && (lane & 15) == a.ce_query - q0;

  for (int kb = 0; kb < N; kb += KB) {
    __syncthreads();
    for (int q = tid; q < KB * 8; q += WAVES * 64) {
      const int r = q >> 3, c = q & 7, key = kb + r;
      uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
      if (key < N) {
        const bf16_t* row = base + (int64_t)key * C3 + h * 64 + c * 8;
        kv = *reinterpret_cast<const uint4*>(row + Cd);
        vv = *reinterpret_cast<const uint4*>(row + 2 * Cd);
      }
      *reinterpret_cast<uint4*>(Ks + r * 64 + ((c ^ (r & 7)) << 3)) = kv;
      const bf16_t* ve = reinterpret_cast<const bf16_t*>(&vv);
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(c * 8 + e) * VT_PITCH + r] = ve[e];
    }
    __syncthreads();

    f32x4 sc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = 16 * t + (lane & 15), c = 4 * s + g;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + r * 64 + ((c ^ (r & 7)) << 3));
        sc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[s], sc[t], 0, 0, 0);
      }
    }
    float bmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = kb + 16 * t + 4 * g + r;
        const float v = key < N ? sc[t][r] * 0.125f : -INFINITY;
        sc[t][r] = v;
        bmax = fmaxf(bmax, v);
      }
    bmax = fmaxf(bmax, __shfl_xor(bmax, 16, 64));
    bmax = fmaxf(bmax, __shfl_xor(bmax, 32, 64));
    if (ce_lane) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kb + 16 * t + 4 * g + r;
          if (key < N) ce_row[key] = sc[t][r];
        }
    }
    const float mnew = fmaxf(m, bmax);
    const float alpha = __expf(m - mnew);
    float psum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(sc[t][r] - mnew);
        sc[t][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;

#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bf16x8 pf;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[r] = (__bf16)sc[2 * u][r];
        pf[4 + r] = (__bf16)sc[2 * u + 1][r];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16_t* vrow = Vt + (16 * dt + (lane & 15)) * VT_PITCH + 32 * u + 4 * g;
        const bf16x4 v0 = *reinterpret_cast<const bf16x4*>(vrow);
        const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(vrow + 16);
        const bf16x8 vf = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf, o[dt], 0, 0, 0);
      }
    }
  }

  const float inv = 1.0f / l;
  if (qi < N) {
    bf16_t* orow = a.out + ((int64_t)b * N + qi) * Cd + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      uint2 w;
      w.x = (uint32_t)f2bf(o[dt][0] * inv) | ((uint32_t)f2bf(o[dt][1] * inv) << 16);
      w.y = (uint32_t)f2bf(o[dt][2] * inv) | ((uint32_t)f2bf(o[dt][3] * inv) << 16);
      *reinterpret_cast<uint2*>(orow + 16 * dt + 4 * g) = w;
    }
  }
  __syncthreads();
  if (ce_wave) {
    const int src = a.ce_query - q0;
    const float mm = __shfl(m, src, 64), ll = __shfl(l, src, 64);
    const int Ls = N - a.ce_lens_t;
    float* dst = a.ce_prob + ((int64_t)b * a.heads + h) * Ls;
    for (int j = lane; j < Ls; j += 64) dst[j] = __expf(ce_row[a.ce_lens_t + j] - mm) / ll;
  }
}

void attention(const AttnArgs& a, hipStream_t s) {
  const int per4 = a.B * a.heads * ((a.N + 63) / 64);
  if (per4 >= 240) {
    dim3 grid((a.N + 63) / 64, a.heads, a.B);
    hipLaunchKernelGGL(attn_kernel<4>, grid, dim3(256), 0, s, a);
  } else if (per4 * 2 >= 240) {
    dim3 grid((a.N + 31) / 32, a.heads, a.B);
    hipLaunchKernelGGL(attn_kernel<2>, grid, dim3(128), 0, s, a);
  } else {
    dim3 grid((a.N + 15) / 16, a.heads, a.B);
    hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(64), 0, s, a);
  }
}

}  // namespace mmt
