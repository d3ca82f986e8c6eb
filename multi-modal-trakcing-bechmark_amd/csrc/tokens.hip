// Bandwidth-bound token kernels of the ViPT path, gfx950: LayerNorm, the
// modality-prompt blocks, candidate elimination, final norm + token recovery.
// Rows are 768 fp32 (one wave per row, 3 x float4 per lane).
#include "kernels.h"

namespace mmt {

constexpr int C768 = 768;
constexpr float LN_EPS = 1e-6f;   // vit_ce_prompt.py:121

struct Row12 { float4 v[3]; };

__device__ __forceinline__ Row12 load_row(const float* p, int lane) {
  Row12 r;
  const float4* q = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) r.v[i] = q[lane + 64 * i];
  return r;
}
__device__ __forceinline__ Row12 zero_row() {
  Row12 r;
#pragma unroll
  for (int i = 0; i < 3; ++i) r.v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  return r;
}

// LayerNorm over 768 (F.layer_norm semantics: biased variance, eps inside sqrt)
__device__ __forceinline__ Row12 ln_row(const Row12& x, const float* w, const float* b, int lane) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) s += x.v[i].x + x.v[i].y + x.v[i].z + x.v[i].w;
  const float mean = wave_sum(s) * (1.0f / C768);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 d = make_float4(x.v[i].x - mean, x.v[i].y - mean, x.v[i].z - mean, x.v[i].w - mean);
    q += d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w;
  }
  const float rstd = 1.0f / sqrtf(wave_sum(q) * (1.0f / C768) + LN_EPS);
  Row12 y;
  const float4* w4 = reinterpret_cast<const float4*>(w);
  const float4* b4 = reinterpret_cast<const float4*>(b);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 ww = w4[lane + 64 * i], bb = b4[lane + 64 * i];
    y.v[i] = make_float4((x.v[i].x - mean) * rstd * ww.x + bb.x, (x.v[i].y - mean) * rstd * ww.y + bb.y,
                         (x.v[i].z - mean) * rstd * ww.z + bb.z, (x.v[i].w - mean) * rstd * ww.w + bb.w);
  }
  return y;
}

__device__ __forceinline__ void store_bf16(bf16_t* p, const Row12& y, int lane) {
  uint2* q = reinterpret_cast<uint2*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    uint2 o;
    o.x = (uint32_t)f2bf(y.v[i].x) | ((uint32_t)f2bf(y.v[i].y) << 16);
    o.y = (uint32_t)f2bf(y.v[i].z) | ((uint32_t)f2bf(y.v[i].w) << 16);
    q[lane + 64 * i] = o;
  }
}
__device__ __forceinline__ void store_bf16_lo(bf16_t* p, const Row12& y, int lane) {   // y - bf16(y)
  uint2* q = reinterpret_cast<uint2*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 v = y.v[i];
    uint2 o;
    o.x = (uint32_t)f2bf(v.x - bf2f(f2bf(v.x))) | ((uint32_t)f2bf(v.y - bf2f(f2bf(v.y))) << 16);
    o.y = (uint32_t)f2bf(v.z - bf2f(f2bf(v.z))) | ((uint32_t)f2bf(v.w - bf2f(f2bf(v.w))) << 16);
    q[lane + 64 * i] = o;
  }
}
__device__ __forceinline__ void store_f32(float* p, const Row12& y, int lane) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) q[lane + 64 * i] = y.v[i];
}

// ------------------------------------------------------------------ LayerNorm (optionally fused CE gather)
__global__ __launch_bounds__(256) void ln_kernel(const float* x, const float* w, const float* b, bf16_t* ob,
                                                 bf16_t* olo, float* of, int rows, int rows_per_seq,
                                                 const int* gather, int in_rows_per_seq, float* xcopy) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  int64_t src = r;
  if (gather) {
    const int bs = r / rows_per_seq;
    src = (int64_t)bs * in_rows_per_seq + gather[r];
  }
  const Row12 xv = load_row(x + src * C768, lane);
  if (xcopy) store_f32(xcopy + (int64_t)r * C768, xv, lane);
  const Row12 y = ln_row(xv, w, b, lane);
  if (ob) store_bf16(ob + (int64_t)r * C768, y, lane);
  if (olo) store_bf16_lo(olo + (int64_t)r * C768, y, lane);
  if (of) store_f32(of + (int64_t)r * C768, y, lane);
}

void layernorm(const float* x, const float* w, const float* b, bf16_t* out_bf16, bf16_t* out_lo, float* out_f32,
               int rows, int rows_per_seq, const int* gather, int in_rows_per_seq, float* xcopy, hipStream_t s) {
  hipLaunchKernelGGL(ln_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, x, w, b, out_bf16, out_lo, out_f32, rows,
                     rows_per_seq, gather, in_rows_per_seq, xcopy);
}

// ------------------------------------------------------------------ prompt block, part 1
// For every slot s of every sequence: a8 = conv0_0(LN_A(srcA[s])), c8 = conv0_1(LN_B(srcB[s]))
// (Prompt_block.forward, vit_ce_prompt.py:62-68, on token2feature maps; a pruned search slot
// is a zero row, vit_ce_prompt.py:276-283, whose LN is the LN bias).
// The two 8 x 768 conv weights live in LDS; a wave handles PR_ROWS rows; the 8 per-lane partial
// dot products are reduced with a transposing butterfly (10 shuffles instead of 8 x 6).
constexpr int PR_ROWS = 4;

// out[c] (valid in lane c for c < 8) = sum over the wave of part[c]
__device__ __forceinline__ float reduce8(float (&part)[8], int lane) {
  // stage xor 32: lanes < 32 keep channels 0-3, others 4-7
  float v4[4];
  const bool hi32 = lane & 32;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float send = hi32 ? part[i] : part[i + 4];
    const float keep = hi32 ? part[i + 4] : part[i];
    v4[i] = keep + __shfl_xor(send, 32, 64);
  }
  float v2[2];
  const bool hi16 = lane & 16;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float send = hi16 ? v4[i] : v4[i + 2];
    const float keep = hi16 ? v4[i + 2] : v4[i];
    v2[i] = keep + __shfl_xor(send, 16, 64);
  }
  const bool hi8 = lane & 8;
  float v1 = (hi8 ? v2[1] : v2[0]) + __shfl_xor(hi8 ? v2[0] : v2[1], 8, 64);
  v1 += __shfl_xor(v1, 4, 64);
  v1 += __shfl_xor(v1, 2, 64);
  v1 += __shfl_xor(v1, 1, 64);
  // lane holds channel ((lane>>5)&1)*4 + ((lane>>4)&1)*2 + ((lane>>3)&1); gather to lane c
  const int c = lane & 7;
  const int src = ((c >> 2) & 1) * 32 + ((c >> 1) & 1) * 16 + (c & 1) * 8;
  return __shfl(v1, src, 64);
}

__device__ __forceinline__ void dot8_lds(const Row12& y, const float* Ws, float (&part)[8], int lane) {
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const float4* w4 = reinterpret_cast<const float4*>(Ws + c * C768);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float4 ww = w4[lane + 64 * i];
      s += y.v[i].x * ww.x + y.v[i].y * ww.y + y.v[i].z * ww.z + y.v[i].w * ww.w;
    }
    part[c] = s;
  }
}

__global__ __launch_bounds__(256) void prompt_reduce_kernel(const PromptArgs a) {
  __shared__ __attribute__((aligned(16))) float W0[8 * C768];
  __shared__ __attribute__((aligned(16))) float W1[8 * C768];
  for (int i = threadIdx.x; i < 8 * C768 / 4; i += 256) {
    reinterpret_cast<float4*>(W0)[i] = reinterpret_cast<const float4*>(a.w00)[i];
    reinterpret_cast<float4*>(W1)[i] = reinterpret_cast<const float4*>(a.w01)[i];
  }
  __syncthreads();
  const int L = a.Lz + a.Lx, lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * PR_ROWS;
  const float ba = lane < 8 ? a.b00[lane] : 0.f, bb = lane < 8 ? a.b01[lane] : 0.f;
  for (int rr = 0; rr < PR_ROWS; ++rr) {
    const int row = row0 + rr;
    if (row >= a.B * L) return;
    const int b = row / L, s = row - b * L;
    Row12 xa;
    if (a.layer == 0) {
      xa = load_row(a.srcA + (int64_t)row * C768, lane);
    } else {
      const int pos = s < a.Lz ? s : a.slot2pos[b * a.Lx + (s - a.Lz)];
      xa = pos >= 0 ? load_row(a.srcA + ((int64_t)b * a.srcA_rows + pos) * C768, lane) : zero_row();
    }
    const Row12 xb = load_row(a.srcB + (int64_t)row * C768, lane);
    float part[8];
    dot8_lds(ln_row(xa, a.lnA_w, a.lnA_b, lane), W0, part, lane);
    const float ra = reduce8(part, lane);
    dot8_lds(ln_row(xb, a.lnB_w, a.lnB_b, lane), W1, part, lane);
    const float rb = reduce8(part, lane);
    if (lane < 8) {
      a.a8[(int64_t)row * 8 + lane] = ra + ba;
      a.c8[(int64_t)row * 8 + lane] = rb + bb;
    }
  }
}

// Deep layers: conv0_0(LN_A(recovered X)) with conv0_0 held in registers (each lane keeps its 12
// columns x 8 outputs) over a grid-strided run of rows; conv0_1(LN_B(P_prev)) from the previous s8 and
// the folded constants (PromptFold) -- 8 floats per token instead of a 768-float prompt row.
constexpr int PD_BLOCKS = 512;

__global__ __launch_bounds__(256) void prompt_reduce_deep_kernel(const PromptArgs a) {
  __shared__ float fold[FOLD_N];
  for (int i = threadIdx.x; i < FOLD_N; i += 256) fold[i] = a.fold[i];
  __syncthreads();
  const int L = a.Lz + a.Lx, lane = threadIdx.x & 63;
  float4 w[8][3];
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int i = 0; i < 3; ++i) w[k][i] = reinterpret_cast<const float4*>(a.w00 + k * C768)[lane + 64 * i];
  const float ba = lane < 8 ? a.b00[lane] : 0.f;
  const int kk = lane & 7;
  const int nw = gridDim.x * 4;
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < a.B * L; row += nw) {
    const int b = row / L, s = row - b * L;
    const int pos = s < a.Lz ? s : a.slot2pos[b * a.Lx + (s - a.Lz)];
    const Row12 xa = pos >= 0 ? load_row(a.srcA + ((int64_t)b * a.srcA_rows + pos) * C768, lane) : zero_row();
    const Row12 y = ln_row(xa, a.lnA_w, a.lnA_b, lane);
    float part[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        t += y.v[i].x * w[k][i].x + y.v[i].y * w[k][i].y + y.v[i].z * w[k][i].z + y.v[i].w * w[k][i].w;
      part[k] = t;
    }
    const float ra = reduce8(part, lane);
    // c8 from the previous prompt's s8
    const float4* sp = reinterpret_cast<const float4*>(a.s8 + (int64_t)row * 8);
    const float4 s0 = sp[0], s1 = sp[1];
    const float sv[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    float var = fold[FOLD_gb];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gj = 2.f * fold[FOLD_g + j];
#pragma unroll
      for (int l = 0; l < 8; ++l) gj += fold[FOLD_G + j * 8 + l] * sv[l];
      var += gj * sv[j];
    }
    const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + LN_EPS);
    float mk = fold[FOLD_mc + kk];
#pragma unroll
    for (int j = 0; j < 8; ++j) mk += fold[FOLD_MC + kk * 8 + j] * sv[j];
    const float rb = rstd * mk + fold[FOLD_cb + kk];
    if (lane < 8) {
      a.a8[(int64_t)row * 8 + lane] = ra + ba;
      a.c8[(int64_t)row * 8 + lane] = rb;
    }
  }
}

void prompt_reduce(const PromptArgs& a, hipStream_t s) {
  const int rows = a.B * (a.Lz + a.Lx);
  if (a.layer == 0) {
    const int waves = (rows + PR_ROWS - 1) / PR_ROWS;
    hipLaunchKernelGGL(prompt_reduce_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, a);
  } else {
    const int blocks = min(PD_BLOCKS, (rows + 3) / 4);   // small batches: one row per wave
    hipLaunchKernelGGL(prompt_reduce_deep_kernel, dim3(blocks), dim3(256), 0, s, a);
  }
}

// ------------------------------------------------------------------ prompt block, part 2
// Fovea (vit_ce_prompt.py:33-47): per channel, softmax over the part's h*w positions of
// x*smooth, times x; + conv0_1 branch -> s8 (kept: the next layer folds LN_B + conv0_1 onto it);
// conv1x1 8 -> 768 (+bias) -> prompt P (full slot layout, each thread holding the conv1x1 rows of its
// 3 columns across the block's 16 tokens).  The residual update that consumes P is fused into the
// next LayerNorm (ln_prompt below).
constexpr int PCHUNK = 16;

__global__ __launch_bounds__(256) void prompt_expand_kernel(const PromptArgs a) {
  __shared__ float red[256];
  __shared__ float smax[8], ssum[8];
  __shared__ float f[PCHUNK][8];
  const int L = a.Lz + a.Lx, b = blockIdx.y, tid = threadIdx.x;
  const int nbz = (a.Lz + PCHUNK - 1) / PCHUNK;
  int lo, n, t0;
  if ((int)blockIdx.x < nbz) {
    lo = 0; n = a.Lz; t0 = blockIdx.x * PCHUNK;
  } else {
    lo = a.Lz; n = a.Lx; t0 = a.Lz + (blockIdx.x - nbz) * PCHUNK;
  }
  const int t1 = min(t0 + PCHUNK, lo + n);
  const float* a8 = a.a8 + (int64_t)b * L * 8;
  const float* c8 = a.c8 + (int64_t)b * L * 8;
  const float sm = a.smooth;
  const int c = tid & 7, stripe = tid >> 3;
  float mx = -INFINITY;
  for (int t = lo + stripe; t < lo + n; t += 32) mx = fmaxf(mx, a8[t * 8 + c] * sm);
  mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  if ((tid & 63) < 8) red[(tid >> 6) * 8 + c] = mx;
  __syncthreads();
  if (tid < 8) smax[tid] = fmaxf(fmaxf(red[tid], red[8 + tid]), fmaxf(red[16 + tid], red[24 + tid]));
  __syncthreads();
  const float cm = smax[c];
  float sum = 0.f;
  for (int t = lo + stripe; t < lo + n; t += 32) sum += __expf(a8[t * 8 + c] * sm - cm);
  sum += __shfl_xor(sum, 8, 64);
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  __syncthreads();
  if ((tid & 63) < 8) red[(tid >> 6) * 8 + c] = sum;
  __syncthreads();
  if (tid < 8) ssum[tid] = (red[tid] + red[8 + tid]) + (red[16 + tid] + red[24 + tid]);
  __syncthreads();
  if (tid < (t1 - t0) * 8) {
    const int t = t0 + tid / 8, ch = tid & 7;
    const float v = a8[t * 8 + ch];
    const float msk = __expf(v * sm - smax[ch]) / ssum[ch];
    const float sv = msk * v + c8[t * 8 + ch];
    f[tid / 8][ch] = sv;
    a.s8[((int64_t)b * L + t) * 8 + ch] = sv;   // kept for the next layer's folded LN_B + conv0_1
  }
  __syncthreads();
  float w1r[3][8], b1r[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int col = tid + 256 * k;
    const float4* w4 = reinterpret_cast<const float4*>(a.w1 + col * 8);
    const float4 p0 = w4[0], p1 = w4[1];
    w1r[k][0] = p0.x; w1r[k][1] = p0.y; w1r[k][2] = p0.z; w1r[k][3] = p0.w;
    w1r[k][4] = p1.x; w1r[k][5] = p1.y; w1r[k][6] = p1.z; w1r[k][7] = p1.w;
    b1r[k] = a.b1[col];
  }
  for (int t = t0; t < t1; ++t) {
    float* prow = a.P + ((int64_t)b * L + t) * C768;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float v = b1r[k];
#pragma unroll
      for (int ch = 0; ch < 8; ++ch) v += w1r[k][ch] * f[t - t0][ch];
      prow[tid + 256 * k] = v;
    }
  }
}

void prompt_expand(const PromptArgs& a, hipStream_t s) {
  const int nb = (a.Lz + PCHUNK - 1) / PCHUNK + (a.Lx + PCHUNK - 1) / PCHUNK;
  hipLaunchKernelGGL(prompt_expand_kernel, dim3(nb, a.B), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ LN1 with the prompt residual fused
// mode 1 (layer 0):  X[r] = (tok_rgb[r] + P[r]) + pos[t]          (vit_ce_prompt.py:218, 240-241)
// mode 2 (layer i):  X[r] = X[r] + P[b][slot(t)], slot(t) = t < Lz ? t : gidx[b][t-Lz]
//                    (candidate_elimination_prompt + x_ori add, attn_blocks.py:9-18, vit_ce_prompt.py:310)
// then out = LN(X[r]) (norm1 of the block).
__global__ __launch_bounds__(256) void ln_prompt_kernel(const LnPromptArgs a) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= a.rows) return;
  const int b = r / a.rows_per_seq, t = r - b * a.rows_per_seq;
  const int L = a.Lz + a.Lx;
  Row12 x;
  if (a.mode == 1) {
    const Row12 tk = load_row(a.tok_rgb + (int64_t)r * C768, lane);
    const Row12 pp = load_row(a.P + (int64_t)r * C768, lane);
    const Row12 ps = load_row(a.pos + (int64_t)t * C768, lane);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      x.v[i] = make_float4((tk.v[i].x + pp.v[i].x) + ps.v[i].x, (tk.v[i].y + pp.v[i].y) + ps.v[i].y,
                           (tk.v[i].z + pp.v[i].z) + ps.v[i].z, (tk.v[i].w + pp.v[i].w) + ps.v[i].w);
  } else {
    const int slot = t < a.Lz ? t : a.Lz + a.gidx[b * (a.rows_per_seq - a.Lz) + (t - a.Lz)];
    const Row12 xo = load_row(a.X + (int64_t)r * C768, lane);
    const Row12 pp = load_row(a.P + ((int64_t)b * L + slot) * C768, lane);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      x.v[i] = make_float4(xo.v[i].x + pp.v[i].x, xo.v[i].y + pp.v[i].y, xo.v[i].z + pp.v[i].z,
                           xo.v[i].w + pp.v[i].w);
  }
  store_f32(a.X + (int64_t)r * C768, x, lane);
  const Row12 y = ln_row(x, a.w, a.b, lane);
  store_bf16(a.out + (int64_t)r * C768, y, lane);
  if (a.out_lo) store_bf16_lo(a.out_lo + (int64_t)r * C768, y, lane);
}

void prompt_expand_ln(const PromptArgs& pa, const LnPromptArgs& a, hipStream_t s) {
  prompt_expand(pa, s);
  hipLaunchKernelGGL(ln_prompt_kernel, dim3((a.rows + 3) / 4), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ candidate elimination
// attn_blocks.py:37-73: score = mean over heads of the CTR_POINT template row of P over the
// search keys, sort descending, keep ceil(ratio * Ls); ties broken by the lower index.
__device__ __forceinline__ bool before(float ka, int va, float kb, int vb) {
  return ka > kb || (ka == kb && va < vb);
}

// Rank selection instead of a sort network: every search token's position in the descending order
// (ties -> lower index, the order "before" defines) is the number of tokens before it, counted in
// one parallel pass over LDS (Ls <= 1024), so there is a single barrier instead of log^2 stages.
__global__ __launch_bounds__(512) void ce_select_kernel(const CEArgs a) {
  __shared__ float key[1024];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* prob = a.prob + (int64_t)b * a.heads * a.Ls;
  for (int i = tid; i < a.Ls; i += 512) {
    float s = 0.f;
    for (int h = 0; h < a.heads; ++h) s += prob[h * a.Ls + i];
    key[i] = s / (float)a.heads;
  }
  __syncthreads();
  const int Ln = a.Lz + a.keep;
  for (int i = tid; i < a.Ls; i += 512) {
    const float ki = key[i];
    int rank = 0;
    for (int j = 0; j < a.Ls; ++j) rank += before(key[j], j, ki, i) ? 1 : 0;
    const int slot = a.gidx_in[b * a.Ls + i];
    if (rank < a.keep) {
      a.gidx_out[b * a.keep + rank] = slot;
      a.gather[b * Ln + a.Lz + rank] = a.Lz + i;
      a.slot2pos[b * a.Lx + slot] = a.Lz + rank;
    } else {
      a.removed[b * a.Lx + a.removed_off + (rank - a.keep)] = slot;
      a.slot2pos[b * a.Lx + slot] = -1;
    }
  }
  for (int t = tid; t < a.Lz; t += 512) a.gather[b * Ln + t] = t;
}

void ce_select(const CEArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ce_select_kernel, dim3(a.B), dim3(512), 0, s, a);
}

__global__ void init_indices_kernel(int* gidx, int* slot2pos, int B, int Lz, int Lx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Lx) return;
  const int j = i % Lx;
  gidx[i] = j;
  slot2pos[i] = Lz + j;
}

void init_indices(int* gidx, int* slot2pos, int B, int Lz, int Lx, hipStream_t s) {
  hipLaunchKernelGGL(init_indices_kernel, dim3((B * Lx + 255) / 256), dim3(256), 0, s, gidx, slot2pos, B, Lz, Lx);
}

// ------------------------------------------------------------------ final norm + recover_tokens
// vit_ce_prompt.py:318-339: LN over the surviving tokens, then scatter the search tokens back
// to their 16x16 slots; pruned slots are exact zeros.
__global__ __launch_bounds__(256) void final_norm_kernel(const float* X, int rows_per_seq, const int* slot2pos,
                                                         const float* w, const float* b, int B, int Lz, int Lx,
                                                         bf16_t* feat, bf16_t* feat_lo, float* dbg) {
  const int L = Lz + Lx;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= B * L) return;
  const int bs = r / L, s = r - bs * L;
  int pos = s < Lz ? s : slot2pos[bs * Lx + (s - Lz)];
  Row12 y = zero_row();
  if (pos >= 0) y = ln_row(load_row(X + ((int64_t)bs * rows_per_seq + pos) * C768, lane), w, b, lane);
  if (s >= Lz) store_bf16(feat + ((int64_t)bs * Lx + (s - Lz)) * C768, y, lane);
  if (s >= Lz && feat_lo) store_bf16_lo(feat_lo + ((int64_t)bs * Lx + (s - Lz)) * C768, y, lane);
  if (dbg) store_f32(dbg + (int64_t)r * C768, y, lane);
}

void final_norm_recover(const float* X, int rows_per_seq, const int* slot2pos, const float* w, const float* b,
                        int B, int Lz, int Lx, bf16_t* feat, bf16_t* feat_lo, float* feat_f32_dbg, hipStream_t s) {
  const int rows = B * (Lz + Lx);
  hipLaunchKernelGGL(final_norm_kernel, dim3((rows + 3) / 4), dim3(256), 0, s, X, rows_per_seq, slot2pos, w, b, B,
                     Lz, Lx, feat, feat_lo, feat_f32_dbg);
}

}  // namespace mmt
