// Bandwidth-bound token kernels of the ViPT path, gfx950: LayerNorm, the
// modality-prompt blocks, candidate elimination, final norm + token recovery.
// Rows are 768 fp32 (one wave per row, 3 x float4 per lane).
#include "kernels.h"

namespace mmt {

constexpr int C768 = 768;
constexpr float LN_EPS = 1e-6f;   // vit_ce_prompt.py:121

#if defined(ROW_STAMPS)   // tuning builds only (tools/b1_row_stamps.py): per-block phase cycles of the row kernels
// [kind][block][8]: s_memtime at four phase points of wave 0, s_memrealtime at entry and end; kind 0 = ln_kernel<true>,
// 1 = ln_prompt_kernel, 2 = prompt_reduce_deep_kernel (the last launch of each kind in a frame)
__device__ unsigned long long* g_row_stamps = nullptr;
extern "C" int mmt_row_stamps(void* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_row_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}
#define RSTAMP_DECL unsigned long long* const rst_ = g_row_stamps
#define RSTAMP_AT(kind, k, v)                                                                               \
  do {                                                                                                      \
    if (rst_ && threadIdx.x == 0)                                                                           \
      rst_[((size_t)(kind) * 4096 + blockIdx.x + (size_t)blockIdx.y * gridDim.x) * 8 + (k)] = (v);          \
  } while (0)
#define RSTAMP(kind, k) RSTAMP_AT(kind, k, __builtin_amdgcn_s_memtime())
#define RSTAMP_RT(kind, k) RSTAMP_AT(kind, k, __builtin_amdgcn_s_memrealtime())
#define RSTAMP_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define RSTAMP_DECL
#define RSTAMP(kind, k) do { } while (0)
#define RSTAMP_RT(kind, k) do { } while (0)
#define RSTAMP_DRAIN() do { } while (0)
#endif

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

// LayerNorm over 768 (F.layer_norm semantics: biased variance, eps inside sqrt).  The arithmetic is spelled out
// (contraction off, the fused multiply-adds written as fmaf) so that every kernel inlining it rounds the same way:
// left to the compiler, ln_kernel and the fused CE + LN2 kernel contracted different products and their rows
// differed in the last bits (tools/runs_r5/r5_run15.sh)
__device__ __forceinline__ float sumsq4(float4 d, float acc) {
#pragma clang fp contract(off)
  float t = d.x * d.x;
  t = __builtin_fmaf(d.y, d.y, t);
  t = __builtin_fmaf(d.z, d.z, t);
  t = __builtin_fmaf(d.w, d.w, t);
  return acc + t;
}
// the LayerNorm affine of one lane's 12 columns, requested at kernel entry: loaded inside ln_row, after a store of
// the residual row, it was a second dependent memory round trip per launch (the compiler may not move a load above
// a store it cannot prove disjoint)
struct LnAffine { float4 w[3], b[3]; };
__device__ __forceinline__ LnAffine load_affine(const float* w, const float* b, int lane) {
  LnAffine a;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    a.w[i] = reinterpret_cast<const float4*>(w)[lane + 64 * i];
    a.b[i] = reinterpret_cast<const float4*>(b)[lane + 64 * i];
  }
  return a;
}
__device__ __forceinline__ Row12 ln_row(const Row12& x, const LnAffine& af) {
#pragma clang fp contract(off)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) s += ((x.v[i].x + x.v[i].y) + x.v[i].z) + x.v[i].w;
  const float mean = wave_sum(s) * (1.0f / C768);
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i)
    q = sumsq4(make_float4(x.v[i].x - mean, x.v[i].y - mean, x.v[i].z - mean, x.v[i].w - mean), q);
  const float rstd = 1.0f / sqrtf(__builtin_fmaf(wave_sum(q), 1.0f / C768, LN_EPS));
  Row12 y;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 ww = af.w[i], bb = af.b[i];
    y.v[i] = make_float4(__builtin_fmaf((x.v[i].x - mean) * rstd, ww.x, bb.x),
                         __builtin_fmaf((x.v[i].y - mean) * rstd, ww.y, bb.y),
                         __builtin_fmaf((x.v[i].z - mean) * rstd, ww.z, bb.z),
                         __builtin_fmaf((x.v[i].w - mean) * rstd, ww.w, bb.w));
  }
  return y;
}

// (x - mean) * rstd, the affine applied by the caller (or folded into the consumer's weights)
__device__ __forceinline__ Row12 ln_hat(const Row12& x) {
#pragma clang fp contract(off)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 3; ++i) s += ((x.v[i].x + x.v[i].y) + x.v[i].z) + x.v[i].w;
  const float mean = wave_sum(s) * (1.0f / C768);
  float q = 0.f;
  Row12 d;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    d.v[i] = make_float4(x.v[i].x - mean, x.v[i].y - mean, x.v[i].z - mean, x.v[i].w - mean);
    q = sumsq4(d.v[i], q);
  }
  const float rstd = 1.0f / sqrtf(__builtin_fmaf(wave_sum(q), 1.0f / C768, LN_EPS));
#pragma unroll
  for (int i = 0; i < 3; ++i) d.v[i] = make_float4(d.v[i].x * rstd, d.v[i].y * rstd, d.v[i].z * rstd, d.v[i].w * rstd);
  return d;
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
// the f16x3 halves of y * scale (common.h)
__device__ __forceinline__ void store_split(bf16_t* hi, bf16_t* lo, const Row12& y, float scale, int lane) {
  uint2* qh = reinterpret_cast<uint2*>(hi);
  uint2* ql = reinterpret_cast<uint2*>(lo);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float v[4] = {y.v[i].x * scale, y.v[i].y * scale, y.v[i].z * scale, y.v[i].w * scale};
    uint16_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) split_h(v[e], h[e], l[e]);
    qh[lane + 64 * i] = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
    ql[lane + 64 * i] = make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
  }
}
__device__ __forceinline__ void store_f32(float* p, const Row12& y, int lane) {
  float4* q = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int i = 0; i < 3; ++i) q[lane + 64 * i] = y.v[i];
}

// X row + its pending split-K update (RowReduce): the slabs summed in slice order, then store4's
// EPI_RESID_F32 arithmetic -- the bits of the splitk_reduce launch this replaces.  All slab loads are issued
// before the first add.
constexpr int kMaxDeferSlabs = 8;
// the pending split-K update of a residual row in two halves: the loads of the row's slabs and bias (issued early by a
// kernel that has the row index early), then the sum in slice order, scale, bias and residual add
struct SlabRow {
  f32x4 p[kMaxDeferSlabs][3];
  float4 bias[3];
};
__device__ __forceinline__ void load_slabs(const RowReduce& rr, int64_t row, int lane, SlabRow& q) {
  const float* base = rr.ws + row * C768;
#pragma unroll
  for (int i = 0; i < 3; ++i) q.bias[i] = reinterpret_cast<const float4*>(rr.bias)[lane + 64 * i];
#pragma unroll
  for (int sl = 0; sl < kMaxDeferSlabs; ++sl)
    if (sl < rr.ks)
#pragma unroll
      for (int i = 0; i < 3; ++i) q.p[sl][i] = reinterpret_cast<const f32x4*>(base + sl * rr.slab)[lane + 64 * i];
}
__device__ __forceinline__ Row12 combine_slabs(const Row12& x, const RowReduce& rr, const SlabRow& q) {
  Row12 o;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    f32x4 acc = q.p[0][i];
#pragma unroll
    for (int sl = 1; sl < kMaxDeferSlabs; ++sl)
      if (sl < rr.ks) acc += q.p[sl][i];
    const float4 bv = q.bias[i];
    const float sc = rr.inv;
    // (explicit fmaf: the same rounding in every consumer kernel, see ln_row)
    const float v[4] = {__builtin_fmaf(acc[0], sc, bv.x), __builtin_fmaf(acc[1], sc, bv.y),
                        __builtin_fmaf(acc[2], sc, bv.z), __builtin_fmaf(acc[3], sc, bv.w)};
    const float4 r = x.v[i];
    o.v[i] = make_float4(r.x + v[0], r.y + v[1], r.z + v[2], r.w + v[3]);
  }
  return o;
}
__device__ __forceinline__ Row12 apply_reduce(const Row12& x, const RowReduce& rr, int64_t row, int lane) {
  SlabRow q;
  load_slabs(rr, row, lane, q);
  return combine_slabs(x, rr, q);
}

// ------------------------------------------------------------------ fovea statistics (vit_ce_prompt.py:33-47)
// Per (sequence, part) and channel: the max over the part's slots of a8 * smooth and the sum of
// exp(a8 * smooth - max), part 0 = template slots [0, Lz), part 1 = search slots [Lz, L).  The reduction order is
// that of the former standalone fovea kernel (256 threads per part, channel = tid & 7, slot stripes of 32, four
// 64-thread groups combined pairwise), so every block that needs a sequence's statistics forms the same bits.
// st[part * 16 + c] = max, st[part * 16 + 8 + c] = sum.
// The sequence's a8 first goes to LDS with coalesced 16-B loads (fovea_stage, issued by the caller with its other
// early loads; fovea_stats stores them and reduces from LDS, as the former fovea kernel did).
constexpr int FOVEA_MAX_TOKENS = 1024;
constexpr int FOVEA_STAGE = FOVEA_MAX_TOKENS * 8 / 4 / 512;   // float4 per thread (512-thread blocks)
struct FoveaStage { float4 v[FOVEA_STAGE]; };
__device__ __forceinline__ FoveaStage fovea_stage(const float* a8seq, int L) {
  FoveaStage f;
#pragma unroll
  for (int k = 0; k < FOVEA_STAGE; ++k) {
    const int e = threadIdx.x + 512 * k;
    if (e < L * 2) f.v[k] = reinterpret_cast<const float4*>(a8seq)[e];
  }
  return f;
}
// (a thread's slots -- n / 32 of them, 8 at the 256-slot search part -- are read once into registers for both
// passes, and the max and sum partials of the four groups go to separate LDS rows: three barriers fewer than the
// former kernel's six, the same operations in the same order)
constexpr int FOVEA_KV = 8;
__device__ __forceinline__ void fovea_stats(const FoveaStage& fs, int Lz, int Lx, float sm, float* va, float* red,
                                            float* st) {
#pragma unroll
  for (int k = 0; k < FOVEA_STAGE; ++k) {
    const int e = threadIdx.x + 512 * k;
    if (e < (Lz + Lx) * 2) reinterpret_cast<float4*>(va)[e] = fs.v[k];
  }
  __syncthreads();
  const int tid = threadIdx.x, part = tid >> 8, t = tid & 255;
  const int lo = part ? Lz : 0, n = part ? Lx : Lz;
  const int c = t & 7, stripe = t >> 3;
  float* rm = red + part * 32;        // [group][channel] maxima
  float* rs = red + 64 + part * 32;   // [group][channel] sums
  const int cnt = n > stripe ? (n - stripe + 31) / 32 : 0;   // this thread's slots stripe, stripe + 32, ...
  const bool regs = cnt <= FOVEA_KV;                         // (n <= 256: every thread)
  float v[FOVEA_KV];
  float mx = -INFINITY;
  if (regs) {
#pragma unroll
    for (int j = 0; j < FOVEA_KV; ++j) v[j] = j < cnt ? va[(lo + stripe + 32 * j) * 8 + c] : 0.f;
#pragma unroll
    for (int j = 0; j < FOVEA_KV; ++j)
      if (j < cnt) mx = fmaxf(mx, v[j] * sm);
  } else {
    for (int k = stripe; k < n; k += 32) mx = fmaxf(mx, va[(lo + k) * 8 + c] * sm);
  }
  mx = fmaxf(mx, dpp<DPP_ROR8>(mx));
  mx = xmax16(mx);
  mx = xmax32(mx);
  if ((t & 63) < 8) rm[(t >> 6) * 8 + c] = mx;
  __syncthreads();
  const float cm = fmaxf(fmaxf(rm[c], rm[8 + c]), fmaxf(rm[16 + c], rm[24 + c]));
  float sum = 0.f;
  if (regs) {
#pragma unroll
    for (int j = 0; j < FOVEA_KV; ++j)
      if (j < cnt) sum += __expf(__builtin_fmaf(v[j], sm, -cm));
  } else {
    for (int k = stripe; k < n; k += 32) sum += __expf(__builtin_fmaf(va[(lo + k) * 8 + c], sm, -cm));
  }
  sum += dpp<DPP_ROR8>(sum);
  sum = xsum16(sum, sum);
  sum = xsum32(sum, sum);
  if ((t & 63) < 8) rs[(t >> 6) * 8 + c] = sum;
  __syncthreads();
  if (t < 8) {
    st[part * 16 + t] = cm;
    st[part * 16 + 8 + t] = (rs[t] + rs[8 + t]) + (rs[16 + t] + rs[24 + t]);
  }
  __syncthreads();
}
// s8[c] of one slot (lane c < 8 of the caller): fovea mask * a8 + c8 (the former fovea kernel's expression)
// (the arithmetic spelled out, as ln_row: the deep prompt, LN1 and fused prompt + LN1 kernels form the same bits)
__device__ __forceinline__ float fovea_s8(float a, float cc, const float* st, int part, int c, float sm) {
  return __builtin_fmaf(__expf(__builtin_fmaf(a, sm, -st[part * 16 + c])) / st[part * 16 + 8 + c], a, cc);
}

// ------------------------------------------------------------------ LayerNorm (optionally fused CE gather)
// RR: a pending split-K update may be applied (its up-to-8 slabs take 96 VGPRs: the variant without them keeps
// more waves per CU)
template <bool RR>
__global__ __launch_bounds__(256) void ln_kernel(const float* x, const float* w, const float* b, bf16_t* ob,
                                                 bf16_t* olo, float oscale, float* of, int rows, int rows_per_seq,
                                                 const int* gather, int in_rows_per_seq, float* xcopy,
                                                 const RowReduce rr) {
  RSTAMP_DECL;
  RSTAMP_RT(RR ? 0 : 3, 4);
  RSTAMP(RR ? 0 : 3, 0);
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= rows) return;
  const LnAffine af = load_affine(w, b, lane);
  int64_t src = r;
  if (gather) {
    const int bs = r / rows_per_seq;
    src = (int64_t)bs * in_rows_per_seq + gather[r];
  }
  Row12 xv = load_row(x + src * C768, lane);
  if (RR && rr.ws) {   // the pending split-K update of the residual stream (proj / fc2), then X is current again
    xv = apply_reduce(xv, rr, src, lane);
    if (!xcopy) store_f32(const_cast<float*>(x) + src * C768, xv, lane);
  }
  if (xcopy) store_f32(xcopy + (int64_t)r * C768, xv, lane);
  RSTAMP(RR ? 0 : 3, 1);   // (the row and its slabs landed: the combine consumed them)
  const Row12 y = ln_row(xv, af);
  RSTAMP(RR ? 0 : 3, 2);
  if (olo) store_split(ob + (int64_t)r * C768, olo + (int64_t)r * C768, y, oscale, lane);
  else if (ob) store_bf16(ob + (int64_t)r * C768, y, lane);
  if (of) store_f32(of + (int64_t)r * C768, y, lane);
  RSTAMP_DRAIN();
  RSTAMP(RR ? 0 : 3, 3);
  RSTAMP_RT(RR ? 0 : 3, 5);
}

// rows per workgroup: 4, or 1 for the few rows of one or two sequences -- each workgroup's row, split-K slabs and
// affine then come into a CU of their own instead of four rows' worth into one (the launch is per-CU intake bound
// there: a row with four fc2 slabs is 15 KB)
static int rows_per_block(int rows) {
  static const int few = getenv("MMT_ROW_FEW") ? atoi(getenv("MMT_ROW_FEW")) : 1024;
  return rows <= few ? 1 : 4;
}

void layernorm(const float* x, const float* w, const float* b, bf16_t* out_bf16, bf16_t* out_lo, float out_scale,
               float* out_f32, int rows, int rows_per_seq, const int* gather, int in_rows_per_seq, float* xcopy,
               hipStream_t s, const RowReduce& rr) {
  const int rpb = rows_per_block(rows);
  const dim3 grid((rows + rpb - 1) / rpb), block(64 * rpb);
  if (rr.ws)
    hipLaunchKernelGGL(ln_kernel<true>, grid, block, 0, s, x, w, b, out_bf16, out_lo, out_scale, out_f32, rows,
                       rows_per_seq, gather, in_rows_per_seq, xcopy, rr);
  else
    hipLaunchKernelGGL(ln_kernel<false>, grid, block, 0, s, x, w, b, out_bf16, out_lo, out_scale, out_f32, rows,
                       rows_per_seq, gather, in_rows_per_seq, xcopy, rr);
}

// ------------------------------------------------------------------ prompt block, part 1
// For every slot s of every sequence: a8 = conv0_0(LN_A(srcA[s])), c8 = conv0_1(LN_B(srcB[s]))
// (Prompt_block.forward, vit_ce_prompt.py:62-68, on token2feature maps; a pruned search slot
// is a zero row, vit_ce_prompt.py:276-283, whose LN is the LN bias).
// The two 8 x 768 conv weights live in LDS; a wave handles PR_ROWS rows; the 8 per-lane partial
// dot products are reduced with a transposing butterfly (10 shuffles instead of 8 x 6).
constexpr int PR_ROWS = 4;

// out[c] (valid in lane c for c < 8) = sum over the wave of part[c]: a transposing butterfly, the
// 32 / 16-lane stages as permlane half-exchanges, the rest DPP (one ds_bpermute for the final gather)
__device__ __forceinline__ float reduce8(float (&part)[8], int lane) {
  // stage 32: lanes < 32 keep channels 0-3, others 4-7
  float v4[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v4[i] = xsum32(part[i], part[i + 4]);
  // stage 16: rows 0 / 2 keep the lower pair, rows 1 / 3 the upper
  float v2[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) v2[i] = xsum16(v4[i], v4[i + 2]);
  const bool hi8 = lane & 8;
  float v1 = (hi8 ? v2[1] : v2[0]) + dpp<DPP_ROR8>(hi8 ? v2[0] : v2[1]);
  // the 8 lanes of a channel: xor 1, xor 2 (quad_perm), then the quads' sums meet by row_half_mirror
  v1 += dpp<DPP_XOR1>(v1);
  v1 += dpp<DPP_XOR2>(v1);
  v1 += dpp<0x141>(v1);
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
  const LnAffine afA = load_affine(a.lnA_w, a.lnA_b, lane), afB = load_affine(a.lnB_w, a.lnB_b, lane);
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
    dot8_lds(ln_row(xa, afA), W0, part, lane);
    const float ra = reduce8(part, lane);
    dot8_lds(ln_row(xb, afB), W1, part, lane);
    const float rb = reduce8(part, lane);
    if (lane < 8) {
      a.a8[(int64_t)row * 8 + lane] = ra + ba;
      a.c8[(int64_t)row * 8 + lane] = rb + bb;
    }
  }
}

// Deep layers: conv0_0(LN_A(recovered X)) with conv0_0 (LN_A's affine folded in) in LDS; conv0_1(LN_B(P_prev))
// from the previous prompt's s8 and the folded constants (PromptFold) -- 8 floats per token instead of a
// 768-float prompt row.  s8_prev = fovea(a8_prev) + c8_prev is re-formed per slot from the previous block's
// a8 / c8 and the fovea statistics of the slot's sequence, which this block computes (fovea_stats).
// One block = 8 slots of one sequence (grid: slot blocks x sequences), one slot per wave; every global load
// the wave needs -- the slot's compact position, its X row (and pending fc2 split-K slabs), the previous
// a8 / c8 -- is issued before the block's weight fill, statistics and barriers.
constexpr int TOK_THREADS = 512;   // 8 waves per block share one LDS copy of the weights
constexpr int TOK_ROWS = TOK_THREADS / 64;
// the blocks of a deep-prompt / LN1 launch walk the 1 536 float4 of their 8 x 768 weight fill from one of eight
// offsets, so they do not all request the same lines in the same order (one sequence +0.2 %, r06_b1_row_stamps.txt)
#define WFILL_IDX(i) (((i) + (int)((blockIdx.x + 5 * blockIdx.y) % 8) * 192) % (8 * C768 / 4))

// One slot of a deep prompt block (the wave's x row, already current; live = the slot has a row): returns, valid in
// lanes 0-7, a8 = conv0_0(LN_A(x)) + b00 (LN_A's affine folded into W0 / b00 by pack_weights) and c8 from the previous
// prompt's s8 (ap, cp: the previous a8 / c8 of the slot, stp: their fovea statistics) through the folded LN_B + conv0_1.
// The arithmetic is spelled out (contraction off): the deep prompt kernel and the fused prompt + LN1 kernel inline it.
__device__ __forceinline__ float2 deep_slot(const Row12& x, bool live, int part_id, float ap, float cp, const float* stp,
                                            const float* fold, const float* W0, float ba, float smooth_p, int lane) {
#pragma clang fp contract(off)
  const int kk = lane & 7;
  // s8_prev of the slot in lanes 0-7, then the lane's pair of it for the LN_B variance form
  const float s8v = lane < 8 ? fovea_s8(ap, cp, stp, part_id, lane, smooth_p) : 0.f;
  const float sp = __shfl(s8v, kk, 64), sq = __shfl(s8v, lane >> 3, 64);
  // the lane's coefficients of the LN_B variance form: G[q][p] s_p s_q (+ 2 g_q s_q for p = 0, + gb in lane 0)
  const float vG = fold[FOLD_G + lane], vg = kk == 0 ? 2.f * fold[FOLD_g + (lane >> 3)] : 0.f;
  const float vb = lane == 0 ? fold[FOLD_gb] : 0.f;
  float ra = 0.f;   // a pruned slot is a zero row: its LN is 0 and a8 = b00 exactly
  if (live) {       // wave-uniform
    const Row12 y = ln_hat(x);
    float part[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const float4 w = reinterpret_cast<const float4*>(W0 + k * C768)[lane + 64 * i];
        t = __builtin_fmaf(y.v[i].x, w.x, t);
        t = __builtin_fmaf(y.v[i].y, w.y, t);
        t = __builtin_fmaf(y.v[i].z, w.z, t);
        t = __builtin_fmaf(y.v[i].w, w.w, t);
      }
      part[k] = t;
    }
    ra = reduce8(part, lane);
  }
  // c8 from the previous prompt's s8: var = s^T G s + 2 g.s + gb, one (q, p) term per lane
  const float var = wave_sum(__builtin_fmaf(__builtin_fmaf(vG, sp, vg), sq, vb));
  const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + LN_EPS);
  // lane kk < 8: mk = mc[kk] + MC[kk][:] . s   (s[q] is lane 8q's sq)
  float mk = fold[FOLD_mc + kk];
#pragma unroll
  for (int q = 0; q < 8; ++q)
    mk = __builtin_fmaf(fold[FOLD_MC + kk * 8 + q], u2f(__builtin_amdgcn_readlane(f2u(sq), 8 * q)), mk);
  return make_float2(ra + ba, __builtin_fmaf(rstd, mk, fold[FOLD_cb + kk]));
}

// R: slots per wave (the block's weight fill and fovea statistics shared by R x 8 slots; 2 at large batches)
// (two-slot 128-thread blocks for one sequence -- four times the blocks, each with its 24-KB weight fill -- measured
// 4.1 -> 6.7 us per block and one sequence -2.5 %, profiles/r06_b1_row_stamps.txt)
template <bool RR, int R>
__global__ __launch_bounds__(TOK_THREADS) void prompt_reduce_deep_kernel(const PromptArgs a) {
  __shared__ float fold[FOLD_N];
  __shared__ __attribute__((aligned(16))) float W0[8 * C768];   // conv0_0 (LN_A affine folded in)
  extern __shared__ __attribute__((aligned(16))) float va[];   // [L][8] (dynamic: sized by the launch)
  __shared__ float red[128], st[32];
  RSTAMP_DECL;
  RSTAMP_RT(2, 4);
  RSTAMP(2, 0);
  const int L = a.Lz + a.Lx, lane = threadIdx.x & 63, b = blockIdx.y;
  // the previous a8's fovea statistics: as the previous LN1 wrote them (32 floats), else reduced here
  const bool pre = a.fstat_p != nullptr;
  FoveaStage fsg;
  if (!pre) fsg = fovea_stage(a.a8p + (int64_t)b * L * 8, L);
  const float stv = pre && threadIdx.x < 32 ? a.fstat_p[b * 32 + threadIdx.x] : 0.f;
  int sv[R], posv[R];
  int64_t xrowv[R];
  Row12 xv[R];
  float apv[R], cpv[R];
  static_assert(!RR || R == 1, "the slab-holding variant keeps one slot per wave");
  SlabRow slabs;   // RR: the pending fc2 slabs of the wave's row, requested with the row (not after the barrier)
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int s = (blockIdx.x * R + rr) * TOK_ROWS + (threadIdx.x >> 6);   // slot of this wave
    const int pos = s >= L ? -1 : s < a.Lz ? s : a.slot2pos[b * a.Lx + (s - a.Lz)];   // wave-uniform
    sv[rr] = s;
    posv[rr] = pos;
    xrowv[rr] = (int64_t)b * a.srcA_rows + max(pos, 0);
    xv[rr] = load_row(a.srcA + xrowv[rr] * C768, lane);
    if (RR && a.rr.ws) load_slabs(a.rr, xrowv[rr], lane, slabs);
    const int64_t srow = ((int64_t)b * L + min(s, L - 1)) * 8;
    apv[rr] = lane < 8 ? a.a8p[srow + lane] : 0.f;
    cpv[rr] = lane < 8 ? a.c8p[srow + lane] : 0.f;
  }
  constexpr int WV = 8 * C768 / 4 / TOK_THREADS;
  float4 wst[WV];
#pragma unroll
  for (int k = 0; k < WV; ++k) wst[k] = reinterpret_cast<const float4*>(a.w00)[WFILL_IDX(threadIdx.x + TOK_THREADS * k)];
  const float fo = threadIdx.x < FOLD_N ? a.fold[threadIdx.x] : 0.f;
  const float ba = lane < 8 ? a.b00[lane] : 0.f;
#pragma unroll
  for (int k = 0; k < WV; ++k) reinterpret_cast<float4*>(W0)[WFILL_IDX(threadIdx.x + TOK_THREADS * k)] = wst[k];
  if (threadIdx.x < FOLD_N) fold[threadIdx.x] = fo;
  RSTAMP(2, 1);   // (wave 0's weight share landed: stored to the LDS)
  if (pre) {
    if (threadIdx.x < 32) st[threadIdx.x] = stv;
    __syncthreads();
  } else {
    fovea_stats(fsg, a.Lz, a.Lx, a.smooth_p, va, red, st);   // ends with a barrier
  }
  RSTAMP(2, 2);
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
  const int s = sv[rr], pos = posv[rr];
  const int64_t xrow = xrowv[rr];
  Row12 x = xv[rr];
  const float ap = apv[rr], cp = cpv[rr];
  if (s >= L) break;   // wave-uniform; later slots of the wave lie further out
  if (RR && pos >= 0 && a.rr.ws) {   // the previous block's fc2 update of this slot's residual row, written back
    x = combine_slabs(x, a.rr, slabs);
    store_f32(const_cast<float*>(a.srcA) + xrow * C768, x, lane);
  }
  const float2 ac = deep_slot(x, pos >= 0, s < a.Lz ? 0 : 1, ap, cp, st, fold, W0, ba, a.smooth_p, lane);
  if (lane < 8) {
    const int64_t row = (int64_t)b * L + s;
    a.a8[row * 8 + lane] = ac.x;
    a.c8[row * 8 + lane] = ac.y;
  }
  }
  RSTAMP_DRAIN();
  RSTAMP(2, 3);
  RSTAMP_RT(2, 5);
}

// slots per wave of the deep prompt / LN1 kernels: 2 from 8 sequences up (the weight fill and fovea statistics of a
// block amortised over 16 rows), 1 below (a sequence's rows spread over more blocks); MMT_TOK_R (tuning) forces it
static int tok_rows_per_wave(int B) {
  static const int forced = getenv("MMT_TOK_R") ? atoi(getenv("MMT_TOK_R")) : 0;
  if (forced == 1 || forced == 2 || forced == 4) return forced;
  return B >= 8 ? 2 : 1;
}

void prompt_reduce(const PromptArgs& a, hipStream_t s) {
  const int L = a.Lz + a.Lx;
  if (a.layer == 0) {
    const int waves = (a.B * L + PR_ROWS - 1) / PR_ROWS;
    hipLaunchKernelGGL(prompt_reduce_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, a);
  } else {
    // the sequence's a8 in LDS takes L x 32 B, not the 32-KB maximum: at 320 tokens four blocks fit a CU instead
    // of two, so the 640 blocks of a 16-sequence half run in one round
    const int R = a.rr.ws ? 1 : tok_rows_per_wave(a.B);   // the slab-holding variant keeps one slot per wave
    const dim3 grid((L + TOK_ROWS * R - 1) / (TOK_ROWS * R), a.B);
    const size_t va_bytes = a.fstat_p ? 0 : (size_t)L * 8 * sizeof(float);
    if (a.rr.ws)
      hipLaunchKernelGGL((prompt_reduce_deep_kernel<true, 1>), grid, dim3(TOK_THREADS), va_bytes, s, a);
    else if (R == 4)
      hipLaunchKernelGGL((prompt_reduce_deep_kernel<false, 4>), grid, dim3(TOK_THREADS), va_bytes, s, a);
    else if (R == 2)
      hipLaunchKernelGGL((prompt_reduce_deep_kernel<false, 2>), grid, dim3(TOK_THREADS), va_bytes, s, a);
    else
      hipLaunchKernelGGL((prompt_reduce_deep_kernel<false, 1>), grid, dim3(TOK_THREADS), va_bytes, s, a);
  }
}

// ------------------------------------------------------------------ LN1 with the prompt residual fused
// The prompt block's output s8[slot] = fovea(a8)[slot] + c8[slot] (Fovea, vit_ce_prompt.py:33-47: per channel a
// softmax over the part's h*w positions of a8 * smooth, times a8), formed per row from the block's fovea
// statistics of the sequence; P[slot] = conv1x1(s8[slot]) + b1 (vit_ce_prompt.py:69-71) from the 32 bytes of
// s8 and the block's LDS copy of conv1x1 (neither s8 nor P is ever written to HBM).
// mode 1 (layer 0):  X[r] = (tok_rgb[r] + P[r]) + pos[t]          (vit_ce_prompt.py:218, 240-241)
// mode 2 (layer i):  X[r] = X[r] + P[b][slot(t)], slot(t) = t < Lz ? t : gidx[b][t-Lz]
//                    (candidate_elimination_prompt + x_ori add, attn_blocks.py:9-18, vit_ce_prompt.py:310)
// then out = LN(X[r]) (norm1 of the block).  One block = 8 compact rows of one sequence, one per wave; the
// slot, rows and weights are all requested before the statistics and barriers.
//
// One compact row r (the wave's; xv its X row -- mode 1: tok_rgb -- q its position row in mode 1, av / cv the slot's
// a8 / c8 in lanes 0-7, st the sequence's fovea statistics, W1t / cst the block's LDS copies): the arithmetic
// spelled out (contraction off), as the fused prompt + LN1 kernel inlines it too
template <int MODE>
__device__ __forceinline__ void ln_prompt_row(const Row12& xv, const Row12& q, float av, float cv, int part_id,
                                              const float* st, const float* W1t, const float* cst,
                                              const LnPromptArgs& a, int64_t r, int lane) {
#pragma clang fp contract(off)
  const float s8v = lane < 8 ? fovea_s8(av, cv, st, part_id, lane, a.smooth) : 0.f;
  float f[8];
#pragma unroll
  for (int ch = 0; ch < 8; ++ch) f[ch] = u2f(__builtin_amdgcn_readlane(f2u(s8v), ch));
  Row12 x;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 b1 = reinterpret_cast<const float4*>(cst)[lane + 64 * i];
    float pv[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
      const float4 wv = reinterpret_cast<const float4*>(W1t + ch * C768)[lane + 64 * i];
      pv[0] = __builtin_fmaf(wv.x, f[ch], pv[0]);
      pv[1] = __builtin_fmaf(wv.y, f[ch], pv[1]);
      pv[2] = __builtin_fmaf(wv.z, f[ch], pv[2]);
      pv[3] = __builtin_fmaf(wv.w, f[ch], pv[3]);
    }
    const float4 xx = xv.v[i];
    if (MODE == 1) {
      const float4 ps = q.v[i];
      x.v[i] = make_float4((xx.x + pv[0]) + ps.x, (xx.y + pv[1]) + ps.y, (xx.z + pv[2]) + ps.z, (xx.w + pv[3]) + ps.w);
    } else {
      x.v[i] = make_float4(xx.x + pv[0], xx.y + pv[1], xx.z + pv[2], xx.w + pv[3]);
    }
  }
  store_f32(a.X + r * C768, x, lane);
  Row12 y = ln_hat(x);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 gw = reinterpret_cast<const float4*>(cst + C768)[lane + 64 * i];
    const float4 gb = reinterpret_cast<const float4*>(cst + 2 * C768)[lane + 64 * i];
    y.v[i] = make_float4(__builtin_fmaf(y.v[i].x, gw.x, gb.x), __builtin_fmaf(y.v[i].y, gw.y, gb.y),
                         __builtin_fmaf(y.v[i].z, gw.z, gb.z), __builtin_fmaf(y.v[i].w, gw.w, gb.w));
  }
  if (a.out_lo) store_split(a.out + r * C768, a.out_lo + r * C768, y, a.out_scale, lane);
  else store_bf16(a.out + r * C768, y, lane);
}

template <int MODE, int R>
// LNP_WPE (build-time tuning): waves per SIMD the register allocation targets; 6 (80 VGPRs, three blocks per CU)
// spills 5 VGPRs in mode 2 and measured -0.35 % at 32 sequences against the default (tests/r3_run23.sh)
#ifndef LNP_WPE
#define LNP_WPE 1
#endif
__global__ __launch_bounds__(TOK_THREADS) __attribute__((amdgpu_waves_per_eu(LNP_WPE))) void ln_prompt_kernel(const LnPromptArgs a) {
  __shared__ __attribute__((aligned(16))) float W1t[8 * C768];
  __shared__ __attribute__((aligned(16))) float cst[3 * C768];   // conv1x1 bias, norm1 weight, norm1 bias
  extern __shared__ __attribute__((aligned(16))) float va[];   // [L][8] (dynamic: sized by the launch)
  __shared__ float red[128], st[32];
  RSTAMP_DECL;
  RSTAMP_RT(1, 4);
  RSTAMP(1, 0);
  const int lane = threadIdx.x & 63, b = blockIdx.y, L = a.Lz + a.Lx;
  const FoveaStage fsg = fovea_stage(a.a8 + (int64_t)b * L * 8, L);
  int tv[R], slotv[R];
  int64_t rv[R];
  Row12 xvv[R], qv[R];
  float avv[R], cvv[R];
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const int t = (blockIdx.x * R + rr) * TOK_ROWS + (threadIdx.x >> 6);
    const int tc = min(t, a.rows_per_seq - 1);
    const int64_t r = (int64_t)b * a.rows_per_seq + tc;
    const int slot = (MODE == 1 || tc < a.Lz) ? tc : a.Lz + a.gidx[b * (a.rows_per_seq - a.Lz) + (tc - a.Lz)];
    tv[rr] = t;
    rv[rr] = r;
    slotv[rr] = slot;
    if (MODE == 1) {
      xvv[rr] = load_row(a.tok_rgb + r * C768, lane);
      qv[rr] = load_row(a.pos + (int64_t)tc * C768, lane);
    } else {
      xvv[rr] = load_row(a.X + r * C768, lane);
    }
    const int64_t srow = ((int64_t)b * L + slot) * 8;
    avv[rr] = lane < 8 ? a.a8[srow + lane] : 0.f;
    cvv[rr] = lane < 8 ? a.c8[srow + lane] : 0.f;
  }
  constexpr int WE = 8 * C768 / 4 / TOK_THREADS;   // 3 float4 of conv1x1 (channel-major, a.w1 = W1t) per thread
  float4 wst[WE];
#pragma unroll
  for (int k = 0; k < WE; ++k) wst[k] = reinterpret_cast<const float4*>(a.w1)[WFILL_IDX(threadIdx.x + TOK_THREADS * k)];
  float cs[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int e = threadIdx.x + TOK_THREADS * k;
    cs[k] = e < C768 ? a.b1[e] : e < 2 * C768 ? a.w[e - C768] : e < 3 * C768 ? a.b[e - 2 * C768] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < WE; ++k) reinterpret_cast<float4*>(W1t)[WFILL_IDX(threadIdx.x + TOK_THREADS * k)] = wst[k];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int e = threadIdx.x + TOK_THREADS * k;
    if (e < 3 * C768) cst[e] = cs[k];
  }
  RSTAMP(1, 1);   // (wave 0's weight share landed: stored to the LDS)
  fovea_stats(fsg, a.Lz, a.Lx, a.smooth, va, red, st);   // ends with a barrier
  RSTAMP(1, 2);
  if (a.fstat && blockIdx.x == 0 && threadIdx.x < 32) a.fstat[b * 32 + threadIdx.x] = st[threadIdx.x];
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
  if (tv[rr] >= a.rows_per_seq) break;   // wave-uniform; later rows of the wave lie further out
  ln_prompt_row<MODE>(xvv[rr], qv[rr], avv[rr], cvv[rr], slotv[rr] < a.Lz ? 0 : 1, st, W1t, cst, a, rv[rr], lane);
  }
  RSTAMP_DRAIN();
  RSTAMP(1, 3);
  RSTAMP_RT(1, 5);
}

void prompt_expand_ln(const LnPromptArgs& a, hipStream_t s) {
  const int B = a.rows / a.rows_per_seq, R = a.mode == 1 ? std::min(tok_rows_per_wave(B), 2) : tok_rows_per_wave(B);
  const dim3 grid((a.rows_per_seq + TOK_ROWS * R - 1) / (TOK_ROWS * R), B);
  const size_t va_bytes = (size_t)(a.Lz + a.Lx) * 8 * sizeof(float);
  if (a.mode == 2 && R == 4)
    hipLaunchKernelGGL((ln_prompt_kernel<2, 4>), grid, dim3(TOK_THREADS), va_bytes, s, a);
  else if (a.mode == 1 && R == 2)
    hipLaunchKernelGGL((ln_prompt_kernel<1, 2>), grid, dim3(TOK_THREADS), va_bytes, s, a);
  else if (a.mode == 1)
    hipLaunchKernelGGL((ln_prompt_kernel<1, 1>), grid, dim3(TOK_THREADS), va_bytes, s, a);
  else if (R == 2)
    hipLaunchKernelGGL((ln_prompt_kernel<2, 2>), grid, dim3(TOK_THREADS), va_bytes, s, a);
  else
    hipLaunchKernelGGL((ln_prompt_kernel<2, 1>), grid, dim3(TOK_THREADS), va_bytes, s, a);
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
// Four threads per search token (a quad) each count a quarter of the keys and the quad's counts meet
// by DPP, so the serial LDS scan is Ls / 4 long; the 12 head rows of a token are requested together.
constexpr int CE_THREADS = 1024, CE_MAX_HEADS = 16;
__global__ __launch_bounds__(CE_THREADS) void ce_select_kernel(const CEArgs a) {
  __shared__ float key[1024];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* prob = a.prob + (int64_t)b * a.heads * a.Ls;
  for (int i = tid; i < a.Ls; i += CE_THREADS) {
    float v[CE_MAX_HEADS];
#pragma unroll
    for (int h = 0; h < CE_MAX_HEADS; ++h) v[h] = h < a.heads ? prob[h * a.Ls + i] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < CE_MAX_HEADS; ++h)
      if (h < a.heads) s += v[h];   // head order 0, 1, ... as before
    for (int h = CE_MAX_HEADS; h < a.heads; ++h) s += prob[h * a.Ls + i];
    s = s / (float)a.heads;
    if (a.keys_out || a.forced) {   // parity diagnostics only
      const int slot = a.gidx_in[b * a.Ls + i];
      if (a.keys_out) a.keys_out[(int64_t)b * a.keys_pitch + slot] = s;
      if (a.forced) s = a.forced[(int64_t)b * a.keys_pitch + slot];
    }
    key[i] = s;
  }
  __syncthreads();
  const int Ln = a.Lz + a.keep;
  const int q = tid & 3, nq = (a.Ls + 3) / 4;   // the quad member's key range [q nq, (q + 1) nq)
  for (int i0 = 0; i0 < a.Ls; i0 += CE_THREADS / 4) {
    const int i = i0 + (tid >> 2);   // quad-uniform
    const int ic = min(i, a.Ls - 1);
    const float ki = key[ic];
    int rank = 0;
    const int j1 = min((q + 1) * nq, a.Ls);
    for (int j = q * nq; j < j1; ++j) rank += before(key[j], j, ki, ic) ? 1 : 0;
    rank += __builtin_bit_cast(int, dpp<DPP_XOR1>(__builtin_bit_cast(float, rank))) ;
    rank += __builtin_bit_cast(int, dpp<DPP_XOR2>(__builtin_bit_cast(float, rank)));
    if (q == 0 && i < a.Ls) {
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
  }
  for (int t = tid; t < a.Lz; t += CE_THREADS) a.gather[b * Ln + t] = t;
}

void ce_select(const CEArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(ce_select_kernel, dim3(a.B), dim3(CE_THREADS), 0, s, a);
}

// Candidate elimination and the LN2 that gathers its survivors in one launch (few sequences: the one-sequence
// frame, where the select kernel is a latency-bound launch of its own).  Grid (row blocks of one sequence, B): every
// workgroup forms the sequence's head-mean keys and ranks (the arithmetic of ce_select_kernel: the same sums in the
// same order, and a rank is an integer count whatever order it is counted in), keeps the inverse (rank -> token) map
// in LDS and LayerNorms its four compact rows from their gathered source rows, as ln_kernel with the gather would;
// workgroup 0 of each sequence also writes the index arrays ce_select_kernel writes.  Ls <= 1024.
template <bool RR>
__global__ __launch_bounds__(256) void ce_ln_kernel(const CEArgs a, const float* x, const float* w, const float* b,
                                                    bf16_t* ob, bf16_t* olo, float oscale, int in_rows_per_seq,
                                                    float* xcopy, const RowReduce rr) {
  __shared__ float key[1024];
  __shared__ int inv[1024];
  const int bs = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const LnAffine af = load_affine(w, b, lane);
  const float* prob = a.prob + (int64_t)bs * a.heads * a.Ls;
  for (int i = tid; i < a.Ls; i += 256) {
    float v[CE_MAX_HEADS];
#pragma unroll
    for (int h = 0; h < CE_MAX_HEADS; ++h) v[h] = h < a.heads ? prob[h * a.Ls + i] : 0.f;
    float sum = 0.f;
#pragma unroll
    for (int h = 0; h < CE_MAX_HEADS; ++h)
      if (h < a.heads) sum += v[h];
    for (int h = CE_MAX_HEADS; h < a.heads; ++h) sum += prob[h * a.Ls + i];
    sum = sum / (float)a.heads;
    if (a.keys_out || a.forced) {   // parity diagnostics only
      const int slot = a.gidx_in[bs * a.Ls + i];
      if (a.keys_out && blockIdx.x == 0) a.keys_out[(int64_t)bs * a.keys_pitch + slot] = sum;
      if (a.forced) sum = a.forced[(int64_t)bs * a.keys_pitch + slot];
    }
    key[i] = sum;
  }
  __syncthreads();
  const int Ln = a.Lz + a.keep;
  for (int i = tid; i < a.Ls; i += 256) {
    const float ki = key[i];
    int rank = 0;
    for (int j = 0; j < a.Ls; ++j) rank += before(key[j], j, ki, i) ? 1 : 0;
    if (rank < a.keep) inv[rank] = i;
    if (blockIdx.x == 0) {
      const int slot = a.gidx_in[bs * a.Ls + i];
      if (rank < a.keep) {
        a.gidx_out[bs * a.keep + rank] = slot;
        a.gather[bs * Ln + a.Lz + rank] = a.Lz + i;
        a.slot2pos[bs * a.Lx + slot] = a.Lz + rank;
      } else {
        a.removed[bs * a.Lx + a.removed_off + (rank - a.keep)] = slot;
        a.slot2pos[bs * a.Lx + slot] = -1;
      }
    }
  }
  if (blockIdx.x == 0)
    for (int t = tid; t < a.Lz; t += 256) a.gather[bs * Ln + t] = t;
  __syncthreads();
  const int p = blockIdx.x * 4 + (tid >> 6);   // compact row of the sequence
  if (p >= Ln) return;
  const int64_t r = (int64_t)bs * Ln + p;
  const int64_t src = (int64_t)bs * in_rows_per_seq + (p < a.Lz ? p : a.Lz + inv[p - a.Lz]);
  Row12 xv = load_row(x + src * C768, lane);
  if (RR && rr.ws) {
    xv = apply_reduce(xv, rr, src, lane);
    if (!xcopy) store_f32(const_cast<float*>(x) + src * C768, xv, lane);
  }
  if (xcopy) store_f32(xcopy + r * C768, xv, lane);
  const Row12 y = ln_row(xv, af);
  if (olo) store_split(ob + r * C768, olo + r * C768, y, oscale, lane);
  else if (ob) store_bf16(ob + r * C768, y, lane);
}

bool ce_layernorm(const CEArgs& a, const float* x, const float* w, const float* b, bf16_t* out_bf16, bf16_t* out_lo,
                  float out_scale, int in_rows_per_seq, float* xcopy, hipStream_t s, const RowReduce& rr) {
  // MMT_CE_FUSED (tuning): 0 never, else the largest batch that takes the fused launch (default 2)
  static const int maxb = getenv("MMT_CE_FUSED") ? atoi(getenv("MMT_CE_FUSED")) : 2;
  if (a.B > maxb || a.Ls > 1024) return false;
  const dim3 grid((a.Lz + a.keep + 3) / 4, a.B);
  if (rr.ws)
    hipLaunchKernelGGL(ce_ln_kernel<true>, grid, dim3(256), 0, s, a, x, w, b, out_bf16, out_lo, out_scale,
                       in_rows_per_seq, xcopy, rr);
  else
    hipLaunchKernelGGL(ce_ln_kernel<false>, grid, dim3(256), 0, s, a, x, w, b, out_bf16, out_lo, out_scale,
                       in_rows_per_seq, xcopy, rr);
  return true;
}

// ------------------------------------------------------------------ final norm + recover_tokens
// vit_ce_prompt.py:318-339: LN over the surviving tokens, then scatter the search tokens back
// to their 16x16 slots; pruned slots are exact zeros.
__global__ __launch_bounds__(256) void final_norm_kernel(const float* X, int rows_per_seq, const int* slot2pos,
                                                         const float* w, const float* b, int B, int Lz, int Lx,
                                                         bf16_t* feat, bf16_t* feat_lo, float fscale, float* dbg,
                                                         const RowReduce rr) {
  const int L = Lz + Lx;
  const int r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= B * L) return;
  const int bs = r / L, s = r - bs * L;
  const LnAffine af = load_affine(w, b, lane);
  int pos = s < Lz ? s : slot2pos[bs * Lx + (s - Lz)];
  Row12 y = zero_row();
  if (pos >= 0) {
    const int64_t row = (int64_t)bs * rows_per_seq + pos;
    Row12 x = load_row(X + row * C768, lane);
    if (rr.ws) x = apply_reduce(x, rr, row, lane);   // the last block's fc2 update (nothing reads X after this)
    y = ln_row(x, af);
  }
  if (s >= Lz && feat_lo)
    store_split(feat + ((int64_t)bs * Lx + (s - Lz)) * C768, feat_lo + ((int64_t)bs * Lx + (s - Lz)) * C768, y, fscale,
                lane);
  else if (s >= Lz)
    store_bf16(feat + ((int64_t)bs * Lx + (s - Lz)) * C768, y, lane);
  if (dbg) store_f32(dbg + (int64_t)r * C768, y, lane);
}

void final_norm_recover(const float* X, int rows_per_seq, const int* slot2pos, const float* w, const float* b,
                        int B, int Lz, int Lx, bf16_t* feat, bf16_t* feat_lo, float feat_scale, float* feat_f32_dbg,
                        hipStream_t s, const RowReduce& rr) {
  const int rows = B * (Lz + Lx), rpb = rows_per_block(rows);
  hipLaunchKernelGGL(final_norm_kernel, dim3((rows + rpb - 1) / rpb), dim3(64 * rpb), 0, s, X, rows_per_seq, slot2pos,
                     w, b, B, Lz, Lx, feat, feat_lo, feat_scale, feat_f32_dbg, rr);
}

}  // namespace mmt
