// MFMA bf16 GEMM with fused epilogues, gfx950 (CDNA4).
//
//   C[m][n] = epi( sum_k A[m][k] * W[n][k] + bias[n] )
//
// The dense contractions of the tracking path (attn.py:17-19 qkv/proj, timm Mlp fc1/fc2,
// patch_embed.py:20 as a k16s16 conv, head.py:8-21 3x3 convs as implicit GEMMs over the NHWC
// token map) all have this shape: activations [tokens x K] and weights [out x K], K-contiguous.
//
// * tiles BM x BN x 64; 4 or 8 waves, each a 64x64 (or smaller) block of v_mfma_f32_16x16x32_bf16;
// * operands move HBM/L2 -> LDS with buffer_load_dwordx4 ... lds (no VGPR staging); each wave-
//   instruction fills 8 LDS rows of 128 B; the 16-B chunks are XOR-swizzled by row (chunk ^ (row&7))
//   by pre-swizzling the per-lane SOURCE address, so the fragment ds_read_b128s are conflict-free;
// * two LDS stages: the loads of K-tile k+1 are in flight while tile k is multiplied;
// * XCD-aware tile order: blocks that share an XCD (b % 8) get a compact rectangle of output tiles
//   (a few W column tiles x all A rows, or an A row slice x all W tiles), so the L2 of each XCD
//   serves the re-reads;
// * SPLIT (fp32-faithful "f16x3" mode, common.h): A = Ah + Al, W = Wh + Wl as fp16 pairs of range-scaled
//   values, acc += Wh*Ah + Wl*Ah + Wh*Al with v_mfma_f32_16x16x32_f16 (22-bit operands: the fp32
//   reference's accuracy, vs ~2e-3 relative for plain bf16), acc * inv in the epilogue;
// * the MFMA is issued W-fragment x A-fragment, so a lane ends with 4 consecutive output columns
//   of one row: 8-B (bf16) / 16-B (fp32) epilogue stores.
#include <type_traits>

#include "kernels.h"

namespace mmt {

__device__ __forceinline__ int swz(int r, int c) { return r * 64 + ((c ^ (r & 7)) << 3); }
// K-tile depth BK = 64: rows of 128 B, 16-B chunk c of row r at c ^ (r & 7).  BK = 32: rows of 64 B
// (four rows per 256-B bank sweep), chunk c at c ^ ((r >> 2) & 2) -- conflict-free for the
// ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... of the fragment reads
template <int BK>
__device__ __forceinline__ int swzk(int r, int c) {
  if constexpr (BK == 64) return swz(r, c);
  else return r * 32 + ((c ^ ((r >> 2) & 2)) << 3);
}

typedef __attribute__((address_space(3))) void* lptr_t;

template <int BM, int BN, int WMW, int WNW, bool SPLIT, int STAGES = 0, int BK = 64>
struct Tile {
  static constexpr int NW = WMW * WNW;
  static constexpr int NT = NW * 64;
  static constexpr int WM = BM / WMW, WN = BN / WNW;
  static constexpr int FM = WM / 16, FN = WN / 16;
  static constexpr int AROWS = SPLIT ? 2 * BM : BM;
  static constexpr int ROWS = AROWS + (SPLIT ? 2 * BN : BN);
  static constexpr int RPW = 512 / BK;              // rows per 1-KB wave-instruction (8 or 16)
  static constexpr int GROUPS = ROWS / RPW;
  static constexpr int STAGE = ROWS * BK;           // bf16 elements per stage
  static constexpr int NSTAGE = STAGES ? STAGES : 2;   // LDS ring depth
  static_assert(GROUPS % NW == 0, "row groups must divide over waves");
};

// logical tile id -> (tm, tn): super-tiles of gm tile-rows x all tile-columns, column-major inside,
// so any 64 consecutive ids cover a ~8 x 8 block of output tiles (A and W slices that fit one L2)
__device__ __forceinline__ void tile_of(int id, int tiles_m, int tiles_n, int gm, int& tm, int& tn) {
  const int per = gm * tiles_n;
  const int grp = id / per, rem = id - grp * per;
  const int first = grp * gm;
  const int h = min(gm, tiles_m - first);
  tn = rem / h;
  tm = first + (rem - tn * h);
}

// optional per-block cycle stamps (tuning: mmt_gemm_stamps); null in production.  The pointer is read ONCE, at
// kernel entry (GEMM_STAMP_DECL, a scalar load before any operand load): re-reading the global inside the kernel
// compiled to a vector load plus s_waitcnt vmcnt(0), which drained every LDS-DMA load in flight at the stamp after
// the prologue -- one dependent memory round trip per tile in production builds (found round 5)
__device__ unsigned long long* g_gemm_stamps = nullptr;
#define GEMM_STAMP_DECL unsigned long long* const gemm_stamps_ = g_gemm_stamps
#define GEMM_STAMP(k)                                                                      \
  do {                                                                                     \
    if (gemm_stamps_ && threadIdx.x == 0)                                                  \
      gemm_stamps_[(size_t)blockIdx.x * 4 + (k)] = __builtin_amdgcn_s_memtime();           \
  } while (0)


// fused epilogue for one lane's 4 consecutive outputs C[m][n..n+3], with the bias bv of those columns and (fp32
// residual / position epilogues) the residual chunk rr already loaded
template <int EPI, bool SPLIT>
__device__ __forceinline__ void store4v(const GemmGroup& g, const GemmArgs& args, int m, int n, const f32x4& a,
                                        const float4& bv, const float4& rr) {
  const float sc = SPLIT ? g.inv : 1.0f;
  float v[4] = {a[0] * sc + bv.x, a[1] * sc + bv.y, a[2] * sc + bv.z, a[3] * sc + bv.w};
  if (EPI == EPI_GELU_BF16)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf(v[e]);
  if (EPI == EPI_RELU_BF16 || EPI == EPI_RELU_F32)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  const int64_t off = (int64_t)m * g.ldc + n;
  if (EPI == EPI_BF16 || EPI == EPI_GELU_BF16 || EPI == EPI_RELU_BF16) {
    if (SPLIT && g.C_lo) {   // the f16x3 pair of v * out_scale
      uint16_t h[4], l[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) split_h(v[e] * g.out_scale, h[e], l[e]);
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.C) + off) =
          make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.C_lo) + off) =
          make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
    } else {
      bf16_t h[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) h[e] = f2bf(v[e]);
      uint2 o;
      o.x = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      o.y = (uint32_t)h[2] | ((uint32_t)h[3] << 16);
      *reinterpret_cast<uint2*>(static_cast<bf16_t*>(g.C) + off) = o;
    }
  } else {
    float4 o = make_float4(v[0], v[1], v[2], v[3]);
    if (EPI == EPI_RESID_F32)
      o = make_float4(rr.x + v[0], rr.y + v[1], rr.z + v[2], rr.w + v[3]);
    else if (EPI == EPI_POS_F32)
      o = make_float4(v[0] + rr.x, v[1] + rr.y, v[2] + rr.z, v[3] + rr.w);
    *reinterpret_cast<float4*>(static_cast<float*>(g.C) + off) = o;
  }
}

constexpr bool epi_has_r(int e) { return e == EPI_RESID_F32 || e == EPI_POS_F32; }

// the same loading its own operands (one fragment: the split-K reduce)
template <int EPI, bool SPLIT>
__device__ __forceinline__ void store4(const GemmGroup& g, const GemmArgs& args, int m, int n, const f32x4& a) {
  const float4 bv = g.bias ? *reinterpret_cast<const float4*>(g.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
  float4 rr = make_float4(0.f, 0.f, 0.f, 0.f);
  if (EPI == EPI_RESID_F32) rr = *reinterpret_cast<const float4*>(g.R + (int64_t)m * g.ldr + n);
  else if (EPI == EPI_POS_F32) rr = *reinterpret_cast<const float4*>(g.R + (int64_t)(m % args.pos_rows) * g.ldr + n);
  store4v<EPI, SPLIT>(g, args, m, n, a, bv, rr);
}

// epilogue operands of a fragment-shaped store pass, requested together before any is used: the bias of a
// column chunk and the residual / position chunk of (row m, column n) through buffer loads that read zeros for
// an absent bias or a row past M (a load behind a branch, as in store4, is waited for in place: one dependent
// round trip per fragment)
__device__ __forceinline__ float4 epi_bias(const rsrc_t& rB, int n) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rB, (uint32_t)n * 4, 0, 0));
}
template <int EPI>
__device__ __forceinline__ float4 epi_resid(const rsrc_t& rR, const GemmGroup& g, const GemmArgs& args, int m, int n,
                                            int M) {
  if constexpr (!epi_has_r(EPI)) return make_float4(0.f, 0.f, 0.f, 0.f);
  const int row = EPI == EPI_POS_F32 ? m % args.pos_rows : m;
  const uint32_t off = m < M ? (uint32_t)(((int64_t)row * g.ldr + n) * 4) : kBufOob;
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rR, off, 0, 0));
}
template <int EPI>
__device__ __forceinline__ rsrc_t epi_resid_rsrc(const GemmGroup& g, const GemmArgs& args, int M) {
  if constexpr (!epi_has_r(EPI)) return make_rsrc(nullptr, 0);
  const int64_t rows = EPI == EPI_POS_F32 ? args.pos_rows : M;
  return make_rsrc(g.R, rows * g.ldr * 4);
}


// ---- LDS-staged epilogue: bias + activation per lane, the tile goes through LDS ([rows][COLS],
// 16-B chunks XOR-swizzled by row so the fragment-shaped writes are conflict-free), then every lane
// stores 16 contiguous bytes of a row (whole 128-B lines per wave instruction) -- fragment-shaped
// 8-B stores scattered over 16 rows are store-issue bound.  The fp32 epilogues add R while streaming.
constexpr bool epi_is_bf16(int e) { return e == EPI_BF16 || e == EPI_GELU_BF16 || e == EPI_RELU_BF16; }

template <int EPI>
__device__ __forceinline__ void epi_values(const float4& bv, const f32x4& a, float* v) {
  v[0] = a[0] + bv.x;
  v[1] = a[1] + bv.y;
  v[2] = a[2] + bv.z;
  v[3] = a[3] + bv.w;
  if (EPI == EPI_GELU_BF16)   // the LDS epilogue serves the bf16 mode only (split keeps store4 + gelu_erf)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = gelu_erf_bf16out(v[e]);
  if (EPI == EPI_RELU_BF16 || EPI == EPI_RELU_F32)
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
}

template <int EPI, int COLS>
struct LdsTile {
  static constexpr int ESZ = epi_is_bf16(EPI) ? 2 : 4;
  static constexpr int CH = 16 / ESZ;                 // elements per 16-B chunk
  static constexpr int NCH = COLS / CH;               // chunks per row
  // the row's chunk XOR stays inside an aligned group of chunks: the largest power of two dividing NCH, at most 16
  // (a 192-wide bf16 tile has 24 chunks per row: XOR with up to 15 would send chunks 16..23 past the row)
  static constexpr int LOWBIT = NCH & -NCH;
  static constexpr int MASK = (LOWBIT < 16 ? LOWBIT : 16) - 1;
  __device__ static int off(int row, int col) {       // byte offset of (row, col), col % 4 == 0
    return row * COLS * ESZ + ((((col / CH) ^ (row & MASK))) << 4) + (col % CH) * ESZ;
  }
  __device__ static void put(char* lds, int row, int col, const float* v) {
    if (ESZ == 2) {
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(lds + off(row, col)) = o;
    } else {
      *reinterpret_cast<float4*>(lds + off(row, col)) = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  static constexpr bool HAS_R = EPI == EPI_RESID_F32 || EPI == EPI_POS_F32;
  // the residual chunk this thread's drain iteration k adds (issued early: see gemm_kernel)
  __device__ static float4 r_chunk(const GemmGroup& g, const GemmArgs& args, int idx, int m_base, int n0, int M) {
    const int r = idx / NCH, c = idx - r * NCH;
    const int m = m_base + r;
    if (m >= M) return make_float4(0.f, 0.f, 0.f, 0.f);
    const int64_t rr = EPI == EPI_POS_F32 ? (int64_t)(m % args.pos_rows) : (int64_t)m;
    return *reinterpret_cast<const float4*>(g.R + rr * g.ldr + n0 + c * CH);
  }
  // rows [0, ROWS) of the LDS tile -> C rows m_base + r (< M), columns n0 ..; RPRE: the residual
  // chunks were prefetched into rpre[k] (k-th iteration of this thread)
  template <int ROWS, int NT, int RPRE = 0>
  __device__ static void drain(const char* lds, const GemmGroup& g, const GemmArgs& args, int m_base, int n0, int M,
                               const float4* rpre = nullptr) {
#pragma unroll
    for (int k = 0; k < (ROWS * NCH + NT - 1) / NT; ++k) {
      const int idx = threadIdx.x + k * NT;
      if (idx >= ROWS * NCH) break;
      const int r = idx / NCH, c = idx - r * NCH;
      const int m = m_base + r;
      if (m >= M) continue;
      const int n = n0 + c * CH;
      const uint4 d = *reinterpret_cast<const uint4*>(lds + r * COLS * ESZ + ((c ^ (r & MASK)) << 4));
      if (ESZ == 2) {
        *reinterpret_cast<uint4*>(static_cast<bf16_t*>(g.C) + (int64_t)m * g.ldc + n) = d;
      } else {
        float4 o = make_float4(__uint_as_float(d.x), __uint_as_float(d.y), __uint_as_float(d.z), __uint_as_float(d.w));
        if constexpr (HAS_R) {
          const float4 R = RPRE ? rpre[k] : r_chunk(g, args, idx, m_base, n0, M);
          o = make_float4(R.x + o.x, R.y + o.y, R.z + o.z, R.w + o.w);
        }
        *reinterpret_cast<float4*>(static_cast<float*>(g.C) + (int64_t)m * g.ldc + n) = o;
      }
    }
  }
};

// scheduling groups: NR times {one LDS read, K MFMAs}
template <int NR, int K>
__device__ __forceinline__ void sched_interleave() {
  if constexpr (NR > 0) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, K, 0);
    sched_interleave<NR - 1, K>();
  }
}
// vmcnt(min(n, MAXN)) for a wave-uniform n: a scalar branch to an immediate
template <int N>
__device__ __forceinline__ void vm_wait_n() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int MAXN>
__device__ __forceinline__ void vm_wait_rt(int n) {   // n wave-uniform; scalar branch to an immediate
  if constexpr (MAXN > 0) {
    if (n >= MAXN) return vm_wait_n<MAXN>();
    return vm_wait_rt<MAXN - 1>(n);
  } else {
    vm_wait_n<0>();
  }
}

template <int BM, int BN, int WMW, int WNW, int EPI, int AM, bool SPLIT, int STAGES, int BK = 64>
__global__ __launch_bounds__(WMW* WNW * 64) void gemm_kernel(const GemmArgs args) {
  static_assert(BK == 64 || (BK == 32 && AM == A_DENSE), "BK 32: dense A only");
  using T = Tile<BM, BN, WMW, WNW, SPLIT, STAGES, BK>;
  __shared__ __attribute__((aligned(16))) bf16_t smem[T::NSTAGE * T::STAGE];
  GEMM_STAMP_DECL;

  const GemmGroup& g = args.g[blockIdx.z];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = args.N / BN, ntiles = tiles_m * tiles_n;
  // XCD-aware remap (bijective): blocks b, b+8, ... (one XCD) take a contiguous logical range
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  const int q = ntiles >> 3, r8 = ntiles & 7;
  const int id = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + j;
  int tm, tn;
  tile_of(id, tiles_m, tiles_n, args.gm, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  GEMM_STAMP(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  // ---- epilogue operands requested now, so their latency hides under the main loop: the bias of
  // the lane's columns and (residual epilogues) the residual chunks of the drain
  using LT = LdsTile<EPI, BN>;
  constexpr bool LDS_EPI = EPI != EPI_PARTIAL && !SPLIT && BM * BN * LT::ESZ <= T::NSTAGE * T::STAGE * 2;
  constexpr int RPRE = (LDS_EPI && LT::HAS_R && (BM * LT::NCH) % T::NT == 0) ? BM * LT::NCH / T::NT : 0;
  float4 bpre[T::FN];
#pragma unroll
  for (int jj = 0; jj < T::FN; ++jj) {
    const int col = n0 + wn * T::WN + jj * 16 + (lane >> 4) * 4;
    bpre[jj] = (LDS_EPI && g.bias) ? *reinterpret_cast<const float4*>(g.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float4 rpre[RPRE > 0 ? RPRE : 1];
  if constexpr (RPRE > 0) {
#pragma unroll
    for (int k = 0; k < RPRE; ++k) rpre[k] = LT::r_chunk(g, args, tid + k * T::NT, m0, n0, M);
  }
  // the fragment-shaped epilogue's bias chunks (split mode), requested now through branch-free raw buffer loads: they
  // are the oldest loads in the queue, so the main loop's first counted wait retires them and the epilogue starts
  // without a dependent round trip (one-sequence qkv / fc1: ~1 us of a ~10 us launch)
  constexpr bool EARLY_BIAS = !LDS_EPI && EPI != EPI_PARTIAL;
  float4 bq[EARLY_BIAS ? T::FN : 1];
  if constexpr (EARLY_BIAS) {
    const rsrc_t rB = make_rsrc(g.bias, g.bias ? (int64_t)args.N * 4 : 0);
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj) bq[jj] = epi_bias(rB, n0 + wn * T::WN + jj * 16 + (lane >> 4) * 4);
  }
  // split fp32 outputs (fc2 / proj residual updates, the patch embedding, the head's last conv): the tile goes through
  // the LDS and leaves as whole 16-B row chunks, the residual chunks of that drain requested here (raw buffer loads,
  // rows past M read zeros) so their round trip hides under the main loop instead of opening the epilogue
  constexpr bool SF32 = SPLIT && (EPI == EPI_RESID_F32 || EPI == EPI_F32 || EPI == EPI_POS_F32 || EPI == EPI_RELU_F32) &&
                        BM * BN * 4 <= T::NSTAGE * T::STAGE * 2 && (BM * (BN / 4)) % T::NT == 0;
  constexpr int SF_N = SF32 ? BM * (BN / 4) / T::NT : 1;   // drain chunks per thread
  constexpr bool SF_R = SF32 && epi_has_r(EPI);
  // (prefetched up to 8 chunks per thread: the 12 of a 128 x 192 tile held over the main loop spill)
  constexpr bool SF_RPRE = SF_R && SF_N <= 8;
  u32x4 rsf[SF_RPRE ? SF_N : 1];
  if constexpr (SF_RPRE) {
    const rsrc_t rR = epi_resid_rsrc<EPI>(g, args, M);
#pragma unroll
    for (int k = 0; k < SF_N; ++k) {
      const int idx = tid + k * T::NT, r = idx / (BN / 4), c = idx - r * (BN / 4), m = m0 + r;
      const int row = EPI == EPI_POS_F32 ? m % args.pos_rows : m;
      const uint32_t o = m < M ? (uint32_t)(((int64_t)row * g.ldr + n0 + 4 * c) * 4) : kBufOob;
      rsf[k] = __builtin_amdgcn_raw_buffer_load_b128(rR, o, 0, 0);
    }
  }

  // ---- loads: buffer_load ... lds with per-lane VGPR offsets fixed over K and the K advance in the
  // SGPR soffset; rows past M fall outside the A resource and read as zero.  Row block i of the
  // tile (rows [i*RPI, (i+1)*RPI)) lies in one operand region, known at compile time.
  constexpr int GPW = T::GROUPS / T::NW;
  constexpr int RPI = T::NW * T::RPW;
  static_assert(BM % RPI == 0 && BN % RPI == 0, "row blocks must not straddle operands");
  // XOR swizzle of the 16-B source chunk so it lands at its swizzled LDS position (swzk)
  const int chunk = (BK == 64 ? ((lane & 7) ^ (lane >> 3)) : ((lane & 3) ^ ((lane >> 4) & 2))) * 16;
  const int64_t a_rows = AM == A_DENSE ? (int64_t)(M - m0) : (int64_t)M;
  const rsrc_t rA = make_rsrc(AM == A_DENSE ? g.A + (int64_t)m0 * g.lda : g.A, a_rows * g.lda * 2);
  const rsrc_t rAl = SPLIT ? make_rsrc(AM == A_DENSE ? g.A_lo + (int64_t)m0 * g.lda : g.A_lo, a_rows * g.lda * 2) : rA;
  const rsrc_t rW = make_rsrc(g.W + (int64_t)n0 * g.ldw, (int64_t)BN * g.ldw * 2);
  const rsrc_t rWl = SPLIT ? make_rsrc(g.W_lo + (int64_t)n0 * g.ldw, (int64_t)BN * g.ldw * 2) : rW;
  uint32_t voff[GPW];
  int conv_b[GPW], conv_y[GPW], conv_x[GPW];   // A_CONV3: map index, pixel of the output row (-1: tail)
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int r0 = i * RPI;                              // compile-time after unrolling
    const int row = r0 + wave * T::RPW + lane / (BK / 8);
    conv_b[i] = -1;
    conv_y[i] = conv_x[i] = 0;
    if (r0 < T::AROWS) {
      const int lr = (SPLIT && r0 >= BM) ? row - BM : row;
      voff[i] = (uint32_t)(lr * g.lda * 2 + chunk);
      if (AM == A_CONV3) {
        const int m = m0 + lr;
        if (m < M) {
          const int hw = args.conv_hw, plane = hw * hw;
          conv_b[i] = m / plane;
          const int pp = m - conv_b[i] * plane;
          conv_y[i] = pp / hw;
          conv_x[i] = pp - conv_y[i] * hw;
        }
      }
    } else {
      const int wr = row - T::AROWS;
      const int lr = (SPLIT && wr >= BN) ? wr - BN : wr;
      voff[i] = (uint32_t)(lr * g.ldw * 2 + chunk);
    }
  }

  auto issue = [&](int kt, int stage) {
    const int k0 = kt * BK;
    bf16_t* sbase = smem + stage * T::STAGE;
    int tap = 0, ch = 0, dy = 0, dx = 0;
    if (AM == A_CONV3) {
      tap = k0 / args.conv_cin;
      ch = k0 - tap * args.conv_cin;
      dy = tap / 3 - 1;
      dx = tap % 3 - 1;
    }
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int r0 = i * RPI;
      lptr_t dst = (lptr_t)(sbase + (r0 + wave * T::RPW) * BK);
      if (r0 < T::AROWS) {
        const rsrc_t rs = (SPLIT && r0 >= BM) ? rAl : rA;
        if (AM == A_CONV3) {
          const int hw = args.conv_hw;
          const int y = conv_y[i] + dy, xx = conv_x[i] + dx;
          const bool ok = conv_b[i] >= 0 && y >= 0 && y < hw && xx >= 0 && xx < hw;
          const uint32_t vo = ok ? (uint32_t)((((conv_b[i] * hw + y) * hw + xx) * g.lda + ch) * 2 + chunk)
                                 : 0x80000000u;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, vo, 0, 0, 0);
        } else {
          const uint32_t vo = voff[i];   // (a subscript directly in the builtin drops the host stub)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, vo, k0 * 2, 0, 0);
        }
      } else {
        const rsrc_t rs = (SPLIT && r0 >= T::AROWS + BN) ? rWl : rW;
        const uint32_t vo = voff[i];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, dst, 16, vo, k0 * 2, 0, 0);
      }
    }
  };

  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one 32-deep K-step, double-buffered in registers: the next step's ds_reads are in flight
  // while this step's MFMAs issue (a barrier-separated read-then-multiply step would leave the MFMA pipe idle
  // for the whole LDS read of every step, all waves phase-locked by the barrier)
  struct Frags {
    bf16x8 ah[T::FM], bh[T::FN];
    bf16x8 al[SPLIT ? T::FM : 1], bl[SPLIT ? T::FN : 1];
  };
  auto read = [&](int stage, int s, Frags& f) {
    const bf16_t* S = smem + stage * T::STAGE;
    const int c = 4 * s + (lane >> 4);
#pragma unroll
    for (int i = 0; i < T::FM; ++i) {
      const int row = wm * T::WM + i * 16 + (lane & 15);
      f.ah[i] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(row, c));
      if (SPLIT) f.al[i] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(BM + row, c));
    }
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj) {
      const int row = T::AROWS + wn * T::WN + jj * 16 + (lane & 15);
      f.bh[jj] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(row, c));
      if (SPLIT) f.bl[jj] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(BN + row, c));
    }
  };
  auto mma = [&](const Frags& f) {
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        acc[i][jj] = mfma16<SPLIT>(f.bh[jj], f.ah[i], acc[i][jj]);
        if (SPLIT) {
          acc[i][jj] = mfma16<SPLIT>(f.bl[jj], f.ah[i], acc[i][jj]);
          acc[i][jj] = mfma16<SPLIT>(f.bh[jj], f.al[i], acc[i][jj]);
        }
      }
  };

  // Split-K (EPI_PARTIAL): workgroup row blockIdx.y takes K-tiles [kbeg, kend) and stores raw sums.
  const int nk_all = K / BK;
  const int kbeg = EPI == EPI_PARTIAL ? (int)((int64_t)blockIdx.y * nk_all / args.ksplit) : 0;
  const int kend = EPI == EPI_PARTIAL ? (int)((int64_t)(blockIdx.y + 1) * nk_all / args.ksplit) : nk_all;
  const int nk = kend - kbeg;
  constexpr int NS = T::NSTAGE, SPK = BK / 32;
  // Register-pipelined loop (DBUF) where the LDS ring already limits the CU to one workgroup (> 80 KB) and a
  // step has enough MFMAs to cover its reads: the second fragment set (146 VGPRs for the 128 x 128 f16x3 tile,
  // 98 without) would otherwise halve the workgroups per CU (proj, 2-stage 32-deep: 47 -> 55 us)
  constexpr int FRAG_REGS = (T::FM + T::FN) * (SPLIT ? 2 : 1) * 4;
#ifndef GEMM_DBUF_ALL
#define GEMM_DBUF_ALL 0
#endif
  constexpr bool DBUF = (T::NSTAGE * T::STAGE * 2 > 80 * 1024 || (GEMM_DBUF_ALL && SPLIT)) && T::FM * T::FN >= 4 &&
                        T::FM * T::FN * 4 + 2 * FRAG_REGS <= 192;
  if constexpr (DBUF) {
    // One 32-deep step at a time (BK / 32 steps per K-tile).  At the last step of K-tile kt the wave retires
    // tile kt + 1's loads (counted vmcnt: younger tiles stay in flight) and its own reads of tile kt
    // (lgkmcnt), and meets the others at a barrier (raw s_barrier: __syncthreads() would drain every in-flight
    // LDS-DMA with vmcnt(0)); tile kt's stage is then free and takes tile kt + NSTAGE.  The next step's
    // fragments are read into the other register set while this step's MFMAs issue.
    for (int p = 0; p < NS; ++p)
      if (p < nk) issue(kbeg + p, p);
    vm_wait_rt<GPW*(NS - 1)>(GPW * (min(NS, nk) - 1));   // tile 0 landed (this wave's part)
    __builtin_amdgcn_s_barrier();
    GEMM_STAMP(1);
    const int nsteps = nk * SPK;
    int stage = 0;   // stage of the K-tile of the current step
    auto boundary = [&](int kt) {
      // loads issued after tile kt + 1: tiles kt + 2 .. min(kt + NS - 1, nk - 1)
      vm_wait_rt<GPW*(NS - 2 > 0 ? NS - 2 : 0)>(GPW * (min(kt + NS - 1, nk - 1) - (kt + 1)));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + NS < nk) issue(kbeg + kt + NS, stage);
      stage = stage + 1 == NS ? 0 : stage + 1;
    };
    Frags f0, f1;
    if (nk > 0) read(0, 0, f0);
    // The next fragments are read unconditionally (after the last step: a harmless re-read of the current
    // stage), so no branch separates them from the MFMAs.  The scheduler is told the order: one MFMA of cur
    // (its lgkmcnt wait sits before it, while no read of nxt is pending), then each read of nxt followed by a
    // few more MFMAs -- left alone it sinks the reads below the MFMAs, into cur's registers.
    auto step = [&](int t, const Frags& cur, Frags& nxt) {
      const int s = SPK == 1 ? 0 : (t & 1);
      if (s == SPK - 1 && t + 1 < nsteps) boundary(t / SPK);
      mma(cur);
      read(stage, s == SPK - 1 ? 0 : s + 1, nxt);
      constexpr int NR = (T::FM + T::FN) * (SPLIT ? 2 : 1), NM = T::FM * T::FN * (SPLIT ? 3 : 1);
      constexpr int KPER = (NM - 1) / NR > 0 ? (NM - 1) / NR : 1;
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      sched_interleave<NR, KPER>();
    };
    for (int t = 0; t < nsteps; t += 2) {
      step(t, f0, f1);
      if (t + 1 < nsteps) step(t + 1, f1, f0);
    }
  } else {
    // tiles kt+1 .. kt+NSTAGE-1 are in flight while tile kt is read and multiplied; a tile is read only after the
    // issuing waves' counted vmcnt retired it AND a barrier
    constexpr int D = NS - 1;
    for (int p = 0; p < D; ++p)
      if (p < nk) issue(kbeg + p, p);
    // tile 0 landed: the min(D, nk) - 1 tiles issued after it may stay in flight (a K shorter than the ring issues
    // fewer; until round 5 a stamp's hidden vmcnt(0) covered the nk < D case this count used to get wrong)
    vm_wait_rt<GPW*(D > 1 ? D - 1 : 0)>(GPW * (min(D, nk) - 1));
    __builtin_amdgcn_s_barrier();
    GEMM_STAMP(1);
    int stage = 0;
    Frags f;
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = kt + D;
      if (ahead < nk) issue(kbeg + ahead, ahead % NS);
#pragma unroll
      for (int s = 0; s < SPK; ++s) {
        read(stage, s, f);
        mma(f);
      }
      stage = stage + 1 == NS ? 0 : stage + 1;
      // retire tile kt+1: the loads issued after it (tiles kt+2 .. min(kt+D, nk-1)) may stay in flight
      const int after = min(kt + D, nk - 1) - (kt + 1);
      if (D > 1 && after >= D - 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GPW * (D - 1)) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  GEMM_STAMP(2);
  // ---- epilogue: lane owns C[m][n..n+3]
  if constexpr (EPI == EPI_PARTIAL) {   // raw partial sums -> workspace slice (blockIdx.z, blockIdx.y)
    GemmGroup gp{};
    gp.C = args.ws + ((int64_t)blockIdx.z * args.ksplit + blockIdx.y) * (int64_t)M * args.N;
    gp.ldc = args.N;
    char* lds = reinterpret_cast<char*>(smem);
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const int col = wn * T::WN + jj * 16 + (lane >> 4) * 4;
        const float v[4] = {acc[i][jj][0], acc[i][jj][1], acc[i][jj][2], acc[i][jj][3]};
        LT::put(lds, wm * T::WM + i * 16 + (lane & 15), col, v);
      }
    __syncthreads();
    LT::template drain<BM, T::NT>(lds, gp, args, m0, n0, M);
  } else if constexpr (LDS_EPI) {
    char* lds = reinterpret_cast<char*>(smem);
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const int col = wn * T::WN + jj * 16 + (lane >> 4) * 4;
        float v[4];
        epi_values<EPI>(bpre[jj], acc[i][jj], v);
        LT::put(lds, wm * T::WM + i * 16 + (lane & 15), col, v);
      }
    __syncthreads();
    LT::template drain<BM, T::NT, RPRE>(lds, g, args, m0, n0, M, rpre);
  } else if constexpr (SF32) {
    using LF = LdsTile<EPI_F32, BN>;   // fp32 [BM][BN], 16-B chunks XOR-swizzled by row
    char* const lds = reinterpret_cast<char*>(smem);
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const f32x4& a = acc[i][jj];
        const float4 bv = bq[jj];
        float v[4] = {a[0] * g.inv + bv.x, a[1] * g.inv + bv.y, a[2] * g.inv + bv.z, a[3] * g.inv + bv.w};
        if (EPI == EPI_RELU_F32)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        LF::put(lds, wm * T::WM + i * 16 + (lane & 15), wn * T::WN + jj * 16 + (lane >> 4) * 4, v);
      }
    __syncthreads();
    const int rows = max(0, min(BM, M - m0));
    const rsrc_t rC = make_rsrc(static_cast<float*>(g.C) + (int64_t)m0 * g.ldc, (int64_t)rows * g.ldc * 4);
#pragma unroll
    for (int k = 0; k < SF_N; ++k) {
      const int idx = tid + k * T::NT, r = idx / (BN / 4), c = idx - r * (BN / 4);
      f32x4 v = *reinterpret_cast<const f32x4*>(lds + r * BN * 4 + ((c ^ (r & LF::MASK)) << 4));
      if constexpr (SF_RPRE) {
        v = __builtin_bit_cast(f32x4, rsf[k]) + v;   // R + (acc * inv + bias), as store4v
      } else if constexpr (SF_R) {
        const rsrc_t rR = epi_resid_rsrc<EPI>(g, args, M);
        const int m = m0 + r, row = EPI == EPI_POS_F32 ? m % args.pos_rows : m;
        const uint32_t o = m < M ? (uint32_t)(((int64_t)row * g.ldr + n0 + 4 * c) * 4) : kBufOob;
        v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rR, o, 0, 0)) + v;
      }
      const uint32_t go = r < rows ? (uint32_t)(((int64_t)r * g.ldc + n0 + 4 * c) * 4) : kBufOob;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rC, go, 0, 0);
    }
  } else if constexpr (SPLIT && epi_is_bf16(EPI) && 2 * BM * BN * 2 <= T::NSTAGE * T::STAGE * 2) {
    // split 16-bit outputs (one-sequence qkv / fc1, the head convs): the tile's hi and lo planes staged in the LDS,
    // then whole 16-B row chunks per lane (fragment-shaped stores write 16 rows x 32 B per wave-instruction; the
    // staged drain, whole 128-B lines: the 256 x 256 kernel's epilogue 35k -> see gemm256s_kernel).  Same bits.
    using LT = LdsTile<EPI_BF16, BN>;
    char* const planeH = reinterpret_cast<char*>(smem);
    char* const planeL = planeH + BM * BN * 2;
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const int row = wm * T::WM + i * 16 + (lane & 15);
        const int col = wn * T::WN + jj * 16 + (lane >> 4) * 4;
        const f32x4& a = acc[i][jj];
        const float4 bv = bq[jj];
        float v[4] = {a[0] * g.inv + bv.x, a[1] * g.inv + bv.y, a[2] * g.inv + bv.z, a[3] * g.inv + bv.w};
        if (EPI == EPI_GELU_BF16) {
          f32x2 g0 = {v[0], v[1]}, g1 = {v[2], v[3]};
          gelu_erf4(g0, g1);
          v[0] = g0.x;
          v[1] = g0.y;
          v[2] = g1.x;
          v[3] = g1.y;
        }
        if (EPI == EPI_RELU_BF16)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        uint16_t hh[4], ll[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) split_h(v[e] * g.out_scale, hh[e], ll[e]);
        const int o = LT::off(row, col);
        *reinterpret_cast<uint2*>(planeH + o) =
            make_uint2((uint32_t)hh[0] | ((uint32_t)hh[1] << 16), (uint32_t)hh[2] | ((uint32_t)hh[3] << 16));
        *reinterpret_cast<uint2*>(planeL + o) =
            make_uint2((uint32_t)ll[0] | ((uint32_t)ll[1] << 16), (uint32_t)ll[2] | ((uint32_t)ll[3] << 16));
      }
    __syncthreads();
    const int rows = max(0, min(BM, M - m0));
    const rsrc_t rC = make_rsrc(static_cast<bf16_t*>(g.C) + (int64_t)m0 * g.ldc, (int64_t)rows * g.ldc * 2);
    const rsrc_t rCl = make_rsrc(static_cast<bf16_t*>(g.C_lo) + (int64_t)m0 * g.ldc, (int64_t)rows * g.ldc * 2);
    static_assert((BM * LT::NCH) % T::NT == 0, "uniform drain");
#pragma unroll
    for (int it = 0; it < BM * LT::NCH / T::NT; ++it) {
      const int idx = tid + it * T::NT, r = idx / LT::NCH, c = idx - r * LT::NCH;
      const int lo = r * BN * 2 + ((c ^ (r & LT::MASK)) << 4);
      const uint32_t go = r < rows ? (uint32_t)(((int64_t)r * g.ldc + n0 + c * 8) * 2) : kBufOob;
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(planeH + lo), rC, go, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(planeL + lo), rCl, go, 0, 0);
    }
  } else {
    const rsrc_t rR = epi_resid_rsrc<EPI>(g, args, M);
    // (the residual chunks of the 32-fragment tiles -- 256 x 256 tuning configs -- would need 128 more VGPRs:
    // those keep one fragment's residual at a time)
    constexpr bool RPRE_ALL = epi_has_r(EPI) && T::FM * T::FN <= 16;
    float4 rq[RPRE_ALL ? T::FM : 1][RPRE_ALL ? T::FN : 1];
    if constexpr (RPRE_ALL) {
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int jj = 0; jj < T::FN; ++jj)
          rq[i][jj] = epi_resid<EPI>(rR, g, args, m0 + wm * T::WM + i * 16 + (lane & 15),
                                     n0 + wn * T::WN + jj * 16 + (lane >> 4) * 4, M);
    }
#pragma unroll
    for (int i = 0; i < T::FM; ++i) {
      const int m = m0 + wm * T::WM + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const int n = n0 + wn * T::WN + jj * 16 + (lane >> 4) * 4;
        if constexpr (RPRE_ALL)
          store4v<EPI, SPLIT>(g, args, m, n, acc[i][jj], bq[jj], rq[i][jj]);
        else
          store4v<EPI, SPLIT>(g, args, m, n, acc[i][jj], bq[jj], epi_resid<EPI>(rR, g, args, m, n, M));
      }
    }
  }
  GEMM_STAMP(3);
}

// ---------------------------------------------------------------------------------------------------
// Persistent variant for the bf16-output GEMMs of the path (qkv, fc1): a grid of two workgroups per
// CU walks the output tiles, and the first K-tile of a workgroup's NEXT output tile is loaded while
// the current one is finishing (issued at the last K-step into the free LDS stage), so the load
// latency that opens every tile of gemm_kernel (its "prologue") hides under the previous tile's last
// MFMAs and epilogue.  The epilogue stages C through the LDS stage just consumed; a tile's bias is
// requested with its second K-tile.  Dense A only (no conv gather), no split mode.
template <int BM, int BN, int WMW, int WNW, int EPI>
__global__ __launch_bounds__(WMW* WNW * 64) void gemm_persist_kernel(const GemmArgs args) {
  using T = Tile<BM, BN, WMW, WNW, false, 2>;
  using LT = LdsTile<EPI, BN>;
  static_assert(LT::ESZ == 2 && BM * BN * 2 <= T::STAGE * 2, "C tile must fit one LDS stage");
  static_assert((BM * LT::NCH) % T::NT == 0, "drain iterations must be uniform");
  __shared__ __attribute__((aligned(16))) bf16_t smem[2 * T::STAGE];
  const GemmGroup& g = args.g[0];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = args.N / BN, ntiles = tiles_m * tiles_n;
  // XCD-aware: the workgroups of XCD x (= b % 8) share the contiguous logical range
  // [x * per, (x + 1) * per) of the super-tile order and take its tiles round-robin
  const int b = blockIdx.x, x = b & 7, j = b >> 3, nb8 = gridDim.x >> 3;
  const int per = (ntiles + 7) >> 3;
  const int lo = x * per, hi = min(ntiles, lo + per);
  int id = lo + j;
  if (id >= hi) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  constexpr int GPW = T::GROUPS / T::NW;
  constexpr int RPI = T::NW * 8;
  constexpr int NST = BM * LT::NCH / T::NT;   // global stores per thread in a full tile's drain
  const int chunk = ((lane & 7) ^ (lane >> 3)) * 16;
  uint32_t voff[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int r0 = i * RPI;
    const int row = r0 + wave * 8 + (lane >> 3);
    voff[i] = r0 < BM ? (uint32_t)(row * g.lda * 2 + chunk) : (uint32_t)((row - BM) * g.ldw * 2 + chunk);
  }
  const int nk = K / 64;

  // tile geometry and buffer resources (plain locals: the rsrc type cannot live in a struct on the host
  // side of the compile, and the builtin's operands are copied to locals, see gemm_kernel)
  auto tile_geom = [&](int tid_, int& m0, int& n0) {
    int tm, tn;
    tile_of(tid_, tiles_m, tiles_n, args.gm, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  auto issue = [&](int m0, int n0, int kt, int stage) {
    const rsrc_t rA = make_rsrc(g.A + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
    const rsrc_t rW = make_rsrc(g.W + (int64_t)n0 * g.ldw, (int64_t)BN * g.ldw * 2);
    bf16_t* sbase = smem + stage * T::STAGE;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int r0 = i * RPI;
      lptr_t dst = (lptr_t)(sbase + (r0 + wave * 8) * 64);
      const uint32_t vo = voff[i];
      const int so = kt * 128;
      if (r0 < BM) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, vo, so, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, dst, 16, vo, so, 0, 0);
    }
  };
  auto load_bias = [&](int n0, float4* bp) {
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj) {
      const int col = n0 + wn * T::WN + jj * 16 + (lane >> 4) * 4;
      bp[jj] = g.bias ? *reinterpret_cast<const float4*>(g.bias + col) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };

  f32x4 acc[T::FM][T::FN];
  auto compute = [&](int stage) {
    const bf16_t* S = smem + stage * T::STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = 4 * s + (lane >> 4);
      bf16x8 ah[T::FM], bh[T::FN];
#pragma unroll
      for (int i = 0; i < T::FM; ++i) ah[i] = *reinterpret_cast<const bf16x8*>(S + swz(wm * T::WM + i * 16 + (lane & 15), c));
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj)
        bh[jj] = *reinterpret_cast<const bf16x8*>(S + swz(BM + wn * T::WN + jj * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int jj = 0; jj < T::FN; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[jj], ah[i], acc[i][jj], 0, 0, 0);
    }
  };

  int cm0, cn0;
  tile_geom(id, cm0, cn0);
  float4 bcur[T::FN];
  issue(cm0, cn0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int stage = 0;
  for (;;) {
    const int nid = id + nb8;
    const bool has_next = nid < hi;
    int nm0 = cm0, nn0 = cn0;
    load_bias(cn0, bcur);   // lands with the K-tile loads of the first step; used in the epilogue
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      const bool last = kt + 1 == nk;
      if (!last) {
        issue(cm0, cn0, kt + 1, stage ^ 1);
      } else if (has_next) {   // the next tile's first K-tile, into the stage freed by K-tile kt-1
        tile_geom(nid, nm0, nn0);
        issue(nm0, nn0, 0, stage ^ 1);
      }
      compute(stage);
      if (!last) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        stage ^= 1;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    // epilogue through the stage just consumed (every wave passed the barrier after reading it)
    char* lds = reinterpret_cast<char*>(smem + stage * T::STAGE);
#pragma unroll
    for (int i = 0; i < T::FM; ++i)
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj) {
        const int col = wn * T::WN + jj * 16 + (lane >> 4) * 4;
        float v[4];
        epi_values<EPI>(bcur[jj], acc[i][jj], v);
        LT::put(lds, wm * T::WM + i * 16 + (lane & 15), col, v);
      }
    // LDS visibility of the C tile without __syncthreads(): its fence would also wait (vmcnt(0)) for
    // the next tile's K-tile in flight
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    LT::template drain<BM, T::NT>(lds, g, args, cm0, cn0, M);
    if (!has_next) break;
    // every wave has read its C rows out of LDS before the next tile's loads land in this stage;
    // the next tile's first K-tile (issued before the drain's stores) must have landed: with a full
    // tile exactly NST stores per thread follow it in the in-order vmcnt queue (M-tail tiles: all)
    if (cm0 + BM <= M) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    stage ^= 1;
    cm0 = nm0;
    cn0 = nn0;
    id = nid;
  }
}

// ---------------------------------------------------------------------------------------------------
// Persistent ring GEMM for the bf16-output GEMMs (qkv, fc1), no LDS in the epilogue.
//
// A grid of up to two workgroups per CU walks its XCD's tile range (as gemm_persist_kernel), and the
// K-tiles of ALL of a workgroup's output tiles form one stream s = t * nk + kt through an NS-deep LDS
// ring: step s + NS - 1 is issued while step s is multiplied, across tile boundaries, so the loads of
// the next tile are in flight while the current tile's epilogue runs (a tile boundary costs no
// prologue).  The epilogue never touches LDS (the ring keeps streaming): bias + activation per lane,
// then a 4 x 4 transpose of 8-byte bf16 quads across the wave's four 16-lane groups
// (v_permlane32_swap + v_permlane16_swap) so a lane holds 16 consecutive columns of one row, and
// 16-B buffer stores (rows past M fall outside the C resource and are dropped, so every tile issues
// the same number of stores).  vmcnt bookkeeping: a step's wait lets the younger ring loads stay in
// flight and, within NS - 1 steps after an epilogue, that epilogue's stores and the next tile's bias
// loads (issued after it) as well.


template <int BM, int BN, int WMW, int WNW, int EPI, int NS, int BK>
__global__ __launch_bounds__(WMW* WNW * 64) void gemm_ring_kernel(const GemmArgs args) {
  using T = Tile<BM, BN, WMW, WNW, false, NS, BK>;
  static_assert(epi_is_bf16(EPI) && T::FN % 4 == 0, "bf16 outputs, wave tiles of 64-column multiples");
  constexpr int D = NS - 1;
  constexpr int GPW = T::GROUPS / T::NW;
  constexpr int RPI = T::NW * T::RPW;
  static_assert(BM % RPI == 0 && BN % RPI == 0, "row blocks must not straddle operands");
  constexpr int NSTORE = T::FM * (T::FN / 4) * 2;   // 16-B stores per lane per tile
  constexpr int NBIAS = 1;                          // bias LDS-DMA pieces per wave per tile
  static_assert(BN <= 256, "one 1-KB bias piece per tile");
  __shared__ __attribute__((aligned(16))) bf16_t smem[NS * T::STAGE];
  __shared__ __attribute__((aligned(16))) float sbias[2][256];   // bias of tile t in slot t & 1

  const GemmGroup& g = args.g[0];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = args.N / BN, ntiles = tiles_m * tiles_n;
  const int b = blockIdx.x, x = b & 7, j = b >> 3, nb8 = gridDim.x >> 3;
  const int per = (ntiles + 7) >> 3;
  const int lo = x * per, hi = min(ntiles, lo + per);
  const int first = lo + j;
  if (first >= hi) return;
  const int nt = (hi - first + nb8 - 1) / nb8;
  const int nk = K / BK, G = nt * nk;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  const int chunk = (BK == 64 ? ((lane & 7) ^ (lane >> 3)) : ((lane & 3) ^ ((lane >> 4) & 2))) * 16;
  uint32_t voff[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int r0 = i * RPI;
    const int row = r0 + wave * T::RPW + lane / (BK / 8);
    voff[i] = r0 < BM ? (uint32_t)(row * g.lda * 2 + chunk) : (uint32_t)((row - BM) * g.ldw * 2 + chunk);
  }
  auto geom = [&](int t, int& m0, int& n0) {
    int tm, tn;
    tile_of(first + t * nb8, tiles_m, tiles_n, args.gm, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  // issue cursor: the next K-step to load (tile is_t, K-tile is_kt, ring slot is_slot); the tile's
  // geometry and buffer resources are recomputed once per tile, not per step
  int is_t = 0, is_kt = 0, is_slot = 0;
  int im0, in0;
  geom(0, im0, in0);
  rsrc_t rA = make_rsrc(g.A + (int64_t)im0 * g.lda, (int64_t)(M - im0) * g.lda * 2);
  rsrc_t rW = make_rsrc(g.W + (int64_t)in0 * g.ldw, (int64_t)BN * g.ldw * 2);
  auto issue_next = [&]() {
    bf16_t* sbase = smem + is_slot * T::STAGE;
    const int so = is_kt * BK * 2;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int r0 = i * RPI;
      lptr_t dst = (lptr_t)(sbase + (r0 + wave * T::RPW) * BK);
      const uint32_t vo = voff[i];
      if (r0 < BM) __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, dst, 16, vo, so, 0, 0);
      else __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, dst, 16, vo, so, 0, 0);
    }
    is_slot = is_slot + 1 == NS ? 0 : is_slot + 1;
    if (++is_kt == nk) {
      is_kt = 0;
      if (++is_t < nt) {
        geom(is_t, im0, in0);
        rA = make_rsrc(g.A + (int64_t)im0 * g.lda, (int64_t)(M - im0) * g.lda * 2);
        rW = make_rsrc(g.W + (int64_t)in0 * g.ldw, (int64_t)BN * g.ldw * 2);
      }
    }
  };
  // the tile's bias goes to LDS by DMA (every wave issues the same 1-KB piece, so each wave's own vmcnt
  // covers the bytes it reads); no VGPR-destination load exists in the kernel, so the compiler inserts
  // no vmcnt wait of its own
  auto load_bias = [&](int n0, int slot) {
    const rsrc_t rB = make_rsrc(g.bias ? g.bias + n0 : nullptr, g.bias ? BN * 4 : 0);
    const uint32_t vo = (uint32_t)((lane % (BN / 4)) * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lptr_t)&sbias[slot][0], 16, vo, 0, 0, 0);
  };
  f32x4 acc[T::FM][T::FN];
#pragma unroll
  for (int i = 0; i < T::FM; ++i)
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int slot) {
    const bf16_t* S = smem + slot * T::STAGE;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      const int c = 4 * s + (lane >> 4);
      bf16x8 ah[T::FM], bh[T::FN];
#pragma unroll
      for (int i = 0; i < T::FM; ++i) ah[i] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(wm * T::WM + i * 16 + (lane & 15), c));
#pragma unroll
      for (int jj = 0; jj < T::FN; ++jj)
        bh[jj] = *reinterpret_cast<const bf16x8*>(S + swzk<BK>(BM + wn * T::WN + jj * 16 + (lane & 15), c));
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int jj = 0; jj < T::FN; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[jj], ah[i], acc[i][jj], 0, 0, 0);
    }
  };
  auto epilogue = [&](int m0, int n0, int slot) {
    float4 bias[T::FN];
#pragma unroll
    for (int jj = 0; jj < T::FN; ++jj)
      bias[jj] = *reinterpret_cast<const float4*>(&sbias[slot][wn * T::WN + jj * 16 + (lane >> 4) * 4]);
    const rsrc_t rC = make_rsrc(static_cast<bf16_t*>(g.C) + (int64_t)m0 * g.ldc, (int64_t)(M - m0) * g.ldc * 2);
#pragma unroll
    for (int i = 0; i < T::FM; ++i) {
      const int row = wm * T::WM + i * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < T::FN / 4; ++q) {
        uint32_t px[4], py[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          float v[4];
          epi_values<EPI>(bias[4 * q + jj], acc[i][4 * q + jj], v);
          px[jj] = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
          py[jj] = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        }
        // lane group G (= lane >> 4) holds columns 16 jj + 4 G .. + 3 in quad jj; afterwards quad jj
        // of group G holds columns 16 G + 4 jj .. + 3 (a 4 x 4 transpose of quads)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          auto r = __builtin_amdgcn_permlane32_swap(px[jj], px[jj + 2], false, false);
          px[jj] = r[0];
          px[jj + 2] = r[1];
          r = __builtin_amdgcn_permlane32_swap(py[jj], py[jj + 2], false, false);
          py[jj] = r[0];
          py[jj + 2] = r[1];
        }
#pragma unroll
        for (int jj = 0; jj < 4; jj += 2) {
          auto r = __builtin_amdgcn_permlane16_swap(px[jj], px[jj + 1], false, false);
          px[jj] = r[0];
          px[jj + 1] = r[1];
          r = __builtin_amdgcn_permlane16_swap(py[jj], py[jj + 1], false, false);
          py[jj] = r[0];
          py[jj + 1] = r[1];
        }
        const int col = n0 + wn * T::WN + q * 64 + (lane >> 4) * 16;
        const int off = (row * (int)g.ldc + col) * 2;
        const u32x4 lo4 = {px[0], py[0], px[1], py[1]};
        const u32x4 hi4 = {px[2], py[2], px[3], py[3]};
        __builtin_amdgcn_raw_buffer_store_b128(lo4, rC, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(hi4, rC, off + 16, 0, 0);
      }
    }
  };

  int m0, n0;
  geom(0, m0, n0);
  load_bias(n0, 0);
  for (int p = 0; p < D; ++p)
    if (p < G) issue_next();
  vm_wait_rt<GPW * D>(GPW * (min(D, G) - 1));
  __builtin_amdgcn_s_barrier();
  int kt = 0, t = 0, e_last = -(1 << 20), slot = 0;
  for (int s = 0; s < G; ++s) {
    const bool steady = s + D < G;
    if (steady) issue_next();
    compute(slot);
    slot = slot + 1 == NS ? 0 : slot + 1;
    // step s + 1 must have landed; younger: the ring loads of steps s + 2 .. min(s + D, G - 1) and, within
    // D steps after an epilogue, its stores and bias piece
    const bool extra = s + 1 <= e_last + D;
    if (steady) {
      if (extra) vm_wait_n<GPW * (D - 1) + NSTORE + NBIAS>();
      else vm_wait_n<GPW * (D - 1)>();
    } else if (s + 1 < G) {
      vm_wait_rt<GPW * (D - 1) + NSTORE + NBIAS>(GPW * (G - 2 - s) + (extra ? NSTORE + NBIAS : 0));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (++kt == nk) {
      epilogue(m0, n0, t & 1);
      kt = 0;
      ++t;
      if (t < nt) geom(t, m0, n0);
      load_bias(n0, t & 1);   // next tile's bias (after the last tile a harmless reload: a constant count)
      e_last = s;
#pragma unroll
      for (int i = 0; i < T::FM; ++i)
#pragma unroll
        for (int jj = 0; jj < T::FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

// ---------------------------------------------------------------------------------------------------
// 256 x 256 tile, 8 waves (2 x 4), four phases per 64-deep K-tile (one 128 x 128 C quadrant per
// phase; each wave owns a 64 x 32 piece of every quadrant).
//
// LDS holds 8 half-tile slots of 128 rows x 64 k (16 KB): {A rows 0-127, W rows 0-127, W rows
// 128-255, A rows 128-255} x 2 K-tile buffers.  Half-tile loads are numbered L = 4 kt + pos and
// load L is issued at global phase L - 6 (5-6 phases ahead of its first read, >= 2 phases after the
// last read of the slot it overwrites).  Phase reads (register reuse): p0 A rows 0-127 + W rows
// 0-127, p1 W rows 128-255, p2 A rows 128-255, p3 none (12 / 4 / 8 / 0 ds_read_b128).  Each phase: fragment reads, counted vmcnt for what the
// next phase reads, one half-tile load (2 x buffer_load_dwordx4 ... lds per lane), s_barrier, 16
// MFMAs at raised priority, s_barrier.  Waves 4-7 run one barrier behind waves 0-3, so on every
// SIMD one wave multiplies while its partner reads fragments and issues loads.
template <int EPI>
__global__ __launch_bounds__(512) void gemm256_kernel(const GemmArgs args) {
  __shared__ __attribute__((aligned(16))) bf16_t smem[8 * 128 * 64];
  GEMM_STAMP_DECL;
  const GemmGroup& g = args.g[blockIdx.z];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + 255) / 256, tiles_n = args.N / 256, ntiles = tiles_m * tiles_n;
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  const int q = ntiles >> 3, r8 = ntiles & 7;
  const int id = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + j;
  int tm, tn;
  tile_of(id, tiles_m, tiles_n, args.gm, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  float4 bpre[2][2];   // bias of the lane's epilogue columns, requested before the main loop
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
      bpre[qb][jj] = g.bias ? *reinterpret_cast<const float4*>(g.bias + n0 + qb * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
  GEMM_STAMP(0);

  const int chunk = ((lane & 7) ^ (lane >> 3)) * 16;
  const rsrc_t rA = make_rsrc(g.A + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
  const rsrc_t rW = make_rsrc(g.W + (int64_t)n0 * g.ldw, (int64_t)256 * g.ldw * 2);
  const uint32_t va = (uint32_t)((wave * 8 + (lane >> 3)) * g.lda * 2 + chunk);
  const uint32_t vw = (uint32_t)((wave * 8 + (lane >> 3)) * g.ldw * 2 + chunk);
  const uint32_t a64 = 64u * g.lda * 2, w64 = 64u * g.ldw * 2;
  const int nk = K / 64, NL = 4 * nk;

  // half-tile L (pos = L & 3: 0 A rows 0-127, 1 W rows 0-127, 2 W rows 128-255, 3 A rows 128-255)
  auto issue = [&](int L, auto pos_c) {
    constexpr int pos = decltype(pos_c)::value;
    const int kt = L >> 2;
    bf16_t* dst = smem + ((kt & 1) * 4 + pos) * 8192 + wave * 512;
    const int soff = kt * 128;
    const rsrc_t rs = (pos == 0 || pos == 3) ? rA : rW;
    const uint32_t v0 = pos == 0 ? va : pos == 3 ? va + 2 * a64 : pos == 1 ? vw : vw + 2 * w64;
    const uint32_t v1 = v0 + ((pos == 0 || pos == 3) ? a64 : w64);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lptr_t)dst, 16, v0, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lptr_t)(dst + 4096), 16, v1, soff, 0, 0);
  };
  auto wait_vm = [&](int n) {   // n half-tiles (2 loads each) may stay in flight
    if (n >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  f32x4 acc[4][4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[a][i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 Ar[4][2], B0r[2][2], B1r[2][2];

  auto read_a = [&](const bf16_t* S) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = wr * 64 + i * 16 + (lane & 15), c = 4 * s2 + (lane >> 4);
        Ar[i][s2] = *reinterpret_cast<const bf16x8*>(S + swz(row, c));
      }
  };
  auto read_b = [&](const bf16_t* S, bf16x8 (&Br)[2][2]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = wc * 32 + jj * 16 + (lane & 15), c = 4 * s2 + (lane >> 4);
        Br[jj][s2] = *reinterpret_cast<const bf16x8*>(S + swz(row, c));
      }
  };
  auto mma = [&](f32x4 (&C)[4][2], bf16x8 (&Br)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          C[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Br[jj][s2], Ar[i][s2], C[i][jj], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // half-tiles that may stay in flight at phase P's wait (before its own load): everything issued
  // after the last one phase P + 1 reads (p0: B1 = P+2, p1: A1 = P+2, p2: A1 = P+1, p3: B0' = P+2)
  auto n_after = [&](int P, int p) {
    const int need = P + (p == 2 ? 1 : 2);
    return max(min(P + 6, NL) - need - 1, 0);
  };

  auto ktile = [&](int kt, auto steady_c) {
    constexpr bool STEADY = decltype(steady_c)::value;   // every load of this K-tile's phases exists
    const bf16_t* S = smem + (kt & 1) * 4 * 8192;
    const int P0 = 4 * kt;
    // phase 0: quadrant (A rows 0-127, W rows 0-127)
    read_b(S + 8192, B0r);
    read_a(S);
    if (STEADY) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else wait_vm(n_after(P0, 0));
    if (STEADY || P0 + 6 < NL) issue(P0 + 6, std::integral_constant<int, 2>{});
    __builtin_amdgcn_s_barrier();
    mma(acc[0], B0r);
    __builtin_amdgcn_s_barrier();
    // phase 1: (A rows 0-127, W rows 128-255)
    read_b(S + 2 * 8192, B1r);
    if (STEADY) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else wait_vm(n_after(P0 + 1, 1));
    if (STEADY || P0 + 7 < NL) issue(P0 + 7, std::integral_constant<int, 3>{});
    __builtin_amdgcn_s_barrier();
    mma(acc[1], B1r);
    __builtin_amdgcn_s_barrier();
    // phase 2: (A rows 128-255, W rows 128-255)
    read_a(S + 3 * 8192);
    if (STEADY) asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); else wait_vm(n_after(P0 + 2, 2));
    if (STEADY || P0 + 8 < NL) issue(P0 + 8, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_barrier();
    mma(acc[2], B1r);
    __builtin_amdgcn_s_barrier();
    // phase 3: (A rows 128-255, W rows 0-127)
    if (STEADY) asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); else wait_vm(n_after(P0 + 3, 3));
    if (STEADY || P0 + 9 < NL) issue(P0 + 9, std::integral_constant<int, 1>{});
    __builtin_amdgcn_s_barrier();
    mma(acc[3], B0r);
    __builtin_amdgcn_s_barrier();
  };

  // prologue: half-tiles 0..5 (tile 0 and the first half of tile 1), wait for A0(0) and B0(0)
  issue(0, std::integral_constant<int, 0>{});
  issue(1, std::integral_constant<int, 1>{});
  issue(2, std::integral_constant<int, 2>{});
  issue(3, std::integral_constant<int, 3>{});
  if (nk > 1) {
    issue(4, std::integral_constant<int, 0>{});
    issue(5, std::integral_constant<int, 1>{});
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  GEMM_STAMP(1);
  if (wr) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 one barrier behind

  // steady K-tiles: all of their phase loads (up to half-tile P+9 < 4 nk) exist
  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, std::true_type{});
  for (; kt < nk; ++kt) ktile(kt, std::false_type{});
  if (!wr) __builtin_amdgcn_s_barrier();  // balance the stagger
  GEMM_STAMP(2);

  // epilogue: quadrant order (0,0), (0,1), (1,1), (1,0); through LDS (bf16: the whole 256 x 256 tile,
  // fp32: two 128-row halves)
  constexpr int QA[4] = {0, 0, 1, 1}, QB[4] = {0, 1, 1, 0};
  using LT = LdsTile<EPI, 256>;
  char* lds = reinterpret_cast<char*>(smem);
  constexpr int HALVES = LT::ESZ == 2 ? 1 : 2;
#pragma unroll
  for (int h = 0; h < HALVES; ++h) {
    if (h) __syncthreads();
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      if (HALVES == 2 && QA[qd] != h) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int col = QB[qd] * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4;
          const int row = (HALVES == 2 ? 0 : QA[qd] * 128) + wr * 64 + i * 16 + (lane & 15);
          float v[4];
          epi_values<EPI>(bpre[QB[qd]][jj], acc[qd][i][jj], v);
          LT::put(lds, row, col, v);
        }
    }
    __syncthreads();
    LT::template drain<256 / HALVES, 512>(lds, g, args, m0 + h * 128, n0, M);
  }
  GEMM_STAMP(3);
}

template <int EPI>
static void launch256(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + 255) / 256;
  a.gm = tiles_m < 4 ? tiles_m : 4;
  dim3 grid(tiles_m * (a.N / 256), 1, a.groups);
  hipLaunchKernelGGL(gemm256_kernel<EPI>, grid, dim3(512), 0, s, a);
}

static void launch256_epi(const GemmArgs& a, int epi, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return launch256<EPI_BF16>(a, s);
    case EPI_GELU_BF16: return launch256<EPI_GELU_BF16>(a, s);
    case EPI_RESID_F32: return launch256<EPI_RESID_F32>(a, s);
    case EPI_F32: return launch256<EPI_F32>(a, s);
    case EPI_POS_F32: return launch256<EPI_POS_F32>(a, s);
    default: break;
  }
}

// ---------------------------------------------------------------------------------------------------
// f16x3 (split) 256 x 256 tile in the 8-phase structure of gemm256_kernel, at BK = 32: a half-tile slot
// (16 KB) holds 128 rows x 32 k of BOTH halves (hi image, then lo image), so the LDS stays at 128 KB and
// the per-phase load is still two buffer_load ... lds per lane (hi, lo).  The 2-barrier K-loop of
// gemm_kernel stalls every K-step on the tile it has just asked for (all its tile shapes measured
// 240-260 TF/s, 29-31 % of the pipe); here loads run 5-6 phases ahead and the two wave groups (waves 0-3,
// 4-7, one barrier apart) alternate MFMA and fragment/load work on every SIMD.  Each phase multiplies
// one 128 x 128 quadrant: per wave 64 x 32 = 4 x 2 fragment pairs x 3 products = 24 MFMAs.
//
// MI = 5 (round 6): the same kernel on 320 x 256 tiles, for the bf16-output GEMMs (qkv, fc1) whose 256 x 256 tiles
// take two rounds of the chip's one-workgroup-per-CU slots for a little over one round of work while 320-row tiles
// fit one (the candidate-eliminated layers: qkv at 2 x 16 x 244 rows, 288 -> 234 tiles; fc1 at 2 x 16 x 190 rows,
// 288 -> 240).  A quadrant is 160 x 128, a wave's share 80 x 32 = 5 x 2 fragment pairs (30 MFMAs per phase, 160
// accumulators).  An A half-tile is 160 rows: the two planes' rows 0..127 load as in the 256-row kernel, rows
// 128..159 by one more instruction on waves 0-3 (waves 0, 1: hi; 2, 3: lo), so those waves count 3 loads per A
// half-tile in their vmcnt waits and waves 4-7 count 2.  The bias goes to the LDS (one DMA by wave 0) instead of
// 16 VGPRs and is read back after the K loop, when the fragment registers are free; the epilogue stages a
// 160-row half (hi + lo planes: the whole 160 KB).
template <int EPI, int MI>
__global__ __launch_bounds__(512) void gemm256s_kernel(const GemmArgs args) {
  static_assert(MI == 4 || (MI == 5 && epi_is_bf16(EPI)), "320-row tiles: 16-bit epilogues only");
  constexpr int BM = 64 * MI, HR = BM / 2;                   // tile rows; rows per A half-tile
  constexpr int AH = HR * 32;                                // elements of one A half-tile plane
  constexpr int P1 = 2 * AH, P2 = P1 + 8192, P3 = P2 + 8192;  // stage offsets of W0, W1, A1 (A0 at 0)
  constexpr int STG = P3 + 2 * AH;                           // elements per stage
  constexpr bool BIAS_LDS = MI > 4;
  constexpr int SMEM_OPS = 2 * STG + (BIAS_LDS ? 512 : 0);
  constexpr int SMEM_EPI = epi_is_bf16(EPI) ? HR * 256 * 2 : 0;
  constexpr int SMEM = SMEM_OPS > SMEM_EPI ? SMEM_OPS : SMEM_EPI;
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");
#ifdef GEMM_PHASE_STAMPS
  // tuning build (256-row tiles): per phase, wave 0 and wave 4 stamp (before the counted wait, after the first
  // barrier = MFMA start, after the second barrier) into an LDS tail of the one staging array; copied to
  // mmt_gemm_stamps' buffer at the end
  constexpr int PS_PH = 3 * 96;
  constexpr int PSE = MI == 4 ? 2 * PS_PH * 4 : 0;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM + PSE];
  unsigned long long* const pst = reinterpret_cast<unsigned long long*>(smem + SMEM);
#define PSTAMP(slot)                                                                                           \
  do {                                                                                                         \
    if (MI == 4 && (threadIdx.x & 255) == 0 && (slot) < PS_PH)                                                 \
      pst[(threadIdx.x >> 8) * PS_PH + (slot)] = __builtin_amdgcn_s_memtime();                                 \
  } while (0)
#else
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];
#define PSTAMP(slot) do { } while (0)
#endif
  GEMM_STAMP_DECL;
  const GemmGroup& g = args.g[blockIdx.z];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = args.N / 256, ntiles = tiles_m * tiles_n;
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  const int q = ntiles >> 3, r8 = ntiles & 7;
  const int id = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + j;
  int tm, tn;
  tile_of(id, tiles_m, tiles_n, args.gm, tm, tn);
  const int m0 = tm * BM, n0 = tn * 256;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  GEMM_STAMP(0);
  // the bias: MI = 4, the lane's 4 bias chunks (2 column halves x 2), requested before the first half-tile loads (the
  // prologue's counted wait retires them; the epilogue then starts without a dependent round trip); MI = 5, the
  // tile's 256 values DMA'd to the LDS tail by wave 0 ahead of its operand loads (retired by the same wait)
  const rsrc_t rB = make_rsrc(g.bias, g.bias ? (int64_t)args.N * 4 : 0);
  float4 bq[2][2];
  float* const bias_lds = reinterpret_cast<float*>(smem + 2 * STG);
  if constexpr (BIAS_LDS) {
    if (wave == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lptr_t)bias_lds, 16, (uint32_t)(n0 + lane * 4) * 4, 0, 0, 0);
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) bq[h][jj] = epi_bias(rB, n0 + h * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4);
  }

  // half-tile loads: a wave-instruction fills 16 rows x 64 B (swzk<32> image, source chunk pre-swizzled)
  const int chunk = ((lane & 3) ^ ((lane >> 4) & 2)) * 16;
  const int lrow = wave * 16 + (lane >> 2);
  const rsrc_t rA = make_rsrc(g.A + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
  const rsrc_t rAl = make_rsrc(g.A_lo + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
  const rsrc_t rW = make_rsrc(g.W + (int64_t)n0 * g.ldw, (int64_t)256 * g.ldw * 2);
  const rsrc_t rWl = make_rsrc(g.W_lo + (int64_t)n0 * g.ldw, (int64_t)256 * g.ldw * 2);
  const uint32_t va = (uint32_t)(lrow * g.lda * 2 + chunk), vw = (uint32_t)(lrow * g.ldw * 2 + chunk);
  const uint32_t aH = (uint32_t)HR * g.lda * 2, w128 = 128u * g.ldw * 2;
  // MI = 5: rows 128..159 of an A half-tile (waves 0-3: wave & 1 picks the 16-row group, wave & 2 the plane)
  const uint32_t vx = (uint32_t)((128 + (wave & 1) * 16 + (lane >> 2)) * g.lda * 2 + chunk);
  const int nk = K / 32, NL = 4 * nk;

  // half-tile L (pos = L & 3: 0 A rows 0..HR-1, 1 W rows 0-127, 2 W rows 128-255, 3 A rows HR..BM-1)
  auto issue = [&](int L, auto pos_c) {
    constexpr int pos = decltype(pos_c)::value;
    constexpr bool isA = pos == 0 || pos == 3;
    constexpr int poff = pos == 0 ? 0 : pos == 1 ? P1 : pos == 2 ? P2 : P3;
    constexpr int plo = isA ? AH : 4096;
    const int kt = L >> 2;
    bf16_t* const slot = smem + (kt & 1) * STG + poff;
    bf16_t* dst = slot + wave * 512;
    const int soff = kt * 64;
    const uint32_t v = pos == 0 ? va : pos == 3 ? va + aH : pos == 1 ? vw : vw + w128;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rA : rW, (lptr_t)dst, 16, v, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? rAl : rWl, (lptr_t)(dst + plo), 16, v, soff, 0, 0);
    if constexpr (isA && MI == 5) {
      if (wave < 4)
        __builtin_amdgcn_raw_ptr_buffer_load_lds((wave & 2) ? rAl : rA,
                                                 (lptr_t)(slot + ((wave & 2) ? AH : 0) + 128 * 32 + (wave & 1) * 512),
                                                 16, pos == 0 ? vx : vx + aH, soff, 0, 0);
    }
  };
  auto wait_vm = [&](int n) {   // n half-tiles (2 loads each) may stay in flight
    if (n >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // steady-state wait of one phase: G0 loads may stay in flight on waves 0-3, G1 on waves 4-7 (MI = 4: the same)
  auto wait_steady = [&](auto g0_c, auto g1_c) {
    constexpr int G0 = decltype(g0_c)::value, G1 = decltype(g1_c)::value;
    if constexpr (G0 == G1) vm_wait_n<G0>();
    else if (wr == 0) vm_wait_n<G0>();
    else vm_wait_n<G1>();
  };
  using I6 = std::integral_constant<int, 6>;
  using I8 = std::integral_constant<int, 8>;
  using I7 = std::integral_constant<int, 7>;
  using I10 = std::integral_constant<int, 10>;

  f32x4 acc[4][MI][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[a][i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 Ah[MI], Al[MI], B0h[2], B0l[2], B1h[2], B1l[2];
  const int c = lane >> 4;
  auto read_a = [&](const bf16_t* S) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int row = wr * (16 * MI) + i * 16 + (lane & 15);
      Ah[i] = *reinterpret_cast<const bf16x8*>(S + swzk<32>(row, c));
      Al[i] = *reinterpret_cast<const bf16x8*>(S + AH + swzk<32>(row, c));
    }
  };
  auto read_b = [&](const bf16_t* S, bf16x8 (&Bh)[2], bf16x8 (&Bl)[2]) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = wc * 32 + jj * 16 + (lane & 15);
      Bh[jj] = *reinterpret_cast<const bf16x8*>(S + swzk<32>(row, c));
      Bl[jj] = *reinterpret_cast<const bf16x8*>(S + 4096 + swzk<32>(row, c));
    }
  };
  // the phase's MFMAs at priority 1 (per-phase flips: 6 279 frames/s against 6 140 for waves 4-7 at a static priority 1
  // and 6 140 for no priorities, profiles/r06_ab_256s_prio.txt)
  auto mma = [&](f32x4 (&C)[MI][2], const bf16x8 (&Bh)[2], const bf16x8 (&Bl)[2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bh[jj], Ah[i], C[i][jj]);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bl[jj], Ah[i], C[i][jj]);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bh[jj], Al[i], C[i][jj]);
    __builtin_amdgcn_s_setprio(0);
  };
  // half-tiles that may stay in flight at phase P's wait (before its own load): everything issued
  // after the last one phase P + 1 reads (p0: B1 = P+2, p1: A1 = P+2, p2: A1 = P+1, p3: B0' = P+2)
  auto n_after = [&](int P, int p) {
    const int need = P + (p == 2 ? 1 : 2);
    return max(min(P + 6, NL) - need - 1, 0);
  };
  // the tail phases' wait: MI = 4, n_after half-tiles of 2 loads; MI = 5, those half-tiles' loads counted one by one
  // (an A half-tile is 3 loads on waves 0-3)
  auto wait_tail = [&](int P, int p) {
    const int n = n_after(P, p);
    if constexpr (MI == 4) {
      wait_vm(n);
    } else {
      const int need = P + (p == 2 ? 1 : 2), na = wr == 0 ? 3 : 2;
      int loads = 0;
      for (int L = need + 1; L <= need + n; ++L) loads += ((L & 3) == 0 || (L & 3) == 3) ? na : 2;
      vm_wait_rt<16>(loads);
    }
  };
  auto ktile = [&](int kt, auto steady_c) {
    constexpr bool STEADY = decltype(steady_c)::value;
    const bf16_t* S = smem + (kt & 1) * STG;
    const int P0 = 4 * kt;
    read_b(S + P1, B0h, B0l);
    read_a(S);
    PSTAMP(3 * P0);
    if (STEADY) {
      if constexpr (MI == 4) wait_steady(I6{}, I6{}); else wait_steady(I8{}, I6{});
    } else {
      wait_tail(P0, 0);
    }
    if (STEADY || P0 + 6 < NL) issue(P0 + 6, std::integral_constant<int, 2>{});
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 1);
    mma(acc[0], B0h, B0l);
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 2);
    read_b(S + P2, B1h, B1l);
    PSTAMP(3 * P0 + 3);
    if (STEADY) {
      if constexpr (MI == 4) wait_steady(I6{}, I6{}); else wait_steady(I7{}, I6{});
    } else {
      wait_tail(P0 + 1, 1);
    }
    if (STEADY || P0 + 7 < NL) issue(P0 + 7, std::integral_constant<int, 3>{});
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 4);
    mma(acc[1], B1h, B1l);
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 5);
    read_a(S + P3);
    PSTAMP(3 * P0 + 6);
    if (STEADY) {
      if constexpr (MI == 4) wait_steady(I8{}, I8{}); else wait_steady(I10{}, I8{});
    } else {
      wait_tail(P0 + 2, 2);
    }
    if (STEADY || P0 + 8 < NL) issue(P0 + 8, std::integral_constant<int, 0>{});
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 7);
    mma(acc[2], B1h, B1l);
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 8);
    PSTAMP(3 * P0 + 9);
    if (STEADY) {
      if constexpr (MI == 4) wait_steady(I6{}, I6{}); else wait_steady(I8{}, I6{});
    } else {
      wait_tail(P0 + 3, 3);
    }
    if (STEADY || P0 + 9 < NL) issue(P0 + 9, std::integral_constant<int, 1>{});
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 10);
    mma(acc[3], B0h, B0l);
    __builtin_amdgcn_s_barrier();
    PSTAMP(3 * P0 + 11);
  };

  issue(0, std::integral_constant<int, 0>{});
  issue(1, std::integral_constant<int, 1>{});
  issue(2, std::integral_constant<int, 2>{});
  issue(3, std::integral_constant<int, 3>{});
  // half-tiles 0 and 1 (A0, W0) landed: 2..5 (or 2, 3) may stay in flight
  if (nk > 1) {
    issue(4, std::integral_constant<int, 0>{});
    issue(5, std::integral_constant<int, 1>{});
    if constexpr (MI == 4) wait_steady(I8{}, I8{}); else wait_steady(I10{}, I8{});
  } else {
    if constexpr (MI == 4) vm_wait_n<4>();
    else if (wr == 0) vm_wait_n<5>();
    else vm_wait_n<4>();
  }
  __builtin_amdgcn_s_barrier();
  GEMM_STAMP(1);
  if (wr) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 one barrier behind

  int kt = 0;
  for (; kt + 2 < nk; ++kt) ktile(kt, std::true_type{});
  for (; kt < nk; ++kt) ktile(kt, std::false_type{});
  if (!wr) __builtin_amdgcn_s_barrier();  // balance the stagger
  GEMM_STAMP(2);

  constexpr int QA[4] = {0, 0, 1, 1}, QB[4] = {0, 1, 1, 0};
  if constexpr (epi_is_bf16(EPI)) {
    // 16-bit outputs (qkv, fc1): per HR-row half, the hi and lo planes of the half go to the LDS (the whole staging
    // array), then every lane stores whole 16-B row chunks, eight lanes per 128-B line.  Stored straight from the
    // fragments, a wave-instruction wrote 16 rows x 32 B and the epilogue took ~35k of a tile's ~145k cycles
    // (round-5 phase stamps, tools/gemm256s_phases.py); same values, same bits.
    if constexpr (BIAS_LDS) {   // the bias back from the LDS tail before the staging overwrites it
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          bq[h][jj] = *reinterpret_cast<const float4*>(bias_lds + h * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4);
    }
    using LT = LdsTile<EPI_BF16, 256>;   // [HR][256] 16-bit, 16-B chunks XOR-swizzled by row
    char* const planeH = reinterpret_cast<char*>(smem);
    char* const planeL = planeH + HR * 256 * 2;
    const int tid = threadIdx.x;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      __syncthreads();   // h = 0: every wave's last fragment (and bias) reads are done; h = 1: the first half is drained
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        if (QA[qd] != h) continue;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const int row = wr * (16 * MI) + i * 16 + (lane & 15);
            const int col = QB[qd] * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4;
            const f32x4& a = acc[qd][i][jj];
            const float4 bv = bq[QB[qd]][jj];
            float v[4] = {a[0] * g.inv + bv.x, a[1] * g.inv + bv.y, a[2] * g.inv + bv.z, a[3] * g.inv + bv.w};
            if (EPI == EPI_GELU_BF16) {
              f32x2 g0 = {v[0], v[1]}, g1 = {v[2], v[3]};
              gelu_erf4(g0, g1);
              v[0] = g0.x;
              v[1] = g0.y;
              v[2] = g1.x;
              v[3] = g1.y;
            }
            if (EPI == EPI_RELU_BF16)
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
            uint16_t hh[4], ll[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) split_h(v[e] * g.out_scale, hh[e], ll[e]);
            const int o = LT::off(row, col);
            *reinterpret_cast<uint2*>(planeH + o) =
                make_uint2((uint32_t)hh[0] | ((uint32_t)hh[1] << 16), (uint32_t)hh[2] | ((uint32_t)hh[3] << 16));
            *reinterpret_cast<uint2*>(planeL + o) =
                make_uint2((uint32_t)ll[0] | ((uint32_t)ll[1] << 16), (uint32_t)ll[2] | ((uint32_t)ll[3] << 16));
          }
      }
      __syncthreads();
      // HR rows x 32 chunks per plane; rows past M fall outside the C resources (zero-sized tail) and are dropped
      const int rows = max(0, min(HR, M - (m0 + h * HR)));
      const rsrc_t rC = make_rsrc(static_cast<bf16_t*>(g.C) + (int64_t)(m0 + h * HR) * g.ldc, (int64_t)rows * g.ldc * 2);
      const rsrc_t rCl = make_rsrc(static_cast<bf16_t*>(g.C_lo) + (int64_t)(m0 + h * HR) * g.ldc,
                                   (int64_t)rows * g.ldc * 2);
#pragma unroll
      for (int it = 0; it < HR * 32 / 512; ++it) {
        const int idx = tid + it * 512, r = idx >> 5, c = idx & 31;
        const int lo = r * 512 + ((c ^ (r & 15)) << 4);
        const uint32_t go = r < rows ? (uint32_t)(((int64_t)r * g.ldc + n0 + c * 8) * 2) : kBufOob;
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(planeH + lo), rC, go, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(planeL + lo), rCl, go, 0, 0);
      }
    }
    GEMM_STAMP(3);
#ifdef GEMM_PHASE_STAMPS
    if constexpr (MI == 4) {
      __syncthreads();
      if (gemm_stamps_ && blockIdx.x < 256)
        for (int e = threadIdx.x; e < 2 * PS_PH; e += 512)
          gemm_stamps_[65536 + (size_t)blockIdx.x * 2 * PS_PH + e] = pst[e];
    }
#endif
    return;
  } else if constexpr (EPI == EPI_RESID_F32 && MI == 4) {
    // fp32 residual output (the long-K residual GEMM, MMT_FC2_256S): per 128-row half the residual chunks are requested
    // first, the half's acc * inv + bias goes to the LDS ([128][256] fp32, 16-B chunks XOR-swizzled by row), then every
    // lane stores whole 16-B row chunks of R + value (store4v's arithmetic: the same bits)
    using LF = LdsTile<EPI_F32, 256>;
    char* const lds = reinterpret_cast<char*>(smem);
    const rsrc_t rR = epi_resid_rsrc<EPI>(g, args, M);
    const int tid = threadIdx.x;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int mb = m0 + h * 128;
      u32x4 rv[128 * 64 / 512];
#pragma unroll
      for (int k = 0; k < 128 * 64 / 512; ++k) {
        const int idx = tid + k * 512, r = idx >> 6, cc = idx & 63, m = mb + r;
        const uint32_t o = m < M ? (uint32_t)(((int64_t)m * g.ldr + n0 + 4 * cc) * 4) : kBufOob;
        rv[k] = __builtin_amdgcn_raw_buffer_load_b128(rR, o, 0, 0);
      }
      __syncthreads();   // h = 0: every wave's last fragment reads are done; h = 1: the first half is drained
#pragma unroll
      for (int qd = 0; qd < 4; ++qd) {
        if (QA[qd] != h) continue;
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
            const f32x4& a = acc[qd][i][jj];
            const float4 bv = bq[QB[qd]][jj];
            const float v[4] = {a[0] * g.inv + bv.x, a[1] * g.inv + bv.y, a[2] * g.inv + bv.z, a[3] * g.inv + bv.w};
            LF::put(lds, wr * 64 + i * 16 + (lane & 15), QB[qd] * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4, v);
          }
      }
      __syncthreads();
      const int rows = max(0, min(128, M - mb));
      const rsrc_t rC = make_rsrc(static_cast<float*>(g.C) + (int64_t)mb * g.ldc, (int64_t)rows * g.ldc * 4);
#pragma unroll
      for (int k = 0; k < 128 * 64 / 512; ++k) {
        const int idx = tid + k * 512, r = idx >> 6, cc = idx & 63;
        const f32x4 v = *reinterpret_cast<const f32x4*>(lds + r * 256 * 4 + ((cc ^ (r & LF::MASK)) << 4));
        const f32x4 o = __builtin_bit_cast(f32x4, rv[k]) + v;
        const uint32_t go = r < rows ? (uint32_t)(((int64_t)r * g.ldc + n0 + 4 * cc) * 4) : kBufOob;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rC, go, 0, 0);
      }
    }
    GEMM_STAMP(3);
  } else {
    // (the remaining fp32 epilogues, not used by the path's launches, keep the per-fragment store4)
    const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int qd = 0; qd < 4; ++qd)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0 + QA[qd] * HR + wr * (16 * MI) + i * 16 + (lane & 15);
        if (m >= M) continue;
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          if constexpr (epi_has_r(EPI))
            store4<EPI, true>(g, args, m, n0 + QB[qd] * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4, acc[qd][i][jj]);
          else
            store4v<EPI, true>(g, args, m, n0 + QB[qd] * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4, acc[qd][i][jj],
                               bq[QB[qd]][jj], zero4);
      }
    GEMM_STAMP(3);
#ifdef GEMM_PHASE_STAMPS
    __syncthreads();
    if (gemm_stamps_ && blockIdx.x < 256)   // blocks' phase stamps after the [blocks][4] kernel stamps
      for (int e = threadIdx.x; e < 2 * PS_PH; e += 512)
        gemm_stamps_[65536 + (size_t)blockIdx.x * 2 * PS_PH + e] = pst[e];
#endif
  }
}
#undef PSTAMP

template <int EPI, int MI>
static void launch256s(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + 64 * MI - 1) / (64 * MI);
  static const int gm256 = getenv("MMT_GM256") ? atoi(getenv("MMT_GM256")) : 4;   // tuning: super-tile height
  a.gm = tiles_m < gm256 ? tiles_m : gm256;
  hipLaunchKernelGGL((gemm256s_kernel<EPI, MI>), dim3(tiles_m * (a.N / 256), 1, a.groups), dim3(512), 0, s, a);
}

// t320: the 320 x 256 tiles (16-bit epilogues; false if the epilogue has none)
static bool launch256s_epi(const GemmArgs& a, int epi, hipStream_t s, bool t320 = false) {
  if (a.N % 256 || a.K % 32 || a.K < 64 || a.amode != A_DENSE) return false;
  if (t320) {
    switch (epi) {
      case EPI_BF16: return launch256s<EPI_BF16, 5>(a, s), true;
      case EPI_GELU_BF16: return launch256s<EPI_GELU_BF16, 5>(a, s), true;
      default: return false;
    }
  }
  switch (epi) {
    case EPI_BF16: return launch256s<EPI_BF16, 4>(a, s), true;
    case EPI_GELU_BF16: return launch256s<EPI_GELU_BF16, 4>(a, s), true;
    case EPI_RESID_F32: return launch256s<EPI_RESID_F32, 4>(a, s), true;
    case EPI_F32: return launch256s<EPI_F32, 4>(a, s), true;
    case EPI_POS_F32: return launch256s<EPI_POS_F32, 4>(a, s), true;
    default: return false;
  }
}

// ---------------------------------------------------------------------------------------------------
// f16x3 128 x 256 tile in the staggered two-group structure of gemm256s_kernel (round 6), for the N = 768 fp32-output
// GEMMs (proj, fc2): 3 column tiles of 256 and one row block of 128 per tile -- where its tiles fill one round of the
// one-workgroup-per-CU slots and 128 x 128 tiles would take two (the 256-row kernel would leave half the CUs idle).
// A 32-deep K-tile is three half-tiles (A rows 0..127, W rows 0..127, W rows 128..255; hi then lo plane, 16 KB each)
// in a 3-stage LDS ring (144 KB), multiplied in two phases: A x W0 into acc[0], A x W1 into acc[1] (per wave 64 x 32
// of each 128 x 128 quadrant: 4 x 2 fragment pairs x 3 products = 24 MFMAs per phase; A's fragments are read once per
// K-tile).  Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave's MFMAs overlap the other's fragment
// reads and load issue; the half-tile slots are refilled five phases ahead of their first read (the loop below).
// Fragment reads are not drained before a barrier (the MFMA after it waits for them): a slot's refill is issued after
// a later barrier and lands hundreds of cycles after any read issued before it (drained, the K loop ran 10 % slower;
// the eight-phase kernel relies on the same order).  Per-block stamps: ~1 000 cycles per phase against 768 of MFMAs.
// Each output accumulates over the same K order, three products per 32-deep step in the same order, as every other
// f16x3 tile: the same bits as gemm_kernel / gemm256s_kernel (test_gemm_f16x3_w256).
template <int EPI>
__global__ __launch_bounds__(512) void gemm128w_kernel(const GemmArgs args) {
  static_assert(EPI == EPI_RESID_F32 || EPI == EPI_F32 || EPI == EPI_POS_F32, "fp32-output epilogues");
  constexpr int PW0 = 8192, PW1 = 16384, STG = 24576;   // elements: A (hi, lo) at 0, W0 (hi, lo), W1 (hi, lo)
  __shared__ __attribute__((aligned(16))) bf16_t smem[3 * STG];   // the epilogue's [128][256] fp32 tile reuses it
  GEMM_STAMP_DECL;
  const GemmGroup& g = args.g[blockIdx.z];
  const int M = args.M, K = args.K;
  const int tiles_m = (M + 127) / 128, tiles_n = args.N / 256, ntiles = tiles_m * tiles_n;
  const int b = blockIdx.x, x = b & 7, j = b >> 3;
  const int q = ntiles >> 3, r8 = ntiles & 7;
  const int id = (x < r8 ? x * (q + 1) : r8 * (q + 1) + (x - r8) * q) + j;
  int tm, tn;
  tile_of(id, tiles_m, tiles_n, args.gm, tm, tn);
  const int m0 = tm * 128, n0 = tn * 256;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  GEMM_STAMP(0);
  // the lane's bias chunks, requested before the operand loads (the prologue's counted wait retires them)
  const rsrc_t rB = make_rsrc(g.bias, g.bias ? (int64_t)args.N * 4 : 0);
  float4 bq[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) bq[h][jj] = epi_bias(rB, n0 + h * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4);

  // half-tile loads: a wave-instruction fills 16 rows x 64 B (swzk<32> image, source chunk pre-swizzled); rows past M
  // fall outside the A resources and read zeros
  const int chunk = ((lane & 3) ^ ((lane >> 4) & 2)) * 16;
  const int lrow = wave * 16 + (lane >> 2);
  const rsrc_t rA = make_rsrc(g.A + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
  const rsrc_t rAl = make_rsrc(g.A_lo + (int64_t)m0 * g.lda, (int64_t)(M - m0) * g.lda * 2);
  const rsrc_t rW = make_rsrc(g.W + (int64_t)n0 * g.ldw, (int64_t)256 * g.ldw * 2);
  const rsrc_t rWl = make_rsrc(g.W_lo + (int64_t)n0 * g.ldw, (int64_t)256 * g.ldw * 2);
  const uint32_t va = (uint32_t)(lrow * g.lda * 2 + chunk), vw = (uint32_t)(lrow * g.ldw * 2 + chunk);
  const uint32_t vw1 = vw + (uint32_t)(128u * g.ldw * 2);
  const int nk = K / 32;
  // half-tile issue: A and W0 of a K-tile together (four wave-instructions), W1 alone (two)
  auto issue_aw0 = [&](int kt) {
    bf16_t* const d = smem + (kt % 3) * STG + wave * 512;
    const int soff = kt * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lptr_t)d, 16, va, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rAl, (lptr_t)(d + 4096), 16, va, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lptr_t)(d + PW0), 16, vw, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rWl, (lptr_t)(d + PW0 + 4096), 16, vw, soff, 0, 0);
  };
  auto issue_w1 = [&](int kt) {
    bf16_t* const d = smem + (kt % 3) * STG + wave * 512;
    const int soff = kt * 64;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rW, (lptr_t)(d + PW1), 16, vw1, soff, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rWl, (lptr_t)(d + PW1 + 4096), 16, vw1, soff, 0, 0);
  };
  f32x4 acc[2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) acc[a][i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 Ah[4], Al[4], Bh[2], Bl[2];
  const int c = lane >> 4;
  auto read_a = [&](const bf16_t* S) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 64 + i * 16 + (lane & 15);
      Ah[i] = *reinterpret_cast<const bf16x8*>(S + swzk<32>(row, c));
      Al[i] = *reinterpret_cast<const bf16x8*>(S + 4096 + swzk<32>(row, c));
    }
  };
  auto read_b = [&](const bf16_t* S) {
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int row = wc * 32 + jj * 16 + (lane & 15);
      Bh[jj] = *reinterpret_cast<const bf16x8*>(S + swzk<32>(row, c));
      Bl[jj] = *reinterpret_cast<const bf16x8*>(S + 4096 + swzk<32>(row, c));
    }
  };
  auto mma = [&](f32x4 (&C)[4][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bh[jj], Ah[i], C[i][jj]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bl[jj], Ah[i], C[i][jj]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) C[i][jj] = mfma16<true>(Bh[jj], Al[i], C[i][jj]);
    __builtin_amdgcn_s_setprio(0);
  };

  // Each half-tile slot is refilled as soon as both groups are past their last read of it: A / W0 of K-tile kt + 3 at
  // phase 1 of K-tile kt (the slots of A / W0 (kt), last read in phase 0), W1 of kt + 2 at phase 0 of kt (the slot of
  // W1 (kt - 1)); so every half-tile is requested five phases before its first read.  A wave waits for its own loads of
  // a half-tile before the barrier that precedes the first read of it by either group: group 1 (one barrier behind)
  // before its pre-MFMA barrier, group 0 before its post-MFMA one.  Counts: the wave-instructions issued after the
  // awaited half-tile (12 in steady state).
  issue_aw0(0);
  issue_w1(0);
  if (nk > 1) {
    issue_aw0(1);
    issue_w1(1);
  }
  if (nk > 2) issue_aw0(2);
  vm_wait_rt<12>((nk > 1 ? 6 : 0) + (nk > 2 ? 4 : 0) + 2);   // A / W0 of K-tile 0 landed
  __builtin_amdgcn_s_barrier();
  GEMM_STAMP(1);
  if (wr) __builtin_amdgcn_s_barrier();   // stagger: waves 4-7 one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const bf16_t* S = smem + (kt % 3) * STG;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk, n3 = kt + 3 < nk;
    // phase 0: A x W0
    if (n2) issue_w1(kt + 2);
    read_b(S + PW0);
    read_a(S);
    const int c0 = (n1 ? 6 : 0) + (n2 ? 6 : 0);   // issued after W1 (kt)
    if (wr) vm_wait_rt<12>(c0);
    __builtin_amdgcn_s_barrier();
    mma(acc[0]);
    if (!wr) vm_wait_rt<12>(c0);
    __builtin_amdgcn_s_barrier();
    // phase 1: A x W1
    if (n3) issue_aw0(kt + 3);
    read_b(S + PW1);
    const int c1 = 2 + (n2 ? 6 : 0) + (n3 ? 4 : 0);   // issued after A / W0 (kt + 1)
    if (wr && n1) vm_wait_rt<12>(c1);
    __builtin_amdgcn_s_barrier();
    mma(acc[1]);
    if (!wr && n1) vm_wait_rt<12>(c1);
    __builtin_amdgcn_s_barrier();
  }
  if (!wr) __builtin_amdgcn_s_barrier();  // balance the stagger
  GEMM_STAMP(2);

  // epilogue: the residual / position chunks requested first, acc * inv + bias staged through the LDS ([128][256]
  // fp32, 16-B chunks XOR-swizzled by row), then every lane stores whole 16-B row chunks of R + value (store4v's
  // arithmetic: the same bits)
  using LF = LdsTile<EPI_F32, 256>;
  char* const lds = reinterpret_cast<char*>(smem);
  const int tid = threadIdx.x;
  u32x4 rv[epi_has_r(EPI) ? 16 : 1];
  if constexpr (epi_has_r(EPI)) {
    // (requested at kernel entry instead, they moved ~5k cycles from the epilogue into the prologue: level)
    const rsrc_t rR = epi_resid_rsrc<EPI>(g, args, M);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int idx = tid + k * 512, r = idx >> 6, cc = idx & 63, m = m0 + r;
      const int row = EPI == EPI_POS_F32 ? m % args.pos_rows : m;
      const uint32_t o = m < M ? (uint32_t)(((int64_t)row * g.ldr + n0 + 4 * cc) * 4) : kBufOob;
      rv[k] = __builtin_amdgcn_raw_buffer_load_b128(rR, o, 0, 0);
    }
  }
  __syncthreads();   // every wave's last fragment reads are done
#pragma unroll
  for (int qd = 0; qd < 2; ++qd)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const f32x4& a = acc[qd][i][jj];
        const float4 bv = bq[qd][jj];
        const float v[4] = {a[0] * g.inv + bv.x, a[1] * g.inv + bv.y, a[2] * g.inv + bv.z, a[3] * g.inv + bv.w};
        LF::put(lds, wr * 64 + i * 16 + (lane & 15), qd * 128 + wc * 32 + jj * 16 + (lane >> 4) * 4, v);
      }
  __syncthreads();
  const int rows = max(0, min(128, M - m0));
  const rsrc_t rC = make_rsrc(static_cast<float*>(g.C) + (int64_t)m0 * g.ldc, (int64_t)rows * g.ldc * 4);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int idx = tid + k * 512, r = idx >> 6, cc = idx & 63;
    f32x4 v = *reinterpret_cast<const f32x4*>(lds + r * 256 * 4 + ((cc ^ (r & LF::MASK)) << 4));
    if constexpr (epi_has_r(EPI)) v = __builtin_bit_cast(f32x4, rv[k]) + v;
    const uint32_t go = r < rows ? (uint32_t)(((int64_t)r * g.ldc + n0 + 4 * cc) * 4) : kBufOob;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rC, go, 0, 0);
  }
  GEMM_STAMP(3);
}

static int super_rows(int tiles_m, int K);

template <int EPI>
static void launch128w(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + 127) / 128;
  a.gm = super_rows(tiles_m, a.K);
  hipLaunchKernelGGL((gemm128w_kernel<EPI>), dim3(tiles_m * (a.N / 256), 1, a.groups), dim3(512), 0, s, a);
}

static bool launch128w_epi(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.N % 256 || a.K % 32 || a.K < 32 || a.amode != A_DENSE) return false;
  switch (epi) {
    case EPI_RESID_F32: return launch128w<EPI_RESID_F32>(a, s), true;
    case EPI_F32: return launch128w<EPI_F32>(a, s), true;
    case EPI_POS_F32: return launch128w<EPI_POS_F32>(a, s), true;
    default: return false;
  }
}

// super-tile height (tile rows walked together, column-major inside): 8 rows x all columns keeps a short-K
// GEMM's weight slab shared per XCD; a long-K GEMM (fc2: K = 3072; the head conv: K = 6912) re-fetches its
// large A row blocks once per column tile unless the row's column tiles run close together (gm = 4: head
// conv 359 -> 331 us at 32 sequences, fc2 level, tests/sweep_gm_b32.sh; +0.5 % over gm = 2, ab_env.sh)
static int super_rows(int tiles_m, int K) {
  static const int gm_env = getenv("MMT_GM") ? atoi(getenv("MMT_GM")) : 0;
  static const int gm_long = getenv("MMT_GM_LONGK") ? atoi(getenv("MMT_GM_LONGK")) : 4;
  const int gm = gm_env > 0 ? gm_env : (K >= 2048 ? gm_long : 8);
  return tiles_m < gm ? tiles_m : gm;
}

template <int BM, int BN, int WMW, int WNW, int EPI, int AM, bool SPLIT, int ST, int BK = 64>
static void launch_one(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = a.N / BN;
  (void)tiles_n;
  a.gm = super_rows(tiles_m, a.K);
  dim3 grid(tiles_m * tiles_n, 1, a.groups);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WMW, WNW, EPI, AM, SPLIT, ST, BK>), grid, dim3(WMW * WNW * 64), 0, s, a);
}

template <int EPI>
static void launch_persist(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + 127) / 128, ntiles = tiles_m * (a.N / 128);
  a.gm = tiles_m < 8 ? tiles_m : 8;
  static const int slots = 2 * num_cus();   // two 64-KB-LDS workgroups per CU
  const int grid = (ntiles < slots ? ntiles : slots) & ~7;
  hipLaunchKernelGGL((gemm_persist_kernel<128, 128, 4, 2, EPI>), dim3(grid), dim3(512), 0, s, a);
}

template <int BM, int BN, int WMW, int WNW, int EPI, int NS, int BK, int WG_PER_CU>
static void launch_ring(const GemmArgs& a0, hipStream_t s) {
  GemmArgs a = a0;
  const int tiles_m = (a.M + BM - 1) / BM, ntiles = tiles_m * (a.N / BN);
  a.gm = tiles_m < 8 ? tiles_m : 8;
  static const int slots = WG_PER_CU * num_cus();
  int grid = (ntiles < slots ? ntiles : slots) & ~7;
  if (grid < 8) grid = 8;
  hipLaunchKernelGGL((gemm_ring_kernel<BM, BN, WMW, WNW, EPI, NS, BK>), dim3(grid), dim3(WMW * WNW * 64), 0, s, a);
}

template <int BM, int BN, int WMW, int WNW, int NS, int BK, int WG_PER_CU>
static bool launch_ring_epi(const GemmArgs& a, int epi, hipStream_t s) {
  // K / BK >= NS: a tile's bias (issued after the previous epilogue) has landed before its own epilogue
  if (a.N % BN != 0 || a.groups != 1 || a.amode != A_DENSE || a.K % BK != 0 || a.K / BK < NS) return false;
  if (epi == EPI_BF16) return launch_ring<BM, BN, WMW, WNW, EPI_BF16, NS, BK, WG_PER_CU>(a, s), true;
  if (epi == EPI_GELU_BF16) return launch_ring<BM, BN, WMW, WNW, EPI_GELU_BF16, NS, BK, WG_PER_CU>(a, s), true;
  return false;
}

template <int BM, int BN, int WMW, int WNW, bool SPLIT, int ST = 2, int BK = 64>
static void launch_cfg(const GemmArgs& a, int epi, hipStream_t s) {
  if (a.amode == A_CONV3) {
    if constexpr (BK == 64) {   // the conv gather walks 64-channel K-tiles
      if (epi == EPI_RELU_BF16) return launch_one<BM, BN, WMW, WNW, EPI_RELU_BF16, A_CONV3, SPLIT, ST>(a, s);
      if (epi == EPI_RELU_F32) return launch_one<BM, BN, WMW, WNW, EPI_RELU_F32, A_CONV3, SPLIT, ST>(a, s);
    }
    return;
  }
  switch (epi) {
    case EPI_BF16: return launch_one<BM, BN, WMW, WNW, EPI_BF16, A_DENSE, SPLIT, ST, BK>(a, s);
    case EPI_GELU_BF16: return launch_one<BM, BN, WMW, WNW, EPI_GELU_BF16, A_DENSE, SPLIT, ST, BK>(a, s);
    case EPI_RESID_F32: return launch_one<BM, BN, WMW, WNW, EPI_RESID_F32, A_DENSE, SPLIT, ST, BK>(a, s);
    case EPI_F32: return launch_one<BM, BN, WMW, WNW, EPI_F32, A_DENSE, SPLIT, ST, BK>(a, s);
    case EPI_POS_F32: return launch_one<BM, BN, WMW, WNW, EPI_POS_F32, A_DENSE, SPLIT, ST, BK>(a, s);
    default: break;
  }
}

// split-K reduction: C = epi(sum_s partial_s + bias) in a fixed order (deterministic)
template <int EPI, bool SPLIT>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const GemmArgs args) {
  const GemmGroup& g = args.g[blockIdx.z];
  const int64_t MN = (int64_t)args.M * args.N;
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (idx >= MN) return;
  const int m = (int)(idx / args.N), n = (int)(idx - (int64_t)m * args.N);
  const float* p = args.ws + (int64_t)blockIdx.z * args.ksplit * MN + idx;
  f32x4 acc = *reinterpret_cast<const f32x4*>(p);
  for (int s = 1; s < args.ksplit; ++s) acc += *reinterpret_cast<const f32x4*>(p + s * MN);
  store4<EPI, SPLIT>(g, args, m, n, acc);
}

// K splits of the last gemm() call on this host thread (1: no split); with defer_reduce a split run leaves its
// slabs for the consumer (RowReduce, kernels.h) and skips the reduce launch
static thread_local int g_last_ks = 1;
constexpr int kMaxDeferKs = 8;   // tokens.hip apply_reduce holds at most this many slabs per row

template <int BM, int BN, int WMW, int WNW, int AM, bool SPLIT, int ST>
static void launch_splitk(const GemmArgs& a0, int epi, int ks, hipStream_t s) {
  GemmArgs a = a0;
  a.ksplit = ks;
  const int tiles_m = (a.M + BM - 1) / BM;
  a.gm = tiles_m < 8 ? tiles_m : 8;
  if (a.defer_reduce && a.groups == 1 && epi == EPI_RESID_F32 && ks <= kMaxDeferKs) {
    hipLaunchKernelGGL((gemm_kernel<BM, BN, WMW, WNW, EPI_PARTIAL, AM, SPLIT, ST>), dim3(tiles_m * (a.N / BN), ks, 1),
                       dim3(WMW * WNW * 64), 0, s, a);
    g_last_ks = ks;
    return;
  }
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WMW, WNW, EPI_PARTIAL, AM, SPLIT, ST>), dim3(tiles_m * (a.N / BN), ks, a.groups),
                     dim3(WMW * WNW * 64), 0, s, a);
  const dim3 rg((unsigned)(((int64_t)a.M * a.N / 4 + 255) / 256), 1, a.groups);
  switch (epi) {
    case EPI_BF16: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_BF16, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_GELU_BF16: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_GELU_BF16, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_RESID_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_RESID_F32, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_RELU_BF16: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_RELU_BF16, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_F32, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_RELU_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_RELU_F32, SPLIT>), rg, dim3(256), 0, s, a); break;
    case EPI_POS_F32: hipLaunchKernelGGL((splitk_reduce_kernel<EPI_POS_F32, SPLIT>), rg, dim3(256), 0, s, a); break;
    default: break;
  }
}

static int g_force_cfg = -1;   // tuning override (mmt_gemm_force_config), -1 = heuristic

template <bool SPLIT>
static void gemm_dispatch(const GemmArgs& a, int epi, hipStream_t s) {
  if constexpr (SPLIT) {   // tuning override of the f16x3 tile (MMT_SPLIT_CFG), dense A only
    static const int scfg = getenv("MMT_SPLIT_CFG") ? atoi(getenv("MMT_SPLIT_CFG")) : -1;
    if (scfg >= 0 && a.amode == A_DENSE) {
      switch (scfg) {
        case 0: return launch_cfg<128, 128, 4, 2, true, 2, 64>(a, epi, s);
        case 1: return launch_cfg<256, 128, 4, 2, true, 3, 32>(a, epi, s);
        case 2: return launch_cfg<128, 128, 2, 2, true, 2, 64>(a, epi, s);
        case 3: return launch_cfg<128, 128, 2, 2, true, 3, 32>(a, epi, s);
        case 4: return launch_cfg<256, 128, 4, 2, true, 2, 32>(a, epi, s);
        case 5: return launch_cfg<128, 256, 2, 4, true, 3, 32>(a, epi, s);
        case 6: return launch_cfg<256, 256, 2, 4, true, 2, 32>(a, epi, s);
        case 7: return launch_cfg<128, 128, 4, 2, true, 3, 32>(a, epi, s);
        case 8: return launch_cfg<128, 64, 2, 2, true, 2, 64>(a, epi, s);
        case 9: return launch_cfg<128, 128, 4, 2, true, 2, 32>(a, epi, s);
        case 10: return launch_cfg<128, 128, 2, 2, true, 2, 32>(a, epi, s);
        case 11: return launch_cfg<128, 64, 2, 2, true, 2, 32>(a, epi, s);
        case 12: return launch_cfg<128, 128, 4, 2, true, 4, 32>(a, epi, s);
        case 13: return launch_cfg<128, 256, 2, 4, true, 2, 32>(a, epi, s);
        case 14: if (launch256s_epi(a, epi, s)) return; break;
        case 15: if (a.N >= 2048 && launch256s_epi(a, epi, s)) return; break;
        case 16: return launch_cfg<64, 64, 2, 2, true, 8, 32>(a, epi, s);
        case 17: return launch_cfg<64, 64, 2, 2, true, 4, 32>(a, epi, s);
        case 18: return launch_cfg<64, 64, 2, 2, true, 6, 32>(a, epi, s);
        case 19: return launch_cfg<64, 64, 2, 2, true, 3, 64>(a, epi, s);
        default: break;
      }
    }
  }
  if constexpr (SPLIT) {
    // f16x3: the 8-phase 256 x 256 kernel where there are enough 256-wide column tiles (qkv, fc1: 250-300
    // TF/s vs 240-250 for the 2-barrier 128 x 128 kernel); N = 768 stays on 128-row tiles (3 column tiles of
    // 256 leave most CUs idle)
    static const int t256_min = getenv("MMT_256S_MIN") ? atoi(getenv("MMT_256S_MIN")) : 128;
    // the residual GEMMs (fc2, proj: N = 768) on the eight-phase kernel where its 256 x 256 tiles fill at least three
    // quarters of a round of the chip, counting the concurrent stream part: OSTrack-384's 720- and 548-token layers
    // (270 / 210 tiles; OSTrack 2 987 -> 3 045 frames/s with fc2 and proj at a full round, r06_ab_resid_256s.txt).  The
    // ViT layers' 120 tiles stay on the 128-row kernels: fc2 there lost 10 % (four times the work per tile lengthens
    // each stream half's chain).  MMT_RESID_256S: 0 never, 2 always (tuning)
    static const int resid_256s = getenv("MMT_RESID_256S") ? atoi(getenv("MMT_RESID_256S")) : 1;
    if (resid_256s && epi == EPI_RESID_F32 && a.groups == 1 && a.N % 256 == 0 &&
        (resid_256s == 2 || 4 * (a.conc > 1 ? a.conc : 1) * ((a.M + 255) / 256) * (a.N / 256) >= 3 * num_cus()) &&
        launch256s_epi(a, epi, s))
      return;
    // 320 x 256 tiles where they take fewer rounds of the one-workgroup-per-CU slots than 256 x 256 ones by more than
    // their 1.25x work per tile, counting the concurrent stream part (qkv of the 244-token layers, fc1 of the
    // 190-token ones at 2 x 16 sequences: two rounds -> one; OSTrack-384 2 914 -> 3 000 frames/s, r06_ab_t320_ostrack.txt;
    // ties, 5 rounds of 320-row tiles for 5 of 256-row ones, measured -0.6 %).  MMT_T320: 0 never, 1 the rule, 2 always
    // (tuning)
    static const int t320 = getenv("MMT_T320") ? atoi(getenv("MMT_T320")) : 1;
    bool use320 = false;
    if (t320 && a.groups == 1 && (epi == EPI_BF16 || epi == EPI_GELU_BF16)) {
      const int conc = a.conc > 1 ? a.conc : 1, slots = num_cus();
      const int r256 = (conc * ((a.M + 255) / 256) * (a.N / 256) + slots - 1) / slots;
      const int r320 = (conc * ((a.M + 319) / 320) * (a.N / 256) + slots - 1) / slots;
      use320 = t320 == 2 || 5 * r320 < 4 * r256;
    }
    // 128 x 256 two-group tiles (gemm128w_kernel) for the fp32-output N = 768 GEMMs where the 256-row kernel's tiles
    // would leave most CUs idle.  MMT_W256: 0 never, 1 the rule, 2 always (tuning); mmt_gemm_force_config(128) pins it
    static const int w256 = getenv("MMT_W256") ? atoi(getenv("MMT_W256")) : 1;
    if (g_force_cfg == 128 && launch128w_epi(a, epi, s)) return;
    if (w256 && g_force_cfg < 0 && epi == EPI_RESID_F32 && a.groups == 1 && a.N % 256 == 0 && a.N < 2048) {
      // the rule: its tiles fill at least 90 % of one round of the one-workgroup-per-CU slots, counting the concurrent
      // stream part, where 128 x 128 tiles would take two rounds or more
      const int conc = a.conc > 1 ? a.conc : 1, slots = num_cus();
      const int tw = conc * ((a.M + 127) / 128) * (a.N / 256), t128 = conc * ((a.M + 127) / 128) * (a.N / 128);
      if ((w256 == 2 || (tw <= slots && 10 * tw >= 9 * slots && t128 > slots)) && launch128w_epi(a, epi, s)) return;
    }
    const bool forced = g_force_cfg == 320 || g_force_cfg == 256;   // tests: pin the tile (any tile count)
    if (forced) use320 = g_force_cfg == 320 && (epi == EPI_BF16 || epi == EPI_GELU_BF16);
    if ((a.N >= 2048 || forced) && ((a.M + 255) / 256 * (a.N / 256) * a.groups >= t256_min || forced) &&
        launch256s_epi(a, epi, s, use320))
      return;
  }
  if constexpr (!SPLIT) {
    if (g_force_cfg >= 0 && a.amode == A_DENSE) {
      switch (g_force_cfg) {
        case 1: return launch_cfg<256, 128, 4, 2, false, 3>(a, epi, s);
        case 2: return launch_cfg<256, 128, 4, 2, false, 2>(a, epi, s);
        case 3: return launch_cfg<128, 128, 2, 2, false, 2>(a, epi, s);
        case 4: return launch_cfg<128, 128, 2, 2, false, 3>(a, epi, s);
        case 5: return launch_cfg<128, 128, 4, 2, false, 2>(a, epi, s);
        case 6: return launch_cfg<256, 256, 4, 2, false, 2>(a, epi, s);
        case 7: return launch_cfg<128, 256, 2, 4, false, 2>(a, epi, s);
        case 8: return launch_cfg<64, 128, 2, 2, false, 2>(a, epi, s);
        case 9: if (a.N % 256 == 0) return launch256_epi(a, epi, s); break;
        case 11: return launch_cfg<128, 128, 4, 2, false, 4, 32>(a, epi, s);
        case 12: return launch_cfg<128, 128, 4, 2, false, 3, 32>(a, epi, s);
        case 13: return launch_cfg<128, 64, 2, 2, false, 4, 32>(a, epi, s);
        case 14: return launch_cfg<256, 128, 4, 2, false, 3, 32>(a, epi, s);
        case 15: return launch_cfg<256, 128, 4, 2, false, 4, 32>(a, epi, s);
        case 16: if (launch_ring_epi<256, 128, 4, 2, 3, 32, 2>(a, epi, s)) return; break;
        case 17: if (launch_ring_epi<128, 128, 4, 2, 4, 32, 2>(a, epi, s)) return; break;
        case 18: if (launch_ring_epi<128, 128, 4, 2, 2, 64, 2>(a, epi, s)) return; break;
        case 19: if (launch_ring_epi<256, 256, 4, 2, 3, 32, 1>(a, epi, s)) return; break;
        case 20: if (launch_ring_epi<256, 128, 4, 2, 2, 64, 1>(a, epi, s)) return; break;
        case 21: return launch_cfg<128, 64, 4, 2, false, 2>(a, epi, s);
        case 22: return launch_cfg<64, 128, 2, 4, false, 2>(a, epi, s);
        case 23: return launch_cfg<128, 64, 4, 2, false, 3>(a, epi, s);
        case 24: return launch_cfg<64, 128, 2, 4, false, 3>(a, epi, s);
        case 10:
          if (a.N % 128 == 0 && a.groups == 1 && (epi == EPI_BF16 || epi == EPI_GELU_BF16))
            return epi == EPI_BF16 ? launch_persist<EPI_BF16>(a, s) : launch_persist<EPI_GELU_BF16>(a, s);
          break;
        default: break;
      }
    }
  }
  // Measured on the path's shapes (tests/bench_gemm.py, MI355X): 128x128 tiles with 8 waves (32x64
  // per wave) and a 2-deep LDS ring (64 KB, two workgroups per CU, so one tile's prologue/epilogue
  // overlaps the other's MFMAs) beat 256x128 / 256x256 / 3-deep rings on every K=768/3072 GEMM.
  const int target = 200;   // aim for at least ~one tile per CU of the 256
  const int t128 = (a.M + 127) / 128, t64 = (a.M + 63) / 64;
  // bf16-output GEMMs with several 128 x 128 tiles per workgroup slot: the persistent kernel (the next
  // tile's first K-tile loads under the current tile's tail)
  static const int persist_min = getenv("MMT_PERSIST_MIN") ? atoi(getenv("MMT_PERSIST_MIN")) : 1;
  if (!SPLIT && persist_min > 0 && a.amode == A_DENSE && a.groups == 1 && a.N % 128 == 0 &&
      t128 * (a.N / 128) >= persist_min * 2 * num_cus()) {
    if (epi == EPI_BF16) return launch_persist<EPI_BF16>(a, s);
    if (epi == EPI_GELU_BF16) return launch_persist<EPI_GELU_BF16>(a, s);
  }
  // a little under one 128 x 128 tile per CU (the N = 768 GEMMs of the CE-pruned layers): 128 x 64 tiles
  // with 8 waves put two workgroups on most CUs (fc2 at M = 4896: 41.4 -> 34.8 us)
  const int t128n = t128 * (a.N / 128) * a.groups;
  if constexpr (SPLIT) {
    // f16x3 N = 768 GEMMs (proj, fc2, patch): 128 x 128 tiles from 128 tiles up -- every M of the path in a
    // two-stream half (the 128 x 64 tiles that suit bf16's under-filled launches are slower here: the split
    // GEMMs are 3x longer per tile, and the other half fills the tail; from 64 tiles: +1.8 % vs 200 and +1.9 %
    // more vs 128 once the head convs (grouped, N = 3 x 128) take it too, sweep_t128.sh / ab_env.sh); a short
    // K streams 32-deep K-tiles (proj 51 -> 48 us, patch 98 -> 85 us at 32 sequences, tests/sweep_split_cfg_b32.sh),
    // fc2's K = 3072 keeps 64-deep ones (144 -> 135 us)
    static const int t128_min = getenv("MMT_SPLIT_T128") ? atoi(getenv("MMT_SPLIT_T128")) : 64;
    // (not for one sequence's few rows: fc1 at M = 320 keeps 240 64 x 64 workgroups instead of 72; the head's implicit
    // 3x3 conv, A_CONV3 with K = 6912, gathers 64-channel K-tiles)
    if (a.N % 128 == 0 && t128n >= t128_min && t128 >= 8) {
      // 128 x 192 tiles where all of them fit one round of the chip's one-workgroup-per-CU slots and 128 x 128 tiles
      // would take two or more, counting the launches of the other stream parts that run beside this one (a.conc):
      // the head's conv1 at 2 x 16 sequences (256 tiles in one round instead of 384: 287 -> 196 us alone), fc2 / proj
      // after candidate elimination (fc2 123.6 -> 107.4 us per launch; the line +0.8 %, profiles/r05_ab_t192.txt).
      // Where the 192-wide tiles take several rounds too (OSTrack-384's long layers: 3 against 5) they lost 1 %, so
      // a one-round fit is the rule.  MMT_T192: 0 never, 2 always (tuning)
      static const int t192 = getenv("MMT_T192") ? atoi(getenv("MMT_T192")) : 1;
      if (t192 && a.N % 192 == 0 && a.groups == 1 && (a.amode == A_CONV3 || a.K % 64 == 0)) {
        const int conc = a.conc > 1 ? a.conc : 1, slots = num_cus();
        const int r128 = (conc * t128 * (a.N / 128) + slots - 1) / slots;
        const int r192 = (conc * t128 * (a.N / 192) + slots - 1) / slots;
        if (t192 == 2 || (r192 == 1 && r128 >= 2)) return launch_cfg<128, 192, 4, 2, true, 2, 64>(a, epi, s);
      }
      // (the N = 768 GEMMs -- proj, patch -- take the register-pipelined 64-deep tile since it exists: proj at one
      // half's rows 31 -> 25 us (5 120 rows) .. 27 -> 22 us (2 432), tests/r3_run33.sh; the wide qkv / fc1 fallbacks
      // keep the 32-deep ring, level or better there)
      if (a.K <= 1024 && a.amode == A_DENSE && a.N > 768) return launch_cfg<128, 128, 4, 2, true, 2, 32>(a, epi, s);
      return launch_cfg<128, 128, 4, 2, true, 2, 64>(a, epi, s);
    }
  }
  if (a.N % 128 == 0 && t128n >= target && t128n < num_cus()) return launch_cfg<128, 64, 4, 2, SPLIT>(a, epi, s);
  if (a.N % 128 == 0 && t128n >= target) return launch_cfg<128, 128, 4, 2, SPLIT>(a, epi, s);
  if (a.N % 64 == 0) {
    if (t128 * (a.N / 64) * a.groups >= target) return launch_cfg<128, 64, 2, 2, SPLIT>(a, epi, s);
    // few 64 x 64 tiles and a long K (small batches): split K over workgroups (fp32 partials in the
    // workspace, fixed-order reduction with the epilogue), at least 4 K-tiles per split
    const int tiles = t64 * (a.N / 64) * a.groups, nk = a.K / 64;
    // (100, not 128: qkv of the 129..192-row CE layers at one sequence -- 108 tiles -- runs unsplit without its
    // reduce launch, 1092 -> 1100 frames/s, profiles/r05_ab_splitk_tiles_b1.txt)
    static const int sk_tiles = getenv("MMT_SPLITK_TILES") ? atoi(getenv("MMT_SPLITK_TILES")) : 100;
    static const int sk_target = getenv("MMT_SPLITK_TARGET") ? atoi(getenv("MMT_SPLITK_TARGET")) : 256;
    static const int sk_minkt = getenv("MMT_SPLITK_MINKT") ? atoi(getenv("MMT_SPLITK_MINKT")) : 4;
    static const int sk_max = getenv("MMT_SPLITK_MAX") ? atoi(getenv("MMT_SPLITK_MAX")) : 8;
    // slices per tile rounded DOWN, so the slices of every tile run in one round of workgroups (fc2 at one
    // sequence: 60 tiles x 4 = 240 workgroups of 768-deep slices beat 300 of 614 that take two rounds on 44
    // CUs; 823 -> 906 frames/s, round 2).  64 x 64 few-tile GEMMs with 8 waves (16 x 32 each): twice
    // the waves issuing each K-tile's LDS-DMA loads -- at one sequence these GEMMs are bound by what a CU can take in
    // (one tile per CU, ~400 KB of hi + lo operands at ~45 GB/s), 906 -> 929 frames/s against 4 waves
    // (tests/few_w8_ab.sh)
    if (a.ws && a.ws_elems > 0 && tiles < sk_tiles && nk >= 2 * sk_minkt) {
      int ks = sk_target / tiles;
      ks = ks < nk / sk_minkt ? ks : nk / sk_minkt;
      ks = ks < sk_max ? ks : sk_max;
      while (ks > 1 && (int64_t)ks * a.groups * a.M * a.N > a.ws_elems) --ks;
      if (ks > 1) {
        // f16x3: a 3-deep ring (96 KB of LDS) beat 4-deep at one sequence (tests/sweep_ring_b1.sh)
        constexpr int SKST = SPLIT ? 3 : 4;
        if (a.amode == A_CONV3) return launch_splitk<64, 64, 4, 2, A_CONV3, SPLIT, SKST>(a, epi, ks, s);
        return launch_splitk<64, 64, 4, 2, A_DENSE, SPLIT, SKST>(a, epi, ks, s);
      }
    }
    // few tiles (small batches): each workgroup walks the whole K serially, so keep K-tiles in flight
    // (bf16: 4-deep LDS ring, an 8-deep one measured no better at M = 320; f16x3: 3-deep, qkv 17.3 ->
    // 15.4 us and fc1 16.8 -> 16.5 us at one sequence, tests/sweep_ring_b1.sh)
    if (a.K >= 6 * 64) return launch_cfg<64, 64, 4, 2, SPLIT, SPLIT ? 3 : 4>(a, epi, s);
    return launch_cfg<64, 64, 2, 2, SPLIT>(a, epi, s);
  }
  if (t64 * (a.N / 32) * a.groups >= target) return launch_cfg<64, 32, 4, 1, SPLIT>(a, epi, s);
  return launch_cfg<32, 32, 2, 1, SPLIT>(a, epi, s);
}

int gemm(const GemmArgs& a, int epi, hipStream_t s) {
  g_last_ks = 1;
  // the f16x3 16-bit epilogues (gemm_kernel's staged split epilogue, gemm256s) always store a lo plane: a caller
  // without one is a programming error, not a bf16 fallback
  if (a.split && epi_is_bf16(epi))
    for (int i = 0; i < a.groups; ++i)
      if (!a.g[i].C_lo) {
        fprintf(stderr, "mmt: f16x3 GEMM with a 16-bit epilogue needs C_lo (group %d)\n", i);
        abort();
      }
  if (a.split)
    gemm_dispatch<true>(a, epi, s);
  else
    gemm_dispatch<false>(a, epi, s);
  return g_last_ks;
}

void gemm_force_config(int cfg) { g_force_cfg = cfg; }

int gemm_set_stamps(void* dev_buf) {
  unsigned long long* p = static_cast<unsigned long long*>(dev_buf);
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_stamps), &p, sizeof(p)) == hipSuccess ? 0 : -1;
}

}  // namespace mmt
