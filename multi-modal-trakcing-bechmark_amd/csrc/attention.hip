// Joint template-search self-attention (attn.py:33-59) with the candidate-
// elimination side output (attn_blocks.py:44-53), gfx950.
//
// One workgroup = WAVES waves, each wave 16 query rows of one (sequence, head).
// K/V tiles of 64 keys are staged in LDS as 16-B chunks, both row-major with
// the chunk XOR-swizzled by row; V^T fragments come from ds_read_b64_tr_b16
// (the hardware transposed read), so staging is a straight copy.  Workgroups
// of one (sequence, head) are mapped to one XCD (their K/V tiles are shared
// through that XCD's L2).  Scores are computed swapped, S^T = K Q^T, with
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
typedef __attribute__((address_space(3))) bf16x4* lds_bf16x4_t;
typedef __attribute__((address_space(3))) void* lds_void_t;

constexpr int KB = 64;         // keys per LDS tile
constexpr int CE_MAX = 1024;   // max tokens for the exported CE row
// bf16 kernels of 4+ waves: ask for 4 waves per SIMD (114 VGPRs instead of 128 + 16 AGPRs -> 3 waves)
#ifndef ATTN_WPE
#define ATTN_WPE 4
#endif
// f16x3 4-wave kernel: no cap (145 VGPRs + 16 AGPRs, 3 waves per SIMD); 4 waves per SIMD spills 13 VGPRs
#ifndef ATTN_WPE_SPLIT
#define ATTN_WPE_SPLIT 1
#endif

// byte offset of 16-B chunk c of row r in a [64][64] bf16 tile (128-B rows, chunk XOR row)
__device__ __forceinline__ int tile_off(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

// KSPLIT: the WAVES waves of a workgroup share ONE 16-query row block and split its keys (wave w takes key
// tiles w, w + WAVES, ...; each stages its own tiles), then merge their (max, sum, O) in wave order -- for
// few (sequence, head) pairs (one sequence: 12), where a lone wave per row block would load every K / V tile
// by itself
template <int WAVES, bool SPLIT, int RB = 1, bool KSPLIT = false>
// (the 8-wave f16x3 kernel is held to 128 VGPRs: two workgroups per CU)
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(WAVES < 4 || KSPLIT ? 1 : (SPLIT ? (WAVES >= 8 ? 4 : ATTN_WPE_SPLIT) : ATTN_WPE)))) void attn_kernel(const AttnArgs a) {
  // SPLIT (fp32-faithful f16x3, common.h): every operand is an (hi, lo) fp16 pair of a range-scaled
  // value and each product is hi*hi + lo*hi + hi*lo; the LDS images of K and V^T hold both halves.
  // RB: 16-query row blocks per wave, multiplied together against each K / V fragment (fragment
  // reads shared, RB independent softmax chains interleaved).
  static_assert(RB == 1 || !SPLIT, "split mode uses one row block per wave");
  static_assert(RB == 1 || !KSPLIT, "key split: one row block");
  constexpr int NH = SPLIT ? 2 : 1;
  constexpr int QW = 16 * RB;   // queries per wave
  constexpr int QWAVES = KSPLIT ? 1 : WAVES;   // waves with distinct queries
  // DMA: K / V tiles go HBM -> LDS by buffer_load ... lds (no VGPRs, no LDS writes by the waves) into a ring of two
  // stages, one barrier per tile.  The key split, and the f16x3 kernels of fewer than 8 waves (whose 68-KB ring
  // would cost them workgroups per CU), stage through registers into one slot per wave / per workgroup.
  constexpr bool DMA = !KSPLIT && (WAVES >= 8 || !SPLIT);
  constexpr int KW = KSPLIT ? WAVES : (DMA ? 2 : 1);   // K / V staging slots (per wave, ring stages, or one)
  // CE_V: the 5-wave key split (N <= 320, one key tile per wave) fills all 160 KB with its K / V slots, so each wave
  // keeps its tile's CE logits in registers and stores them after the loop into the V slots' space (free by then)
  constexpr bool CE_V = KSPLIT && WAVES == 5;
  constexpr int KV_BYTES = KW * NH * KB * 64 * 2;   // the K (or V) slots
  __shared__ __attribute__((aligned(16))) char lds_raw[2 * KV_BYTES + (CE_V ? 0 : CE_MAX * 4)];
  bf16_t(&KsAll)[KW][NH][KB * 64] = *reinterpret_cast<bf16_t(*)[KW][NH][KB * 64]>(lds_raw);
  bf16_t(&VsAll)[KW][NH][KB * 64] = *reinterpret_cast<bf16_t(*)[KW][NH][KB * 64]>(lds_raw + KV_BYTES);
  float* const ce_row = reinterpret_cast<float*>(lds_raw + (CE_V ? KV_BYTES : 2 * KV_BYTES));
  float cel[CE_V ? 16 : 1];
  int cekb = -1;

  // XCD-aware order: logical id = (b * heads + h) * nqt + qt; blocks bid, bid + 8, ... (one XCD) take a
  // contiguous logical range, so the query tiles of one (b, h) share an L2
  const int nqt = (a.N + QW * QWAVES - 1) / (QW * QWAVES);
  const int nblk = nqt * a.heads * a.B;
  const int bid = blockIdx.x, xcd = bid & 7, jx = bid >> 3;
  const int q8 = nblk >> 3, r8 = nblk & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + jx;
  const int qt = lid % nqt, bh = lid / nqt;
  const int b = bh / a.heads, h = bh - b * a.heads;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int N = a.N, Cd = 64 * a.heads, C3 = 3 * Cd;
  const bf16_t* base = a.qkv + (int64_t)b * N * C3;
  const int q0 = qt * (QW * QWAVES) + (KSPLIT ? 0 : wave * QW);
  const int g = lane >> 4;

  const bf16_t* base_lo = SPLIT ? a.qkv_lo + (int64_t)b * N * C3 : nullptr;
  bf16x8 qf[RB][NH][2];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int qi = q0 + 16 * rb + (lane & 15);
#pragma unroll
    for (int hl = 0; hl < NH; ++hl)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16_t* bb = hl ? base_lo : base;
        if (qi < N) {
          // the softmax scale 64^-0.5 = 2^-3 folded into Q: exact in bf16, and MFMA products and sums
          // commute with a power-of-two scale, so S = K (Q / 8)^T is the scaled score bit for bit
          const bf16x8 qv = *reinterpret_cast<const bf16x8*>(bb + (int64_t)qi * C3 + h * 64 + 32 * s + 8 * g);
          if (SPLIT) {   // f16x3: the 1/8 is folded into qk_inv
            qf[rb][hl][s] = qv;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) qf[rb][hl][s][e] = (__bf16)((float)qv[e] * 0.125f);
          }
        } else {
          qf[rb][hl][s] = bf16x8{};
        }
      }
  }

  f32x4 o[RB][4];
  float m[RB], l[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[rb][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    m[rb] = -INFINITY;
    l[rb] = 0.f;
  }
  const float qks = SPLIT ? a.qk_inv : 1.0f;   // the logits' scale (f16x3: applied in the exponent, see below)
  const bool ce_wave = a.ce_query >= q0 && a.ce_query < q0 + QW;
  const int ce_rb = ce_wave ? (a.ce_query - q0) >> 4 : -1;
  const bool ce_lane = ce_wave && (lane & 15) == ((a.ce_query - q0) & 15);

  // K/V staging, software-pipelined: the next tile's 16-B chunks are loaded into registers while the
  // current tile is multiplied, then copied to LDS
  constexpr int NCHUNK = NH * KB * 8;                               // 16-B chunks of K (and of V) per tile
  constexpr int LT = KSPLIT ? 64 : WAVES * 64;                      // threads staging one tile
  constexpr int NCHT = (NCHUNK + LT - 1) / LT;                      // per thread
  constexpr bool CH_EXACT = NCHUNK % LT == 0;
  const int ltid = KSPLIT ? lane : tid;
  // a key-split wave syncs only with itself: its LDS operations complete in order
  auto tile_sync = [&]() {
    if constexpr (KSPLIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else __syncthreads();
  };
  // LDS-DMA pieces: one wave-instruction fills 8 key rows x 128 B of one image (K or V, hi or lo); lane l lands at
  // byte 16 l of the piece = row l >> 3, chunk position l & 7, so it loads the source chunk (l & 7) ^ (l >> 3) that
  // tile_off puts there.  Keys past N read zeros (offset past the resource).
  constexpr int NPIECE = 2 * NH * 8, PPW = NPIECE / WAVES;
  static_assert(!DMA || NPIECE % WAVES == 0, "pieces must divide over the waves");
  const rsrc_t rq = make_rsrc(base, (int64_t)N * C3 * 2);
  const rsrc_t rql = SPLIT ? make_rsrc(base_lo, (int64_t)N * C3 * 2) : rq;
  auto issue = [&](int kb, int st) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int p = wave * PPW + j;                        // wave-uniform
      const int kv = p / (8 * NH), hl = (p / 8) % NH, rb = p % 8;
      const int key = kb + rb * 8 + (lane >> 3), c = (lane & 7) ^ (lane >> 3);
      const uint32_t vo = key < N ? (uint32_t)(((int64_t)key * C3 + (kv ? 2 * Cd : Cd) + h * 64 + c * 8) * 2) : kBufOob;
      bf16_t* img = kv ? &VsAll[st][hl][0] : &KsAll[st][hl][0];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(hl ? rql : rq, (lds_void_t)(img + rb * 8 * 64), 16, vo, 0, 0, 0);
    }
  };

  uint4 kreg[NCHT], vreg[NCHT];
  auto fetch = [&](int kb) {
#pragma unroll
    for (int i = 0; i < NCHT; ++i) {
      const int q = ltid + i * LT;
      if (!CH_EXACT && q >= NCHUNK) break;
      const int hl = q / (KB * 8), qq = q - hl * (KB * 8);
      const int r = qq >> 3, c = qq & 7, key = kb + r;
      kreg[i] = make_uint4(0, 0, 0, 0);
      vreg[i] = make_uint4(0, 0, 0, 0);
      if (key < N) {
        const bf16_t* row = (hl ? base_lo : base) + (int64_t)key * C3 + h * 64 + c * 8;
        kreg[i] = *reinterpret_cast<const uint4*>(row + Cd);
        vreg[i] = *reinterpret_cast<const uint4*>(row + 2 * Cd);
      }
    }
  };
  const int kb0 = KSPLIT ? wave * KB : 0;
  constexpr int KSTEP = KSPLIT ? WAVES * KB : KB;
  if constexpr (DMA) {
    if (kb0 < N) issue(kb0, 0);
  } else {
    if (kb0 < N) fetch(kb0);
  }
  int stage = 0;
#ifdef ATTN_STAMPS
  // tuning build (abx variant, never the product): wave 0's cycles per loop part, summed over the key tiles and printed
  // by the first workgroups -- landed (this tile's DMA waited for), wait (the barrier + the next tile's issue), S issue,
  // softmax (incl. the S results), PV issue
  unsigned long long st_l = 0, st_w = 0, st_s = 0, st_x = 0, st_p = 0, st_t0 = __builtin_amdgcn_s_memtime(), st_q = 0, st_e = 0;
  int st_n = 0;
#define ATTN_ST(v)                                            \
  do {                                                        \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    v += t_ - st_q;                                           \
    st_q = t_;                                                \
  } while (0)
#else
#define ATTN_ST(v) do { } while (0)
#endif
  for (int kb = kb0; kb < N; kb += KSTEP) {
#ifdef ATTN_STAMPS
    st_q = __builtin_amdgcn_s_memtime();
    ++st_n;
#endif
    if constexpr (DMA) {
      // this tile's pieces landed (the only loads in flight) and every wave is past the previous tile, whose
      // stage then takes the next tile
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      ATTN_ST(st_l);
      __builtin_amdgcn_s_barrier();
      if (kb + KSTEP < N) issue(kb + KSTEP, stage ^ 1);
      ATTN_ST(st_w);
    } else {
      tile_sync();
#pragma unroll
      for (int i = 0; i < NCHT; ++i) {
        const int q = ltid + i * LT;
        if (!CH_EXACT && q >= NCHUNK) break;
        const int hl = q / (KB * 8), qq = q - hl * (KB * 8);
        const int r = qq >> 3, c = qq & 7;
        *reinterpret_cast<uint4*>(reinterpret_cast<char*>(KsAll[KSPLIT ? wave : 0][hl]) + tile_off(r, c)) = kreg[i];
        *reinterpret_cast<uint4*>(reinterpret_cast<char*>(VsAll[KSPLIT ? wave : 0][hl]) + tile_off(r, c)) = vreg[i];
      }
      tile_sync();
      if (kb + KSTEP < N) fetch(kb + KSTEP);
    }
    bf16_t(&Ks)[NH][KB * 64] = KsAll[DMA ? stage : (KSPLIT ? wave : 0)];
    bf16_t(&Vs)[NH][KB * 64] = VsAll[DMA ? stage : (KSPLIT ? wave : 0)];
    stage ^= 1;
    // a wave whose queries all lie past N (the last query tile of a sequence: at 153 tokens 6 of its 8 waves) still
    // stages its share of the K / V tiles and meets the barriers, but multiplies nothing: its MFMA and softmax issue
    // slots go to the other waves of its SIMDs (wave-uniform)
    if (!KSPLIT && q0 >= N) continue;

    f32x4 sc[RB][4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) sc[rb][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r = 16 * t + (lane & 15), c = 4 * s + g;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(Ks[0]) + tile_off(r, c));
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) sc[rb][t] = mfma16<SPLIT>(kf, qf[rb][0][s], sc[rb][t]);
        if (SPLIT) {
          const bf16x8 kl =
              *reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(Ks[NH - 1]) + tile_off(r, c));
          sc[0][t] = mfma16<SPLIT>(kl, qf[0][0][s], sc[0][t]);
          sc[0][t] = mfma16<SPLIT>(kf, qf[0][NH - 1][s], sc[0][t]);
        }
      }
      // (f16x3: S = (K s)(Q s)^T / s^2 / 8 -- qk_inv, a power of two, is folded into the exponent's scale below:
      // the same bits as scaling the scores, 16 multiplies fewer per tile)
    }
    ATTN_ST(st_s);
    bf16x8 pf[RB][2], pl[RB][2];
    const bool tail = kb + KB > N;   // only the last key tile has keys past N (wave-uniform)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      float bmax = -INFINITY;
      if (tail) {
        const int lim = N - kb - 4 * g;   // this lane's keys 16 t + 4 g + r are valid below N
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * t + r >= lim) sc[rb][t][r] = -INFINITY;
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) bmax = fmaxf(bmax, sc[rb][t][r]);
      bmax = xmax16(bmax);   // xor 16, xor 32 by permlane half-exchanges (no LDS round trip)
      bmax = xmax32(bmax);
      if (ce_lane && rb == ce_rb) {
        // the tile's 64 logits (keys past N land in ce_row's slack, CE_MAX >= N + 64, and are never read)
        if constexpr (CE_V) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) cel[4 * t + r] = sc[rb][t][r];
          cekb = kb;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) ce_row[kb + 16 * t + 4 * g + r] = sc[rb][t][r];
        }
      }
      // f16x3: m, the logits and ce_row stay in the unscaled units of the accumulator; the scale qk_inv = 2^k
      // enters through lg = qk_inv log2(e) (exact: a power of two times log2(e)), so fma(s, lg, -m lg) is bit for bit
      // fma(s qk_inv, log2(e), -(m qk_inv) log2(e)) and the maxima commute with the positive scale
      const float lg = qks * 1.44269504f;
      const float mnew = fmaxf(m[rb], bmax);
      const float alpha = __expf((m[rb] - mnew) * qks);
      // p = e^(s - m) = 2^(s log2e - m log2e): one FMA + v_exp_f32 per score
      const float ml2 = mnew * lg;
      float psum = 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(sc[rb][t][r], lg, -ml2));
          sc[rb][t][r] = p;
          psum += p;
        }
      psum = xsum16(psum, psum);
      psum = xsum32(psum, psum);
      l[rb] = l[rb] * alpha + psum;
      m[rb] = mnew;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[rb][dt] *= alpha;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (SPLIT) {   // f16x3 halves of p * 2^14
            uint16_t h0, l0, h1, l1;
            split_h(sc[rb][2 * u][r] * 16384.0f, h0, l0);
            split_h(sc[rb][2 * u + 1][r] * 16384.0f, h1, l1);
            pf[rb][u][r] = __builtin_bit_cast(__bf16, h0);
            pf[rb][u][4 + r] = __builtin_bit_cast(__bf16, h1);
            pl[rb][u][r] = __builtin_bit_cast(__bf16, l0);
            pl[rb][u][4 + r] = __builtin_bit_cast(__bf16, l1);
          } else {
            pf[rb][u][r] = (__bf16)sc[rb][2 * u][r];
            pf[rb][u][4 + r] = (__bf16)sc[rb][2 * u + 1][r];
          }
        }
    }

    ATTN_ST(st_x);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      // V^T fragment of keys {32u + 4g + 0..3} and {32u + 16 + 4g + 0..3} (the P element order) at
      // dim 16 dt + (lane & 15): two transposed reads; lane 4q + p of a 16-lane group addresses key
      // row q, dims 16 dt + 4p .. + 3
      const int qq = (lane & 15) >> 2, pp = lane & 3;
      const int vrow = 32 * u + 4 * g + qq;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int c = 2 * dt + (pp >> 1), half = (pp & 1) * 8;
        const int oA = tile_off(vrow, c) + half, oB = tile_off(vrow + 16, c) + half;
        const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(reinterpret_cast<char*>(Vs[0]) + oA));
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(reinterpret_cast<char*>(Vs[0]) + oB));
        const bf16x8 vf = __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) o[rb][dt] = mfma16<SPLIT>(vf, pf[rb][u], o[rb][dt]);
        if (SPLIT) {
          const bf16x4 w0 =
              __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(reinterpret_cast<char*>(Vs[NH - 1]) + oA));
          const bf16x4 w1 =
              __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t)(reinterpret_cast<char*>(Vs[NH - 1]) + oB));
          const bf16x8 vl = __builtin_shufflevector(w0, w1, 0, 1, 2, 3, 4, 5, 6, 7);
          o[0][dt] = mfma16<SPLIT>(vl, pf[0][u], o[0][dt]);
          o[0][dt] = mfma16<SPLIT>(vf, pl[0][u], o[0][dt]);
        }
      }
    }
    ATTN_ST(st_p);
  }
#ifdef ATTN_STAMPS
  st_e = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0 && blockIdx.x < 24)
    printf("attn_stamps block %d waves %d N %d tiles %d: total %llu wait %llu s %llu softmax %llu pv %llu landed %llu\n",
           (int)blockIdx.x, WAVES, N, st_n, st_e - st_t0, st_w, st_s, st_x, st_p, st_l);
#endif

  if constexpr (KSPLIT) {
    // merge the waves' partial softmax states in wave order: m = max m_w, l = sum l_w e^(m_w - m),
    // O = sum O_w e^(m_w - m); the K / V slots are free once every wave is past its last tile
    __syncthreads();
    if constexpr (CE_V) {   // each wave's tile of the CE query's logits, now that every V slot is free
      if (ce_lane && cekb >= 0)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) ce_row[cekb + 16 * t + 4 * g + r] = cel[4 * t + r];
    }
    float* st = reinterpret_cast<float*>(&KsAll[0][0][0]);   // [WAVES][18][64]
    if (wave > 0) {
      float* my = st + wave * 18 * 64 + lane;
      my[0] = m[0];
      my[64] = l[0];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) my[(2 + 4 * dt + r) * 64] = o[0][dt][r];
    }
    __syncthreads();
    if (wave > 0) return;
    float mw[WAVES];
    mw[0] = m[0];
    float mm = m[0];
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
      mw[w] = st[w * 18 * 64 + lane];
      mm = fmaxf(mm, mw[w]);
    }
    const float f0 = __expf((mw[0] - mm) * qks);
    float ll = l[0] * f0;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[0][dt] *= f0;
#pragma unroll
    for (int w = 1; w < WAVES; ++w) {
      const float* ow = st + w * 18 * 64 + lane;
      const float f = __expf((mw[w] - mm) * qks);
      ll += ow[64] * f;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[0][dt][r] += ow[(2 + 4 * dt + r) * 64] * f;
    }
    m[0] = mm;
    l[0] = ll;
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int qi = q0 + 16 * rb + (lane & 15);
    const float inv = SPLIT ? a.pv_inv / l[rb] : 1.0f / l[rb];
    if (qi < N) {
      const int64_t orow = ((int64_t)b * N + qi) * Cd + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        float v[4];
        uint16_t hv[4], lv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = o[rb][dt][r] * inv;
          if (SPLIT) split_h(v[r] * a.out_scale, hv[r], lv[r]);
          else hv[r] = f2bf(v[r]);
        }
        *reinterpret_cast<uint2*>(a.out + orow + 16 * dt + 4 * g) =
            make_uint2((uint32_t)hv[0] | ((uint32_t)hv[1] << 16), (uint32_t)hv[2] | ((uint32_t)hv[3] << 16));
        if (SPLIT)
          *reinterpret_cast<uint2*>(a.out_lo + orow + 16 * dt + 4 * g) =
              make_uint2((uint32_t)lv[0] | ((uint32_t)lv[1] << 16), (uint32_t)lv[2] | ((uint32_t)lv[3] << 16));
      }
    }
  }
  if constexpr (!KSPLIT) __syncthreads();   // (key split: every wave's ce_row logits landed before the merge)
  if (ce_wave) {
    const int src = (a.ce_query - q0) & 15;
    float cm = m[0], cl = l[0];
#pragma unroll
    for (int rb = 1; rb < RB; ++rb)
      if (rb == ce_rb) {
        cm = m[rb];
        cl = l[rb];
      }
    const float mm = __shfl(cm, src, 64), ll = __shfl(cl, src, 64);
    const int Ls = N - a.ce_lens_t;
    float* dst = a.ce_prob + ((int64_t)b * a.heads + h) * Ls;
    for (int j = lane; j < Ls; j += 64) dst[j] = __expf((ce_row[a.ce_lens_t + j] - mm) * qks) / ll;
  }
}

template <bool SPLIT>
static void attention_t(const AttnArgs& a, hipStream_t s) {
  const int per4 = a.B * a.heads * ((a.N + 63) / 64);
  const int bh = a.B * a.heads;
  // long joint sequences (OSTrack-384, N = 720) in bf16: 8 waves x 16 queries per workgroup -- one
  // K/V staging shared by 128 queries, half the L2 re-reads of 4 waves (-24 % kernel time, +2.5 %
  // end to end; at the ViPT lengths N <= 320 it measured level in isolation and -0.4 % end to end)
  static const int w8 = getenv("MMT_ATTN_W") ? atoi(getenv("MMT_ATTN_W")) : 0;
  static const bool ks4 = getenv("MMT_ATTN_NOKS") == nullptr;   // tuning: one wave per row block instead
  if (!SPLIT && bh >= 128 && (w8 == 8 || (w8 == 0 && a.N > 320))) {
    hipLaunchKernelGGL((attn_kernel<8, false>), dim3((a.N + 127) / 128 * bh), dim3(512), 0, s, a);
    return;
  }
  // f16x3: 8 waves share one K / V (hi + lo) staging -- 116 VGPRs (4 waves per SIMD, no spills) against 145 +
  // 16 AGPRs for 4 waves (+0.6 % end to end at 32 sequences, tests/ab_env.sh)
  if (SPLIT && bh >= 128 && (w8 == 8 || w8 == 0)) {
    hipLaunchKernelGGL((attn_kernel<8, true>), dim3((a.N + 127) / 128 * bh), dim3(512), 0, s, a);
    return;
  }
  if (per4 >= 240) {
    hipLaunchKernelGGL((attn_kernel<4, SPLIT>), dim3((a.N + 63) / 64 * bh), dim3(256), 0, s, a);
  } else if (per4 * 2 >= 240) {
    hipLaunchKernelGGL((attn_kernel<2, SPLIT>), dim3((a.N + 31) / 32 * bh), dim3(128), 0, s, a);
  } else if (SPLIT && ks4) {
    // few (sequence, head) pairs: 4 waves split the keys of each 16-query block (one sequence, N = 320:
    // 240 workgroups whose K / V tiles load 4 waves at a time instead of one).  f16x3 only: the merge
    // changes the fp32 rounding with the batch size, which the bf16 mode keeps bit-exact (its kernel
    // choice does not change a query's arithmetic; test_batch_equals_single)
    // (257..320 keys: five tiles, so five waves take one each instead of the first wave taking two; MMT_ATTN_KS5=0,
    // tuning: four)
    static const bool ks5 = !getenv("MMT_ATTN_KS5") || atoi(getenv("MMT_ATTN_KS5")) != 0;
    if (ks5 && a.N > 4 * KB && a.N <= 5 * KB)
      hipLaunchKernelGGL((attn_kernel<5, SPLIT, 1, true>), dim3((a.N + 15) / 16 * bh), dim3(320), 0, s, a);
    else
      hipLaunchKernelGGL((attn_kernel<4, SPLIT, 1, true>), dim3((a.N + 15) / 16 * bh), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_kernel<1, SPLIT>), dim3((a.N + 15) / 16 * bh), dim3(64), 0, s, a);
  }
}

void attention(const AttnArgs& a, hipStream_t s) {
  if (a.qkv_lo)
    attention_t<true>(a, s);
  else
    attention_t<false>(a, s);
}

}  // namespace mmt
