// DiMP / mfDiMP target-classifier inner loop on gfx950 (fp32):
//   apply_filter           RGBD/models/DeT/ltr/models/layers/filter.py:5-54   (per-sequence correlation, pad k//2)
//   apply_feat_transpose   filter.py:57-148   (its filter gradient)
//   DistanceMap + label / target-mask / spatial-weight predictors   distance.py:17-39, optimizer.py:111-125
//   DiMPSteepestDescentGN  optimizer.py:132-168  (LeakyReluPar score activation, Gauss-Newton step length)
// All reductions are block-partial arrays combined in fixed order (bitwise reproducible, no atomics).
#include "dimp.h"

namespace mmt {

__global__ __launch_bounds__(256) void dimp_maps_kernel(DimpMaps m) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int n = m.Ho * m.Wo;
  if (idx >= m.IS * n) return;
  const int is = idx / n, p = idx - is * n;
  if (m.ctl && m.ctl[is % m.S].num_iter <= 0) return;
  const int y = p / m.Wo, x = p - y * m.Wo;
  const float d0 = (float)y - m.centers[2 * is], d1 = (float)x - m.centers[2 * is + 1];
  const float dist = sqrtf(d0 * d0 + d1 * d1);
  float lab = 0.f, msk = 0.f, spw = 0.f;
  for (int k = 0; k < m.nbins; ++k) {
    const float diff = dist / m.bin_disp - (float)k;
    const float v = k < m.nbins - 1 ? fmaxf(1.0f - fabsf(diff), 0.f) : fminf(fmaxf(1.0f + diff, 0.f), 1.f);
    lab += m.label_w[k] * v;
    msk += m.mask_w[k] * v;
    spw += m.spatial_w[k] * v;
  }
  m.label[idx] = lab;
  m.mask[idx] = 1.0f / (1.0f + expf(-msk));
  m.sw[idx] = m.sqrt_sw[is] * spw;
}

// Both correlation kernels stage their operands through the LDS in double-buffered chunks: each thread
// issues its share of the next chunk's global loads (kDimpStage registers) before it multiplies the current
// one, so a chunk's load latency hides under the previous chunk's FMAs.  Out-of-map taps are staged as
// zeros (the padded image), so the inner loops carry no bounds checks; a zero tap adds an exact zero.

// scores[i,s,y,x] = sum_c,ky,kx feat[i,s,c,y+ky-P,x+kx-P] * w[s,c,ky,kx]; mode 1/2 epilogues below.
// One workgroup per (image * sequence, band of RB output rows, RB * Wo <= 64 positions): the 4 waves take
// interleaved channels (c = wave + 4 k) of chunks of CC channels, every lane one output position; the 4
// partial sums combine in a fixed order, the band's squares (mode 1 / 2) in position order into
// partial[is][band].  ctl: sequence s skips (no output) when it >= ctl[s].num_iter or i >= n_samples.
// STRIP (4 x 4 filters, <= 16 four-position strips per band, CC % 16 == 0): register-blocked -- lane (strip,
// channel subgroup) keeps four adjacent positions' sums and reads each feature value once per 4 x 7 window row
// (8-B reads) and its channel's 16 weights as four 16-B reads: 20 LDS reads per 64 FMAs instead of 32 per 16; the
// 16 channel groups (c = group + 16 k) combine in group order.  Explicit fmaf: a `+=` of a product lets the backend
// split some of them into a separately rounded multiply and add (it did, for packed pairs, in one build), so the bits
// would depend on instruction selection.
// STG: staged floats per thread and chunk (kDimpStage; 10 for the STRIP kernel's 16-channel chunks, its default:
// 72 -> 30 staging / offset registers, four workgroups per CU)
template <int FH, int FW, bool STRIP = false, int STG = kDimpStage>
__global__ __launch_bounds__(256) void dimp_filter_kernel(DimpFilter a) {
  extern __shared__ float sm[];   // 2 x ([CC][rows][Wp] padded feature rows + [CC][T] weights)
  __shared__ float red[STRIP ? 16 : 4][64];
  if constexpr (FH > 0) {
    a.fh = FH;
    a.fw = FW;
  }
  const int is = blockIdx.x, band = blockIdx.y;
  const int i = is / a.S, s = is - i * a.S;
  if (a.ctl && (a.it >= a.ctl[s].num_iter || i >= a.ctl[s].n_samples)) return;   // uniform over the workgroup
  const int T = a.fh * a.fw, P0 = a.fh / 2, P1 = a.fw / 2;
  const int y0 = band * a.RB, nrow = min(a.RB, a.Ho - y0);
  const int Wp = a.Wo + a.fw - 1, plane = (a.RB + a.fh - 1) * Wp, CC = a.CC;
  const int fsz = CC * plane, stage = fsz + CC * T;
  const float* f = a.feat + (int64_t)i * a.img_stride + (int64_t)s * a.seq_stride;
  const float* wsrc = a.w + (int64_t)s * a.C * T;
  const int nch = (a.C + CC - 1) / CC;
  const int t = threadIdx.x;
  // each staged element's source offset within its chunk (fixed over the chunks; -1: a zero pad tap), so a
  // chunk's fetch is one add and one load per register
  int soff[STG];
#pragma unroll
  for (int k = 0; k < STG; ++k) {
    const int e = t + k * 256;
    int o = -1;
    if (e < fsz) {
      const int c = e / plane, r = e - c * plane, py = r / Wp, px = r - py * Wp;
      const int yy = y0 + py - P0, xx = px - P1;
      if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) o = c * a.H * a.W + yy * a.W + xx;
    } else if (e < stage) {
      o = e - fsz;
    }
    soff[k] = o;
  }
  // the STRIP kernel keeps two chunks in flight (registers ra / rb alternate; its multiply is short enough that one
  // chunk's latency was the bound), the 4-group kernel one (ra)
  float ra[STG], rb[STG];
  auto fetch = [&](int ch, float (&rg)[STG]) {
    const float* fb = f + (int64_t)ch * CC * a.H * a.W;   // C % CC == 0 (dimp_geo)
    const float* wb = wsrc + ch * CC * T;
#pragma unroll
    for (int k = 0; k < STG; ++k) {
      const int e = t + k * 256;
      rg[k] = soff[k] < 0 ? 0.f : (e < fsz ? fb : wb)[soff[k]];
    }
  };
  auto put = [&](int buf, const float (&rg)[STG]) {
    float* d = sm + buf * stage;
#pragma unroll
    for (int k = 0; k < STG; ++k) {
      const int e = t + k * 256;
      if (e < stage) d[e] = rg[k];
    }
  };
  const int g = t >> 6, slot = t & 63;
  const int ly = slot / a.Wo, x = slot - ly * a.Wo;
  const bool pv = slot < nrow * a.Wo;
  float acc = 0.f;
  // STRIP: lane = strip (ly_s, 4 sx) + 16 x channel subgroup; channel group cg = 4 g + subgroup
  const int nsx = (a.Wo + 3) >> 2, st = t & 15, cg = 4 * g + ((t >> 4) & 3);
  const int sly = st / nsx, sx0 = 4 * (st - sly * nsx);
  const bool sv = STRIP && sly < nrow;
  float sacc[4] = {0.f, 0.f, 0.f, 0.f};
  auto mult_strip = [&](int ch) {
    const float* sf = sm + (ch & 1) * stage;
    const float* sw = sf + fsz;
    if (sv) {
        for (int c = cg; c < CC; c += 16) {
          const float4* wq = reinterpret_cast<const float4*>(sw + c * 16);
          float wv[16];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float4 w4 = wq[q];
            wv[4 * q] = w4.x;
            wv[4 * q + 1] = w4.y;
            wv[4 * q + 2] = w4.z;
            wv[4 * q + 3] = w4.w;
          }
#pragma unroll
          for (int ky = 0; ky < 4; ++ky) {
            const float2* fr = reinterpret_cast<const float2*>(sf + c * plane + (sly + ky) * Wp + sx0);
            float fv[8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float2 f2 = fr[q];
              fv[2 * q] = f2.x;
              fv[2 * q + 1] = f2.y;
            }
#pragma unroll
            for (int kx = 0; kx < 4; ++kx)
#pragma unroll
              for (int e = 0; e < 4; ++e) sacc[e] = fmaf(fv[e + kx], wv[ky * 4 + kx], sacc[e]);   // fused always
          }
        }
    }
  };
  if constexpr (STRIP) {
    fetch(0, ra);
    if (nch > 1) fetch(1, rb);
    put(0, ra);
    __syncthreads();
    for (int ch = 0; ch < nch; ch += 2) {
      if (ch + 2 < nch) fetch(ch + 2, ra);   // rb holds ch + 1
      mult_strip(ch);
      if (ch + 1 < nch) put((ch + 1) & 1, rb);
      __syncthreads();
      if (ch + 1 >= nch) break;
      if (ch + 3 < nch) fetch(ch + 3, rb);   // ra holds ch + 2
      mult_strip(ch + 1);
      if (ch + 2 < nch) put((ch + 2) & 1, ra);
      __syncthreads();
    }
  } else {
  fetch(0, ra);
  put(0, ra);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) fetch(ch + 1, ra);
    const float* sf = sm + (ch & 1) * stage;
    const float* sw = sf + fsz;
    if (pv) {
      for (int c = g; c < CC; c += 4) {
        const float* fp = sf + c * plane + ly * Wp + x;
        const float* wp = sw + c * T;
        if constexpr (FH > 0) {
#pragma unroll
          for (int ky = 0; ky < FH; ++ky)
#pragma unroll
            for (int kx = 0; kx < FW; ++kx) acc += fp[ky * Wp + kx] * wp[ky * FW + kx];
        } else {
          for (int ky = 0; ky < a.fh; ++ky)
            for (int kx = 0; kx < a.fw; ++kx) acc += fp[ky * Wp + kx] * wp[ky * a.fw + kx];
        }
      }
    }
    if (ch + 1 < nch) put((ch + 1) & 1, ra);
    __syncthreads();
  }
  }
  if constexpr (STRIP) {
    if (sv)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (sx0 + e < a.Wo) red[cg][sly * a.Wo + sx0 + e] = sacc[e];
  } else {
    red[g][slot] = acc;
  }
  __syncthreads();
  float r2 = 0.f;
  if (g == 0 && pv) {
    if constexpr (STRIP) {
      acc = red[0][slot];
#pragma unroll
      for (int k = 1; k < 16; ++k) acc += red[k][slot];
    } else {
      acc = ((red[0][slot] + red[1][slot]) + red[2][slot]) + red[3][slot];
    }
    const int npos = a.Ho * a.Wo;
    const int64_t o = (int64_t)is * npos + (y0 + ly) * a.Wo + x;
    if (a.mode == 0) {
      a.out[o] = acc;
    } else if (a.mode == 1) {            // residuals (optimizer.py:137-146)
      const float m = a.mask[o], sw = a.sw[o];
      const float sa = (1.0f - m) / 2.0f * fabsf(acc) + (1.0f + m) / 2.0f * acc;
      const float sg = acc > 0.f ? 1.f : (acc < 0.f ? -1.f : 0.f);
      const float dm = (1.0f - m) / 2.0f * sg + (1.0f + m) / 2.0f;
      const float r = sw * (sa - a.label[o]);
      if (a.out) a.out[o] = dm * (sw * r);
      if (a.smask) a.smask[o] = dm;
      r2 = r * r;
    } else {                              // scores_grad (optimizer.py:151-152)
      const float gs = a.sw[o] * (a.smask[o] * acc);
      r2 = gs * gs;
    }
  }
  if (!a.partial) return;   // uniform over the workgroup
  __syncthreads();          // every group has read the sums
  if (g == 0) red[0][slot] = r2;
  __syncthreads();
  if (t == 0) {
    float tot = 0.f;
    for (int k = 0; k < nrow * a.Wo; ++k) tot += red[0][k];
    a.partial[(int64_t)is * gridDim.y + band] = tot;
  }
}

// grad[s,c,ky,kx] = sum_i,y,x r[i,s,y,x] * feat[i,s,c,y+ky-P,x+kx-P] (+ reg * w).  One workgroup per
// (sequence, CT channels), looping over the samples i < I (ctl: < n_samples; the sequence skips when it >=
// num_iter): the sample's padded planes of the CT channels and its residual map are staged double-buffered;
// G = 256 / (CT T) threads per (channel, tap) take interleaved positions, combined in a fixed order.
// STRIP (4 x 4, even padded row pitch): each lane takes four-position strips of its channel -- four residuals and a
// 4 x 8 window read once (8-B reads) feed 64 FMAs (explicit fmaf), instead of 17 LDS reads per 16 FMAs; the PG lanes
// of a channel combine in lane order.  Buffers start on 16-B boundaries (stage rounded up to 4 floats).
template <int FH, int FW, bool STRIP = false>
__global__ __launch_bounds__(256) void dimp_transpose_kernel(DimpTranspose a) {
  extern __shared__ float sm[];   // 2 x ([CT][Hp][Wp] padded planes + [npos] residuals)
  __shared__ float red[256];
  if constexpr (FH > 0) {
    a.fh = FH;
    a.fw = FW;
  }
  const int s = blockIdx.x, c0 = blockIdx.y * a.CT;
  if (a.ctl && a.it >= a.ctl[s].num_iter) return;
  const int nI = a.ctl ? min(a.I, a.ctl[s].n_samples) : a.I;
  const int T = a.fh * a.fw, P0 = a.fh / 2, P1 = a.fw / 2, npos = a.Ho * a.Wo;
  const int Wp = a.Wo + a.fw - 1, plane = (a.Ho + a.fh - 1) * Wp, CT = a.CT;
  const int fsz = CT * plane, stage = STRIP ? (fsz + npos + 3) & ~3 : fsz + npos;
  const int t = threadIdx.x;
  int soff[kDimpStage];   // as dimp_filter_kernel: fixed over the samples
#pragma unroll
  for (int k = 0; k < kDimpStage; ++k) {
    const int e = t + k * 256;
    int o = -1;
    if (e < fsz) {
      const int c = e / plane, r = e - c * plane, py = r / Wp, px = r - py * Wp;
      const int yy = py - P0, xx = px - P1;
      if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) o = (c0 + c) * a.H * a.W + yy * a.W + xx;
    } else if (e < fsz + npos) {   // the residual map (STRIP's rounding-up pad stays a zero)
      o = e - fsz;
    }
    soff[k] = o;
  }
  float rg[kDimpStage];
  auto fetch = [&](int i) {
    const float* f = a.feat + (int64_t)i * a.img_stride + (int64_t)s * a.seq_stride;
    const float* rs = a.r + ((int64_t)i * a.S + s) * npos;
#pragma unroll
    for (int k = 0; k < kDimpStage; ++k) {
      const int e = t + k * 256;
      rg[k] = soff[k] < 0 ? 0.f : (e < fsz ? f : rs)[soff[k]];
    }
  };
  auto put = [&](int buf) {
    float* d = sm + buf * stage;
#pragma unroll
    for (int k = 0; k < kDimpStage; ++k) {
      const int e = t + k * 256;
      if (e < stage) d[e] = rg[k];
    }
  };
  if (nI > 0) {
    fetch(0);
    put(0);
  }
  __syncthreads();
  float gv = 0.f;
  const bool own = t < CT * T && c0 + t / T < a.C;
  if constexpr (FH > 0) {
    // register-blocked: thread (channel c, position group pg) keeps all FH x FW taps of its channel in registers
    // and reads each residual once and each padded-plane value once per tap it feeds (~1 LDS read per FMA
    // instead of 2); the PG group sums of a (channel, tap) combine in group order at the end
    constexpr int TT = FH * FW;
    const int PG = 256 / CT;
    const int c = t / PG, pg = t - c * PG;
    float accb[TT];
#pragma unroll
    for (int k = 0; k < TT; ++k) accb[k] = 0.f;
    const int nsx = (a.Wo + 3) >> 2, nstrips = a.Ho * nsx;
    for (int i = 0; i < nI; ++i) {
      if (i + 1 < nI) fetch(i + 1);
      const float* sf = sm + (i & 1) * stage;
      const float* sr = sf + fsz;
      if constexpr (STRIP) {
        if (c < CT) {
          for (int st = pg; st < nstrips; st += PG) {
            const int y = st / nsx, x0 = 4 * (st - y * nsx);
            float rv[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) rv[e] = x0 + e < a.Wo ? sr[y * a.Wo + x0 + e] : 0.f;
#pragma unroll
            for (int ky = 0; ky < 4; ++ky) {
              const float2* fr = reinterpret_cast<const float2*>(sf + c * plane + (y + ky) * Wp + x0);
              float fv[8];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const float2 f2 = fr[q];
                fv[2 * q] = f2.x;
                fv[2 * q + 1] = f2.y;
              }
#pragma unroll
              for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int kx = 0; kx < 4; ++kx) accb[ky * 4 + kx] = fmaf(rv[e], fv[e + kx], accb[ky * 4 + kx]);
            }
          }
        }
      } else if (c < CT) {
        int y = pg / a.Wo, x = pg - y * a.Wo;
        for (int p = pg; p < npos; p += PG) {
          const float rv = sr[p];
          const float* fp = sf + c * plane + y * Wp + x;
#pragma unroll
          for (int ky = 0; ky < FH; ++ky)
#pragma unroll
            for (int kx = 0; kx < FW; ++kx) accb[ky * FW + kx] += rv * fp[ky * Wp + kx];
          x += PG;
          while (x >= a.Wo) {
            x -= a.Wo;
            ++y;
          }
        }
      }
      if (i + 1 < nI) put((i + 1) & 1);
      __syncthreads();
    }
    float* part = sm;   // the staging buffers are free now: [CT][TT][PG]
    if (c < CT)
#pragma unroll
      for (int k = 0; k < TT; ++k) part[(c * TT + k) * PG + pg] = accb[k];
    __syncthreads();
    if (own)
      for (int u = 0; u < PG; ++u) gv += part[t * PG + u];
  } else {
    const int G = 256 / (CT * T);
    const int pair = t / G, sub = t - pair * G;
    const bool active = pair < CT * T;
    const int c = pair / T, tt = pair - c * T, ky = tt / a.fw, kx = tt - ky * a.fw;
    float acc = 0.f;
    for (int i = 0; i < nI; ++i) {
      if (i + 1 < nI) fetch(i + 1);
      const float* sf = sm + (i & 1) * stage;
      const float* sr = sf + fsz;
      if (active) {
        const float* fp = sf + c * plane + ky * Wp + kx;
        int y = sub / a.Wo, x = sub - y * a.Wo;
        for (int p = sub; p < npos; p += G) {
          acc += sr[p] * fp[y * Wp + x];
          x += G;
          while (x >= a.Wo) {
            x -= a.Wo;
            ++y;
          }
        }
      }
      if (i + 1 < nI) put((i + 1) & 1);
      __syncthreads();
    }
    red[t] = acc;
    __syncthreads();
    if (own)
      for (int u = 0; u < G; ++u) gv += red[t * G + u];
  }
  if (own) {
    const int64_t o = ((int64_t)s * a.C + c0) * T + t;
    gv += a.w ? a.reg * a.w[o] : 0.f;
    a.grad[o] = gv;
  }
  __syncthreads();
  if (own) red[t] = gv;
  __syncthreads();
  if (a.gsq && t < CT && c0 + t < a.C) {
    float sq = 0.f;
    for (int k = 0; k < T; ++k) sq += red[t * T + k] * red[t * T + k];
    a.gsq[(int64_t)s * a.C + c0 + t] = sq;
  }
}

// alpha = |g|^2 / (|J g|^2 + (reg + eps)|g|^2), w -= step * alpha * g   (optimizer.py:155-160); one block per s
__global__ __launch_bounds__(256) void dimp_update_kernel(DimpUpdate a) {
  __shared__ float red[256];
  __shared__ float num_sh, den_sh;
  const int s = blockIdx.x;
  if (a.ctl && a.it >= a.ctl[s].num_iter) return;
  const int nI = a.ctl ? min(a.I, a.ctl[s].n_samples) : a.I;
  float v = 0.f;
  for (int c = threadIdx.x; c < a.C; c += 256) v += a.gsq[(int64_t)s * a.C + c];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) num_sh = red[0];
  __syncthreads();
  v = 0.f;
  for (int k = threadIdx.x; k < nI * a.nby; k += 256) {
    const int i = k / a.nby, by = k - i * a.nby;
    v += a.sgsq[((int64_t)i * a.S + s) * a.nby + by];
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) den_sh = fmaxf(red[0] + (a.reg + a.alpha_eps) * num_sh, 1e-8f);
  __syncthreads();
  const float alpha = num_sh / den_sh;
  const int T = a.fh * a.fw;
  for (int k = threadIdx.x; k < a.C * T; k += 256) {
    const int64_t o = (int64_t)s * a.C * T + k;
    a.w[o] = a.w[o] - (a.step * alpha) * a.grad[o];
  }
}

// loss = (sum r^2 + reg * sum w^2) / S   (optimizer.py:142-143, 165-168)
__global__ __launch_bounds__(256) void dimp_loss_kernel(const float* rsq, int nparts, const float* w, int nw, float reg,
                                                        int S, float* loss) {
  __shared__ float red[256];
  float a = 0.f, b = 0.f;
  for (int k = threadIdx.x; k < nparts; k += 256) a += rsq[k];
  for (int k = threadIdx.x; k < nw; k += 256) b += w[k] * w[k];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  const float ra = red[0];
  __syncthreads();
  red[threadIdx.x] = b;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (ra + reg * red[0]) / (float)S;
}

__global__ __launch_bounds__(256) void dimp_prep_kernel(DimpPrep a) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= a.IS) return;
  const int i = k / a.S, sq = k - i * a.S;
  const float* b = a.bb + i * a.bb_i + sq * a.bb_s;
  a.centers[2 * k] = (b[1] + b[3] / 2) / a.feat_stride - a.off0;       // flip((1,)) -> (y, x)
  a.centers[2 * k + 1] = (b[0] + b[2] / 2) / a.feat_stride - a.off1;
  a.sqrtsw[k] = a.sw ? sqrtf(a.sw[i * a.sw_i + sq * a.sw_s]) : (float)sqrt(1.0 / a.I);
}
__global__ __launch_bounds__(256) void dimp_prep_args_kernel(DimpPrepArgs a) {
  const int j = threadIdx.x;
  if (j >= a.n) return;
  const int k = a.k0 + j;
  const float* b = a.bb + 4 * j;
  a.centers[2 * k] = (b[1] + b[3] / 2) / a.feat_stride - a.off0;
  a.centers[2 * k + 1] = (b[0] + b[2] / 2) / a.feat_stride - a.off1;
  a.sqrtsw[k] = a.has_sw ? sqrtf(a.sw[j]) : (float)sqrt(1.0 / a.I);
}
__global__ __launch_bounds__(384) void dimp_params_kernel(DimpParamArgs a) { a.dst[threadIdx.x] = a.v[threadIdx.x]; }

void dimp_prep(const DimpPrep& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_prep_kernel, dim3((a.IS + 255) / 256), dim3(256), 0, s, a);
}
void dimp_prep_args(const DimpPrepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_prep_args_kernel, dim3(1), dim3(256), 0, s, a);
}
void dimp_params(const DimpParamArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_params_kernel, dim3(1), dim3(384), 0, s, a);
}

void dimp_maps(const DimpMaps& m, hipStream_t s) {
  const int n = m.IS * m.Ho * m.Wo;
  hipLaunchKernelGGL(dimp_maps_kernel, dim3((n + 255) / 256), dim3(256), 0, s, m);
}
void dimp_filter(const DimpFilter& a_, hipStream_t s) {
  DimpFilter a = a_;
  const DimpGeo g = dimp_geo(a.C, a.H, a.W, a.fh, a.fw);
  a.RB = g.RB;
  a.CC = g.CC;
  const size_t lds = 2 * (size_t)g.filter_stage * sizeof(float);
  const dim3 grid(a.I * a.S, g.nbands);
  static const bool strip_off = getenv("MMT_DIMP_NOSTRIP") != nullptr;   // tuning A/B: the 4-group kernel
  // 16-channel chunks (one channel per lane and chunk; 108 VGPRs, four workgroups per CU): GN steps 50.5 -> 43.9 us,
  // the per-frame scores 44.4 -> 37.4 us, mfDiMP +0.9 % (tools/runs_r4/r4_run14.sh); MMT_DIMP_STRIP_CC=32 (tuning)
  static const int strip_cc = getenv("MMT_DIMP_STRIP_CC") ? atoi(getenv("MMT_DIMP_STRIP_CC")) : 16;
  const int nstrips = g.RB * ((g.Wo + 3) / 4);
  const int fplane = (g.RB + 3) * (g.Wo + 3);
  const bool strip = a.fh == 4 && a.fw == 4 && !strip_off && nstrips <= 16 && g.CC % 16 == 0 && fplane % 2 == 0 &&
                     (g.Wo + 3) % 2 == 0;
  if (strip && strip_cc == 16 && 16 * (fplane + 16) <= 10 * 256) {
    a.CC = 16;
    hipLaunchKernelGGL((dimp_filter_kernel<4, 4, true, 10>), grid, dim3(256), 2 * (size_t)16 * (fplane + 16) * 4, s, a);
  } else if (strip)
    hipLaunchKernelGGL((dimp_filter_kernel<4, 4, true>), grid, dim3(256), lds, s, a);
  else if (a.fh == 4 && a.fw == 4)
    hipLaunchKernelGGL((dimp_filter_kernel<4, 4>), grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((dimp_filter_kernel<0, 0>), grid, dim3(256), lds, s, a);
}
void dimp_transpose(const DimpTranspose& a_, hipStream_t s) {
  DimpTranspose a = a_;
  const DimpGeo g = dimp_geo(a.C, a.H, a.W, a.fh, a.fw);
  a.CT = g.CT;
  const size_t lds = 2 * (size_t)g.transpose_stage * sizeof(float);
  const dim3 grid(a.S, (a.C + g.CT - 1) / g.CT);
  static const bool strip_off = getenv("MMT_DIMP_NOSTRIP") != nullptr;   // tuning A/B
  const int stage4 = (g.transpose_stage + 3) & ~3;
  if (a.fh == 4 && a.fw == 4 && !strip_off && (g.Wo + 3) % 2 == 0 && 256 % g.CT == 0 &&
      2 * g.transpose_stage >= 256 * 16 && stage4 <= kDimpStage * 256)
    hipLaunchKernelGGL((dimp_transpose_kernel<4, 4, true>), grid, dim3(256), 2 * (size_t)stage4 * sizeof(float), s, a);
  else if (a.fh == 4 && a.fw == 4 && 2 * g.transpose_stage >= 256 * 16)   // the blocked form's group sums fit the staging
    hipLaunchKernelGGL((dimp_transpose_kernel<4, 4>), grid, dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((dimp_transpose_kernel<0, 0>), grid, dim3(256), lds, s, a);
}
void dimp_update(const DimpUpdate& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_update_kernel, dim3(a.S), dim3(256), 0, s, a);
}
void dimp_loss(const float* rsq, int nparts, const float* w, int nw, float reg, int S, float* loss, hipStream_t s) {
  hipLaunchKernelGGL(dimp_loss_kernel, dim3(1), dim3(256), 0, s, rsq, nparts, w, nw, reg, S, loss);
}

}  // namespace mmt
