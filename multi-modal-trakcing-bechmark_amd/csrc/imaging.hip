// Frame-side kernels of the tracking path, gfx950:
//  * crop_patchify: sample_target (processing_utils.py:14-81: square crop, zero pad, cv2 INTER_LINEAR
//    resize) + PreprocessorMM normalisation (data_utils.py:20-24) + the k16s16 patch unfold that feeds
//    the patch-embed GEMM, in one pass straight from the HBM-resident H x W x C uint8 frame (the padded
//    crop is never materialised);
//  * decode: the CENTER head's conv5 1x1 + sigmoid/clamp (head.py:110-124, 177-201), the Hann window
//    (vipt.py:79-80) and cal_bbox's first-occurrence argmax + gather (head.py:142-160);
//  * xcorr: SiamFC / DiMP per-sequence cross-correlation (grouped conv2d).
#include "cvresize.h"
#include "kernels.h"

namespace mmt {

__constant__ float kMean[6] = {0.485f, 0.456f, 0.406f, 0.485f, 0.456f, 0.406f};
__constant__ float kStd[6] = {0.229f, 0.224f, 0.225f, 0.229f, 0.224f, 0.225f};

// padded-crop pixel: image row y1 + r is real only for 0 <= y <= H-2 (the reference slices
// im[y1+y1_pad : y2-y2_pad] with y2_pad = max(y2-H+1, 0), which drops the last row/col)
__device__ __forceinline__ int crop_px(const CropParam& p, int r, int x, int c) {
  const int yy = p.y1 + r, xx = p.x1 + x;
  if (yy < 0 || yy > p.H - 2 || xx < 0 || xx > p.W - 2) return 0;
  return p.frame[(int64_t)yy * p.stride + (int64_t)xx * p.C + c];
}

// processing_utils.py:32-41: crop_sz = ceil(sqrt(w h) factor) ('Too small bounding box.' if < 1),
// x1 = round(x + w/2 - crop_sz/2) with python's round (half to even)
__device__ void geometry_of(const double box[4], double factor, int out_sz, CropParam& p, double& rf, int& err) {
#pragma clang fp contract(off)
  const double x = box[0], y = box[1], w = box[2], h = box[3];
  const double cs = ceil(sqrt(w * h) * factor);
  err = 0;
  if (!(cs >= 1.0)) err = -5;           // MMT_E_BOX
  else if (cs > 1e6) err = -1;          // MMT_E_ARG
  if (err) {                            // a harmless crop; the frame's result is discarded
    p.x1 = p.y1 = 0;
    p.crop_sz = 1;
    rf = 1.0;
  } else {
    p.crop_sz = (int)cs;
    p.x1 = (int)rint(x + 0.5 * w - cs * 0.5);
    p.y1 = (int)rint(y + 0.5 * h - cs * 0.5);
    rf = (double)out_sz / cs;
  }
}
// FUSED_GEOM (launches that are not split into stream parts: the one-sequence frame): the geometry kernel's work
// done here -- every workgroup derives its sequence's crop from the device state (and the frame from the host ring
// entry) itself; workgroup 0 of each sequence stores the parameters, rf / err and the token index reset, and
// records the ring entry for decode, which advances the counter (g.ring_advance) -- one launch fewer
// (fused mode: the geometry fields x1, y1, crop_sz of params[b] are written by workgroup 0 and read by nobody in this
// launch -- every workgroup forms its own -- and the frame fields are only read: from the ring entry, or, without the
// ring, from params[b], where the host put them and nothing in this launch writes them)
template <bool FUSED_GEOM>
__global__ __launch_bounds__(256) void crop_kernel(const CropArgs a) {
  const int b = blockIdx.y;
  CropParam p;
  if constexpr (FUSED_GEOM) {
    const GeomArgs& g = a.geom;
    const int e = g.use_ring ? *g.ring.ctr : 0;
    const CropParam& h = g.use_ring ? g.ring.params[(int64_t)e * g.ring.pitch + b] : a.params[b];
    p.frame = h.frame;
    p.stride = h.stride;
    p.H = h.H;
    p.W = h.W;
    p.C = h.C;
    double rf;
    int err;
    geometry_of(g.state[b].box, g.factor, a.out_sz, p, rf, err);
    if (blockIdx.x == 0) {
      if (threadIdx.x == 0) {
        CropParam* const dst = const_cast<CropParam*>(a.params) + b;
        if (g.use_ring) {   // the frame fields too (decode and the host read params after the launch)
          dst->frame = p.frame;
          dst->stride = p.stride;
          dst->H = p.H;
          dst->W = p.W;
          dst->C = p.C;
        }
        dst->x1 = p.x1;
        dst->y1 = p.y1;
        dst->crop_sz = p.crop_sz;
        g.state[b].rf = rf;
        g.state[b].err = err;
        if (g.use_ring && b == 0) *g.ring.cur = e;
      }
      if (g.gidx)
        for (int j = threadIdx.x; j < g.Lx; j += blockDim.x) {
          g.gidx[b * g.Lx + j] = j;
          g.slot2pos[b * g.Lx + j] = g.Lz + j;
        }
    }
  } else {
    p = a.params[b];
  }
  const int O = a.out_sz;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= O * O) return;
  // thread -> (patch, pixel within the patch): a wave's 64 pixels are 64 consecutive elements of each channel plane
  // of a patch row (within = (oy & 15) * 16 + (ox & 15)), so every store instruction writes whole 128-B lines
  // (an output-row order wrote 4 separate 32-B pieces per instruction, each line finished by 4 other workgroups)
  const int np = O / 16;
  const int patch = idx >> 8, within = idx & 255;
  const int oy = (patch / np) * 16 + (within >> 4), ox = (patch % np) * 16 + (within & 15);
  int u8[6];
  cv_linear_u8([&](int r, int x, int c) { return crop_px(p, r, x, c); }, p.crop_sz, O, oy, ox, a.C, u8);
  const int64_t rowoff = ((int64_t)b * a.rows_per_seq + a.row0 + patch) * 768;
  for (int c = 0; c < a.C; ++c) {
    const float t = ((float)u8[c] / 255.0f - kMean[c]) / kStd[c];
    const int64_t o = rowoff + (c % 3) * 256 + within;
    bf16_t* lo = c < 3 ? a.A_rgb_lo : a.A_aux_lo;
    if (lo) {   // f16x3 halves of t * 2^12
      uint16_t h, l;
      split_h(t * kPixScale, h, l);
      (c < 3 ? a.A_rgb : a.A_aux)[o] = h;
      lo[o] = l;
    } else {
      (c < 3 ? a.A_rgb : a.A_aux)[o] = f2bf(t);
    }
    if (a.dbg_patch) a.dbg_patch[((int64_t)b * O * O + oy * O + ox) * a.C + c] = (uint8_t)u8[c];
  }
}

void crop_patchify(const CropArgs& a, hipStream_t s) {
  const dim3 grid((a.out_sz * a.out_sz + 255) / 256, a.B);
  if (a.geom.state)
    hipLaunchKernelGGL(crop_kernel<true>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(crop_kernel<false>, grid, dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ decode
__device__ __forceinline__ float sigmoid_clamp(float x) {
  const float y = 1.0f / (1.0f + expf(-x));
  return fminf(fmaxf(y, 1e-4f), 1.0f - 1e-4f);
}

// ------------------------------------------------------------------ tracker state on the device
// No FMA contraction in update_state and geometry_of (pragma at the top of each body): every product and sum
// rounds as in the reference's python doubles (and float32 tensor ops where it computes on tensors).
__device__ __forceinline__ double dmax(double a, double b) { return a < b ? b : a; }   // std::max / python max
__device__ __forceinline__ double dmin(double a, double b) { return b < a ? b : a; }   // std::min / python min

// geometry_of into the device parameters and state (geometry_kernel)
__device__ void geometry_one(CropParam* params, SeqState* state, int i, double factor, int out_sz) {
  SeqState& st = state[i];
  double rf;
  int err;
  geometry_of(st.box, factor, out_sz, params[i], rf, err);
  st.rf = rf;
  st.err = err;
}

// one workgroup: every thread reads the launch counter before thread 0 advances it.  It also resets the
// launch's token index arrays (gidx[b][j] = j, slot2pos[b][j] = Lz + j: every search token kept, before the
// first candidate elimination), which would otherwise take a launch of their own
__global__ __launch_bounds__(256) void geometry_kernel(CropParam* params, SeqState* state, int n, double factor,
                                                       int out_sz, RingArgs ring, int use_ring, int* gidx,
                                                       int* slot2pos, int Lz, int Lx) {
  if (gidx)
    for (int i = threadIdx.x; i < n * Lx; i += blockDim.x) {
      const int j = i % Lx;
      gidx[i] = j;
      slot2pos[i] = Lz + j;
    }
  int e = 0;
  if (use_ring) e = *ring.ctr;   // kept in [0, kring): launches mod kring, as the host's tickets count them
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    if (use_ring) {
      const CropParam h = ring.params[(int64_t)e * ring.pitch + i];
      CropParam& p = params[i];
      p.frame = h.frame;
      p.stride = h.stride;
      p.H = h.H;
      p.W = h.W;
      p.C = h.C;
    }
    geometry_one(params, state, i, factor, out_sz);
  }
  if (use_ring) {
    __syncthreads();
    if (threadIdx.x == 0) {
      *ring.cur = e;
      *ring.ctr = e + 1 == ring.kring ? 0 : e + 1;   // never overflows however long the engine runs
    }
  }
}

void crop_geometry(CropParam* params, SeqState* state, int n, double factor, int out_sz, const RingArgs* ring,
                   int* gidx, int* slot2pos, int Lz, int Lx, hipStream_t s) {
  hipLaunchKernelGGL(geometry_kernel, dim3(1), dim3(256), 0, s, params, state, n, factor, out_sz,
                     ring ? *ring : RingArgs{}, ring ? 1 : 0, gidx, slot2pos, Lz, Lx);
}

// vipt.py:84-88 (pred_box * S / resize_factor in float32 tensors, then python floats) + map_box_back
// + clip_box (box_ops.py:97-106, margin 10)
__device__ void update_state(const DecodeArgs& a, int b, const float* r) {
#pragma clang fp contract(off)
  SeqState& st = a.state[b];
  TrackOut& o = a.out[b];
  o.score = r[4];
  o.err = st.err;
  if (st.err) {
    for (int k = 0; k < 4; ++k) o.box[k] = st.box[k];
    return;
  }
  const float S = (float)a.search_size;
  const float frf = (float)st.rf;
  const double cx = (double)((r[0] * S) / frf), cy = (double)((r[1] * S) / frf);
  const double w = (double)((r[2] * S) / frf), h = (double)((r[3] * S) / frf);
  const double cx_prev = st.box[0] + 0.5 * st.box[2], cy_prev = st.box[1] + 0.5 * st.box[3];
  const double half = 0.5 * a.search_size / st.rf;
  const double cxr = cx + (cx_prev - half), cyr = cy + (cy_prev - half);
  double x1 = cxr - 0.5 * w, y1 = cyr - 0.5 * h;
  const double margin = 10;
  double x2 = x1 + w, y2 = y1 + h;
  const double Ww = a.params[b].W, Hh = a.params[b].H;
  x1 = dmin(dmax(0.0, x1), Ww - margin);
  x2 = dmin(dmax(margin, x2), Ww);
  y1 = dmin(dmax(0.0, y1), Hh - margin);
  y2 = dmin(dmax(margin, y2), Hh);
  const double bw = dmax(margin, x2 - x1), bh = dmax(margin, y2 - y1);
  st.box[0] = x1;
  st.box[1] = y1;
  st.box[2] = bw;
  st.box[3] = bh;
  for (int k = 0; k < 4; ++k) o.box[k] = st.box[k];
}

__device__ void ring_out(const DecodeArgs& a, int b) {   // the launch's result row into the host ring entry
  if (a.ring_outs) a.ring_outs[(int64_t)(*a.ring_cur) * a.ring_pitch + a.row0 + b] = a.out[b];
}

__global__ __launch_bounds__(256) void decode_kernel(const DecodeArgs a) {
  __shared__ float sv[256];
  __shared__ int si[256];
  __shared__ float sw[5 * 32 + 5];
  const int b = blockIdx.x, tid = threadIdx.x, n = a.fs * a.fs;
  // (a crop with the geometry fused in read the ring counter; the launch's last kernel advances it)
  if (a.ring_ctr && b == 0 && tid == 0) {
    const int e = *a.ring_cur;
    *a.ring_ctr = e + 1 == a.ring_kring ? 0 : e + 1;
  }
  if (tid < 165) sw[tid] = tid < 160 ? a.w5[tid] : a.b5[tid - 160];
  __syncthreads();
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int p = tid; p < n; p += 256) {
    float acc[5];
#pragma unroll
    for (int o = 0; o < 5; ++o) acc[o] = sw[160 + o];
    const int br_of[5] = {0, 1, 1, 2, 2};
#pragma unroll
    for (int o = 0; o < 5; ++o) {
      const float* h = a.h4 + ((int64_t)br_of[o] * a.B * n + (int64_t)b * n + p) * 32;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += h[k] * sw[o * 32 + k];
      acc[o] += s;
    }
    const float ctr = sigmoid_clamp(acc[0]);
    const float resp = a.hann[p] * ctr;
    if (a.maps) {
      float* mp = a.maps + (int64_t)b * 5 * n;
      mp[p] = ctr;
      mp[n + p] = sigmoid_clamp(acc[3]);
      mp[2 * n + p] = sigmoid_clamp(acc[4]);
      mp[3 * n + p] = acc[1];
      mp[4 * n + p] = acc[2];
    }
    if (resp > best) { best = resp; bidx = p; }
  }
  sv[tid] = best;
  si[tid] = bidx;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (tid < st) {
      const float v2 = sv[tid + st];
      const int i2 = si[tid + st];
      if (v2 > sv[tid] || (v2 == sv[tid] && i2 < si[tid])) { sv[tid] = v2; si[tid] = i2; }
    }
    __syncthreads();
  }
  if (tid == 0) {
    const int p = si[0];
    float acc[5];
    const int br_of[5] = {0, 1, 1, 2, 2};
    for (int o = 0; o < 5; ++o) {
      const float* h = a.h4 + ((int64_t)br_of[o] * a.B * n + (int64_t)b * n + p) * 32;
      float s = 0.f;
      for (int k = 0; k < 32; ++k) s += h[k] * sw[o * 32 + k];
      acc[o] = sw[160 + o] + s;
    }
    const int iy = p / a.fs, ix = p - iy * a.fs;
    float* r = a.res + (int64_t)b * 8;
    r[0] = ((float)ix + acc[1]) / (float)a.fs;
    r[1] = ((float)iy + acc[2]) / (float)a.fs;
    r[2] = sigmoid_clamp(acc[3]);
    r[3] = sigmoid_clamp(acc[4]);
    r[4] = sv[0];
    r[5] = (float)p;
    r[6] = 0.f;
    r[7] = 0.f;
    if (a.state) {
      update_state(a, b, r);
      ring_out(a, b);
    }
  }
}

void decode(const DecodeArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(decode_kernel, dim3(a.B), dim3(256), 0, s, a);
}

// ------------------------------------------------------------------ cross-correlation
// One thread per output pixel, channel loop with the exemplar staged in LDS per 16-channel slab.
// NCHW correlation: a workgroup takes 16 output pixels of one batch entry; its 256 threads are 16 pixels x 16
// channel slices (slice s sums channels s, s + 16, ...; 16 neighbouring pixels read neighbouring x), the exemplar
// staged in the LDS a chunk of channels at a time, the 16 slice sums of a pixel added in slice order (same bits
// on every run)
constexpr int kXcLds = 16384;   // floats of exemplar per chunk
__global__ __launch_bounds__(256) void xcorr_kernel(const float* __restrict__ Z, const float* __restrict__ X,
                                                    float* __restrict__ out, int C, int hz, int wz, int hx, int wx,
                                                    float scale, float bias) {
  __shared__ float zs[kXcLds];
  __shared__ float part[16][17];
  const int b = blockIdx.y, t = threadIdx.x, o = t & 15, sl = t >> 4;
  const int ho = hx - hz + 1, wo = wx - wz + 1, zsz = hz * wz;
  const int p = blockIdx.x * 16 + o;
  const bool live = p < ho * wo;
  const int y = live ? p / wo : 0, x = live ? p - (p / wo) * wo : 0;
  const int cc = (kXcLds / zsz) & ~15;   // channels per chunk (a multiple of the 16 slices; zsz <= 1024)
  float acc = 0.f;
  for (int c0 = 0; c0 < C; c0 += cc) {
    const int cn = min(cc, C - c0);
    __syncthreads();
    for (int i = t; i < cn * zsz; i += 256) zs[i] = Z[((int64_t)b * C + c0) * zsz + i];
    __syncthreads();
    if (live)
      for (int c = sl; c < cn; c += 16) {
        const float* xp = X + (((int64_t)b * C + c0 + c) * hx + y) * wx + x;
        const float* zp = zs + c * zsz;
        for (int i = 0; i < hz; ++i)
          for (int j = 0; j < wz; ++j) acc += xp[i * wx + j] * zp[i * wz + j];
      }
  }
  part[sl][o] = acc;
  __syncthreads();
  if (t < 16 && live) {
    float sum = part[0][t];
    for (int k = 1; k < 16; ++k) sum += part[k][t];
    out[(int64_t)b * ho * wo + p] = sum * scale + bias;
  }
}

void xcorr(const float* Z, const float* X, float* out, int B, int C, int hz, int wz, int hx, int wx, float scale,
           float bias, hipStream_t s) {
  const int n = (hx - hz + 1) * (wx - wz + 1);
  hipLaunchKernelGGL(xcorr_kernel, dim3((n + 15) / 16, B), dim3(256), 0, s, Z, X, out, C, hz, wz, hx, wx, scale, bias);
}

// NHWC correlation: one wave per output pixel, lanes over channels (float4 when C % 4 == 0), the exemplar in
// LDS, the wave's partial sums combined in a fixed butterfly order (same bits on every run)
__global__ __launch_bounds__(256) void xcorr_nhwc_kernel(const float* __restrict__ Z, int64_t z_bstride,
                                                         const float* __restrict__ X, float* __restrict__ out, int C,
                                                         int hz, int wz, int hx, int wx, float scale, float bias) {
  extern __shared__ __attribute__((aligned(16))) float zsh[];
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int ho = hx - hz + 1, wo = wx - wz + 1;
  const int n = hz * wz * C;
  const float* zb = Z + b * z_bstride;
  for (int i = threadIdx.x; i < n; i += 256) zsh[i] = zb[i];
  __syncthreads();
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= ho * wo) return;
  const int y = p / wo, x = p - y * wo;
  const float* xb = X + (int64_t)b * hx * wx * C;
  float acc = 0.f;
  if ((C & 3) == 0) {
    const int c4 = C >> 2;
    for (int i = 0; i < hz; ++i)
      for (int j = 0; j < wz; ++j) {
        const float4* xr = reinterpret_cast<const float4*>(xb + ((int64_t)(y + i) * wx + x + j) * C);
        const float4* zr = reinterpret_cast<const float4*>(zsh + (i * wz + j) * C);
        for (int c = lane; c < c4; c += 64) {
          const float4 u = xr[c], v = zr[c];
          acc += u.x * v.x + u.y * v.y + u.z * v.z + u.w * v.w;
        }
      }
  } else {
    for (int i = 0; i < hz; ++i)
      for (int j = 0; j < wz; ++j) {
        const float* xr = xb + ((int64_t)(y + i) * wx + x + j) * C;
        const float* zr = zsh + (i * wz + j) * C;
        for (int c = lane; c < C; c += 64) acc += xr[c] * zr[c];
      }
  }
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) out[(int64_t)b * ho * wo + p] = acc * scale + bias;
}

void xcorr_nhwc(const float* Z, int64_t z_bstride, const float* X, float* out, int B, int C, int hz, int wz, int hx,
                int wx, float scale, float bias, hipStream_t s) {
  const int n = (hx - hz + 1) * (wx - wz + 1);
  hipLaunchKernelGGL(xcorr_nhwc_kernel, dim3((n + 3) / 4, B), dim3(256), (size_t)hz * wz * C * sizeof(float), s, Z,
                     z_bstride, X, out, C, hz, wz, hx, wx, scale, bias);
}

}  // namespace mmt
