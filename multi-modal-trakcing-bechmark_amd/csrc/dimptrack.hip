// The DiMP tracker's per-frame state machine on the device, batched over a GPU's sequences (gfx950).
//
// pytracking/tracker/dimp/dimp.py (DeT, RGBD/models/DeT/pytracking/tracker/dimp/dimp.py) with the
// DeT_DiMP50_Max parameters and use_iou_net False keeps per sequence a position, a scale, a 50-sample memory
// with its weights and boxes, and after every frame decides -- from the 19 x 19 classifier scores -- where the
// target went, whether the frame is a new training sample, and whether the filter gets Gauss-Newton steps.
// Here that state lives in device memory (DimpState, one per sequence) and two launches per frame advance
// every sequence of a batch at once, so only boxes, scores and flags cross PCIe:
//   dimp_sample_kernel     get_centered_sample_pos + sample_patch geometry (dimp.py:309-312,
//                          preprocessing.py:49-125) from the device state, the 288 x 288 patch into the batch
//   dimp_localize_kernel   get_sample_location, localize_advanced, update_state, get_iounet_box,
//                          update_classifier's memory bookkeeping (update_sample_weights) and its choice of
//                          Gauss-Newton iterations (dimp.py:101-166, 232-301, 538-607) -- one workgroup per
//                          sequence; then dimp_memory_kernel copies the frame's features into the chosen slot.
// The arithmetic is the reference's: float32 tensor ops with Python scalars cast to float32, .item() values
// compared and rounded in double (Python floats), torch.max / torch.min first-index ties.  One deliberate
// difference: sw.sum() (50 weights) is a sequential float32 sum here, where ATen's vectorised CPU sum may
// round differently in the last bit (the tracker golden pins the resulting boxes, flags and confidences).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmtrack.h"

#pragma clang fp contract(off)

namespace mmt {

constexpr int kMem = MMT_DIMP_MEMORY;   // sample_memory_size

// flags (dimp.py localize_advanced return values)
enum { F_NORMAL = 0, F_NOT_FOUND = 1, F_UNCERTAIN = 2, F_HARD_NEGATIVE = 3 };

__device__ __forceinline__ float pyf(double v) { return (float)v; }   // a Python float in a float32 tensor op

// ---- sample_patch geometry from the device state (the host version: dimp_tracker.DiMP._sample_patch)
struct Geom {
  int df, os_y, os_x, tl_y, tl_x, sz_h, sz_w, H2, W2;
  float coords[4];
};
__device__ __forceinline__ int64_t floordiv(int64_t a, int64_t b) {
  const int64_t q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}
__device__ __forceinline__ int64_t floormod(int64_t a, int64_t b) { return a - floordiv(a, b) * b; }

__device__ Geom dimp_geometry(const mmt_dimp_state& st, const mmt_dimp_track_params& p, int H, int W) {
  // get_centered_sample_pos: pos + ((feature_sz + kernel_size) % 2) * target_scale * img_support_sz / (2 feature_sz)
  float pc[2];
  for (int d = 0; d < 2; ++d) {
    const float odd = fmodf(p.feature_sz[d] + p.kernel_size[d], 2.0f);
    pc[d] = st.pos[d] + odd * st.target_scale * p.img_sample_sz[d] / (2.0f * p.feature_sz[d]);
  }
  // sample_sz = target_scale * scale_factors[0] * img_sample_sz, output_sz = img_sample_sz
  float ssz[2];
  for (int d = 0; d < 2; ++d) ssz[d] = st.target_scale * 1.0f * p.img_sample_sz[d];
  const float rf = fminf(ssz[0] / p.img_sample_sz[0], ssz[1] / p.img_sample_sz[1]);
  const double rfd = (double)rf - 0.1;
  int df = (int)rfd;            // int(resize_factor - 0.1): truncation
  df = df < 1 ? 1 : df;
  Geom g{};
  g.df = df;
  int64_t posl[2], os[2] = {0, 0}, szl[2], tl[2], br[2];
  for (int d = 0; d < 2; ++d) {
    posl[d] = (int64_t)pc[d];   // Tensor.long(): truncation toward zero
    if (df > 1) {
      os[d] = floormod(posl[d], df);
      posl[d] = floordiv(posl[d] - os[d], df);
    }
    const float sz = ssz[d] / (float)df;
    const float r = rintf(sz);   // torch.round: half to even
    szl[d] = (int64_t)fmaxf(r, 2.0f);
    tl[d] = posl[d] - floordiv(szl[d] - 1, 2);
    br[d] = posl[d] + floordiv(szl[d], 2) + 1;
  }
  g.os_y = (int)os[0];
  g.os_x = (int)os[1];
  g.tl_y = (int)tl[0];
  g.tl_x = (int)tl[1];
  g.sz_h = (int)szl[0];
  g.sz_w = (int)szl[1];
  g.H2 = (H - g.os_y + df - 1) / df;
  g.W2 = (W - g.os_x + df - 1) / df;
  g.coords[0] = (float)(df * tl[0]);
  g.coords[1] = (float)(df * tl[1]);
  g.coords[2] = (float)(df * br[0]);
  g.coords[3] = (float)(df * br[1]);
  return g;
}

__device__ __forceinline__ float frame_at(const uint8_t* f, int64_t rs, int C, const Geom& g, int cy, int cx, int c) {
  int r = g.tl_y + cy, q = g.tl_x + cx;
  r = min(max(r, 0), g.H2 - 1);
  q = min(max(q, 0), g.W2 - 1);
  return (float)f[(int64_t)(g.os_y + r * g.df) * rs + (int64_t)(g.os_x + q * g.df) * C + c];
}

// grid (pixel blocks, sequences): patch [n][C][oh][ow] from the sequence's frame; block 0 stores the sample
// coordinates.  Pixels as sample_patch_kernel (dimpnet.hip): replicate padding, ATen's CPU bilinear with its
// fma contraction.
// NORM4 (6-channel frames): instead of the NCHW patch, each pixel's two 3-channel halves normalised as
// normalize_kernel does (dimpnet.hip, oc = 4: v / 255, - mean, / std, zero fourth channel) into outa / outb
// [n][oh][ow][4] -- the same values, so the same bits as the two launches
struct NormArgs {
  float mean[3], sd[3];
  float* outa;
  float* outb;
  float* zero;     // optional: words to clear (the backbones' max words)
  int64_t nzero;
};
template <bool NORM4>
__global__ __launch_bounds__(256) void dimp_sample_kernel(mmt_dimp_state* states, const mmt_dimp_frame* frames,
                                                          mmt_dimp_track_params p, int oh, int ow, float* out,
                                                          NormArgs na) {
  const int s = blockIdx.y;
  if (NORM4 && na.zero) {   // the backbones' max words cleared here, before their first producer (no fill launch)
    const int64_t nt = (int64_t)gridDim.x * gridDim.y * 256;
    for (int64_t k = ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x; k < na.nzero; k += nt)
      na.zero[k] = 0.f;
  }
  const mmt_dimp_frame fr = frames[s];
  const Geom g = dimp_geometry(states[s], p, fr.H, fr.W);
  if (blockIdx.x == 0 && threadIdx.x < 4) states[s].coords[threadIdx.x] = g.coords[threadIdx.x];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)oh * ow) return;
  const int C = NORM4 ? 6 : fr.C;
  float* o = out + (int64_t)s * C * oh * ow;
  float v6[6];
  auto put = [&](int c, float v) {
    if constexpr (NORM4) v6[c] = v;
    else o[(int64_t)c * oh * ow + i] = v;
  };
  auto flush = [&]() {
    if constexpr (NORM4) {
      float n[6];
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        float v = v6[c] / 255.f;
        v = v - na.mean[c % 3];
        n[c] = v / na.sd[c % 3];
      }
      const int64_t q = (int64_t)s * oh * ow + i;
      reinterpret_cast<float4*>(na.outa)[q] = make_float4(n[0], n[1], n[2], 0.f);
      reinterpret_cast<float4*>(na.outb)[q] = make_float4(n[3], n[4], n[5], 0.f);
    }
  };
  const int oy = (int)(i / ow), ox = (int)(i - (int64_t)oy * ow);
  if (g.sz_h == oh && g.sz_w == ow) {
    for (int c = 0; c < C; ++c) put(c, frame_at(fr.data, fr.stride, C, g, oy, ox, c));
    flush();
    return;
  }
  const float sy = (float)g.sz_h / (float)oh, sx = (float)g.sz_w / (float)ow;
  float fy = __builtin_fmaf(sy, (float)oy + 0.5f, -0.5f), fx = __builtin_fmaf(sx, (float)ox + 0.5f, -0.5f);
  fy = fy < 0.f ? 0.f : fy;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = (int)fy, x0 = (int)fx;
  const int y1 = y0 + (y0 < g.sz_h - 1 ? 1 : 0), x1 = x0 + (x0 < g.sz_w - 1 ? 1 : 0);
  const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
  for (int c = 0; c < C; ++c) {
    const float t0 = __builtin_fmaf(frame_at(fr.data, fr.stride, C, g, y0, x1, c), lx1,
                                    frame_at(fr.data, fr.stride, C, g, y0, x0, c) * lx0);
    const float t1 = __builtin_fmaf(frame_at(fr.data, fr.stride, C, g, y1, x1, c), lx1,
                                    frame_at(fr.data, fr.stride, C, g, y1, x0, c) * lx0);
    put(c, __builtin_fmaf(t1, ly1, t0 * ly0));
  }
  flush();
}

// pytracking dcf.max2d over an h x w map in LDS: the maximum and its (row, col) as torch.max(dim=-2) then
// torch.max(dim=-1) choose them (first maximal index along each reduction)
__device__ void max2d(const float* m, int h, int w, float* red_v, int* red_i, float& mx, int& row, int& col) {
  // column maxima (over rows, first row on ties), then the first column with the maximal column maximum
  const int t = threadIdx.x;
  if (t < w) {
    float best = m[t];
    int bi = 0;
    for (int r = 1; r < h; ++r)
      if (m[r * w + t] > best) {
        best = m[r * w + t];
        bi = r;
      }
    red_v[t] = best;
    red_i[t] = bi;
  }
  __syncthreads();
  float best = red_v[0];
  int bc = 0;
  for (int c = 1; c < w; ++c)
    if (red_v[c] > best) {
      best = red_v[c];
      bc = c;
    }
  mx = best;
  col = bc;
  row = red_i[bc];
  __syncthreads();
}

// update_sample_weights (dimp.py:585-607) on sw[kMem]; returns the replaced index
__device__ int update_sample_weights(float* sw, int num_samp, int num_init, int prev_ind, double lr,
                                     const mmt_dimp_track_params& p) {
  const bool init_w = p.init_samples_minimum_weight != 0;   // 0 -> None
  const int s_ind = init_w ? num_init : 0;
  int r_ind;
  if (num_samp == 0 || lr == 1.0) {
    for (int k = 0; k < kMem; ++k) sw[k] = 0.f;
    sw[0] = 1.f;
    r_ind = 0;
  } else {
    if (num_samp < kMem) {
      r_ind = num_samp;
    } else {
      r_ind = s_ind;
      for (int k = s_ind + 1; k < kMem; ++k)
        if (sw[k] < sw[r_ind]) r_ind = k;   // torch.min: first minimal index
    }
    const float den = pyf(1.0 - lr);
    if (prev_ind < 0) {
      for (int k = 0; k < kMem; ++k) sw[k] = sw[k] / den;
      sw[r_ind] = pyf(lr);
    } else {
      sw[r_ind] = sw[prev_ind] / den;
    }
  }
  float tot = 0.f;
  for (int k = 0; k < kMem; ++k) tot += sw[k];
  for (int k = 0; k < kMem; ++k) sw[k] = sw[k] / tot;
  if (init_w) {
    float init_sum = 0.f;
    for (int k = 0; k < num_init; ++k) init_sum += sw[k];
    // sw[:num_init].sum() < init_samp_weight: a float32 tensor against a Python float, compared in float32
    if (init_sum < pyf(p.init_samples_minimum_weight)) {
      float rest = 0.f;
      for (int k = num_init; k < kMem; ++k) rest += sw[k];
      const float d = pyf(p.init_samples_minimum_weight) + rest;
      for (int k = 0; k < kMem; ++k) sw[k] = sw[k] / d;
      const float v = pyf((double)p.init_samples_minimum_weight / num_init);
      for (int k = 0; k < num_init; ++k) sw[k] = v;
    }
  }
  return r_ind;
}

// one workgroup (256 threads) per sequence: scores [n][sh][sw] of this frame -> the tracker's update
__global__ __launch_bounds__(256) void dimp_localize_kernel(mmt_dimp_state* states, const float* scores, int sh, int sw_,
                                                            mmt_dimp_track_params p, mmt_dimp_result* results,
                                                            mmt_dimp_result* host_results) {
  __shared__ float sm[1024];
  __shared__ float red_v[64];
  __shared__ int red_i[64];
  __shared__ mmt_dimp_result sres;   // thread 0's decisions, broadcast to the block
  const int s = blockIdx.x, t = threadIdx.x;
  mmt_dimp_state& st = states[s];
  const int n = sh * sw_;
  for (int k = t; k < n; k += 256) sm[k] = scores[(int64_t)s * n + k];
  __syncthreads();
  float ms1;
  int r1, c1;
  max2d(sm, sh, sw_, red_v, red_i, ms1, r1, c1);
  mmt_dimp_result res{};
  if (t == 0) {
    st.frame_num += 1;   // track(): self.frame_num += 1 (dimp.py:98)
    // get_sample_location (dimp.py:314-319)
    const float* co = st.coords;
    float spos[2], ratio[2];
    for (int d = 0; d < 2; ++d) {
      spos[d] = 0.5f * (co[d] + co[d + 2] - 1.0f);
      ratio[d] = (co[d + 2] - co[d]) / p.img_sample_sz[d];
    }
    const float sscale = sqrtf(ratio[0] * ratio[1]);
    // localize_advanced (dimp.py:232-301), one scale
    const float score_sz[2] = {(float)sh, (float)sw_};
    float output_sz[2], score_center[2], disp1[2], tv1[2];
    for (int d = 0; d < 2; ++d) {
      output_sz[d] = score_sz[d] - fmodf(p.kernel_size[d] + 1.0f, 2.0f);
      score_center[d] = (score_sz[d] - 1.0f) / 2.0f;
    }
    const float md1[2] = {(float)r1, (float)c1};
    float unit[2];
    for (int d = 0; d < 2; ++d) {
      unit[d] = p.img_sample_sz[d] / output_sz[d];   // img_support_sz / output_sz
      disp1[d] = md1[d] - score_center[d];
      tv1[d] = disp1[d] * unit[d] * sscale;
    }
    int flag;
    float tv[2] = {tv1[0], tv1[1]};
    if ((double)ms1 < p.target_not_found_threshold) {
      flag = F_NOT_FOUND;
    } else if ((double)ms1 < p.uncertain_threshold) {
      flag = F_UNCERTAIN;
    } else if ((double)ms1 < p.hard_sample_threshold) {
      flag = F_HARD_NEGATIVE;
    } else {
      // the second peak outside the target neighbourhood
      float neigh[2];
      for (int d = 0; d < 2; ++d)
        neigh[d] = pyf(p.target_neighborhood_scale) * (st.target_sz[d] / sscale) * (output_sz[d] / p.img_sample_sz[d]);
      const int top = max((int)rint((double)md1[0] - (double)neigh[0] / 2), 0);
      const int bottom = min((int)rint((double)md1[0] + (double)neigh[0] / 2 + 1), sh);
      const int left = max((int)rint((double)md1[1] - (double)neigh[1] / 2), 0);
      const int right = min((int)rint((double)md1[1] + (double)neigh[1] / 2 + 1), sw_);
      res.aux[0] = top;   // passed to the whole block below through the result record
      res.aux[1] = bottom;
      res.aux[2] = left;
      res.aux[3] = right;
      flag = -1;          // decided after the masked maximum
    }
    res.flag = flag;
    res.tv[0] = tv[0];
    res.tv[1] = tv[1];
    res.sample_pos[0] = spos[0];
    res.sample_pos[1] = spos[1];
    res.sample_scale = sscale;
    res.max_score = ms1;
    sres = res;
  }
  __syncthreads();
  res = sres;
  if (res.flag < 0) {
    for (int k = t; k < n; k += 256) {
      const int r = k / sw_, c = k - r * sw_;
      if (r >= res.aux[0] && r < res.aux[1] && c >= res.aux[2] && c < res.aux[3]) sm[k] = 0.f;
    }
    __syncthreads();
  }
  float ms2 = 0.f;
  int r2 = 0, c2 = 0;
  if (res.flag < 0) max2d(sm, sh, sw_, red_v, red_i, ms2, r2, c2);
  if (t != 0) return;
  const float score_center[2] = {((float)sh - 1.0f) / 2.0f, ((float)sw_ - 1.0f) / 2.0f};
  const float output_sz[2] = {(float)sh - fmodf(p.kernel_size[0] + 1.0f, 2.0f), (float)sw_ - fmodf(p.kernel_size[1] + 1.0f, 2.0f)};
  float unit[2];
  for (int d = 0; d < 2; ++d) unit[d] = p.img_sample_sz[d] / output_sz[d];
  const float sscale = res.sample_scale;
  int flag = res.flag;
  float tv[2] = {res.tv[0], res.tv[1]};
  if (flag < 0) {
    const float disp1[2] = {(float)r1 - score_center[0], (float)c1 - score_center[1]};
    const float disp2[2] = {(float)r2 - score_center[0], (float)c2 - score_center[1]};
    float tv2[2], prev[2];
    for (int d = 0; d < 2; ++d) {
      tv2[d] = disp2[d] * unit[d] * sscale;
      prev[d] = (st.pos[d] - res.sample_pos[d]) / (unit[d] * sscale);
    }
    if (ms2 > pyf(p.distractor_threshold) * ms1) {
      const float a0 = disp1[0] - prev[0], a1 = disp1[1] - prev[1];
      const float b0 = disp2[0] - prev[0], b1 = disp2[1] - prev[1];
      const float n1 = sqrtf(a0 * a0 + a1 * a1), n2 = sqrtf(b0 * b0 + b1 * b1);
      const float thr = pyf(p.dispalcement_scale * sqrt((double)sh * sw_) / 2);
      if (n2 > thr && n1 < thr) {
        flag = F_HARD_NEGATIVE;
      } else if (n2 < thr && n1 > thr) {
        flag = F_HARD_NEGATIVE;
        tv[0] = tv2[0];
        tv[1] = tv2[1];
      } else {
        flag = F_UNCERTAIN;
      }
    } else if (ms2 > pyf(p.hard_negative_threshold) * ms1 && ms2 > pyf(p.target_not_found_threshold)) {
      // both tensor-vs-Python-float comparisons (dimp.py:298), so in float32; the max_score1.item() tests above
      // compare Python floats, in double
      flag = F_HARD_NEGATIVE;
    } else {
      flag = F_NORMAL;
    }
  }
  // new position and update_state (dimp.py:121-130, 518-529)
  if (flag != F_NOT_FOUND) {
    const float ts = fminf(fmaxf(sscale, st.min_scale_factor), st.max_scale_factor);
    st.target_scale = ts;
    for (int d = 0; d < 2; ++d) st.target_sz[d] = st.base_target_sz[d] * ts;
    for (int d = 0; d < 2; ++d) {
      const float np_ = res.sample_pos[d] + tv[d];
      const float off = pyf(p.target_inside_ratio - 0.5) * st.target_sz[d];
      st.pos[d] = fmaxf(fminf(np_, st.image_sz[d] - off), off);
    }
  }
  // update_classifier (dimp.py:538-570) bookkeeping: the memory slot and the Gauss-Newton iterations
  res.replace_ind = -1;
  res.num_iter = 0;
  const bool update = flag != F_NOT_FOUND && flag != F_UNCERTAIN;
  const bool hard = flag == F_HARD_NEGATIVE;
  if (update && p.update_classifier) {
    float tb[4];   // get_iounet_box (dimp.py:468-475)
    float c[2], bs[2];
    for (int d = 0; d < 2; ++d) {
      c[d] = (st.pos[d] - res.sample_pos[d]) / sscale + (p.img_sample_sz[d] - 1.0f) / 2.0f;
      bs[d] = st.target_sz[d] / sscale;
    }
    tb[0] = c[1] - (bs[1] - 1.0f) / 2.0f;
    tb[1] = c[0] - (bs[0] - 1.0f) / 2.0f;
    tb[2] = bs[1];
    tb[3] = bs[0];
    const double lr = hard ? p.hard_negative_learning_rate : p.learning_rate;
    if (hard || st.frame_num % p.train_sample_interval == 0) {
      const int r = update_sample_weights(st.sample_weights, st.num_stored, st.num_init, st.prev_replace, lr, p);
      st.prev_replace = r;
      for (int k = 0; k < 4; ++k) st.target_boxes[r][k] = tb[k];
      st.num_stored += 1;
      res.replace_ind = r;
    }
    if (hard) res.num_iter = p.net_opt_hn_iter;
    else if (p.low_score_opt_threshold == p.low_score_opt_threshold && p.low_score_opt_threshold > (double)ms1)
      res.num_iter = p.net_opt_low_iter;
    else if ((st.frame_num - 1) % p.train_skipping == 0) res.num_iter = p.net_opt_update_iter;
  }
  res.flag = flag;
  res.n_samples = min(st.num_stored, kMem);
  res.max_score = ms1;
  // new_state = cat(pos[[1, 0]] - (target_sz[[1, 0]] - 1) / 2, target_sz[[1, 0]])
  res.box[0] = st.pos[1] - (st.target_sz[1] - 1.0f) / 2.0f;
  res.box[1] = st.pos[0] - (st.target_sz[0] - 1.0f) / 2.0f;
  res.box[2] = st.target_sz[1];
  res.box[3] = st.target_sz[0];
  results[s] = res;
  if (host_results) host_results[s] = res;   // the record straight into the caller's pinned buffer (no copy launch)
}

// the frame's features into the memory slot update_sample_weights chose (training_samples[replace_ind] = x)
__global__ __launch_bounds__(256) void dimp_memory_kernel(const mmt_dimp_result* results, const float* x, int64_t feat_elems,
                                                          float* memory) {
  const int s = blockIdx.y;
  const int r = results[s].replace_ind;
  if (r < 0) return;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= feat_elems) return;
  const float4 v = *reinterpret_cast<const float4*>(x + (int64_t)s * feat_elems + i);
  *reinterpret_cast<float4*>(memory + ((int64_t)s * kMem + r) * feat_elems + i) = v;
}

}  // namespace mmt

using namespace mmt;

extern "C" {

size_t mmt_dimp_state_bytes(void) { return sizeof(mmt_dimp_state); }

int mmt_dimp_track_sample(mmt_dimp_state* states, const mmt_dimp_frame* frames, int n,
                          const mmt_dimp_track_params* p, int out_h, int out_w, float* patches, void* stream) {
  if (!states || !frames || !p || !patches || n <= 0 || out_h <= 0 || out_w <= 0) return MMT_E_ARG;
  const dim3 grid((unsigned)(((int64_t)out_h * out_w + 255) / 256), n);
  hipLaunchKernelGGL(dimp_sample_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, states, frames, *p, out_h,
                     out_w, patches, NormArgs{});
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_dimp_track_sample_norm4(mmt_dimp_state* states, const mmt_dimp_frame* frames, int n,
                                const mmt_dimp_track_params* p, int out_h, int out_w, const float mean[3],
                                const float std_[3], float* out_a, float* out_b, float* zero_words, int64_t n_zero,
                                void* stream) {
  if (!states || !frames || !p || !mean || !std_ || !out_a || !out_b || n <= 0 || out_h <= 0 || out_w <= 0 ||
      n_zero < 0 || (n_zero && !zero_words))
    return MMT_E_ARG;
  NormArgs na{{mean[0], mean[1], mean[2]}, {std_[0], std_[1], std_[2]}, out_a, out_b, zero_words, n_zero};
  const dim3 grid((unsigned)(((int64_t)out_h * out_w + 255) / 256), n);
  hipLaunchKernelGGL(dimp_sample_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, states, frames, *p, out_h,
                     out_w, nullptr, na);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_dimp_track_update_pinned(mmt_dimp_state* states, int n, const float* scores, int sh, int sw,
                                 const mmt_dimp_track_params* p, const float* feat, int64_t feat_elems, float* memory,
                                 mmt_dimp_result* results, mmt_dimp_result* host_results, void* stream) {
  if (!states || !scores || !p || !feat || !memory || !results || n <= 0 || sh <= 0 || sw <= 0 || sh * sw > 1024 ||
      sw > 64 || feat_elems <= 0 || feat_elems % 4 || p->sample_memory_size != kMem || p->train_skipping <= 0 ||
      p->train_sample_interval <= 0)
    return MMT_E_ARG;
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(dimp_localize_kernel, dim3(n), dim3(256), 0, s, states, scores, sh, sw, *p, results,
                     host_results);
  hipLaunchKernelGGL(dimp_memory_kernel, dim3((unsigned)((feat_elems / 4 + 255) / 256), n), dim3(256), 0, s, results,
                     feat, feat_elems, memory);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_dimp_track_update(mmt_dimp_state* states, int n, const float* scores, int sh, int sw,
                          const mmt_dimp_track_params* p, const float* feat, int64_t feat_elems, float* memory,
                          mmt_dimp_result* results, void* stream) {
  return mmt_dimp_track_update_pinned(states, n, scores, sh, sw, p, feat, feat_elems, memory, results, nullptr,
                                      stream);
}

}  // extern "C"
