// C ABI of the DiMP classifier inner loop (include/mmtrack.h, mmt_dimp_*).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "../../include/mmtrack.h"
#include "dimp.h"

using namespace mmt;

namespace {

struct WsLayout {
  size_t label, mask, sw, rm, smask, scratch, grad, gsq, rsq, sgsq, loss, centers, sqrtsw, params, total;
};

WsLayout layout(int I, int S, int C, int H, int W, int fh, int fw, int num_iter) {
  const size_t Ho = H + (fh + 1) % 2, Wo = W + (fw + 1) % 2, n = Ho * Wo, IS = (size_t)I * S;
  const size_t nby = dimp_geo(C, H, W, fh, fw).nbands;
  WsLayout L{};
  size_t off = 0;
  auto take = [&](size_t floats) {
    size_t o = off;
    off += (floats * 4 + 255) & ~size_t(255);
    return o;
  };
  L.label = take(IS * n);
  L.mask = take(IS * n);
  L.sw = take(IS * n);
  L.rm = take(IS * n);
  L.smask = take(IS * n);
  L.scratch = take(IS * n);
  L.grad = take((size_t)S * C * fh * fw);
  L.gsq = take((size_t)S * C);
  L.rsq = take(IS * nby);
  L.sgsq = take(IS * nby);
  L.loss = take(num_iter + 1);
  L.centers = take(IS * 2);
  L.sqrtsw = take(IS);
  L.params = take(3 * 128);
  L.total = off;
  return L;
}

bool bad_dims(int I, int S, int C, int H, int W, int fh, int fw) {
  return I <= 0 || S <= 0 || C <= 0 || H <= 0 || W <= 0 || fh <= 0 || fw <= 0 || fh * fw > 25 ||
         !dimp_geo_ok(C, H, W, fh, fw);
}

}  // namespace

extern "C" {

size_t mmt_dimp_workspace_bytes(int I, int S, int C, int H, int W, int fh, int fw, int num_iter) {
  if (bad_dims(I, S, C, H, W, fh, fw) || num_iter < 0) return 0;
  return layout(I, S, C, H, W, fh, fw, num_iter).total;
}

int mmt_dimp_apply_filter(const float* feat, const float* w, float* scores, int I, int S, int C, int H, int W, int fh,
                          int fw, void* stream) {
  if (!feat || !w || !scores || bad_dims(I, S, C, H, W, fh, fw)) return MMT_E_ARG;
  DimpFilter a{};
  a.feat = feat;
  a.w = w;
  a.I = I; a.S = S; a.C = C; a.H = H; a.W = W; a.fh = fh; a.fw = fw;
  a.seq_stride = (int64_t)C * H * W;
  a.img_stride = S * a.seq_stride;
  a.Ho = H + 2 * (fh / 2) - fh + 1;
  a.Wo = W + 2 * (fw / 2) - fw + 1;
  a.mode = 0;
  a.out = scores;
  dimp_filter(a, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_dimp_feat_transpose(const float* feat, const float* r, float* grad, int I, int S, int C, int H, int W, int fh,
                            int fw, void* stream) {
  if (!feat || !r || !grad || bad_dims(I, S, C, H, W, fh, fw)) return MMT_E_ARG;
  DimpTranspose a{};
  a.feat = feat;
  a.r = r;
  a.I = I; a.S = S; a.C = C; a.H = H; a.W = W; a.fh = fh; a.fw = fw;
  a.seq_stride = (int64_t)C * H * W;
  a.img_stride = S * a.seq_stride;
  a.Ho = H + 2 * (fh / 2) - fh + 1;
  a.Wo = W + 2 * (fw / 2) - fw + 1;
  a.grad = grad;
  dimp_transpose(a, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

// the Gauss-Newton loop of mmt_dimp_optimize / _dev once the per-sample constants are in the workspace
// ctl: per-sequence steps / sample counts in device memory (null: num_iter steps over all I samples)
static int optimize_body(const float* feat, int64_t img_stride, int64_t seq_stride, int I, int S, int C, int H, int W,
                         float* weights, int fh, int fw, const mmt_dimp_params* p, int num_iter, char* ws,
                         const WsLayout& L, float* losses, hipStream_t st, const mmt_dimp_result* ctl = nullptr) {
  auto F = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const int IS = I * S;
  const int Ho = H + (fh + 1) % 2, Wo = W + (fw + 1) % 2, nby = dimp_geo(C, H, W, fh, fw).nbands;
  const float step = std::exp(p->log_step_length);
  const float reg = std::fmax(p->filter_reg * p->filter_reg, p->min_filter_reg * p->min_filter_reg);

  DimpMaps m{IS, Ho, Wo, p->num_dist_bins, p->bin_displacement, F(L.centers), F(L.sqrtsw), F(L.params),
             F(L.params) + 128, F(L.params) + 256, F(L.label), F(L.mask), F(L.sw), S, ctl};
  dimp_maps(m, st);

  DimpFilter fa{};
  fa.feat = feat;
  fa.img_stride = img_stride;
  fa.seq_stride = seq_stride;
  fa.I = I; fa.S = S; fa.C = C; fa.H = H; fa.W = W; fa.fh = fh; fa.fw = fw; fa.Ho = Ho; fa.Wo = Wo;
  fa.label = F(L.label);
  fa.mask = F(L.mask);
  fa.sw = F(L.sw);
  fa.smask = F(L.smask);
  fa.ctl = ctl;
  DimpTranspose ta{};
  ta.feat = feat;
  ta.img_stride = img_stride;
  ta.seq_stride = seq_stride;
  ta.r = F(L.rm);
  ta.w = weights;
  ta.reg = reg;
  ta.I = I; ta.S = S; ta.C = C; ta.H = H; ta.W = W; ta.fh = fh; ta.fw = fw; ta.Ho = Ho; ta.Wo = Wo;
  ta.grad = F(L.grad);
  ta.gsq = F(L.gsq);
  ta.ctl = ctl;
  DimpUpdate ua{weights, F(L.grad), F(L.gsq), F(L.sgsq), I, S, C, fh, fw, nby, reg, p->alpha_eps, step, ctl, 0};
  const int nw = S * C * fh * fw;
  for (int it = 0; it < num_iter; ++it) {
    fa.it = ta.it = ua.it = it;
    fa.mode = 1;               // residuals at the current filter
    fa.w = weights;
    fa.out = F(L.rm);
    fa.partial = F(L.rsq);
    dimp_filter(fa, st);
    if (losses) dimp_loss(F(L.rsq), IS * nby, weights, nw, reg, S, F(L.loss) + it, st);
    dimp_transpose(ta, st);    // gradient
    fa.mode = 2;               // |J g|^2
    fa.w = F(L.grad);
    fa.out = nullptr;
    fa.partial = F(L.sgsq);
    dimp_filter(fa, st);
    dimp_update(ua, st);       // Gauss-Newton step
  }
  if (losses) {
    fa.mode = 1;
    fa.w = weights;
    fa.out = F(L.scratch);
    fa.smask = F(L.scratch);
    fa.partial = F(L.rsq);
    dimp_filter(fa, st);
    dimp_loss(F(L.rsq), IS * nby, weights, nw, reg, S, F(L.loss) + num_iter, st);
    if (hipMemcpyAsync(losses, F(L.loss), (num_iter + 1) * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return MMT_E_HIP;
  }
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_dimp_optimize(const float* feat, int I, int S, int C, int H, int W, float* weights, int fh, int fw,
                      const float* bb, const float* sample_weight, const mmt_dimp_params* p, int num_iter,
                      void* workspace, size_t ws_bytes, float* losses, void* stream_) {
  if (!feat || !weights || !bb || !p || !workspace || num_iter < 0 || bad_dims(I, S, C, H, W, fh, fw) ||
      p->num_dist_bins <= 0 || p->num_dist_bins > 128)
    return MMT_E_ARG;
  const WsLayout L = layout(I, S, C, H, W, fh, fw, num_iter);
  if (ws_bytes < L.total) return MMT_E_ARG;
  hipStream_t st = (hipStream_t)stream_;
  char* ws = static_cast<char*>(workspace);
  auto F = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const int IS = I * S;
  // optimizer.py:108-125's per-sample constants from the host values, passed by value to the kernels that
  // store them in the workspace (no host staging buffer, nothing to wait for)
  DimpPrepArgs pa{};
  pa.I = I;
  pa.has_sw = sample_weight ? 1 : 0;
  pa.feat_stride = p->feat_stride;
  pa.off0 = (float)(fh % 2) / 2.0f;
  pa.off1 = (float)(fw % 2) / 2.0f;
  pa.centers = F(L.centers);
  pa.sqrtsw = F(L.sqrtsw);
  for (int k0 = 0; k0 < IS; k0 += kDimpPrepChunk) {
    pa.k0 = k0;
    pa.n = std::min(kDimpPrepChunk, IS - k0);
    std::memcpy(pa.bb, bb + 4 * k0, (size_t)pa.n * 16);
    if (sample_weight) std::memcpy(pa.sw, sample_weight + k0, (size_t)pa.n * 4);
    dimp_prep_args(pa, st);
  }
  DimpParamArgs pr{};
  std::memcpy(pr.v, p->label_w, 128 * 4);
  std::memcpy(pr.v + 128, p->mask_w, 128 * 4);
  std::memcpy(pr.v + 256, p->spatial_w, 128 * 4);
  pr.dst = F(L.params);
  dimp_params(pr, st);
  const int64_t chw = (int64_t)C * H * W;
  return optimize_body(feat, S * chw, chw, I, S, C, H, W, weights, fh, fw, p, num_iter, ws, L, losses, st);
}

int mmt_dimp_optimize_strided(const float* feat, int64_t feat_img_stride, int64_t feat_seq_stride, int I, int S,
                              int C, int H, int W, float* weights, int fh, int fw, const float* bb_dev,
                              int64_t bb_img_stride, int64_t bb_seq_stride, const float* sample_weight_dev,
                              int64_t sw_img_stride, int64_t sw_seq_stride, const mmt_dimp_params* p, int num_iter,
                              void* workspace, size_t ws_bytes, void* stream_) {
  if (!feat || !weights || !bb_dev || !p || !workspace || num_iter < 0 || bad_dims(I, S, C, H, W, fh, fw) ||
      p->num_dist_bins <= 0 || p->num_dist_bins > 128 || feat_img_stride < -1 || feat_seq_stride < -1 ||
      bb_img_stride < -1 || bb_seq_stride < -1 || sw_img_stride < -1 || sw_seq_stride < -1)
    return MMT_E_ARG;
  const WsLayout L = layout(I, S, C, H, W, fh, fw, num_iter);
  if (ws_bytes < L.total) return MMT_E_ARG;
  hipStream_t st = (hipStream_t)stream_;
  char* ws = static_cast<char*>(workspace);
  auto F = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const int64_t chw = (int64_t)C * H * W;
  // strides -1: the contiguous [I][S] layouts (0 is a real stride: one sample broadcast over the sequences)
  if (feat_seq_stride < 0) feat_seq_stride = chw;
  if (feat_img_stride < 0) feat_img_stride = S * feat_seq_stride;
  if (bb_seq_stride < 0) bb_seq_stride = 4;
  if (bb_img_stride < 0) bb_img_stride = S * bb_seq_stride;
  if (sw_seq_stride < 0) sw_seq_stride = 1;
  if (sw_img_stride < 0) sw_img_stride = S * sw_seq_stride;
  DimpPrep pp{bb_dev, sample_weight_dev, bb_img_stride, bb_seq_stride, sw_img_stride, sw_seq_stride, I * S, I, S,
              p->feat_stride, (float)(fh % 2) / 2.0f, (float)(fw % 2) / 2.0f, F(L.centers), F(L.sqrtsw)};
  dimp_prep(pp, st);
  DimpParamArgs pr{};
  std::memcpy(pr.v, p->label_w, 128 * 4);
  std::memcpy(pr.v + 128, p->mask_w, 128 * 4);
  std::memcpy(pr.v + 256, p->spatial_w, 128 * 4);
  pr.dst = F(L.params);
  dimp_params(pr, st);
  return optimize_body(feat, feat_img_stride, feat_seq_stride, I, S, C, H, W, weights, fh, fw, p, num_iter, ws, L,
                       nullptr, st);
}

size_t mmt_dimp_track_optimize_ws_bytes(int n, int C, int H, int W, int fh, int fw, int max_iter) {
  return mmt_dimp_workspace_bytes(MMT_DIMP_MEMORY, n, C, H, W, fh, fw, max_iter);
}

int mmt_dimp_track_optimize(const mmt_dimp_state* states, int n, const mmt_dimp_result* results, const float* memory,
                            int C, int H, int W, float* filters, int fh, int fw, const mmt_dimp_params* p, int max_iter,
                            void* workspace, size_t ws_bytes, void* stream_) {
  constexpr int I = MMT_DIMP_MEMORY;
  if (!states || !results || !memory || !filters || !p || !workspace || n <= 0 || max_iter < 0 ||
      bad_dims(I, n, C, H, W, fh, fw) || p->num_dist_bins <= 0 || p->num_dist_bins > 128)
    return MMT_E_ARG;
  const WsLayout L = layout(I, n, C, H, W, fh, fw, max_iter);
  if (ws_bytes < L.total) return MMT_E_ARG;
  if (max_iter == 0) return MMT_OK;
  hipStream_t st = (hipStream_t)stream_;
  char* ws = static_cast<char*>(workspace);
  auto F = [&](size_t off) { return reinterpret_cast<float*>(ws + off); };
  const int64_t chw = (int64_t)C * H * W, sf = (int64_t)(sizeof(mmt_dimp_state) / sizeof(float));
  static_assert(sizeof(mmt_dimp_state) % sizeof(float) == 0, "state stride in floats");
  // every sequence's boxes / weights in its state, its samples in its memory slot ([n][I][C][H][W])
  DimpPrep pp{states->target_boxes[0], states->sample_weights, 4, sf, 1, sf, I * n, I, n, p->feat_stride,
              (float)(fh % 2) / 2.0f, (float)(fw % 2) / 2.0f, F(L.centers), F(L.sqrtsw)};
  dimp_prep(pp, st);
  DimpParamArgs pr{};
  std::memcpy(pr.v, p->label_w, 128 * 4);
  std::memcpy(pr.v + 128, p->mask_w, 128 * 4);
  std::memcpy(pr.v + 256, p->spatial_w, 128 * 4);
  pr.dst = F(L.params);
  dimp_params(pr, st);
  return optimize_body(memory, chw, I * chw, I, n, C, H, W, filters, fh, fw, p, max_iter, ws, L, nullptr, st,
                       results);
}

}  // extern "C"
