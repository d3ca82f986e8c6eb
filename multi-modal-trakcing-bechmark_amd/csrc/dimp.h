// DiMP classifier kernels (dimp.hip) -- launch interfaces.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmtrack.h"

namespace mmt {

constexpr int kDimpStage = 24;   // staged floats per thread per chunk (6144 per workgroup and LDS buffer)

// launch geometry of the correlation kernels for C channels of H x W maps and an fh x fw filter: dimp_filter
// takes bands of RB output rows (RB * Wo <= 64 positions; partial sums per band: nbands per image * sequence)
// and chunks of CC channels; dimp_transpose CT channels per workgroup (CT * taps <= 128)
struct DimpGeo {
  int Ho, Wo, RB, nbands, CC, CT, filter_stage, transpose_stage;
};
inline DimpGeo dimp_geo(int C, int H, int W, int fh, int fw) {
  DimpGeo g{};
  g.Ho = H + (fh + 1) % 2;
  g.Wo = W + (fw + 1) % 2;
  g.RB = g.Wo >= 64 ? 1 : 64 / g.Wo;
  if (g.RB > g.Ho) g.RB = g.Ho;
  g.nbands = (g.Ho + g.RB - 1) / g.RB;
  const int T = fh * fw, Wp = g.Wo + fw - 1;
  const int fplane = (g.RB + fh - 1) * Wp, tplane = (g.Ho + fh - 1) * Wp;
  g.CC = 32;   // channels per chunk: a divisor of C
  while (g.CC > 1 && (g.CC * (fplane + T) > kDimpStage * 256 || C % g.CC)) g.CC /= 2;
  g.filter_stage = g.CC * (fplane + T);
  g.CT = 16;   // a divisor of C
  while (g.CT > 1 && (g.CT * T > 128 || g.CT * tplane + g.Ho * g.Wo > kDimpStage * 256 || C % g.CT)) g.CT /= 2;
  g.transpose_stage = g.CT * tplane + g.Ho * g.Wo;
  return g;
}
// the shapes the staging supports: a chunk of one channel (filter) / one channel + the residual map
// (transpose) fits the per-thread registers, Wo <= 64
inline bool dimp_geo_ok(int C, int H, int W, int fh, int fw) {
  const DimpGeo g = dimp_geo(C, H, W, fh, fw);
  return g.Wo <= 64 && g.filter_stage <= kDimpStage * 256 && g.transpose_stage <= kDimpStage * 256;
}

struct DimpMaps {                 // label / target-mask / sample-weight maps from the distance bins
  int IS, Ho, Wo, nbins;
  float bin_disp;
  const float* centers;           // [IS][2] (y, x) in feature cells
  const float* sqrt_sw;           // [IS] sqrt of the per-sample weight
  const float* label_w; const float* mask_w; const float* spatial_w;   // [nbins] (device)
  float* label; float* mask; float* sw;                                 // [IS][Ho][Wo]
  int S;                          // sequences (is = i * S + s)
  const mmt_dimp_result* ctl;     // sequences with no steps this frame are skipped (null: none skipped)
};
struct DimpFilter {
  const float* feat;              // [I][S][C][H][W]: sample (i, s) at feat + i * img_stride + s * seq_stride
  int64_t img_stride, seq_stride; // floats
  const float* w;                 // [S][C][fh][fw]
  int I, S, C, H, W, fh, fw, Ho, Wo;
  int mode;                       // 0: scores, 1: residual step (out = mapped residual), 2: |J g|^2 partials
  float* out;
  const float* label; const float* mask; const float* sw;
  float* smask;                   // mode 1 writes the activation derivative, mode 2 reads it
  float* partial;                 // [I*S][nbands] band partial sums of squares (or null)
  const mmt_dimp_result* ctl;     // per-sequence steps / sample counts (device), or null: all
  int it;                         // the Gauss-Newton step this launch belongs to (with ctl)
  int RB, CC;                     // set by dimp_filter (dimp_geo)
};
struct DimpTranspose {
  const float* feat; const float* r;   // r: [I][S][Ho][Wo]
  int64_t img_stride, seq_stride;      // of feat, as DimpFilter
  const float* w; float reg;           // optional: grad += reg * w
  int I, S, C, H, W, fh, fw, Ho, Wo;
  float* grad;                         // [S][C][fh][fw]
  float* gsq;                          // [S][C] partial |g|^2 (or null)
  const mmt_dimp_result* ctl;          // as DimpFilter
  int it;
  int CT;                              // set by dimp_transpose (dimp_geo)
};
struct DimpUpdate {
  float* w; const float* grad; const float* gsq; const float* sgsq;
  int I, S, C, fh, fw, nby;
  float reg, alpha_eps, step;
  const mmt_dimp_result* ctl;     // as DimpFilter
  int it;
};

// optimizer.py:108-125's per-sample constants, formed on the device: centers [IS][2] = ((y + h / 2) / stride - off0,
// (x + w / 2) / stride - off1) of bb [IS][4] (x, y, w, h), sqrtsw [IS] = sqrt(sample_weight) (null: 1 / I)
struct DimpPrep {
  const float* bb; const float* sw;   // device; sample (i, s) at bb + i * bb_i + s * bb_s, sw + i * sw_i + s * sw_s (floats)
  int64_t bb_i, bb_s, sw_i, sw_s;
  int IS, I, S;
  float feat_stride, off0, off1;
  float* centers; float* sqrtsw;
};
constexpr int kDimpPrepChunk = 160;   // samples per by-value launch (kernel arguments <= 4 KB)
struct DimpPrepArgs {                 // the same from host values, by value
  float bb[kDimpPrepChunk * 4];
  float sw[kDimpPrepChunk];
  int k0, n, I, has_sw;
  float feat_stride, off0, off1;
  float* centers; float* sqrtsw;
};
struct DimpParamArgs { float v[3 * 128]; float* dst; };   // label / mask / spatial predictor weights
void dimp_prep(const DimpPrep& a, hipStream_t s);
void dimp_prep_args(const DimpPrepArgs& a, hipStream_t s);
void dimp_params(const DimpParamArgs& a, hipStream_t s);
void dimp_maps(const DimpMaps& m, hipStream_t s);
void dimp_filter(const DimpFilter& a, hipStream_t s);
void dimp_transpose(const DimpTranspose& a, hipStream_t s);
void dimp_update(const DimpUpdate& a, hipStream_t s);
void dimp_loss(const float* rsq, int nparts, const float* w, int nw, float reg, int S, float* loss, hipStream_t s);

}  // namespace mmt
