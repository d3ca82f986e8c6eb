// SiamFC per-frame kernels (RGBE/models/siamfc; the published SiamFC tracker, source absent from the
// reference -- parity unpinned beyond the restated algorithm):
//  * siamfc_crop: crop_and_resize for the exemplar / the 3-scale instance pyramid straight from the
//    HBM-resident H x W x C uint8 frame: square window of side round(size) at round(center - (size-1)/2),
//    constant border = the frame's mean colour (cv2.copyMakeBorder BORDER_CONSTANT), cv2 INTER_LINEAR
//    resize, written as float NCHW or NHWC (raw 0..255, what the AlexNet backbone consumes);
//  * siamfc_response: the post-correlation step of TrackerSiamFC.update -- INTER_CUBIC x16 upsampling
//    of every scale's 17x17 response, scale penalty, first-max scale selection, min/sum normalisation,
//    cosine-window blend in double, first-occurrence argmax.
#include "cvresize.h"
#include "kernels.h"

namespace mmt {

__global__ __launch_bounds__(256) void siamfc_crop_kernel(const SiamCropArgs a) {
  const int n = blockIdx.y;
  const int O = a.out_sz;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= O * O) return;
  const int oy = idx / O, ox = idx - oy * O;
  const int y0 = a.y0[n], x0 = a.x0[n], S = a.size[n];
  auto px = [&](int r, int x, int c) -> int {
    const int yy = y0 + r, xx = x0 + x;
    if (yy < 0 || yy >= a.H || xx < 0 || xx >= a.W) return a.pad[c];
    return a.frame[(int64_t)yy * a.stride + (int64_t)xx * a.C + c];
  };
  int u8[3];
  cv_linear_u8(px, S, O, oy, ox, 3, u8);
  if (a.nhwc) {   // [n][O][O][3]: the HIP AlexNet's input layout
    float* o = a.out + ((int64_t)n * O * O + idx) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] = (float)u8[c];
    return;
  }
  float* o = a.out + (int64_t)n * 3 * O * O + idx;
#pragma unroll
  for (int c = 0; c < 3; ++c) o[(int64_t)c * O * O] = (float)u8[c];
}

void siamfc_crop(const SiamCropArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(siamfc_crop_kernel, dim3((a.out_sz * a.out_sz + 255) / 256, a.n), dim3(256), 0, s, a);
}

constexpr int RT = 1024;

__device__ __forceinline__ float block_reduce_f(float v, float* red, bool is_max, bool is_min) {
  const int t = threadIdx.x;
  for (int o = 32; o >= 1; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, u) : (is_min ? fminf(v, u) : v + u);
  }
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = v;
  __syncthreads();
  if (t < 64) {
    v = t < RT / 64 ? red[t] : (is_max ? -INFINITY : (is_min ? INFINITY : 0.f));
    for (int o = 32; o >= 1; o >>= 1) {
      const float u = __shfl_xor(v, o, 64);
      v = is_max ? fmaxf(v, u) : (is_min ? fminf(v, u) : v + u);
    }
    if (t == 0) red[RT / 64] = v;
  }
  __syncthreads();
  return red[RT / 64];
}

__global__ __launch_bounds__(RT) void siamfc_response_kernel(const SiamRespArgs a) {
#pragma clang fp contract(off)   // numpy's separate float32 / float64 roundings
  __shared__ float red[RT / 64 + 1];
  __shared__ double dv[RT];
  __shared__ int di[RT];
  __shared__ float smax[8];
  const int t = threadIdx.x, U = a.up, UU = U * U, mid = a.n / 2;
  // 1. upsample every scale, penalise the off-centre scales, per-scale max
  for (int s = 0; s < a.n; ++s) {
    const float* src = a.resp + (int64_t)s * a.r * a.r;
    float* dst = a.scratch + (int64_t)s * UU;
    float m = -INFINITY;
    for (int i = t; i < UU; i += RT) {
      const int oy = i / U, ox = i - oy * U;
      float v = cv_cubic_f32(src, a.r, U, oy, ox);
      if (s != mid) v = __fmul_rn(v, a.penalty);
      dst[i] = v;
      m = fmaxf(m, v);
    }
    m = block_reduce_f(m, red, true, false);
    if (t == 0) smax[s] = m;
  }
  __syncthreads();
  int sid = 0;
  for (int s = 1; s < a.n; ++s)
    if (smax[s] > smax[sid]) sid = s;
  const float* r = a.scratch + (int64_t)sid * UU;
  // 2. response -= min; response /= sum + 1e-16
  float mn = INFINITY;
  for (int i = t; i < UU; i += RT) mn = fminf(mn, r[i]);
  mn = block_reduce_f(mn, red, false, true);
  float sm = 0.f;
  for (int i = t; i < UU; i += RT) sm += __fsub_rn(r[i], mn);
  sm = block_reduce_f(sm, red, false, false);
  const float div = (float)((double)sm + 1e-16);
  // 3. (1 - wi) * response + wi * hann (double), first-occurrence argmax
  double best = -1e300;
  int bi = 0x7fffffff;
  for (int i = t; i < UU; i += RT) {
    const int y = i / U, x = i - y * U;
    const float nv = __fdiv_rn(__fsub_rn(r[i], mn), div);
    const double v = (double)__fmul_rn(a.one_minus_wi, nv) + a.wi * ((a.hann1d[y] * a.hann1d[x]) / a.hann_sum);
    if (v > best) { best = v; bi = i; }
  }
  dv[t] = best;
  di[t] = bi;
  __syncthreads();
  for (int st = RT / 2; st > 0; st >>= 1) {
    if (t < st) {
      const double v2 = dv[t + st];
      const int i2 = di[t + st];
      if (v2 > dv[t] || (v2 == dv[t] && i2 < di[t])) { dv[t] = v2; di[t] = i2; }
    }
    __syncthreads();
  }
  if (t == 0) {
    a.result[0] = (float)sid;
    a.result[1] = (float)(di[0] / U);
    a.result[2] = (float)(di[0] % U);
    a.result[3] = (float)dv[0];
  }
}

void siamfc_response(const SiamRespArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(siamfc_response_kernel, dim3(1), dim3(RT), 0, s, a);
}

}  // namespace mmt
