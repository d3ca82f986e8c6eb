// OpenCV cv::resize restatements shared by the crop kernels (device side).
//  * INTER_LINEAR on CV_8U (imgproc/src/resize.cpp): 11-bit fixed-point coefficients, x-border clamp of
//    (sx, fx), y-border row clamp, SIMD vertical rounding (((D0>>4)*b0>>16) + ((D1>>4)*b1>>16) + 2) >> 2;
//    an exact 2x down-scale is INTER_AREA's fast path (a+b+c+d+2)>>2.
//  * INTER_CUBIC on CV_32F: A = -0.75 coefficients in float, replicate borders, separate mul/add.
#pragma once
#include <float.h>

#include "common.h"

namespace mmt {

// px(r, x, c) -> int pixel of the S x S source (already padded); writes u8[0..C)
template <class Px>
__device__ __forceinline__ void cv_linear_u8(const Px& px, int S, int O, int oy, int ox, int C, int* u8) {
  const double scale = 1.0 / ((double)O / (double)S);
  if (fabs(scale - 2.0) < DBL_EPSILON) {
    for (int c = 0; c < C; ++c) {
      const int s = px(2 * oy, 2 * ox, c) + px(2 * oy, 2 * ox + 1, c) + px(2 * oy + 1, 2 * ox, c) +
                    px(2 * oy + 1, 2 * ox + 1, c);
      u8[c] = (s + 2) >> 2;
    }
    return;
  }
  float fx = (float)((ox + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { fx = 0.f; sx = 0; }
  if (sx >= S - 1) { fx = 0.f; sx = S - 1; }
  const int a0 = __float2int_rn((1.f - fx) * 2048.f), a1 = __float2int_rn(fx * 2048.f);
  float fy = (float)((oy + 0.5) * scale - 0.5);
  const int sy = (int)floorf(fy);
  fy -= (float)sy;
  const int b0 = __float2int_rn((1.f - fy) * 2048.f), b1 = __float2int_rn(fy * 2048.f);
  const int r0 = min(max(sy, 0), S - 1), r1 = min(max(sy + 1, 0), S - 1);
  const int sx1 = min(sx + 1, S - 1);
  for (int c = 0; c < C; ++c) {
    const int d0 = px(r0, sx, c) * a0 + px(r0, sx1, c) * a1;
    const int d1 = px(r1, sx, c) * a0 + px(r1, sx1, c) * a1;
    const int v = (((d0 >> 4) * b0) >> 16) + (((d1 >> 4) * b1) >> 16);
    u8[c] = min(max((v + 2) >> 2, 0), 255);
  }
}

// interpolateCubic (resize.cpp): coefficients for fractional offset x, A = -0.75
__device__ __forceinline__ void cv_cubic_coeffs(float x, float* c) {
#pragma clang fp contract(off)   // separate roundings (HIP's __fmul_rn / __fadd_rn are plain operators)
  const float A = -0.75f;
  const float x1 = __fadd_rn(x, 1.f), omx = __fsub_rn(1.f, x);
  c[0] = __fsub_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fsub_rn(__fmul_rn(A, x1), 5.f * A), x1), 8.f * A), x1), 4.f * A);
  c[1] = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(__fmul_rn(A + 2.f, x), A + 3.f), x), x), 1.f);
  c[2] = __fadd_rn(__fmul_rn(__fmul_rn(__fsub_rn(__fmul_rn(A + 2.f, omx), A + 3.f), omx), omx), 1.f);
  c[3] = __fsub_rn(__fsub_rn(__fsub_rn(1.f, c[0]), c[1]), c[2]);
}

// INTER_CUBIC sample (oy, ox) of the O x O resize of an S x S float map (row pitch S)
__device__ __forceinline__ float cv_cubic_f32(const float* src, int S, int O, int oy, int ox) {
#pragma clang fp contract(off)
  const double scale = 1.0 / ((double)O / (double)S);
  float fx = (float)((ox + 0.5) * scale - 0.5), fy = (float)((oy + 0.5) * scale - 0.5);
  const int sx = (int)floorf(fx), sy = (int)floorf(fy);
  fx = __fsub_rn(fx, (float)sx);
  fy = __fsub_rn(fy, (float)sy);
  float ax[4], by[4];
  cv_cubic_coeffs(fx, ax);
  cv_cubic_coeffs(fy, by);
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = min(max(sy + k - 1, 0), S - 1);
    const float* row = src + r * S;
    float h = __fmul_rn(row[min(max(sx - 1, 0), S - 1)], ax[0]);
    h = __fadd_rn(h, __fmul_rn(row[min(max(sx, 0), S - 1)], ax[1]));
    h = __fadd_rn(h, __fmul_rn(row[min(max(sx + 1, 0), S - 1)], ax[2]));
    h = __fadd_rn(h, __fmul_rn(row[min(max(sx + 2, 0), S - 1)], ax[3]));
    acc = k == 0 ? __fmul_rn(h, by[0]) : __fadd_rn(acc, __fmul_rn(h, by[k]));
  }
  return acc;
}

}  // namespace mmt
