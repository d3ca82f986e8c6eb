// RGB-D frame assembly on the GPU: get_rgbd_frame(..., dtype='rgbcolormap',
// depth_clip=True) of ViPT/lib/train/dataset/depth_utils.py:7-58 as used by the RGB-D VOT path
// (ViPT/lib/test/vot/vipt_class.py:79, 92):
//   depth clip   max_depth = min(median(dp) * 3, 10000); dp[dp > max_depth] = max_depth   (uint16)
//   normalise    cv2.normalize(dp, None, 0, 255, NORM_MINMAX): scale = 255 / (max - min) (0 when
//                max == min), shift = -min * scale, out = saturate_cast<ushort>(dp * scale + shift)
//                (OpenCV's convertTo arithmetic: float scale / shift, round to nearest even)
//   colormap     cv2.applyColorMap(u8, COLORMAP_JET): a 256-entry BGR table
//   merge        cv2.merge((rgb, colormap)) -> H x W x 6 uint8 = R G B | B' G' R'
// Parity is unpinned at the OpenCV boundary (no cv2 in this image): the JET table is the published
// piecewise-linear definition unless the caller passes OpenCV's own table.
// Three launches: histogram + min/max (LDS-private per workgroup, then exact integer atomics: deterministic),
// one workgroup to find the median and the normalisation constants, then the per-pixel map.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mmtrack.h"

namespace mmt {

// COLORMAP_JET as the published piecewise-linear definition (lib/train/dataset/depth_utils.py JET_BGR)
__device__ __forceinline__ uint8_t jet_chan(double x, double a, double b) {   // clip(min(4x + a, -4x + b), 0, 1)
  const double v = fmin(fmax(fmin(4.0 * x + a, -4.0 * x + b), 0.0), 1.0);
  return (uint8_t)rint(v * 255.0);
}

struct FrameStats {         // workspace header (device)
  unsigned int dmin, dmax;  // raw depth range
  unsigned int clip;        // clip value (uint16) or 65535 when no clip applies
  unsigned int pad_;
  float scale, shift;       // NORM_MINMAX constants (float, as convertTo uses them)
  unsigned int pad2[2];
  unsigned int hist[65536];
};

__global__ void stats_init_kernel(FrameStats* st) {
  st->dmin = 0xffffffffu;
  st->dmax = 0;
}

// One pass over the depth map: each workgroup counts its pixels into a private 65 536-bin histogram in the LDS
// (two 16-bit counters per word: a workgroup sees at most kHistPix pixels, fewer than 65 536, so a counter never
// carries into its neighbour), then adds its non-zero bins to the global histogram -- one global atomic per
// (workgroup, distinct depth value) instead of one per pixel, exact integer counts in any order.
constexpr int kHistPix = 65535;
template <bool HIST>
__global__ __launch_bounds__(1024) void depth_hist_kernel(const uint16_t* dp, int64_t stride, int H, int W,
                                                          FrameStats* st) {
  constexpr bool want_hist = HIST;
  __shared__ unsigned int lh[HIST ? 32768 : 1];   // packed counters (128 KB)
  __shared__ unsigned int smin, smax;
  const int t = threadIdx.x;
  if (t == 0) { smin = 0xffffffffu; smax = 0; }
  if constexpr (want_hist)
    for (int i = t; i < 32768; i += 1024) lh[i] = 0;
  __syncthreads();
  unsigned int lmin = 0xffffffffu, lmax = 0;
  const int64_t n = (int64_t)H * W;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;   // <= kHistPix (checked at launch)
  const int64_t i0 = (int64_t)blockIdx.x * per, i1 = i0 + per < n ? i0 + per : n;
  for (int64_t i = i0 + t; i < i1; i += 1024) {
    const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
    const unsigned int v = dp[(int64_t)y * stride + x];
    lmin = min(lmin, v);
    lmax = max(lmax, v);
    if constexpr (want_hist) atomicAdd(&lh[v >> 1], 1u << ((v & 1) * 16));
  }
  atomicMin(&smin, lmin);
  atomicMax(&smax, lmax);
  __syncthreads();
  if (t == 0) {
    atomicMin(&st->dmin, smin);
    atomicMax(&st->dmax, smax);
  }
  if constexpr (want_hist)
    for (int i = t; i < 32768; i += 1024) {
      const unsigned int w = lh[i];
      if (w & 0xffffu) atomicAdd(&st->hist[2 * i], w & 0xffffu);
      if (w >> 16) atomicAdd(&st->hist[2 * i + 1], w >> 16);
    }
}

// median (np.median: mean of the two middle order statistics for an even count), clip and scale.  1 024 threads,
// 64 bins each held in registers (16-B loads): per-thread sums, an inclusive scan of them in the LDS, then the
// thread whose range holds an order statistic walks its own 64 bins
__global__ __launch_bounds__(1024) void depth_stats_kernel(FrameStats* st, int64_t n, int depth_clip) {
  __shared__ unsigned int scan[2][1024];
  __shared__ int kv[2];
  const int t = threadIdx.x;
  unsigned int lo = st->dmin, hi = st->dmax;
  unsigned int clip = 65535u;
  if (depth_clip) {
    uint4 h[16];
    const uint4* src = reinterpret_cast<const uint4*>(st->hist) + t * 16;
#pragma unroll
    for (int q = 0; q < 16; ++q) h[q] = src[q];
    unsigned int sum = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) sum += h[q].x + h[q].y + h[q].z + h[q].w;
    // inclusive Hillis-Steele scan over the 1 024 sums (exact integers, n < 2^31)
    int cur = 0;
    scan[0][t] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const unsigned int v = scan[cur][t] + (t >= off ? scan[cur][t - off] : 0u);
      scan[cur ^ 1][t] = v;
      cur ^= 1;
      __syncthreads();
    }
    const int64_t end = scan[cur][t], base = end - sum;
    // order statistics k1 = (n-1)/2, k2 = n/2 (0-based)
    const int64_t k[2] = {(n - 1) / 2, n / 2};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (k[j] >= base && k[j] < end) {
        int64_t c = base;
        int found = t * 64 + 63;
        for (int q = 0; q < 16; ++q) {
          const unsigned int w[4] = {h[q].x, h[q].y, h[q].z, h[q].w};
          bool done = false;
          for (int e = 0; e < 4; ++e) {
            c += w[e];
            if (k[j] < c) { found = t * 64 + q * 4 + e; done = true; break; }
          }
          if (done) break;
        }
        kv[j] = found;
      }
    }
    __syncthreads();
    const double median = 0.5 * ((double)kv[0] + (double)kv[1]);
    const double maxd = fmin(median * 3.0, 10000.0);
    if ((double)hi > maxd) {   // dp[dp > max_depth] = max_depth (float -> uint16 truncates)
      clip = (unsigned int)maxd;
      hi = clip;
      lo = min(lo, clip);
    }
  }
  if (t == 0) {
    const double smin = lo, smax = hi;
    const double scale = (smax - smin) > 2.220446049250313e-16 ? 255.0 / (smax - smin) : 0.0;
    const double shift = 0.0 - smin * scale;
    st->clip = clip;
    st->scale = (float)scale;
    st->shift = (float)shift;
  }
}

__global__ __launch_bounds__(256) void rgbd_map_kernel(const uint8_t* rgb, int64_t rgb_stride, const uint16_t* dp,
                                                       int64_t dp_stride, int H, int W, const FrameStats* st,
                                                       const uint8_t* lut, uint8_t* out, int64_t out_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
  unsigned int d = dp[(int64_t)y * dp_stride + x];
  if (d > st->clip) d = st->clip;
  // saturate_cast<ushort>(d * scale + shift): separate mul / add in float (no FMA contraction: HIP's
  // __fmul_rn is a plain multiply), round half to even
  float f;
  {
#pragma clang fp contract(off)
    f = (float)d * st->scale + st->shift;
  }
  int v = (int)rintf(f);
  v = min(max(v, 0), 65535) & 0xff;   // np.asarray(dp, dtype=np.uint8) keeps the low byte
  const uint8_t* c = rgb + (int64_t)y * rgb_stride + (int64_t)x * 3;
  uint8_t* o = out + (int64_t)y * out_stride + (int64_t)x * 6;
  o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
  if (lut) {
    o[3] = lut[v * 3]; o[4] = lut[v * 3 + 1]; o[5] = lut[v * 3 + 2];
  } else {
    const double xv = v / 255.0;
    o[3] = jet_chan(xv, 0.5, 2.5);    // B
    o[4] = jet_chan(xv, -0.5, 3.5);   // G
    o[5] = jet_chan(xv, -1.5, 4.5);   // R
  }
}

// RGB-T / RGB-E frame assembly: get_x_frame(color, aux, dtype='rgbrgb') (depth_utils.py:71-132 as the
// RGB-T / RGB-E workspaces call it, test_rgbt_mgpus.py:98): both images are read as colour and converted
// BGR -> RGB by the reference (cv2.imread + cvtColor); the host decoders here hand over RGB already, so
// the device step is the channel merge into the HBM frame the tracker reads (a 1-channel aux is
// replicated, as IMREAD_COLOR expands a grayscale file).  One thread per pixel, 6 bytes out.
__global__ __launch_bounds__(256) void rgbx_merge_kernel(const uint8_t* __restrict__ rgb, int64_t rgb_stride,
                                                         const uint8_t* __restrict__ aux, int64_t aux_stride,
                                                         int aux_ch, int H, int W, uint8_t* __restrict__ out,
                                                         int64_t out_stride) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)H * W) return;
  const int y = (int)(i / W), x = (int)(i - (int64_t)y * W);
  const uint8_t* c = rgb + (int64_t)y * rgb_stride + (int64_t)x * 3;
  const uint8_t* a = aux + (int64_t)y * aux_stride + (int64_t)x * aux_ch;
  uint8_t* o = out + (int64_t)y * out_stride + (int64_t)x * 6;
  o[0] = c[0]; o[1] = c[1]; o[2] = c[2];
  if (aux_ch == 3) {
    o[3] = a[0]; o[4] = a[1]; o[5] = a[2];
  } else {
    o[3] = a[0]; o[4] = a[0]; o[5] = a[0];
  }
}

}  // namespace mmt

using namespace mmt;

extern "C" {

size_t mmt_rgbd_workspace_bytes(void) { return sizeof(FrameStats); }

int mmt_rgbd_assemble(const uint8_t* rgb, int64_t rgb_stride, const uint16_t* depth, int64_t depth_stride, int H,
                      int W, int depth_clip, const uint8_t* lut_bgr, uint8_t* out, int64_t out_stride,
                      void* workspace, size_t ws_bytes, void* stream_) {
  if (!rgb || !depth || !out || !workspace || H <= 0 || W <= 0 || ws_bytes < sizeof(FrameStats) ||
      rgb_stride < (int64_t)W * 3 || depth_stride < W || out_stride < (int64_t)W * 6)
    return MMT_E_ARG;
  hipStream_t s = (hipStream_t)stream_;
  FrameStats* st = static_cast<FrameStats*>(workspace);
  hipLaunchKernelGGL(stats_init_kernel, dim3(1), dim3(1), 0, s, st);
  if (depth_clip && hipMemsetAsync(st->hist, 0, sizeof(st->hist), s) != hipSuccess) return MMT_E_HIP;
  const int64_t n = (int64_t)H * W;
  // 1 024-thread workgroups over 4 096 pixels each (at most kHistPix: the 16-bit LDS counters)
  int blocks = (int)((n + 4095) / 4096);
  if (blocks < (int)((n + kHistPix - 1) / kHistPix)) blocks = (int)((n + kHistPix - 1) / kHistPix);
  if (depth_clip)
    hipLaunchKernelGGL(depth_hist_kernel<true>, dim3(blocks), dim3(1024), 0, s, depth, depth_stride, H, W, st);
  else
    hipLaunchKernelGGL(depth_hist_kernel<false>, dim3(blocks), dim3(1024), 0, s, depth, depth_stride, H, W, st);
  hipLaunchKernelGGL(depth_stats_kernel, dim3(1), dim3(1024), 0, s, st, n, depth_clip);
  hipLaunchKernelGGL(rgbd_map_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rgb, rgb_stride, depth,
                     depth_stride, H, W, st, lut_bgr, out, out_stride);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

int mmt_rgbx_merge(const uint8_t* rgb, int64_t rgb_stride, const uint8_t* aux, int64_t aux_stride, int aux_channels,
                   int H, int W, uint8_t* out, int64_t out_stride, void* stream_) {
  if (!rgb || !aux || !out || H <= 0 || W <= 0 || (aux_channels != 1 && aux_channels != 3) ||
      rgb_stride < (int64_t)W * 3 || aux_stride < (int64_t)W * aux_channels || out_stride < (int64_t)W * 6)
    return MMT_E_ARG;
  const int64_t n = (int64_t)H * W;
  hipLaunchKernelGGL(rgbx_merge_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream_, rgb,
                     rgb_stride, aux, aux_stride, aux_channels, H, W, out, out_stride);
  return hipGetLastError() == hipSuccess ? MMT_OK : MMT_E_HIP;
}

}  // extern "C"
