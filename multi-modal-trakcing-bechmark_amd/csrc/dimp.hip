// DiMP / mfDiMP target-classifier inner loop on gfx950 (fp32):
//   apply_filter           RGBD/models/DeT/ltr/models/layers/filter.py:5-54   (per-sequence correlation, pad k//2)
//   apply_feat_transpose   filter.py:57-148   (its filter gradient)
//   DistanceMap + label / target-mask / spatial-weight predictors   distance.py:17-39, optimizer.py:111-125
//   DiMPSteepestDescentGN  optimizer.py:132-168  (LeakyReluPar score activation, Gauss-Newton step length)
// All reductions are block-partial arrays combined in fixed order (bitwise reproducible, no atomics).
#include "dimp.h"

namespace mmt {

constexpr int MAXT = 25;   // filter taps (<= 5x5)

__global__ __launch_bounds__(256) void dimp_maps_kernel(DimpMaps m) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int n = m.Ho * m.Wo;
  if (idx >= m.IS * n) return;
  const int is = idx / n, p = idx - is * n;
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

// scores[i,s,y,x] = sum_c,ky,kx feat[i,s,c,y+ky-P,x+kx-P] * w[s,c,ky,kx]; mode 1/2 epilogues below.
// One workgroup per (image * sequence, tile of kDimpPosPerBlock output positions): the 8 wave halves
// (32 lanes each) take interleaved channel slices (c = group + 8 k) of the same 32 positions, so a frame's
// 15-50 samples still spread over hundreds of workgroups; the 8 partial sums combine in a fixed order.
// FH / FW > 0: the filter size as compile-time constants (the taps unroll, so a channel's loads are all in
// flight together; the same summation order as the generic loop)
template <int FH, int FW>
__global__ __launch_bounds__(256) void dimp_filter_kernel(DimpFilter a) {
  extern __shared__ float wsh[];
  __shared__ float part[8][kDimpPosPerBlock];
  if constexpr (FH > 0) {
    a.fh = FH;
    a.fw = FW;
  }
  const int is = blockIdx.x;                  // image * S + sequence
  const int s = is % a.S;
  const int T = a.fh * a.fw;
  for (int k = threadIdx.x; k < a.C * T; k += 256) wsh[k] = a.w[(int64_t)s * a.C * T + k];
  __syncthreads();
  const int n = a.Ho * a.Wo;
  const int lp = threadIdx.x & (kDimpPosPerBlock - 1), cg = threadIdx.x / kDimpPosPerBlock;
  const int p = blockIdx.y * kDimpPosPerBlock + lp;
  float acc = 0.f;
  if (p < n) {
    const int y = p / a.Wo, x = p - y * a.Wo;
    const int P0 = a.fh / 2, P1 = a.fw / 2;
    const float* f = a.feat + (int64_t)(is / a.S) * a.img_stride + (int64_t)s * a.seq_stride;
#pragma unroll 4
    for (int c = cg; c < a.C; c += 8) {
      const float* fc = f + (int64_t)c * a.H * a.W;
      const float* wc = wsh + c * T;
#pragma unroll
      for (int ky = 0; ky < (FH > 0 ? FH : a.fh); ++ky) {
        const int yy = y + ky - P0;
        if (yy < 0 || yy >= a.H) continue;
#pragma unroll
        for (int kx = 0; kx < (FW > 0 ? FW : a.fw); ++kx) {
          const int xx = x + kx - P1;
          if (xx < 0 || xx >= a.W) continue;
          acc += fc[yy * a.W + xx] * wc[ky * a.fw + kx];
        }
      }
    }
  }
  part[cg][lp] = acc;
  __syncthreads();
  float r2 = 0.f;
  if (cg == 0 && p < n) {
    acc = part[0][lp];
#pragma unroll
    for (int g = 1; g < 8; ++g) acc += part[g][lp];
    const int64_t o = (int64_t)is * n + p;
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
      const float g = a.sw[o] * (a.smask[o] * acc);
      r2 = g * g;
    }
  }
  if (!a.partial) return;   // uniform over the workgroup
  __syncthreads();          // every group has read its sums
  if (cg == 0) part[0][lp] = r2;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < kDimpPosPerBlock; ++k) t += part[0][k];
    a.partial[(int64_t)is * gridDim.y + blockIdx.y] = t;
  }
}

// grad[s,c,ky,kx] = sum_i,y,x r[i,s,y,x] * feat[i,s,c,y+ky-P,x+kx-P] (+ reg * w), one block per (s, c)
__global__ __launch_bounds__(256) void dimp_transpose_kernel(DimpTranspose a) {
  __shared__ float red[256][MAXT + 1];
  const int s = blockIdx.x / a.C, c = blockIdx.x % a.C;
  const int T = a.fh * a.fw, n = a.Ho * a.Wo;
  const int P0 = a.fh / 2, P1 = a.fw / 2;
  float acc[MAXT];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) acc[t] = 0.f;
  for (int q = threadIdx.x; q < a.I * n; q += 256) {
    const int i = q / n, p = q - i * n;
    const int y = p / a.Wo, x = p - y * a.Wo;
    const float r = a.r[((int64_t)i * a.S + s) * n + p];
    const float* fc = a.feat + (int64_t)i * a.img_stride + (int64_t)s * a.seq_stride + (int64_t)c * a.H * a.W;
#pragma unroll
    for (int t = 0; t < MAXT; ++t) {
      if (t >= T) break;
      const int ky = t / a.fw, kx = t - ky * a.fw;
      const int yy = y + ky - P0, xx = x + kx - P1;
      if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) acc[t] += r * fc[yy * a.W + xx];
    }
  }
  for (int t = 0; t < T; ++t) red[threadIdx.x][t] = acc[t];
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if (threadIdx.x < st)
      for (int t = 0; t < T; ++t) red[threadIdx.x][t] += red[threadIdx.x + st][t];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float sq = 0.f;
    for (int t = 0; t < T; ++t) {
      const int64_t o = ((int64_t)s * a.C + c) * T + t;
      const float g = red[0][t] + (a.w ? a.reg * a.w[o] : 0.f);
      a.grad[o] = g;
      sq += g * g;
    }
    if (a.gsq) a.gsq[(int64_t)s * a.C + c] = sq;
  }
}

// alpha = |g|^2 / (|J g|^2 + (reg + eps)|g|^2), w -= step * alpha * g   (optimizer.py:155-160); one block per s
__global__ __launch_bounds__(256) void dimp_update_kernel(DimpUpdate a) {
  __shared__ float red[256];
  __shared__ float num_sh, den_sh;
  const int s = blockIdx.x;
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
  for (int k = threadIdx.x; k < a.I * a.nby; k += 256) {
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
void dimp_filter(const DimpFilter& a, hipStream_t s) {
  const int nby = (a.Ho * a.Wo + kDimpPosPerBlock - 1) / kDimpPosPerBlock;
  const size_t lds = a.C * a.fh * a.fw * sizeof(float);
  if (a.fh == 4 && a.fw == 4)
    hipLaunchKernelGGL((dimp_filter_kernel<4, 4>), dim3(a.I * a.S, nby), dim3(256), lds, s, a);
  else
    hipLaunchKernelGGL((dimp_filter_kernel<0, 0>), dim3(a.I * a.S, nby), dim3(256), lds, s, a);
}
void dimp_transpose(const DimpTranspose& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_transpose_kernel, dim3(a.S * a.C), dim3(256), 0, s, a);
}
void dimp_update(const DimpUpdate& a, hipStream_t s) {
  hipLaunchKernelGGL(dimp_update_kernel, dim3(a.S), dim3(256), 0, s, a);
}
void dimp_loss(const float* rsq, int nparts, const float* w, int nw, float reg, int S, float* loss, hipStream_t s) {
  hipLaunchKernelGGL(dimp_loss_kernel, dim3(1), dim3(256), 0, s, rsq, nparts, w, nw, reg, S, loss);
}

}  // namespace mmt
