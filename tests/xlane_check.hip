// Bitwise check of the LDS-free cross-lane reductions (common.h: wave_sum / wave_max by permlane swaps +
// DPP) against the __shfl_xor (ds_bpermute) butterfly they replace, on random data (GPU tuning check;
// built by tests/Makefile.xlane, run by tests/test_gpu_kernels.py::test_xlane_reductions_bitwise).
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../multi-modal-trakcing-bechmark_amd/csrc/common.h"

__device__ float shfl_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ float shfl_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ void check(const float* x, float* out, int n) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= n) return;
  const float v = x[w * 64 + lane];
  out[(w * 64 + lane) * 6 + 0] = wave_sum(v);
  out[(w * 64 + lane) * 6 + 1] = shfl_sum(v);
  out[(w * 64 + lane) * 6 + 2] = wave_max(v);
  out[(w * 64 + lane) * 6 + 3] = shfl_max(v);
  // the 16 / 32-lane half-exchange sums with distinct operands (reduce8's first stages)
  const float y = v * 3.0f + 1.0f;
  out[(w * 64 + lane) * 6 + 4] = xsum32(v, y);
  const float keep = (lane & 32) ? y : v, send = (lane & 32) ? v : y;   // non-divergent reference
  out[(w * 64 + lane) * 6 + 5] = keep + __shfl_xor(send, 32, 64);
}

int main() {
  const int n = 4096;
  std::vector<float> h(n * 64), o(n * 64 * 6);
  srand(7);
  for (auto& v : h) v = (float)rand() / RAND_MAX * 200.f - 100.f + (float)rand() / RAND_MAX * 1e-3f;
  float *dx, *dout;
  hipMalloc(&dx, h.size() * 4);
  hipMalloc(&dout, o.size() * 4);
  hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check, dim3(n / 4), dim3(256), 0, 0, dx, dout, n);
  hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  int bad[3] = {0, 0, 0};
  for (int i = 0; i < n * 64; ++i) {
    bad[0] += o[i * 6] != o[i * 6 + 1];
    bad[1] += o[i * 6 + 2] != o[i * 6 + 3];
    bad[2] += o[i * 6 + 4] != o[i * 6 + 5];
  }
  printf("xlane mismatches: sum %d max %d xsum32 %d of %d\n", bad[0], bad[1], bad[2], n * 64);
  if (bad[0] || bad[1] || bad[2]) {
    for (int i = 0; i < 8; ++i) printf("lane %d: %.9g %.9g\n", i, o[i * 6], o[i * 6 + 1]);
    return 1;
  }
  return 0;
}
