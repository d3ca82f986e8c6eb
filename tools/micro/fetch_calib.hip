// FETCH_SIZE calibration on gfx950 (tuning tool): known byte counts read by the access patterns the path's kernels
// use, so rocprofv3's FETCH_SIZE (L2 -> fabric read requests x 64 B) can be converted to bytes per pattern.
//   k_lds128: buffer_load_dwordx4 ... lds, each wave instruction 1 KB contiguous (8 full 128-B lines)
//   k_lds64 : buffer_load_dwordx4 ... lds, each wave instruction 16 rows x 64 B at a 128-B row pitch (the BK = 32
//             weight pieces): every 128-B line is read in two halves by two instructions one "K-tile" apart
//   k_vgpr  : global_load_dwordx4 into VGPRs, 1 KB contiguous per wave instruction
// Each kernel reads BYTES once (no re-reads); 512 MB so the 256 MB Infinity Cache cannot hold it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void* lptr_t;
constexpr size_t BYTES = 512ull << 20;
constexpr int WG = 256, NWG = 2048;

__global__ __launch_bounds__(WG) void k_lds128(const char* src, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[WG * 16 * 4];
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, 0x7fffffff, 0x00020000);
  const size_t per = BYTES / NWG;   // 256 KB per workgroup
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (size_t off = 0; off < per; off += WG * 16) {
    const uint32_t vo = (uint32_t)(((size_t)blockIdx.x * per + off) % 0x7fff0000u) + (w * 64 + l) * 16;   // wrap past 2 GB
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)(lds + w * 1024), 16, vo, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[5];
}

__global__ __launch_bounds__(WG) void k_lds64(const char* src, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[WG * 16 * 4];
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), 0, 0x7fffffff, 0x00020000);
  const size_t per = BYTES / NWG;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int row = l >> 2, ch = l & 3;   // 16 rows x 4 chunks of 16 B
  for (size_t off = 0; off < per; off += WG * 16 * 2) {   // a block of 4 waves x 16 rows x 128 B
    for (int half = 0; half < 2; ++half) {
      const uint32_t vo = (uint32_t)(((size_t)blockIdx.x * per + off) % 0x7fff0000u) + (w * 16 + row) * 128 + half * 64 + ch * 16;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lptr_t)(lds + w * 1024), 16, vo, 0, 0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = lds[5];
}

__global__ __launch_bounds__(WG) void k_vgpr(const float4* src, float* sink) {
  const size_t per = BYTES / NWG / 16;
  float acc = 0.f;
  for (size_t i = threadIdx.x; i < per; i += WG) {
    const float4 v = src[(size_t)blockIdx.x * per + i];
    acc += v.x + v.w;
  }
  if (acc == 12345.f) sink[blockIdx.x] = acc;
}

int main() {
  char* src;
  float* sink;
  if (hipMalloc(&src, BYTES) != hipSuccess || hipMalloc(&sink, NWG * 4) != hipSuccess) return 1;
  hipMemset(src, 1, BYTES);
  for (int it = 0; it < 2; ++it) {
    hipLaunchKernelGGL(k_lds128, dim3(NWG), dim3(WG), 0, 0, src, sink);
    hipLaunchKernelGGL(k_lds64, dim3(NWG), dim3(WG), 0, 0, src, sink);
    hipLaunchKernelGGL(k_vgpr, dim3(NWG), dim3(WG), 0, 0, (const float4*)src, sink);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("each kernel reads %zu bytes per launch\n", BYTES);
  return 0;
}
