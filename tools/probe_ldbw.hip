// build: hipcc -O3 --offload-arch=gfx950 tools/probe_ldbw.hip -o probe/ldbw  (run on the GPU box)
// Load-path microbenchmark (tuning tool, not product): bytes/s into the CUs for the GEMM staging
// pattern -- every workgroup repeatedly loads KB-sized tiles of an L2/MALL-resident buffer, waits,
// barriers.  Variants: 0 = buffer_load_dwordx4 ... lds (LDS-DMA), 1 = buffer_load_dwordx4 to VGPRs +
// ds_write_b128, 2 = buffer_load_dwordx4 to VGPRs only (xor-reduced).  DEPTH tiles in flight per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((address_space(3))) void* lptr_t;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// each step: every wave loads LPW x 1 KB (rows of 128 B, 8 rows per instruction) of a tile of the buffer
template <int MODE, int LPW, int DEPTH>
__global__ __launch_bounds__(512) void ldbw(const char* buf, long long bytes, int steps, unsigned* sink) {
  __shared__ __attribute__((aligned(16))) char smem[DEPTH * 8 * LPW * 1024];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const rsrc_t r = make_rsrc(buf, bytes);
  const long long tile = 8LL * LPW * 1024;   // bytes per workgroup step
  const long long ntiles = bytes / tile;
  unsigned acc = 0;
  u32x4 v[DEPTH][LPW];
  auto issue = [&](int s, int slot) {
    const long long t = ((long long)blockIdx.x * 7919 + s * 131) % ntiles;
    const unsigned base = (unsigned)(t * tile);
#pragma unroll
    for (int i = 0; i < LPW; ++i) {
      const unsigned vo = base + (wave * LPW + i) * 1024 + lane * 16;
      if (MODE == 0) {
        lptr_t dst = (lptr_t)(smem + ((slot * 8 + wave) * LPW + i) * 1024);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, vo, 0, 0, 0);
      } else {
        v[slot][i] = __builtin_amdgcn_raw_buffer_load_b128(r, vo, 0, 0);
      }
    }
  };
  for (int p = 0; p < DEPTH - 1; ++p) issue(p, p);
  for (int s = 0; s < steps; ++s) {
    const int slot = s % DEPTH;
    if (s + DEPTH - 1 < steps) issue(s + DEPTH - 1, (s + DEPTH - 1) % DEPTH);
    if (DEPTH == 1 || s + DEPTH - 1 >= steps) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (DEPTH == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPW) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPW * (DEPTH - 1 > 1 ? DEPTH - 1 : 1)) : "memory");
    if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < LPW; ++i)
        *reinterpret_cast<u32x4*>(smem + ((slot * 8 + wave) * LPW + i) * 1024 + lane * 16) = v[slot][i];
    } else if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < LPW; ++i) acc ^= v[slot][i].x ^ v[slot][i].w;
    }
    __builtin_amdgcn_s_barrier();
  }
  if (MODE == 0 || MODE == 1) acc = *reinterpret_cast<unsigned*>(smem + threadIdx.x * 4);
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int MODE, int LPW, int DEPTH>
void run(const char* buf, long long bytes, int grid, unsigned* sink, const char* name) {
  const int steps = 200;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((ldbw<MODE, LPW, DEPTH>), dim3(grid), dim3(512), 0, 0, buf, bytes, steps, sink);
  hipEventRecord(e0);
  const int reps = 5;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL((ldbw<MODE, LPW, DEPTH>), dim3(grid), dim3(512), 0, 0, buf, bytes, steps, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double moved = (double)grid * steps * 8 * LPW * 1024 * reps;
  printf("%-28s grid %4d buf %6.1f MB: %7.2f TB/s  (%5.1f B/clk/CU @2.4GHz, %.2f us/step)\n", name, grid, bytes / 1e6,
         moved / (ms * 1e-3) / 1e12, moved / (ms * 1e-3) / 256 / 2.4e9, ms * 1e3 / reps / steps);
}

int main() {
  const long long bytes = 16LL << 20;
  char* buf;
  unsigned* sink;
  hipMalloc(&buf, bytes);
  hipMalloc(&sink, 64);
  hipMemset(buf, 1, bytes);
  for (int grid : {256, 512}) {
    run<0, 4, 2>(buf, bytes, grid, sink, "ldsdma  32KB d2");
    run<0, 4, 3>(buf, bytes, grid, sink, "ldsdma  32KB d3");
    run<0, 2, 4>(buf, bytes, grid, sink, "ldsdma  16KB d4");
    run<1, 4, 2>(buf, bytes, grid, sink, "vgpr+ds 32KB d2");
    run<1, 4, 3>(buf, bytes, grid, sink, "vgpr+ds 32KB d3");
    run<2, 4, 2>(buf, bytes, grid, sink, "vgpr    32KB d2");
    run<2, 4, 3>(buf, bytes, grid, sink, "vgpr    32KB d3");
  }
  const long long small = 2LL << 20;
  run<0, 4, 2>(buf, small, 512, sink, "ldsdma 32KB d2 (2MB)");
  run<2, 4, 2>(buf, small, 512, sink, "vgpr   32KB d2 (2MB)");
  return 0;
}
