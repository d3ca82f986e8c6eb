// In-launch grid barrier vs kernel boundary on MI355X (tuning tool, not part of the product): the cost a
// persistent per-layer ViT kernel would pay per phase hand-off, measured against the
// dependent-launch floor of tools/micro/launch_floor.hip.
//
// Barrier: every workgroup (all co-resident: one per CU, or two) does its phase's work -- one coalesced
// 1-KB read-modify-write, like a phase's tail -- then one lane releases it with an agent-scope atomic add on a
// phase counter (a vector atomic) and polls the counter with agent-scope acquire loads until every workgroup
// arrived; a bounded poll (an error count instead of a hang) guarantees every wave reaches the end.
// Launch: the same work as one kernel per phase, back to back on a stream and replayed from a hipGraph.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

constexpr int kPollCap = 1 << 22;

__device__ __forceinline__ void phase_work(float* p, int phase) {
  float* q = p + (size_t)blockIdx.x * 256;
  q[threadIdx.x] = q[threadIdx.x] * 1.0001f + (float)phase;
}

__global__ __launch_bounds__(256) void persistent(float* p, unsigned* counter, unsigned* timeouts, int phases) {
  for (int ph = 0; ph < phases; ++ph) {
    phase_work(p, ph);
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(ph + 1) * gridDim.x;
      int n = 0;
      while (__hip_atomic_load(counter, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target && ++n < kPollCap) {
      }
      if (n >= kPollCap) __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

// the same with the arrival counter sharded over 8 lines (workgroup b adds to line b % 8, the XCD it runs on
// under the round-robin dispatch; 32 adders per line instead of 256) and the poll summing the 8 lines
constexpr int kShards = 8, kShardWords = 32;   // one 128-B line per shard
__global__ __launch_bounds__(256) void persistent_sharded(float* p, unsigned* counters, unsigned* timeouts, int phases) {
  for (int ph = 0; ph < phases; ++ph) {
    phase_work(p, ph);
    __syncthreads();
    if (threadIdx.x < 64) {   // one wave: lane 0 adds, lanes 0-7 poll one shard each
      const int lane = threadIdx.x;
      if (lane == 0)
        __hip_atomic_fetch_add(counters + (blockIdx.x % kShards) * kShardWords, 1u, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(ph + 1) * gridDim.x;
      int n = 0;
      unsigned sum = 0;
      do {
        const unsigned v = lane < kShards ? __hip_atomic_load(counters + lane * kShardWords, __ATOMIC_ACQUIRE,
                                                              __HIP_MEMORY_SCOPE_AGENT)
                                          : 0u;
        sum = v;
#pragma unroll
        for (int o = 1; o < kShards; o <<= 1) sum += __shfl_xor(sum, o, 64);
      } while (sum < target && ++n < kPollCap);
      if (lane == 0 && n >= kPollCap) __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void one_phase(float* p, int phase) { phase_work(p, phase); }

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  float* d;
  unsigned *counter, *timeouts;
  CK(hipMalloc(&d, (size_t)4 * cus * 256 * sizeof(float)));
  CK(hipMemset(d, 0, (size_t)4 * cus * 256 * sizeof(float)));
  CK(hipMalloc(&counter, sizeof(unsigned)));
  unsigned* counter8;
  CK(hipMalloc(&counter8, kShards * kShardWords * sizeof(unsigned)));
  CK(hipMalloc(&timeouts, sizeof(unsigned)));
  CK(hipMemset(timeouts, 0, sizeof(unsigned)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int phases = 1000;
  printf("# %d CUs, %d phases per measurement\n", cus, phases);
  for (int per_cu : {1, 2}) {
    const int grid = per_cu * cus;
    float ms;
    // persistent: one launch, phases - 1 grid barriers (+ 1 trailing)
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemsetAsync(counter, 0, sizeof(unsigned), s));
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(persistent, dim3(grid), dim3(256), 0, s, d, counter, timeouts, phases);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    unsigned to = 0;
    CK(hipMemcpy(&to, timeouts, sizeof(unsigned), hipMemcpyDeviceToHost));
    printf("grid barrier   wg=%5d  %.2f us/phase  (poll timeouts %u)\n", grid, 1000.f * ms / phases, to);
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemsetAsync(counter8, 0, kShards * kShardWords * sizeof(unsigned), s));
      CK(hipEventRecord(a, s));
      hipLaunchKernelGGL(persistent_sharded, dim3(grid), dim3(256), 0, s, d, counter8, timeouts, phases);
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
    }
    CK(hipMemcpy(&to, timeouts, sizeof(unsigned), hipMemcpyDeviceToHost));
    printf("sharded bar.   wg=%5d  %.2f us/phase  (poll timeouts %u)\n", grid, 1000.f * ms / phases, to);
    // one launch per phase, stream
    for (int k = 0; k < 50; ++k) hipLaunchKernelGGL(one_phase, dim3(grid), dim3(256), 0, s, d, k);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int k = 0; k < phases; ++k) hipLaunchKernelGGL(one_phase, dim3(grid), dim3(256), 0, s, d, k);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("stream launch  wg=%5d  %.2f us/phase\n", grid, 1000.f * ms / phases);
    // one launch per phase, graph replay
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 100; ++k) hipLaunchKernelGGL(one_phase, dim3(grid), dim3(256), 0, s, d, k);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int k = 0; k < phases / 100; ++k) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("graph launch   wg=%5d  %.2f us/phase\n", grid, 1000.f * ms / phases);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(d));
  CK(hipFree(counter));
  CK(hipFree(counter8));
  CK(hipFree(timeouts));
  return 0;
}
