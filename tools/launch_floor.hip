// Per-launch floor of back-to-back kernels in a hipGraph on one stream (GPU tuning tool, not a test): the
// one-sequence frame is ~117 launches whose shortest kernels last ~4.8 us in the kernel trace, so this measures
// what a launch costs by itself -- an empty kernel of 1 / 256 workgroups, and kernels that leave 1 / 8 MB of dirty
// lines behind (the L2 writeback of a kernel's release) -- as graph replays of 100 launches, timed with events.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_kernel(int* p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}

__global__ void touch_kernel(float4* buf, int n4, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x)
    buf[i] = make_float4(v, v, v, v);
}

__global__ void chain_kernel(const float* in, float* out) {   // one dependent global load + store
  if (threadIdx.x == 0) out[blockIdx.x] = in[blockIdx.x] + 1.f;
}

template <class F>
static void measure(const char* name, hipStream_t s, int n, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < n; ++i) launch(i);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 5; ++w) CK(hipGraphLaunch(ge, s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int reps = 20;
  CK(hipEventRecord(a, s));
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"case\": \"%s\", \"launches\": %d, \"us_per_launch\": %.3f}\n", name, n, ms * 1e3f / (reps * n));
  fflush(stdout);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int* p;
  float *buf, *in, *out;
  CK(hipMalloc(&p, 64));
  CK(hipMemset(p, 0, 64));
  CK(hipMalloc(&buf, 64 << 20));
  CK(hipMalloc(&in, 1 << 20));
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(in, 0, 1 << 20));
  const int n = 100;
  measure("empty_1wg", s, n, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, p); });
  measure("empty_256wg", s, n, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, p); });
  measure("empty_2048wg", s, n, [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(256), 0, s, p); });
  measure("chain_1wg", s, n, [&](int i) {
    hipLaunchKernelGGL(chain_kernel, dim3(1), dim3(64), 0, s, (i & 1) ? out : in, (i & 1) ? in : out);
  });
  measure("chain_256wg", s, n, [&](int i) {
    hipLaunchKernelGGL(chain_kernel, dim3(256), dim3(64), 0, s, (i & 1) ? out : in, (i & 1) ? in : out);
  });
  for (int mb : {1, 4, 16}) {
    char name[64];
    snprintf(name, sizeof name, "touch_%dMB", mb);
    const int n4 = (mb << 20) / 16;
    measure(name, s, n, [&](int i) {
      hipLaunchKernelGGL(touch_kernel, dim3(1024), dim3(256), 0, s, reinterpret_cast<float4*>(buf) + (size_t)(i & 1) * (16 << 20) / 16, n4, (float)i);
    });
  }
  // the same plain launches outside a graph
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, p);
    CK(hipEventRecord(a, s));
    for (int w = 0; w < 2000; ++w) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, p);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"case\": \"empty_1wg_stream\", \"launches\": 2000, \"us_per_launch\": %.3f}\n", ms * 1e3f / 2000);
  }
  CK(hipStreamSynchronize(s));
  printf("done\n");
  return 0;
}
