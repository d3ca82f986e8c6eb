// Launch-cost floor on MI355X: back-to-back dependent launches of a near-empty kernel on one stream,
// plain and captured in a hipGraph, at 1 / 256 / 2048 workgroups (tuning tool, not part of the product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void tiny(float* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 1.0001f + 1.0f;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
  float* d;
  const int n = 2048 * 256;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemset(d, 0, n * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int iters = 2000;
  for (int wg : {1, 256, 2048}) {
    int cnt = wg * 256;
    for (int k = 0; k < 50; ++k) tiny<<<wg, 256, 0, s>>>(d, cnt);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int k = 0; k < iters; ++k) tiny<<<wg, 256, 0, s>>>(d, cnt);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("stream  wg=%5d  %.2f us/launch\n", wg, 1000.f * ms / iters);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < 100; ++k) tiny<<<wg, 256, 0, s>>>(d, cnt);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int k = 0; k < iters / 100; ++k) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    printf("graph   wg=%5d  %.2f us/launch\n", wg, 1000.f * ms / iters);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  CK(hipFree(d));
  return 0;
}
