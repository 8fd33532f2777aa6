// copy_probe.hip — dev probe: how long does a device->host copy queued behind
// a kernel take in a FRESH process, the first time and afterwards?  (The CLI's
// first Render waited ~7 ms for it, profiles/r04_cli_trace.json.)
// build: hipcc --offload-arch=gfx950 -O2 -o build/copy_probe scripts/copy_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void busy(float* p, int n, int iters) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = p[i];
  for (int k = 0; k < iters; ++k) v = v * 0.999f + 1.0f;
  p[i] = v;
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t n = 2 << 20;  // 8 MB of floats
  float* d = nullptr;
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipMalloc(&d, n * 4);
  hipMemsetAsync(d, 0, n * 4, s);
  hipStreamSynchronize(s);
  std::vector<float> pageable(n);
  float* pinned = nullptr;
  hipHostMalloc((void**)&pinned, n * 4, hipHostMallocDefault);
  const char* names[] = {"pageable", "pinned"};
  for (int round = 0; round < 3; ++round) {
    for (int kind = 0; kind < 2; ++kind) {
      float* h = kind ? pinned : pageable.data();
      double t0 = now();
      hipLaunchKernelGGL(busy, dim3((n + 255) / 256), dim3(256), 0, s, d, (int)n, 2000);
      double t1 = now();
      hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s);
      double t2 = now();
      hipStreamSynchronize(s);
      double t3 = now();
      printf("round %d %-8s: launch %.3f ms, memcpyAsync call %.3f ms, sync %.3f ms, total %.3f ms\n", round,
             names[kind], (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t3 - t0) * 1e3);
    }
  }
  // the same with the kernel already finished before the copy is queued
  for (int kind = 0; kind < 2; ++kind) {
    float* h = kind ? pinned : pageable.data();
    hipLaunchKernelGGL(busy, dim3((n + 255) / 256), dim3(256), 0, s, d, (int)n, 2000);
    hipStreamSynchronize(s);
    double t1 = now();
    hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    printf("idle stream %-8s: copy %.3f ms\n", names[kind], (now() - t1) * 1e3);
  }
  // copies after the copy engine sat idle for a while (host sleep)
  for (int idle_ms : {0, 1, 2, 5, 10, 20, 50}) {
    for (int kind = 0; kind < 2; ++kind) {
      float* h = kind ? pinned : pageable.data();
      hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
      const double ts = now();
      while (now() - ts < idle_ms * 1e-3) {
      }
      double t1 = now();
      hipMemcpyAsync(h, d, n * 4, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
      printf("after %2d ms idle %-8s: copy %.3f ms\n", idle_ms, names[kind], (now() - t1) * 1e3);
    }
  }
  // small copies (1.92 MB, the CLI's RGBA image) after idling
  for (int idle_ms : {2, 10}) {
    const double ts = now();
    while (now() - ts < idle_ms * 1e-3) {
    }
    double t1 = now();
    hipMemcpyAsync(pageable.data(), d, 1920000, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    printf("after %2d ms idle pageable 1.92 MB: copy %.3f ms\n", idle_ms, (now() - t1) * 1e3);
  }
  return 0;
}
