// microbench.hip — single-wave latency/throughput probes for the building
// blocks of the render kernel (dev tool; results inform DESIGN.md).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off scripts/microbench.hip -o build/microbench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#include "../include/rt_rng.h"

#define N 1024

struct Sph {
  double c[3], r, r2;
  int mat, obj;
};

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }

// mode 0: dependent f64 division chain; 1: dependent sqrt chain; 2: rng draws (dependent);
// 3: sphere loop via scalar loads (5 spheres) per iteration; 4: same spheres in LDS;
// 5: independent f64 fma throughput (8 chains); 6: rcp+newton chain; 7: 5-sphere test with data in SGPR args
__global__ void probe(int mode, const Sph* __restrict__ sp, int ns, double* out, unsigned long long* cyc) {
  __shared__ Sph lsp[16];
  if (threadIdx.x < ns) lsp[threadIdx.x] = sp[threadIdx.x];
  __syncthreads();
  double x = 1.0 + threadIdx.x * 1e-3, y = 3.0;
  rt_rng r;
  rt_rng_init(&r, 12345, threadIdx.x, 7);
  unsigned long long t0 = now();
  if (mode == 0) {
    for (int i = 0; i < N; ++i) x = y / x;
  } else if (mode == 1) {
    for (int i = 0; i < N; ++i) x = sqrt(x + 1.0);
  } else if (mode == 2) {
    for (int i = 0; i < N; ++i) x += rt_rng_draw(&r);
  } else if (mode == 3 || mode == 4) {
    double ox = 0.1 * threadIdx.x, oy = 0.2, oz = 8.0;
    double dx = 0.01, dy = 0.02, dz = -1.0;
    double a = dx * dx + dy * dy + dz * dz;
    int hits = 0;
    for (int i = 0; i < N / 8; ++i) {
      for (int j = 0; j < ns; ++j) {
        const Sph& S = mode == 3 ? sp[j] : lsp[j];
        double ocx = ox - S.c[0], ocy = oy - S.c[1], ocz = oz - S.c[2];
        double hb = ocx * dx + ocy * dy + ocz * dz;
        double c = (ocx * ocx + ocy * ocy + ocz * ocz) - S.r2;
        double disc = hb * hb - a * c;
        hits += disc >= 0;
      }
      ox += 1e-9;
    }
    x += hits;
  } else if (mode == 5) {
    double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
    for (int i = 0; i < N / 8; ++i) {
      a0 = __builtin_fma(a0, 0.999, 0.001); a1 = __builtin_fma(a1, 0.999, 0.001);
      a2 = __builtin_fma(a2, 0.999, 0.001); a3 = __builtin_fma(a3, 0.999, 0.001);
      a4 = __builtin_fma(a4, 0.999, 0.001); a5 = __builtin_fma(a5, 0.999, 0.001);
      a6 = __builtin_fma(a6, 0.999, 0.001); a7 = __builtin_fma(a7, 0.999, 0.001);
    }
    x = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  } else if (mode == 6) {
    for (int i = 0; i < N; ++i) {
      double r0 = __builtin_amdgcn_rcp(x);
      double e = __builtin_fma(-x, r0, 1.0);
      x = __builtin_fma(r0, e, r0) + 1.0;
    }
  } else if (mode == 8) {
    for (int i = 0; i < N; ++i) x = x * 1.0000001 + 1e-9;  // dependent mul+add
  }
  unsigned long long t1 = now();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  Sph h[5] = {{{0, 0, 0}, 1.0, 1.0, 0, 0}, {{2, 0, 0}, 0.5, 0.25, 1, 1}, {{-2, 0, 0}, 0.7, 0.49, 2, 2},
              {{0, 2, 0}, 0.3, 0.09, 3, 3}, {{0, -2, 0}, 0.4, 0.16, 4, 4}};
  Sph* d;
  double* out;
  unsigned long long* cyc;
  hipMalloc(&d, sizeof h);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  hipMalloc(&out, 1 << 20);
  hipMalloc(&cyc, 1 << 16);
  const char* names[] = {"f64 div chain /op", "f64 sqrt chain /op", "rng draw chain /draw", "5-sphere disc test, scalar loads /sphere",
                         "5-sphere disc test, LDS /sphere", "indep fma x8 /fma", "rcp+newton chain /op", "", "dep mul+add /op"};
  int ops[] = {N, N, N, (N / 8) * 5, (N / 8) * 5, N, N, 1, N};
  for (int mode : {0, 1, 2, 3, 4, 5, 6, 8}) {
    for (int waves : {1, 4}) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64 * waves), 0, 0, mode, d, 5, out, cyc);
      hipDeviceSynchronize();
      hipLaunchKernelGGL(probe, dim3(1), dim3(64 * waves), 0, 0, mode, d, 5, out, cyc);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("%-42s waves/WG=%d: %.1f cycles\n", names[mode], waves, (double)c / ops[mode]);
    }
  }
  return 0;
}
