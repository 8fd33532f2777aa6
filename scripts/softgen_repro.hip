// softgen_repro.hip — reduced repro of the wf_softgen queue-write defect
// (commit e2ca53b).  Dev tool, not part of librtgo.
//
// wf_softgen writes each clear light's 16 soft-ray points into a queue.  The
// pre-e2ca53b code appended with a bumped pointer inside the rejection loop,
//     if (unit_ball_accept(ux, uy, uz)) { *sq++ = entry; ++k; }
// where unit_ball_accept screens in binary32 and lets a binary64 test decide
// a thin shell (rt_device.h).  The 1920x1080x64 wavefront frames then differed
// from run to run.  This program runs that loop (kernel bump) and the
// shipped form (kernel indexed: sq[k] = entry; k += acc) over the same
// streams, 2 lights x 16 points per thread, and compares:
//   - bump vs indexed (a lost increment leaves a stale slot and overwrites
//     the next point: the queues differ wherever the shell branch accepted);
//   - each kernel against itself on a second run (queues pre-filled with a
//     different garbage pattern, so a slot a kernel never writes shows up).
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I ../include -I ../concurrent-raytracer-go_amd/csrc
//        softgen_repro.hip -o softgen_repro       (scripts/softgen_repro.sh; --save-temps keeps the ISA)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rt_rng.h"
#include "rt_device.h"

using namespace rtgo;

constexpr int kThreads = 1 << 20;
constexpr int kPoints = 32;  // 2 lights x 16

__global__ void bump(uint4* q, uint64_t* tries) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  rt_rng rng;
  rt_rng_init(&rng, 0x9E3779B97F4A7C15ull, (uint32_t)t, 7u);
  uint4* sq = q + (size_t)t * kPoints;
  uint64_t n = 0;
  for (int li = 0; li < 2; ++li) {
    for (int k = 0; k < 16;) {
      const uint32_t ux = rt_rng_next(&rng), uy = rt_rng_next(&rng), uz = rt_rng_next(&rng);
      ++n;
      if (unit_ball_accept(ux, uy, uz)) {
        *sq++ = make_uint4((uint32_t)li, ux, uy, uz);
        ++k;
      }
    }
  }
  tries[t] = n;
}

__global__ void indexed(uint4* q, uint64_t* tries) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  rt_rng rng;
  rt_rng_init(&rng, 0x9E3779B97F4A7C15ull, (uint32_t)t, 7u);
  uint4* sq = q + (size_t)t * kPoints;
  uint64_t n = 0;
  int k = 0;
  for (int li = 0; li < 2; ++li) {
    for (const int end = k + 16; k < end;) {
      const uint32_t ux = rt_rng_next(&rng), uy = rt_rng_next(&rng), uz = rt_rng_next(&rng);
      ++n;
      const bool acc = unit_ball_accept(ux, uy, uz);
      if (acc) sq[k] = make_uint4((uint32_t)li, ux, uy, uz);
      k += acc ? 1 : 0;
    }
  }
  tries[t] = n;
}

template <typename K>
static std::vector<uint4> run(K kern, unsigned fill, std::vector<uint64_t>* tries) {
  const size_t n = (size_t)kThreads * kPoints;
  uint4* d = nullptr;
  uint64_t* dt = nullptr;
  if (hipMalloc(&d, n * sizeof(uint4)) != hipSuccess || hipMalloc(&dt, kThreads * 8) != hipSuccess) exit(3);
  if (hipMemset(d, (int)fill, n * sizeof(uint4)) != hipSuccess) exit(3);
  hipLaunchKernelGGL(kern, dim3(kThreads / 256), dim3(256), 0, 0, d, dt);
  if (hipDeviceSynchronize() != hipSuccess) exit(3);
  std::vector<uint4> h(n);
  tries->resize(kThreads);
  if (hipMemcpy(h.data(), d, n * sizeof(uint4), hipMemcpyDeviceToHost) != hipSuccess) exit(3);
  if (hipMemcpy(tries->data(), dt, kThreads * 8, hipMemcpyDeviceToHost) != hipSuccess) exit(3);
  (void)hipFree(d);
  (void)hipFree(dt);
  return h;
}

static size_t differ(const std::vector<uint4>& a, const std::vector<uint4>& b, size_t* threads) {
  size_t n = 0;
  *threads = 0;
  for (size_t t = 0; t < (size_t)kThreads; ++t) {
    bool any = false;
    for (int k = 0; k < kPoints; ++k) {
      const uint4 x = a[t * kPoints + k], y = b[t * kPoints + k];
      if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) {
        ++n;
        any = true;
      }
    }
    *threads += any;
  }
  return n;
}

int main() {
  std::vector<uint64_t> t1, t2, t3, t4;
  const auto b1 = run(bump, 0x00, &t1), b2 = run(bump, 0xA5, &t2);
  const auto i1 = run(indexed, 0x00, &t3), i2 = run(indexed, 0xA5, &t4);
  size_t th = 0;
  const size_t d_bb = differ(b1, b2, &th);
  printf("bump vs bump (garbage 00 vs A5):       %zu slots differ in %zu threads\n", d_bb, th);
  const size_t d_ii = differ(i1, i2, &th);
  printf("indexed vs indexed (garbage 00 vs A5): %zu slots differ in %zu threads\n", d_ii, th);
  const size_t d_bi = differ(b1, i1, &th);
  printf("bump vs indexed:                       %zu slots differ in %zu threads\n", d_bi, th);
  size_t tries = 0, td = 0;
  for (int t = 0; t < kThreads; ++t) {
    tries += t3[t];
    td += t1[t] != t3[t];
  }
  printf("%d threads, %zu rejection tries (%zu threads where the two kernels' try counts differ)\n", kThreads, tries,
         td);
  printf(d_ii == 0 ? "indexed form: deterministic\n" : "indexed form: NOT deterministic\n");
  return 0;
}
