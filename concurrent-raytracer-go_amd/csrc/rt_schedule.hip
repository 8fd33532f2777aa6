// rt_schedule.hip — the work schedule of a rank, built on the GPU.
//
// The reference hands tiles to goroutines in row-major order through a
// channel (createRenderTasks, internal/renderer/renderer.go:398-436); a
// goroutine that draws a slow tile just keeps it while the others continue.
// On the GPU a workgroup is dispatched once and runs to completion, so a
// slow block dispatched late (long multi-bounce paths between mirrors and
// inside glass) runs alone at the end of the launch.  The schedule therefore
// cuts the rank's pixels into work BLOCKS of about equal estimated work and
// dispatches them heaviest first:
//
//   sched_pixels   per pixel, the primary-ray candidate masks (the
//                  primitives whose bounding sphere meets the cone of the
//                  pixel's jittered camera rays, within its tile's masks);
//                  per 64 pixels, a record of the one-sample PILOT render
//   (pilot)        render_kernel<kPilot>: each pixel's path length
//   sched_est      per pixel, the estimated work of one sample: the longest
//                  pilot path among it and its 4 neighbours (+0.02 for the
//                  camera ray), or the tile's projected-primitive estimate
//   sched_blocks   per tile, consecutive pixels grouped while spp * sum(est)
//                  <= block_work (at most big_pixels pixels); a pixel whose
//                  own work exceeds block_work is SPLIT into sample ranges of
//                  at most 64 samples; a tile whose camera rays provably miss
//                  everything becomes 16 black blocks.  Pass 1 counts the
//                  blocks per weight class (log2 buckets, 8 per octave),
//                  pass 2 writes them at the class's cursor, heaviest class
//                  first, with the union of their pixels' masks
//   sched_scan     exclusive scan of the class counts
//
// One small device->host copy (block and split counts) follows, to size the
// launch; no per-pixel data crosses PCIe.  The schedule only partitions and
// orders work: every block is rendered by the same code and every pixel's
// samples are summed in sample order, so the image does not depend on it
// (tests/test_gpu_schedules.py).  The order inside a weight class follows
// the atomics and may differ from run to run; the image does not.
#include <hip/hip_runtime.h>

#include "rt_internal.h"

namespace rtgo {

namespace {

constexpr int kBuckets = 128;  // weight classes: 8 per octave of estimated work

__device__ __forceinline__ int bucket_of(double est) {
  // heaviest first: order index 0 = the largest estimate
  const double l = log2(1.0 + fmax(est, 0.0)) * 8.0;
  const int k = l >= (double)(kBuckets - 1) ? kBuckets - 1 : (int)l;
  return kBuckets - 1 - k;
}

// Does the cone (apex, unit axis, cos/sin of its half-angle) meet the sphere
// (c, r)?  Conservative: radius inflated by ~1e-7, far above binary64
// rounding of the ray directions (same test as the shadow cones, rt_kernel.hip).
__device__ bool cone_meets_sphere(const double* c, double r, const double* apex, const double* axis, double cos_t,
                                  double sin_t) {
  const double v0 = c[0] - apex[0], v1 = c[1] - apex[1], v2 = c[2] - apex[2];
  const double dc2 = v0 * v0 + v1 * v1 + v2 * v2;
  const double dc = sqrt(dc2);
  const double ra = fabs(r) * (1.0 + 1e-7) + 1e-7 * dc + 1e-12;
  if (dc <= ra) return true;
  const double tl = sqrt(fmax(dc2 - ra * ra, 0.0));
  const double vd = v0 * axis[0] + v1 * axis[1] + v2 * axis[2];
  return vd >= cos_t * (1.0 - 1e-9) * tl - (sin_t + 1e-9) * ra - 1e-7 * dc;
}

// The cone around the camera rays of pixel (x, y): getRay direction
// (vw*(u-1/2), 2*(v-1/2), -1) with u in [x/W, (x+1)/W], v in [y/H, (y+1)/H]
// (renderer.go:155-156,377-390).
__device__ void pixel_cone(double vw, int W, int H, int x, int y, double* axis, double* cmin, double* smax) {
  const double dx0 = vw * ((double)x / W - 0.5), dx1 = vw * ((double)(x + 1) / W - 0.5);
  const double dy0 = 2.0 * ((double)y / H - 0.5), dy1 = 2.0 * ((double)(y + 1) / H - 0.5);
  axis[0] = 0.5 * (dx0 + dx1);
  axis[1] = 0.5 * (dy0 + dy1);
  axis[2] = -1.0;
  const double al = sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  for (int k = 0; k < 3; ++k) axis[k] /= al;
  double c = 1.0;  // the widest corner: the angle is quasiconvex on the image plane
  for (int k = 0; k < 4; ++k) {
    const double cx = (k & 1) ? dx1 : dx0, cy = (k & 2) ? dy1 : dy0;
    const double cl = sqrt(cx * cx + cy * cy + 1.0);
    c = fmin(c, (axis[0] * cx + axis[1] * cy - axis[2]) / cl);
  }
  *cmin = c;
  *smax = sqrt(fmax(0.0, 1.0 - c * c));
}

__device__ __forceinline__ unsigned long long wave_or(unsigned long long v) {
  for (int off = 32; off; off >>= 1) v |= __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ void put_u64(int32_t* r, unsigned long long v) {
  r[0] = (int32_t)(uint32_t)v;
  r[1] = (int32_t)(uint32_t)(v >> 32);
}

// K1: one wave per 64 pixels of a local tile.
__global__ __launch_bounds__(64) void sched_pixels(const SchedParams p) {
  const int lt = blockIdx.x >> 4, w = blockIdx.x & 15, lane = threadIdx.x;
  const int q = w * 64 + lane, t = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
  unsigned long long ms = 0, mt = 0;
  if (p.tile_masks) {
    const unsigned long long ts = p.tile_masks[2 * lt], tt = p.tile_masks[2 * lt + 1];
    const int x = (t % p.tiles_x) * 32 + (q & 31), y = (t / p.tiles_x) * 32 + (q >> 5);
    if (t < p.ntiles && (ts | tt) && x < p.W && y < p.H) {
      double axis[3], cmin, smax;
      pixel_cone(p.vw, p.W, p.H, x, y, axis, &cmin, &smax);
      for (unsigned long long b = ts; b; b &= b - 1) {
        const int i = __builtin_ctzll(b);
        if (cone_meets_sphere(p.spheres[i].c, p.spheres[i].r, p.cam, axis, cmin, smax)) ms |= 1ull << i;
      }
      for (unsigned long long b = tt; b; b &= b - 1) {
        const int i = __builtin_ctzll(b);
        if (cone_meets_sphere(p.tris[i].bc, p.tris[i].br, p.cam, axis, cmin, smax)) mt |= 1ull << i;
      }
    }
    p.pixmask[((size_t)lt * 1024 + q) * 2] = ms;
    p.pixmask[((size_t)lt * 1024 + q) * 2 + 1] = mt;
  }
  const unsigned long long live = __ballot((ms | mt) != 0);
  ms = wave_or(ms);
  mt = wave_or(mt);
  if (lane == 0 && p.pilot_blocks) {  // the pilot's block: 64 pixels, sample 0 only
    int32_t* r = p.pilot_blocks + (size_t)blockIdx.x * kBlockInts;
    r[0] = lt;
    r[1] = w * 64;
    r[2] = 64;
    r[3] = 0;
    r[4] = 1;
    r[5] = -1;
    r[6] = 1;
    r[7] = 0;
    put_u64(r + 8, ms);
    put_u64(r + 10, mt);
    put_u64(r + 12, live);
    r[14] = t;
    r[15] = 0;
  }
}

// K2: per pixel, the estimated path work of one sample.
__global__ __launch_bounds__(256) void sched_est(const SchedParams p) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)p.local * 1024) return;
  const int lt = (int)(i >> 10), q = (int)(i & 1023);
  float e;
  bool heavy = false;
  if (p.work_max && p.work_n < p.spp && !p.work_mean) {
    // a pilot of a few samples is a noisy estimate of a pixel's mean: take
    // the neighbourhood's longest path
    const unsigned int* L = p.work_max + (size_t)lt * 1024;
    const int x = q & 31, y = q >> 5;
    unsigned int m = L[q];
    if (x > 0) m = max(m, L[q - 1]);
    if (x < 31) m = max(m, L[q + 1]);
    if (y > 0) m = max(m, L[q - 32]);
    if (y < 31) m = max(m, L[q + 32]);
    e = (float)m + 0.02f;
  } else if (p.work_max) {
    // a measured frame: every sample's path length, so the pixel's mean work
    // per sample; a pixel with a long path is split whatever its mean (its
    // block would otherwise run that path's chain of bounces with many other
    // paths: the launch's tail)
    const size_t i0 = (size_t)lt * 1024 + q;
    e = (float)((double)p.work_sum[i0] / (double)p.work_n) + 0.02f;
    heavy = (int)p.work_max[i0] > p.split_depth;
    if (heavy) e = fmaxf(e, (float)p.work_max[i0]);  // its sub-blocks go first: they hold the long chains
  } else {  // no pilot: every pixel of a tile with geometry weighs half a block
    const float c = p.tile_cost[lt];
    e = c > 0 ? (float)(p.block_work / (2.0 * max(1, p.spp))) * (1.0f + 1e-3f * fminf(c, 100.0f)) : 0.0f;
  }
  // the sign bit marks a pixel to split (est >= 0 otherwise)
  p.est[i] = heavy ? -e - 1e-30f : e;
}

// One record: the block's pixels and samples, the union of its pixels'
// primary masks and the bits of its live pixels.
__device__ void put_record(const SchedParams& p, int pos, int lt, int p0, int np, int s0, int ns, int slot, int nsub,
                           int flags) {
  unsigned long long ms = 0, mt = 0, live = 0;
  if (p.tile_masks) {
    for (int k = 0; k < np && k < 64 && p0 + k < 1024; ++k) {
      const unsigned long long* m = p.pixmask + ((size_t)lt * 1024 + p0 + k) * 2;
      ms |= m[0];
      mt |= m[1];
      if (m[0] | m[1]) live |= 1ull << k;
    }
  }
  int4* r = reinterpret_cast<int4*>(p.blocks + (size_t)pos * kBlockInts);
  r[0] = make_int4(lt, p0, np, s0);
  r[1] = make_int4(ns, slot, nsub, flags);
  r[2] = make_int4((int)(uint32_t)ms, (int)(uint32_t)(ms >> 32), (int)(uint32_t)mt, (int)(uint32_t)(mt >> 32));
  const int tile = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
  r[3] = make_int4((int)(uint32_t)live, (int)(uint32_t)(live >> 32), tile, 0);
}

// K3 (pass 1, kWrite = false) / K5 (pass 2, kWrite = true): one wave per
// local tile.  The blocks are the greedy partition of the tile's pixels
// (row-major): a block starting at pixel p ends at next(p), the first pixel
// it cannot take (a pixel heavier than block_work, big_pixels reached, or
// spp * sum(est) would exceed block_work); a heavy pixel is its own block,
// split into sample ranges.  next() is computed for every pixel at once
// (prefix sums, a suffix minimum, a binary search), and the chain of block
// starts 0, next(0), next(next(0)), ... by pointer doubling: no lane walks
// the tile alone.
template <bool kWrite>
__global__ __launch_bounds__(64) void sched_blocks(const SchedParams p) {
  constexpr int kLevels = 11;                  // 2^10 = 1024 steps at most
  __shared__ double s_pre[1025];               // prefix sums of spp * est
  __shared__ uint16_t s_J[kLevels][1025];      // s_J[k][p] = next^(2^k)(p)
  __shared__ uint16_t s_big[1025];             // first pixel >= p heavier than block_work
  __shared__ int s_nodes, s_nsplit, s_slot0;
  __shared__ int s_cnt[kBuckets], s_base[kBuckets];
  const int lt = blockIdx.x, lane = threadIdx.x;
  const double S = max(p.spp, 1), bw = p.block_work;
  const bool black = p.frustum && p.tile_masks && p.spp > 0 &&
                     (p.tile_masks[2 * lt] | p.tile_masks[2 * lt + 1]) == 0;
  if (black) {  // every camera ray of the tile provably misses: 16 black blocks, dispatched last
    if (lane < 16) {
      const int b = kBuckets - 1;
      if (!kWrite) atomicAdd(&p.hist[b], 1);
      else put_record(p, atomicAdd(&p.cursor[b], 1), lt, lane * 64, 64, 0, p.spp, -1, 1, kBlockBlack);
    }
    return;
  }
  const float* est_raw = p.est + (size_t)lt * 1024;
  // (a negative estimate marks a pixel measured as heavy: split it; its work is -est)
  auto est_of = [&](int q) { return fabsf(est_raw[q]); };
  auto heavy_of = [&](int q) { return p.spp > 1 && (S * (double)fabsf(est_raw[q]) > bw || est_raw[q] < 0.0f); };
  // prefix sums (16 consecutive pixels per lane, then a wave scan) and the
  // suffix minimum of the heavy pixels
  const int q0 = lane * 16;
  double v[16];
  double acc = 0;
  int big = 1024;
  for (int k = 0; k < 16; ++k) {
    v[k] = S * (double)est_of(q0 + k);
    acc += v[k];
  }
  double excl = acc;
  for (int off = 1; off < 64; off <<= 1) {
    const double t = __shfl_up(excl, off);
    if (lane >= off) excl += t;
  }
  excl -= acc;
  for (int k = 15; k >= 0; --k)
    if (v[k] > bw || heavy_of(q0 + k)) big = q0 + k;
  int sbig = big;  // suffix minimum over the lanes above
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_down(sbig, off);
    if (lane + off < 64) sbig = min(sbig, t);
  }
  {
    double a = excl;
    int nb = lane + 1 < 64 ? __shfl_down(sbig, 1) : 1024;
    if (lane == 63) nb = 1024;
    for (int k = 15; k >= 0; --k) {
      if (v[k] > bw || heavy_of(q0 + k)) nb = q0 + k;
      s_big[q0 + k] = (uint16_t)nb;
    }
    for (int k = 0; k < 16; ++k) {
      s_pre[q0 + k] = a;
      a += v[k];
    }
    if (lane == 63) {
      s_pre[1024] = a;
      s_big[1024] = 1024;
    }
  }
  __syncthreads();
  // next(p) for every pixel
  for (int q = lane; q <= 1024; q += 64) {
    int nx = 1024;
    if (q < 1024) {
      if (heavy_of(q)) {
        nx = q + 1;  // split pixel: a block of its own
      } else {
        int hi = min(min(q + p.big_pixels, 1024), (int)s_big[min(q + 1, 1024)]);
        // the largest end e in [q + 1, hi] with pre[e] - pre[q] <= bw
        int lo = q + 1;
        const double lim = s_pre[q] + bw;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (s_pre[mid] <= lim) lo = mid;
          else hi = mid - 1;
        }
        nx = lo;
      }
    }
    s_J[0][q] = (uint16_t)nx;
  }
  __syncthreads();
  for (int k = 1; k < kLevels; ++k) {
    for (int q = lane; q <= 1024; q += 64) s_J[k][q] = s_J[k - 1][s_J[k - 1][q]];
    __syncthreads();
  }
  if (lane == 0) {  // block starts: 0, next(0), ...; their number by doubling
    int pos = 0, m = 0;
    for (int k = kLevels - 1; k >= 0; --k)
      if (s_J[k][pos] < 1024) {
        pos = s_J[k][pos];
        m += 1 << k;
      }
    s_nodes = m + 1;
  }
  __syncthreads();
  const int nodes = s_nodes;
  // the blocks (and the sub-blocks of split pixels) of this tile, per lane:
  // f(bucket, first pixel, pixels, first sample, samples, split slot
  // ordinal or -1, sub-blocks)
  auto visit = [&](auto&& f) {
    for (int m = lane; m < nodes; m += 64) {
      int q = 0;
      for (int k = 0; k < kLevels; ++k)
        if ((m >> k) & 1) q = s_J[k][q];
      const int e = s_J[0][q];
      if (heavy_of(q)) {  // a split pixel (e == q + 1): sample ranges of <= split_samples
        const int nsub = (p.spp + p.split_samples - 1) / p.split_samples;
        const int ord = atomicAdd(&s_nsplit, 1);
        for (int j = 0; j < nsub; ++j) {
          const int s0 = (int)((long long)p.spp * j / nsub), s1 = (int)((long long)p.spp * (j + 1) / nsub);
          f(bucket_of((s1 - s0) * (double)est_of(q)), q, 1, s0, s1 - s0, ord, nsub);
        }
      } else {
        f(bucket_of(s_pre[e] - s_pre[q]), q, e - q, 0, p.spp, -1, 1);
      }
    }
  };
  // counts per class in LDS, then one global atomic per class and tile
  // (the classes are few: per-record global atomics serialized on them)
  for (int b = lane; b < kBuckets; b += 64) s_cnt[b] = 0;
  if (lane == 0) s_nsplit = 0;
  __syncthreads();
  visit([&](int b, int, int, int, int, int, int) { atomicAdd(&s_cnt[b], 1); });
  __syncthreads();
  if (!kWrite) {
    for (int b = lane; b < kBuckets; b += 64)
      if (s_cnt[b]) atomicAdd(&p.hist[b], s_cnt[b]);
    if (lane == 0 && s_nsplit) atomicAdd(&p.totals[1], s_nsplit);
    return;
  }
  for (int b = lane; b < kBuckets; b += 64) {
    s_base[b] = s_cnt[b] ? atomicAdd(&p.cursor[b], s_cnt[b]) : 0;
    s_cnt[b] = 0;
  }
  if (lane == 0) {
    s_slot0 = s_nsplit ? atomicAdd(&p.totals[2], s_nsplit) : 0;
    s_nsplit = 0;
  }
  __syncthreads();
  visit([&](int b, int q, int np, int s0, int ns, int ord, int nsub) {
    const int pos = s_base[b] + atomicAdd(&s_cnt[b], 1);
    put_record(p, pos, lt, q, np, s0, ns, ord < 0 ? -1 : s_slot0 + ord, nsub, 0);
  });
}

// K4: exclusive scan of the class counts (heaviest class first) into the
// write cursors; totals[0] = blocks; the split-slot counter starts at 0.
__global__ __launch_bounds__(kBuckets) void sched_scan(const SchedParams p) {
  __shared__ int s[kBuckets];
  const int i = threadIdx.x;
  s[i] = p.hist[i];
  __syncthreads();
  for (int off = 1; off < kBuckets; off <<= 1) {
    const int v = i >= off ? s[i - off] : 0;
    __syncthreads();
    s[i] += v;
    __syncthreads();
  }
  p.cursor[i] = s[i] - p.hist[i];
  if (i == kBuckets - 1) {
    p.totals[0] = s[i];
    p.totals[2] = 0;
  }
}

// Per local tile (the whole frame in a planning pilot: lt = t), the
// estimated work of its image pixels, spp * sum(est) (the weight sched_blocks
// gives the tile's blocks).  One wave per tile, a fixed reduction order: the
// same inputs give the same bits on every device, so every rank that plans a
// partition from the same pilot derives the same one.
__global__ __launch_bounds__(64) void sched_tile_work(const SchedParams p, float* out) {
  const int lt = blockIdx.x, lane = threadIdx.x;
  const int t = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
  const int x0 = (t % p.tiles_x) * 32, y0 = (t / p.tiles_x) * 32;
  double a = 0;
  for (int k = 0; k < 16; ++k) {
    const int q = k * 64 + lane, x = x0 + (q & 31), y = y0 + (q >> 5);
    if (x < p.W && y < p.H) a += (double)fabsf(p.est[(size_t)lt * 1024 + q]);
  }
  for (int off = 32; off; off >>= 1) a += __shfl_xor(a, off);
  if (lane == 0) out[lt] = (float)(a * (double)max(p.spp, 1));
}

}  // namespace

int sched_launch_tile_work(const SchedParams& p, float* tile_work, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (p.local <= 0) return hipSuccess;
  const unsigned n = (unsigned)(((size_t)p.local * 1024 + 255) / 256);
  hipLaunchKernelGGL(sched_est, dim3(n), dim3(256), 0, s, p);
  hipLaunchKernelGGL(sched_tile_work, dim3(p.local), dim3(64), 0, s, p, tile_work);
  return (int)hipGetLastError();
}

size_t sched_scratch_bytes(int local) {
  // pixmask (2 u64 / pixel) | est (f32 / pixel) | pilot blocks (16 / tile) | hist | cursor | totals
  return (size_t)local * 1024 * 16 + (size_t)local * 1024 * 4 + (size_t)local * 16 * kBlockInts * 4 +
         2 * kBuckets * 4 + 64;
}

void sched_layout(void* scratch, int local, SchedParams* p) {
  char* m = (char*)scratch;
  p->pixmask = (unsigned long long*)m;
  m += (size_t)local * 1024 * 16;
  p->est = (float*)m;
  m += (size_t)local * 1024 * 4;
  p->pilot_blocks = (int32_t*)m;
  m += (size_t)local * 16 * kBlockInts * 4;
  p->hist = (int32_t*)m;
  p->cursor = p->hist + kBuckets;
  p->totals = p->cursor + kBuckets;
}

// (see preload_render_kernels)
int preload_sched_kernels() {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(sched_est));
}

int sched_launch_pixels(const SchedParams& p, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (p.local <= 0) return hipSuccess;
  const hipError_t e = hipMemsetAsync(p.hist, 0, (2 * kBuckets + 4) * sizeof(int32_t), s);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(sched_pixels, dim3(p.local * 16), dim3(64), 0, s, p);
  return (int)hipGetLastError();
}

int sched_launch_blocks(const SchedParams& p, bool write, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (p.local <= 0) return hipSuccess;
  if (!write) {
    const unsigned n = (unsigned)(((size_t)p.local * 1024 + 255) / 256);
    hipLaunchKernelGGL(sched_est, dim3(n), dim3(256), 0, s, p);
    hipLaunchKernelGGL((sched_blocks<false>), dim3(p.local), dim3(64), 0, s, p);
    hipLaunchKernelGGL(sched_scan, dim3(1), dim3(kBuckets), 0, s, p);
  } else {
    hipLaunchKernelGGL((sched_blocks<true>), dim3(p.local), dim3(64), 0, s, p);
  }
  return (int)hipGetLastError();
}

}  // namespace rtgo
