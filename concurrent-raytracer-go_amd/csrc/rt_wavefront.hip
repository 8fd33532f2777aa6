// rt_wavefront.hip — the wavefront path for BVH scenes (> 64 spheres, configs
// C4/C5: 10k spheres).
//
// The megakernel (rt_kernel.hip) keeps a whole path in one lane: its binary64
// path state costs 168 VGPRs, so a SIMD holds 3 waves, and on a 10k-sphere
// scene every BVH traversal is a chain of dependent L2 loads that 3 waves
// cannot hide (C4: 1.4 s, lanes mostly waiting).  Here the bounce loop of
// traceRay (internal/renderer/renderer.go:165-227) is cut into stages, each a
// small kernel over a compacted array of live paths in HBM:
//
//   regen    new camera samples fill the free slots (tracePixel's jitter and
//            getRay, renderer.go:150-163,377-390)
//   extend   closest hit of every live path (hitWorld, renderer.go:333-346,
//            through the BVH); a miss or the depth cut-off ends the path
//   shade1   the HitRecord (sphere.go:42-58) and one hard shadow ray per light
//            (calculateSmartShadow, renderer.go:299-305) into a queue
//   hard     any-hit of the hard shadow rays
//   softgen  per light whose hard ray is clear, in light order, the 16
//            RandomVec3InUnitSphere points (renderer.go:311-318) into a queue
//   soft     any-hit of the soft rays, counted per (path, light)
//   shade2   calculateDirectLighting (renderer.go:229-297) with those counts,
//            Material.Scatter, the traceRay combination; survivors are
//            compacted into the next path array (wave ballot + one atomic)
//
// The traversal kernels need few registers (8 waves per SIMD instead of 3),
// every stage runs on full waves, and the 16 soft rays of one point sit in 16
// adjacent lanes (a coherent packet).  The arithmetic is the megakernel's
// (rt_device.h), each path consumes its RNG stream in the reference's order
// (soft-shadow draws light by light, then the scatter draws), and each sample's
// radiance lands in its own slot; resolve sums a pixel's samples in sample
// order (tracePixel) — so images are bit-identical to the megakernel's and the
// oracle's.  The loop is host-driven with device-side counts: every kernel
// reads its item count from WfCtl, and the host only polls a copy of WfCtl
// one iteration behind to know when the frame is done.
#include <hip/hip_runtime.h>

#include "../../include/rt_rng.h"
#include "rt_device.h"
#include "rt_internal.h"

namespace rtgo {

constexpr int kWfBlock = 256;           // threads per workgroup of every stage
constexpr uint32_t kHardBit = 1u << 16;  // lstate: the hard shadow ray is blocked (low bits: blocked soft rays)

extern __shared__ __attribute__((aligned(16))) unsigned char wf_lds[];

// per-lane BVH stack in dynamic LDS: one region of 64 x depth ints per wave,
// lane-interleaved (closest_hit / any_hit index it with stride 64)
__device__ __forceinline__ int* wf_stack(int depth) {
  return reinterpret_cast<int*>(wf_lds) + (threadIdx.x >> 6) * 64 * depth + (threadIdx.x & 63);
}

// Append `want` (per lane) items to a queue: one atomic per wave; returns the
// lane's first index.
__device__ __forceinline__ int wave_append(int* counter, bool want, int per = 1) {
  const unsigned long long m = __ballot(want);
  if (m == 0) return 0;
  const int lane = (int)(threadIdx.x & 63);
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, per * __popcll(m));
  base = __shfl(base, leader);
  return base + per * __popcll(m & ((1ull << lane) - 1ull));
}

template <bool kCount>
__device__ __forceinline__ void flush_counts(const WfParams& p, Counters& c) {
  if constexpr (kCount) {
    for (int i = 0; i < 9; ++i) {
      unsigned long long v = c.v[i];
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(&p.counts[i], v);
    }
  }
}

__device__ __forceinline__ d3 ld_o(const WfPaths& a, int i) { return mk(a.ox[i], a.oy[i], a.oz[i]); }
__device__ __forceinline__ d3 ld_d(const WfPaths& a, int i) { return mk(a.dx[i], a.dy[i], a.dz[i]); }
__device__ __forceinline__ d3 ld_P(const WfParams& p, int i) { return mk(p.px[i], p.py[i], p.pz[i]); }

// the light vector of a hit point: calculateDirectLighting's lightDir and
// distance (renderer.go:249-254); recomputed wherever needed, same bits
__device__ __forceinline__ void light_vec(const DLight& Lt, d3 P, d3& ldir, double& ldist) {
  const d3 lv = ld3(Lt.pos) - P;
  ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
  ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
}

__device__ __forceinline__ void store_path(const WfPaths& b, int j, d3 o, d3 d, d3 T, d3 L, uint64_t rng,
                                           uint32_t sid, int depth) {
  b.ox[j] = o.x;
  b.oy[j] = o.y;
  b.oz[j] = o.z;
  b.dx[j] = d.x;
  b.dy[j] = d.y;
  b.dz[j] = d.z;
  b.tx[j] = T.x;
  b.ty[j] = T.y;
  b.tz[j] = T.z;
  b.lx[j] = L.x;
  b.ly[j] = L.y;
  b.lz[j] = L.z;
  b.rng[j] = rng;
  b.sid[j] = sid;
  b.depth[j] = depth;
}

__device__ __forceinline__ void finish(const WfParams& p, uint32_t sid, d3 L) {
  double* r = p.rad + (size_t)sid * 3;
  r[0] = L.x;
  r[1] = L.y;
  r[2] = L.z;
}

// ---------------------------------------------------------------- regen
// Samples [next, next + regen_cnt) of the chunk start as paths appended to
// the next array.  Sample id = local pixel * spp + sample: a pixel's samples
// are consecutive, so a wave's camera rays are neighbours.
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_regen(const WfParams p) {
  const WfCtl* ctl = p.ctl;
  const long long nnew = ctl->regen_cnt;
  const long long first = (long long)ctl->next_sample;
  const CamK ck = make_cam(p.seed_key, p.W, p.H, p.aspect, p.cam[0], p.cam[1], p.cam[2]);
  Counters c;
  if constexpr (kCount)
    for (int i = 0; i < 9; ++i) c.v[i] = 0;
  const long long stride = (long long)gridDim.x * blockDim.x;
  // (block-uniform trip count: the ballot in wave_append sees whole waves)
  for (long long b0 = (long long)blockIdx.x * blockDim.x; b0 < nnew; b0 += stride) {
    const long long t = b0 + threadIdx.x;
    bool valid = false;
    const uint32_t sid = (uint32_t)(first + t);
    int x = 0, y = 0, s = 0;
    if (t < nnew) {
      const uint32_t lp = p.lp0 + sid / (uint32_t)p.spp;
      s = (int)(sid - (sid / (uint32_t)p.spp) * (uint32_t)p.spp);
      const int lt = (int)(lp >> 10), tp = (int)(lp & 1023);
      const int tile = p.rank + lt * p.world;
      const int tx = tile % p.tiles_x, ty = tile / p.tiles_x;
      x = tx * 32 + (tp & 31);
      y = ty * 32 + (tp >> 5);
      valid = tile < p.ntiles && x < p.W && y < p.H;
    }
    const int j = wave_append(&p.ctl->n_next, valid);
    if (valid) {
      cnt<kCount>(c, C_CAM);
      rt_rng rng;
      d3 o, d;
      camera_ray_c<kCount>(ck, x, y, s, rng, o, d, c);
      store_path(p.next, j, o, d, mk(1, 1, 1), mk(0, 0, 0), rng.x, sid, 0);
    }
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- extend
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_extend(const WfParams p) {
  const int n = p.ctl->n_cur;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  if (i < n) {
    const WfPaths& a = p.cur;
    bool found = false;
    HitSel hs;
    if (a.depth[i] < p.max_depth) {  // traceRay's depth cut-off comes first
      cnt<kCount>(c, C_BOUNCE);
      const Cand all{~0ull, ~0ull};
      found = closest_hit<kCount>(p.g, ld_o(a, i), ld_d(a, i), hs, wf_stack(p.stack_depth), all, c);
    }
    if (found) {
      p.hidx[i] = hs.idx;
      p.hnum[i] = hs.num;
    } else {  // miss: black (renderer.go:170-173); the path ends with what it has
      p.hidx[i] = -1;
      finish(p, a.sid[i], mk(a.lx[i], a.ly[i], a.lz[i]));
    }
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- shade1
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_shade1(const WfParams p) {
  const int n = p.ctl->n_cur;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const bool hit = i < n && p.hidx[i] >= 0;
  d3 P = mk(0, 0, 0);
  if (hit) {
    // HitRecord of the sphere (sphere.go:42-58), as in the megakernel
    const WfPaths& a = p.cur;
    cnt<kCount>(c, C_SHADE);
    const d3 o = ld_o(a, i), d = ld_d(a, i);
    const DSphere& S0 = p.g.spheres[p.hidx[i]];
    const double t = p.hnum[i] / len2(d);
    P = o + muls(d, t);
    const d3 outward = divs(P - ld3(S0.c), S0.r);
    const bool front = dot(d, outward) < 0;
    const d3 N = front ? outward : neg(outward);
    p.px[i] = P.x;
    p.py[i] = P.y;
    p.pz[i] = P.z;
    p.nx[i] = N.x;
    p.ny[i] = N.y;
    p.nz[i] = N.z;
    p.hinfo[i] = (S0.mat << 1) | (front ? 1 : 0);
  }
  for (int li = 0; li < p.nl; ++li) {
    bool lit = false;
    if (hit) {
      d3 ldir;
      double ldist;
      light_vec(p.lights[li], P, ldir, ldist);
      lit = !(ldist < 0.001);
      p.lstate[(size_t)i * p.nl + li] = 0;
      if (lit) {
        cnt<kCount>(c, C_LIGHT);
        cnt<kCount>(c, C_SHADOW);
      }
    }
    const int j = wave_append(&p.ctl->n_hard, lit);
    if (lit) p.hardq[j] = (uint32_t)i * (uint32_t)p.nl + (uint32_t)li;
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- hard
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_hard(const WfParams p) {
  const int n = p.ctl->n_hard;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  int* stack = wf_stack(p.stack_depth);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint32_t key = p.hardq[j];
    const int i = (int)(key / (uint32_t)p.nl), li = (int)(key - (uint32_t)i * (uint32_t)p.nl);
    const d3 P = ld_P(p, i);
    d3 ldir;
    double ldist;
    light_vec(p.lights[li], P, ldir, ldist);
    if (any_hit<kCount>(p.g, P, ldir, ldist, stack, c)) p.lstate[key] = kHardBit;
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- softgen
// The 16 jittered points of every (path, light) whose hard ray is clear, in
// light order from the path's stream (rejection sampling, vector.go:132-139).
// An owner reserves 16 consecutive queue entries, so its rays are adjacent.
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_softgen(const WfParams p) {
  const int n = p.ctl->n_cur;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const bool hit = i < n && p.hidx[i] >= 0;
  rt_rng rng{hit ? p.cur.rng[i] : 0};
  const d3 P = hit ? ld_P(p, i) : mk(0, 0, 0);
  for (int li = 0; li < p.nl; ++li) {
    bool own = false;
    const uint32_t key = (uint32_t)i * (uint32_t)p.nl + (uint32_t)li;
    if (hit) {
      d3 ldir;
      double ldist;
      light_vec(p.lights[li], P, ldir, ldist);
      own = !(ldist < 0.001) && !(p.lstate[key] & kHardBit);
    }
    const int q = wave_append(&p.ctl->n_soft, own, 16);
    if (own) {
      cnt<kCount>(c, C_SHADOW, 16);
      for (int k = 0; k < 16;) {
        const uint32_t ux = rt_rng_next(&rng), uy = rt_rng_next(&rng), uz = rt_rng_next(&rng);
        cnt<kCount>(c, C_RNG, 3);
        const d3 pt = mk(rt_bits_to_unit(ux) * 2 - 1, rt_bits_to_unit(uy) * 2 - 1, rt_bits_to_unit(uz) * 2 - 1);
        if (len2(pt) < 1) reinterpret_cast<uint4*>(p.softq)[q + k++] = make_uint4(key, ux, uy, uz);
      }
    }
  }
  if (hit) p.cur.rng[i] = rng.x;
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- soft
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_soft(const WfParams p) {
  const int n = p.ctl->n_soft;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  int* stack = wf_stack(p.stack_depth);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
    const uint4 e = reinterpret_cast<const uint4*>(p.softq)[j];
    const int i = (int)(e.x / (uint32_t)p.nl), li = (int)(e.x - (uint32_t)i * (uint32_t)p.nl);
    const d3 P = ld_P(p, i);
    d3 ldir;
    double ldist;
    light_vec(p.lights[li], P, ldir, ldist);
    const d3 pt = mk(rt_bits_to_unit(e.y) * 2 - 1, rt_bits_to_unit(e.z) * 2 - 1, rt_bits_to_unit(e.w) * 2 - 1);
    if (any_hit<kCount>(p.g, P, normalize(ldir + muls(pt, 0.1)), ldist, stack, c)) atomicAdd(&p.lstate[e.x], 1u);
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- shade2
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_shade2(const WfParams p) {
  const int n = p.ctl->n_cur;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if ((int)(blockIdx.x * blockDim.x) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const bool hit = i < n && p.hidx[i] >= 0;
  bool cont = false;
  d3 P = mk(0, 0, 0), nd = mk(0, 0, 0), T = mk(0, 0, 0), L = mk(0, 0, 0);
  rt_rng rng{0};
  uint32_t sid = 0;
  int depth = 0;
  if (hit) {
    const WfPaths& a = p.cur;
    P = ld_P(p, i);
    const d3 N = mk(p.nx[i], p.ny[i], p.nz[i]);
    const int info = p.hinfo[i];
    const bool front = info & 1;
    const DMat* __restrict__ m = p.mats + (info >> 1);
    const d3 d = ld_d(a, i);
    T = mk(a.tx[i], a.ty[i], a.tz[i]);
    L = mk(a.lx[i], a.ly[i], a.lz[i]);
    rng.x = a.rng[i];
    sid = a.sid[i];
    depth = a.depth[i];
    // calculateDirectLighting (renderer.go:229-297), light by light
    d3 D = mk(m->ambient, m->ambient, m->ambient);
    for (int li = 0; li < p.nl; ++li) {
      const DLight& Lt = p.lights[li];
      d3 ldir;
      double ldist;
      light_vec(Lt, P, ldir, ldist);
      if (!(ldist < 0.001)) {
        const uint32_t ls = p.lstate[(size_t)i * p.nl + li];
        const bool occl = ls & kHardBit;
        const int unocc = 16 - (int)(ls & 0xFFFFu);
        const double sf = occl ? 0.0 : (p.soft ? (double)unocc / 16.0 : 1.0);  // shadowSum / 16
        if (sf > 0.0) {
          const double metallic = m->metallic;
          double cos_t = gmax0(dot(N, ldir));
          double intensity = cos_t * Lt.intensity / (ldist * ldist);
          D = D + muls(ld3(m->albedo), m->diffuse_strength * intensity * sf);
          if (metallic > 0.5) {
            d3 view = normalize(neg(P));
            d3 half = normalize(ldir + view);
            double hc = gmax0(dot(N, half));
            const int sp = m->spec_pow;
            double si = sp == 64 ? pow_n<64>(hc) : (sp == 48 ? pow_n<48>(hc) : pow_n<32>(hc));
            D = D + muls(ld3(Lt.color), si * intensity * sf * metallic * 3.0);
          }
        }
      }
    }
    // Material.Scatter and the traceRay combination (renderer.go:181-226)
    const d3 E = ld3(m->emit);
    const Scat sc = scatter<kCount>(m, d, N, front, rng, c);
    if (!sc.ok) {
      L = L + mul(T, E + D);
    } else {
      L = L + mul(T, E + muls(D, m->dw));
      cont = p.recursive && depth + 1 < p.max_depth;
      if (cont) {
        T = mul(T, muls(sc.A, m->rw));
        nd = sc.nd;
        depth += 1;
      }
    }
    if (!cont) finish(p, sid, L);
  }
  const int j = wave_append(&p.ctl->n_next, cont);
  if (cont) store_path(p.next, j, P, nd, T, L, rng.x, sid, depth);
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- bookkeeping
// before regen: how many new samples fit (the free slots of the next array)
__global__ void wf_book_regen(WfCtl* ctl, int capacity) {
  const long long left = (long long)ctl->total - (long long)ctl->next_sample;
  const long long room = capacity - ctl->n_next;
  ctl->regen_cnt = (int)(left < room ? left : room);
}
// after regen: the next array becomes current
__global__ void wf_book_swap(WfCtl* ctl) {
  ctl->next_sample += ctl->regen_cnt;
  ctl->n_cur = ctl->n_next;
  ctl->n_next = 0;
  ctl->n_hard = 0;
  ctl->n_soft = 0;
  ctl->regen_cnt = 0;
  ctl->iter += 1;
}

// ---------------------------------------------------------------- resolve
// tracePixel's in-order sum over the pixel's samples (misses are +0, which
// leaves the sum unchanged), the mean, toneMap, one write per pixel.
__global__ __launch_bounds__(kWfBlock) void wf_resolve(const WfParams p, int npix) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= npix) return;
  const uint32_t lp = p.lp0 + (uint32_t)q;
  const int lt = (int)(lp >> 10), tp = (int)(lp & 1023);
  const int tile = p.rank + lt * p.world;
  const int x = (tile % p.tiles_x) * 32 + (tp & 31), y = (tile / p.tiles_x) * 32 + (tp >> 5);
  if (tile >= p.ntiles || x >= p.W || y >= p.H) return;
  const double* r = p.rad + (size_t)q * p.spp * 3;
  double ax = 0, ay = 0, az = 0;
  for (int s = 0; s < p.spp; ++s) {
    ax += r[3 * s + 0];
    ay += r[3 * s + 1];
    az += r[3 * s + 2];
  }
  const double nn = (double)p.spp;
  const double mx = ax / nn, my = ay / nn, mz = az / nn;  // DivScalar(float64(samples))
  const size_t oi = p.layout == RT_LAYOUT_IMAGE ? (size_t)y * p.W + x : (size_t)lt * 1024 + (size_t)tp;
  if (p.out_linear) {
    p.out_linear[oi * 3 + 0] = (float)mx;
    p.out_linear[oi * 3 + 1] = (float)my;
    p.out_linear[oi * 3 + 2] = (float)mz;
  }
  if (p.out_rgba) *reinterpret_cast<uint32_t*>(p.out_rgba + oi * 4) = tonemap_rgba8(mx, my, mz);
}

// ---------------------------------------------------------------- launches
size_t wf_stack_bytes(const WfParams& p) { return (size_t)kWfBlock * p.stack_depth * sizeof(int); }

template <bool kCount>
static int enqueue_iteration(const WfParams& p, hipStream_t st) {
  const int cap = p.capacity;
  const dim3 b(kWfBlock);
  const dim3 gp((cap + kWfBlock - 1) / kWfBlock);
  const size_t sh = wf_stack_bytes(p);
  // queue kernels: grid-stride over at most this many workgroups
  const dim3 gq(std::min((cap * std::max(p.nl, 1) + kWfBlock - 1) / kWfBlock, 256 * 32));
  hipLaunchKernelGGL((wf_extend<kCount>), gp, b, sh, st, p);
  hipLaunchKernelGGL((wf_shade1<kCount>), gp, b, 0, st, p);
  if (p.nl > 0) {
    hipLaunchKernelGGL((wf_hard<kCount>), gq, b, sh, st, p);
    if (p.soft) {
      hipLaunchKernelGGL((wf_softgen<kCount>), gp, b, 0, st, p);
      hipLaunchKernelGGL((wf_soft<kCount>), gq, b, sh, st, p);
    }
  }
  hipLaunchKernelGGL((wf_shade2<kCount>), gp, b, 0, st, p);
  return (int)hipGetLastError();
}

template <bool kCount>
static int enqueue_regen(const WfParams& p, hipStream_t st) {
  hipLaunchKernelGGL(wf_book_regen, dim3(1), dim3(1), 0, st, p.ctl, p.capacity);
  const dim3 g(std::min((p.capacity + kWfBlock - 1) / kWfBlock, 256 * 32));
  hipLaunchKernelGGL((wf_regen<kCount>), g, dim3(kWfBlock), 0, st, p);
  hipLaunchKernelGGL(wf_book_swap, dim3(1), dim3(1), 0, st, p.ctl);
  return (int)hipGetLastError();
}

int wf_launch_regen(const WfParams& p, bool count, void* stream) {
  return count ? enqueue_regen<true>(p, (hipStream_t)stream) : enqueue_regen<false>(p, (hipStream_t)stream);
}
int wf_launch_iteration(const WfParams& p, bool count, void* stream) {
  return count ? enqueue_iteration<true>(p, (hipStream_t)stream) : enqueue_iteration<false>(p, (hipStream_t)stream);
}
int wf_launch_resolve(const WfParams& p, int npix, void* stream) {
  if (npix <= 0) return hipSuccess;
  hipLaunchKernelGGL(wf_resolve, dim3((npix + kWfBlock - 1) / kWfBlock), dim3(kWfBlock), 0, (hipStream_t)stream, p,
                     npix);
  return (int)hipGetLastError();
}

}  // namespace rtgo
