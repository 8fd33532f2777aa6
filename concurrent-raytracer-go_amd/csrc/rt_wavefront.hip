// rt_wavefront.hip — the wavefront path for BVH scenes (> 64 spheres, configs
// C4/C5: 10k spheres).  DESIGN.md §4.2.
//
// The megakernel (rt_kernel.hip) keeps a whole path in one lane: its binary64
// path state costs 168 VGPRs, so a SIMD holds 3 waves, and on a 10k-sphere
// scene its lanes spend most of the time masked off while the longest
// traversal of the wave finishes.  Here traceRay's bounce loop
// (internal/renderer/renderer.go:165-227) is cut into kernels over dense,
// sharded arrays of live paths and shadow rays in HBM:
//
//   extend    closest hit of every live path (hitWorld, renderer.go:333-346,
//             through the BVH); a miss or the depth cut-off ends the path
//   shade1    the HitRecord (sphere.go:42-58); one hard shadow ray per lit
//             light (calculateSmartShadow, renderer.go:299-305) queued
//   occlude   any-hit of the hard rays (wf_occlude4 / wf_cone4: occlusion and
//             cone walks over the 4-wide tree when it fits the LDS whole, as
//             on C4 / C5; else wf_occlude / wf_cone over the binary one)
//   cone      per light whose hard ray is clear, the shadow cone's candidate
//             spheres (a list of <= 16, a wide list of <= 32, or too many)
//   softgen   the 16 RandomVec3InUnitSphere points (renderer.go:311-318) of
//             each clear light from its own stream (RNG spec v4): 16 queued
//             soft rays, or for a (wide) listed cone its stream state and
//             accepted tries; none for an empty cone
//   listtest  a listed cone's 16 rays against its list, one cone per thread
//   widetest  a wide cone's 16 rays against its list, one ray per lane
//   occlude   any-hit of the other soft rays, blocked ones counted per (path, light)
//   shade     calculateDirectLighting (renderer.go:229-297) with those counts,
//             Material.Scatter, the traceRay combination; survivors appended
//             to the next path array, finished paths write their radiance
//   regen     free slots of the next array take new camera samples
//             (tracePixel / getRay, renderer.go:150-163,377-390)
//
// extend and occlude are PERSISTENT traversal kernels: each wave owns a range
// of jobs and refills idle lanes from it as rays finish (Aila & Laine's
// persistent while-while traversal with dynamic fetch), so waves stay full
// instead of waiting for their longest ray.  Appends aggregate per workgroup
// and go to one of kWfShards queues (a workgroup's shard = its index mod
// kWfShards): one atomic per workgroup and queue, spread over 8 words.
//
// The arithmetic is the megakernel's (rt_device.h).  Each path consumes its
// RNG streams as the spec says (include/rt_rng.h: the sample's stream for
// the camera and scatter draws, one stream per (sample, bounce, light) for
// the soft-shadow points; hard rays draw nothing), and each sample's radiance
// lands in its own slot of a per-frame buffer; resolve sums every pixel's
// samples in sample order (tracePixel) — so images are bit-identical to the
// megakernel's and the oracle's (tests/test_gpu_wavefront.py).  The loop is
// host-driven: the book kernel publishes the live count, and the host polls
// a copy of it one bounce behind the GPU to know when the frame is done.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <tuple>

#include "../../include/rt_rng.h"
#include "rt_device.h"
#include "rt_internal.h"

namespace rtgo {

constexpr int kWfBlock = kWfBlockSlots;  // threads per workgroup of the dense kernels
// Traversal kernels: by default one 1024-thread workgroup per CU (4 waves per
// SIMD), whose LDS holds the lanes' stacks and as much of the quantized BVH as
// fits behind them (10k spheres: all 6,623 nodes, 104 KB).  The launch size
// (p.trav_block <= kTravBlock) and workgroups per CU are host choices.
constexpr int kTravBlock = kWfTravBlock;
#define RT_WF_TRAV_WAVES 4  // waves per SIMD the traversal kernels are compiled for
#define RT_TRAV_ATTR __launch_bounds__(kTravBlock) __attribute__((amdgpu_waves_per_eu(RT_WF_TRAV_WAVES)))
constexpr int kLdsBytes = 160 * 1024;    // LDS per CU (MI355X), all of it available to one workgroup
// (measured r02, C4 per frame with 2^21 path slots: chunk 256 / refill 16
// 640 ms, 128 / 16 596, 64 / 16 594, 32 / 16 641, 64 / 24 591, 64 / 32 593,
// 64 / 48 632, 256 / 32 627; with 2^22 slots: 64 / 24 549, 96 / 24 537,
// 128 / 24 536, 64 / 32 552; guided chunks, min(256, left / (k waves)) with
// k = 2, 4, 8: 551-569.  Smaller chunks shorten each persistent launch's
// drain, where waves still hold unstarted jobs while others have none)
#ifndef RT_WF_REFILL
#define RT_WF_REFILL 24
#endif
#ifndef RT_WF_CHUNK
#define RT_WF_CHUNK 128
#endif
constexpr int kRefill = RT_WF_REFILL;    // persistent traversal: refill once this many lanes are idle
constexpr int kChunk = RT_WF_CHUNK;      // persistent traversal: jobs a wave takes per atomic
// lstate per (path, light): blocked soft rays in the low 16 bits, and
constexpr uint32_t kHardBit = 1u << 16;   // the hard shadow ray is blocked
constexpr uint32_t kUnlitBit = 1u << 17;  // the hit point is within 0.001 of the light (no shadow rays)
constexpr uint32_t kListBit = 1u << 18;   // the light's shadow cone left a candidate list (wf_cone)
constexpr uint32_t kEmptyBit = 1u << 19;  // ... an empty one: no soft ray can be blocked
#ifndef RT_WIDE_EXIT
#define RT_WIDE_EXIT 1
#endif
constexpr uint32_t kWideBit = 1u << 20;   // ... a wide one (kWfConeK < candidates <= kWfConeWide, wf_widetest)
// hidx of a path whose ray hit nothing while a sky is opted in: wf_shade1
// ends it with the sky's radiance (GetSkyColor, atmosphere.go:100-135) --
// kept out of the traversal kernel, whose registers it would cost
constexpr int kSkyMiss = -2;

extern __shared__ __attribute__((aligned(16))) unsigned char wf_lds[];

// per-lane BVH stack in dynamic LDS: one region of 64 x depth ints per wave,
// lane-interleaved (closest_hit / any_hit index it with stride 64)
__device__ __forceinline__ int* wf_stack(int depth) {
  return reinterpret_cast<int*>(wf_lds) + (threadIdx.x >> 6) * 64 * depth + (threadIdx.x & 63);
}

// The first p.lds_nodes quantized nodes (breadth-first order, bvh.cpp: the
// top of the tree, or all of it) copied into LDS behind the stacks, once per
// workgroup of a persistent traversal kernel.  Divergent lanes then read
// their node pairs as ds_read_b128 (~50 cycles, 256 B/clk per CU) instead of
// one vector-L1 line per lane.  Every thread must call it.
// (Typed address spaces keep the two loads of descend apart: through generic
// pointers the compiler merges them into one select + flat load.)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4 lds_node;
typedef __attribute__((address_space(1))) const u32x4 glb_node;
__device__ __forceinline__ uint4 as_uint4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ lds_node* stage_tree(const WfParams& p) {
  uint4* t = reinterpret_cast<uint4*>(wf_lds + (size_t)p.trav_block * p.stack_depth * sizeof(int));
  const uint4* src = reinterpret_cast<const uint4*>(p.qbvh);
  for (int i = threadIdx.x; i < p.lds_nodes; i += p.trav_block) t[i] = src[i];
  __syncthreads();
  return (lds_node*)t;
}

// The 4-wide tree (bvh.cpp qbvh4), staged whole behind stacks of p.stack4
// entries per lane (the host sets use4 only when it fits).
__device__ __forceinline__ lds_node* stage_tree4(const WfParams& p) {
  uint4* t = reinterpret_cast<uint4*>(wf_lds + (size_t)p.trav_block * p.stack4 * sizeof(int));
  const uint4* src = reinterpret_cast<const uint4*>(p.qbvh4);
  for (int i = threadIdx.x; i < p.nodes4; i += p.trav_block) t[i] = src[i];
  __syncthreads();
  return (lds_node*)t;
}

// Block-wide exclusive prefix of a per-lane count over the workgroup (wave
// scans, one LDS word per wave); sets `total`.  Every thread must call it.
__device__ __forceinline__ int block_prefix(int v, int* s_wave, int& total) {
  const int lane = (int)(threadIdx.x & 63), w = (int)(threadIdx.x >> 6);
  int incl = v;
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(incl, off);
    if (lane >= off) incl += t;
  }
  if (lane == 63) s_wave[w] = incl;
  __syncthreads();
  int before = 0;
  total = 0;
  for (int k = 0; k < kWfBlock / 64; ++k) {
    const int x = s_wave[k];
    before += k < w ? x : 0;
    total += x;
  }
  __syncthreads();  // s_wave is reused by the next call
  return before + incl - v;
}

// Append `v` entries per thread to the workgroup's shard of a sharded queue:
// one atomic per workgroup; returns this thread's first entry index within
// the shard.  Every thread must call it.
__device__ __forceinline__ int block_append(int v, int32_t* shard_cnt, int* s_wave, int* s_base) {
  int total;
  const int before = block_prefix(v, s_wave, total);
  if (threadIdx.x == 0 && total > 0) *s_base = atomicAdd(shard_cnt, total);
  __syncthreads();
  return *s_base + before;
}

// Dense index over the kWfShards shards of an array or queue (counts at
// cnt[32 s]): start[s] = entries before shard s.  Constant indices only, so
// start[] stays in registers.
struct Dense {
  int start[kWfShards + 1];
};
__device__ __forceinline__ Dense dense(const int32_t* cnt) {
  Dense d;
  d.start[0] = 0;
#pragma unroll
  for (int s = 0; s < kWfShards; ++s) d.start[s + 1] = d.start[s] + cnt[s * 32];
  return d;
}
// entry j (< total) -> physical index shard * cap + offset
__device__ __forceinline__ size_t dense_at(const Dense& d, int j, size_t cap) {
  int s = 0, off = 0;
#pragma unroll
  for (int k = 1; k < kWfShards; ++k)
    if (j >= d.start[k]) {
      s = k;
      off = d.start[k];
    }
  return (size_t)s * cap + (size_t)(j - off);
}

// (group: the kernel also adds its counts to its own slots of rt_counts --
// kGroupSoft: the soft-shadow stage (rt_counts.soft_occlusion); kGroupHard:
// the hard-ray traversal (rt_counts.hard_occlusion) -- in both the
// shadow-ray slot counts the rays the kernel traced, kept in c.v[kSoftJobs]
// and left out of the totals (softgen and shade1 count them there);
// kGroupExtend: the closest-hit traversal (rt_counts.extend) -- for each
// kernel's own roofline)
constexpr int kSoftJobs = C_SHADOW;
template <bool kCount>
__device__ __forceinline__ void flush_counts(const WfParams& p, Counters& c, int group = 0) {
  if constexpr (kCount) {
    for (int i = 0; i < kCounters; ++i) {
      unsigned long long v = c.v[i];
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if ((threadIdx.x & 63) == 0 && v) {
        if (!((group == kGroupSoft || group == kGroupHard) && i == kSoftJobs)) atomicAdd(&p.counts[i], v);
        if (group) atomicAdd(&p.counts[group * kCounters + i], v);
      }
    }
  }
}

__device__ __forceinline__ d3 ld_o(const WfPaths& a, size_t i) { return mk(a.ox[i], a.oy[i], a.oz[i]); }
__device__ __forceinline__ d3 ld_d(const WfPaths& a, size_t i) { return mk(a.dx[i], a.dy[i], a.dz[i]); }
__device__ __forceinline__ d3 ld_P(const WfParams& p, int i) { return mk(p.px[i], p.py[i], p.pz[i]); }

// the light vector of a hit point: calculateDirectLighting's lightDir and
// distance (renderer.go:249-254); recomputed wherever needed, same bits
__device__ __forceinline__ void light_vec(const DLight& Lt, d3 P, d3& ldir, double& ldist) {
  const d3 lv = ld3(Lt.pos) - P;
  ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
  ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
}

__device__ __forceinline__ void store_path(const WfPaths& b, size_t j, d3 o, d3 d, d3 T, d3 L, uint64_t rng,
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

// ---------------------------------------------------------------- traversal
// Slab tests against the quantized BVH (DQNode: 16-bit grid indices, bounds
// rounded outward, bvh.cpp).  For a grid index q on axis k the slab distance
// is t = (q0 + q qd - o) inv = q A + B with A = qd inv, B = (q0 - o) inv
// (binary64).  The kernel evaluates it in binary32 (ray_q_axis: the error
// bound e_k and its derivation); e_k is folded into the coefficient used for
// the near and for the far bound of axis k (pushed outward: down for the near
// side, up for the far side), so every computed near distance is <= the
// exact one and every far distance >= it; max/min/med3 and the final compare
// are exact, so a box the exact interval meets is never rejected.  tmin /
// tmax enter rounded outward (t_lo32 / t_hi32).  A ray whose coefficients are
// not finite or too large tests every box as hit (A = 0, B = -1e30 / +1e30
// per axis: the interval becomes [tmin, tmax]): slower, exact.
// Node words (bvh.cpp): w[k] = lo_k | hi_k << 16 for axes k = 0..2, w[3] the
// child code.  Per ray and axis the near bound is lo when the direction is
// positive, else hi; a per-ray byte selector `s` picks it, so the near and
// far grid indices of an axis come out of two v_perm_b32 as the float bits
// of 2^23 + q (exact), and one packed fma (with the 2^23 folded into B,
// below) gives (t_near, t_far) with no per-box min/max.
typedef float f2 __attribute__((ext_vector_type(2)));
struct RayQ {
  float ax, ay, az;  // A per axis
  f2 bx, by, bz;     // (B - e, B + e): the near and the far bound's coefficient
  uint32_t sx, sy, sz;  // v_perm selector of the near half (the far half: s ^ 0x0202)
};
constexpr uint32_t kSelLo = 0x070c0100u, kSelHi = 0x070c0302u;  // bytes {q, q, 0x00, 0x4B}
// The kernel evaluates t = fma(Q, A, B') with Q = 2^23 + q (the float whose
// bits v_perm_b32 builds, no subtraction) and B' = B - 2^23 A, so that
// Q A + B' = q A + B.  Error against the exact t: |Q (fl(A) - A)| <= |A|
// (Q < 2^24), fl(B') - B' <= 2^-24 (|B| + 2^23 |A|), and the fma's one
// rounding 2^-24 |t| <= 2^-24 (65537 |A| + |B|): in all < 1.51 |A| +
// 2^-23 |B|.  The bound e = 2 |A| + 2^-22 (65536 |A| + |B|) covers it (|A| is
// one grid step of t: the test widens boxes by about two steps, 2 / 65000 of
// the scene extent), and is folded outward into B' as before.
__device__ __forceinline__ void ray_q_axis(double q0, double qd, double o, double id, float& a, f2& b, uint32_t& sel,
                                           bool& ok) {
  const double ik = fmin(fmax(id, -1e30), 1e30);
  const double A = qd * ik, B = (q0 - o) * ik;
  const double e = 2.0 * fabs(A) + (65536.0 * fabs(A) + fabs(B)) * 0x1p-22;
  const double Bp = B - 8388608.0 * A;
  // the near side is pushed down, the far side up
  const double bn = Bp - e, bf = Bp + e;
  a = (float)A;
  b = f2{(float)bn, (float)bf};
  sel = ik > 0 ? kSelLo : kSelHi;  // t = q A + B grows with q when A > 0: near = lo
  ok = ok && __builtin_isfinite(A) && __builtin_isfinite(bn) && __builtin_isfinite(bf) && fabs(bn) < 1e37 &&
       fabs(bf) < 1e37 && fabs(A) < 1e30;
}
__device__ __forceinline__ RayQ ray_q(const WfParams& p, d3 o, d3 id) {
  RayQ r;
  bool ok = true;
  ray_q_axis(p.q0[0], p.qd[0], o.x, id.x, r.ax, r.bx, r.sx, ok);
  ray_q_axis(p.q0[1], p.qd[1], o.y, id.y, r.ay, r.by, r.sy, ok);
  ray_q_axis(p.q0[2], p.qd[2], o.z, id.z, r.az, r.bz, r.sz, ok);
  if (!ok) {
    r.ax = r.ay = r.az = 0.f;
    r.bx = r.by = r.bz = f2{-1e30f, 1e30f};
  }
  return r;
}
// (near, far) of one axis word as Q = 2^23 + q, exact floats
__device__ __forceinline__ f2 q_near_far(uint32_t w, uint32_t sel) {
  return f2{__builtin_bit_cast(float, __builtin_amdgcn_perm(0x4B000000u, w, sel)),
            __builtin_bit_cast(float, __builtin_amdgcn_perm(0x4B000000u, w, sel ^ 0x0202u))};
}
__device__ __forceinline__ bool box_q(const uint4 n, const RayQ& r, float tmin, float tmax, float& tn) {
  const f2 tx = __builtin_elementwise_fma(q_near_far(n.x, r.sx), f2{r.ax, r.ax}, r.bx);
  const f2 ty = __builtin_elementwise_fma(q_near_far(n.y, r.sy), f2{r.ay, r.ay}, r.by);
  const f2 tz = __builtin_elementwise_fma(q_near_far(n.z, r.sz), f2{r.az, r.az}, r.bz);
  // (med3 with a huge bound clamps by the loop-invariant tmin / tmax without
  // the per-iteration canonicalisation fmaxf / fminf of them costs)
  tn = fmaxf(fmaxf(tx.x, ty.x), __builtin_amdgcn_fmed3f(tz.x, tmin, 3.4e38f));
  const float tf = fminf(fminf(tx.y, ty.y), __builtin_amdgcn_fmed3f(tz.y, -3.4e38f, tmax));
  return tn <= tf;
}

// One step of the while-while traversal of a lane (the closest_hit / any_hit
// order of rt_device.h over the same tree): descend internal nodes, nearer
// child first, until `cur` is a leaf (count 1..4) or -1 (done).
// Node pairs below `nlds` come from the LDS copy `lt` (stage_tree), the rest
// from global memory.
// kFull: the whole tree is staged (no global-memory branch).
template <bool kFull>
__device__ __forceinline__ void load_pair(glb_node* __restrict__ qb, lds_node* __restrict__ lt, int nlds, int first,
                                          uint4& L, uint4& R) {
  if (kFull || first < nlds) {  // nlds is odd or the whole tree: a staged pair is whole
    L = as_uint4(lt[first]);
    R = as_uint4(lt[first + 1]);
  } else {
    L = as_uint4(qb[first]);
    R = as_uint4(qb[first + 1]);
  }
}
template <bool kCount, bool kFull>
__device__ __forceinline__ void descend(glb_node* __restrict__ qb, lds_node* __restrict__ lt, int nlds,
                                        const RayQ& r, float tminf, float tmaxf, int& cur, int& sp, int* stack,
                                        Counters& c) {
  while ((cur & 7) == 0) {
    uint4 L, R;
    load_pair<kFull>(qb, lt, nlds, cur >> 3, L, R);
    cnt<kCount>(c, C_BOX, 2);
    float tl, tr;
    const bool hl = box_q(L, r, tminf, tmaxf, tl), hr = box_q(R, r, tminf, tmaxf, tr);
    if (hl || hr) {
      const bool lfirst = hl && (!hr || tl <= tr);
      if (hl && hr) {
        stack[sp * 64] = lfirst ? (int)R.w : (int)L.w;
        ++sp;
      }
      cur = lfirst ? (int)L.w : (int)R.w;
    } else {
      cur = sp == 0 ? -1 : stack[--sp * 64];
    }
  }
}

// The closest-hit descent with an early exit (wf_extend): the lanes that
// have reached a leaf idle in `descend` until the deepest-descending lane
// of the wave gets there (C4: 14.6 % of the lanes active per VALU
// instruction).  Here the descent stops for every lane once at most
// 1/kDescendFrac of the lanes that entered it are still descending; those
// keep their node and stack and go on in the next round, while the others
// test their leaves now.  (The node order and the tests are the same: only
// when each lane's steps run changes, not which.)
// (C4 per frame, scripts/c4_tuning_probe.py, one MI355X, two frames each,
// profiles/r06_c4_descend.jsonl: closest hit 102.5-102.9 ms without the exit,
// 103.9-104.3 at 1/2, 98.0-98.4 at 1/4, 98.6-99.0 at 1/8; frame 373.8-374.2 ->
// 369.1-369.2 ms at 1/4; the image checksum unchanged)
#ifndef RT_DESCEND_FRAC
#define RT_DESCEND_FRAC 4
#endif
constexpr int kDescendFrac = RT_DESCEND_FRAC;
template <bool kCount, bool kFull>
__device__ __forceinline__ void descend_x(glb_node* __restrict__ qb, lds_node* __restrict__ lt, int nlds,
                                          const RayQ& r, float tminf, float tmaxf, int& cur, int& sp, int* stack,
                                          Counters& c) {
  if constexpr (kDescendFrac <= 0) {
    descend<kCount, kFull>(qb, lt, nlds, r, tminf, tmaxf, cur, sp, stack, c);
  } else {
    const int entered = __popcll(__ballot(true));
    while ((cur & 7) == 0) {
      uint4 L, R;
      load_pair<kFull>(qb, lt, nlds, cur >> 3, L, R);
      cnt<kCount>(c, C_BOX, 2);
      float tl, tr;
      const bool hl = box_q(L, r, tminf, tmaxf, tl), hr = box_q(R, r, tminf, tmaxf, tr);
      if (hl || hr) {
        const bool lfirst = hl && (!hr || tl <= tr);
        if (hl && hr) {
          stack[sp * 64] = lfirst ? (int)R.w : (int)L.w;
          ++sp;
        }
        cur = lfirst ? (int)L.w : (int)R.w;
      } else {
        cur = sp == 0 ? -1 : stack[--sp * 64];
      }
      // (the lanes still in this loop are the active ones: the ballot counts them)
      if (__popcll(__ballot((cur & 7) == 0)) * kDescendFrac <= entered) break;
    }
  }
}

// The any-hit descent over the 4-wide tree (bvh.cpp qbvh4: groups of 2..4
// child boxes): a group's boxes are tested at once, the first hit child in
// slot order is entered and the other hit children are pushed.  Half the
// dependent LDS round trips of the binary walk.  No distance order: an
// occlusion query ends at any hit, and sorting the children (full sort, or
// the nearest first) measured slower, as did the 4-wide tree for closest hit
// (DESIGN.md §4.2).  The order does not change which rays are blocked.
// (the same early exit as descend_x, 1/RT_OCC_FRAC; 0: none)
#ifndef RT_OCC_FRAC
#define RT_OCC_FRAC 4
#endif
template <bool kCount>
__device__ __forceinline__ void descend4(lds_node* __restrict__ lt, const RayQ& r, float tminf, float tmaxf, int& cur,
                                         int& sp, int* stack, Counters& c) {
  const int entered = RT_OCC_FRAC > 0 ? __popcll(__ballot(true)) : 0;
  while ((cur & 7) == 0) {
    const int base = cur >> 5, nk = ((cur >> 3) & 3) + 1;  // the group's first slot and size (bvh.cpp)
    const uint4 n0 = as_uint4(lt[base]), n1 = as_uint4(lt[base + 1]), n2 = as_uint4(lt[base + 2]),
                n3 = as_uint4(lt[base + 3]);
    cnt<kCount>(c, C_BOX, nk);
    float t0, t1, t2, t3;
    const int cs[4] = {(int)n0.w, (int)n1.w, (int)n2.w, (int)n3.w};
    const bool hs[4] = {box_q(n0, r, tminf, tmaxf, t0), box_q(n1, r, tminf, tmaxf, t1),
                        box_q(n2, r, tminf, tmaxf, t2) && nk > 2, box_q(n3, r, tminf, tmaxf, t3) && nk > 3};
    bool taken = false;
#pragma unroll
    for (int k = 3; k >= 0; --k)
      if (hs[k]) {
        if (taken) stack[sp++ * 64] = cur;
        cur = cs[k];
        taken = true;
      }
    if (!taken) cur = sp == 0 ? -1 : stack[--sp * 64];
    if (RT_OCC_FRAC > 0 && __popcll(__ballot((cur & 7) == 0)) * RT_OCC_FRAC <= entered) break;
  }
}

// The spheres of a leaf: the loads of the first kLeafBatch are issued
// together, before any test, so a leaf costs one memory round trip instead of
// one per sphere (the tests stop early in occlusion, which kept the compiler
// from hoisting the loads).  Indices past the leaf reload its last sphere.
constexpr int kLeafBatch = 4;  // = the BVH's largest leaf (bvh.cpp)
__device__ __forceinline__ void load_leaf(const DSphere* __restrict__ sp, int first, int count, DSphere* out) {
#pragma unroll
  for (int k = 0; k < kLeafBatch; ++k) out[k] = sp[first + min(k, count - 1)];
}
__device__ __forceinline__ const DSphere& leaf_sphere(const DSphere* sp, const DSphere* ls, int first, int i) {
  return i - first < kLeafBatch ? ls[i - first] : sp[i];
}

// Dynamic job distribution of the persistent traversal kernels.  The dense
// job space [0, n) is cut into kWfShards ranges, each with a head counter
// (heads[32 s], reset by wf_book); a wave takes chunks of kChunk jobs from
// its home range (its workgroup index mod kWfShards, i.e. its XCD under the
// round-robin dispatch), then from the other ranges.  (A static split of the
// jobs over the waves left the SIMDs idle half the time: traversal lengths
// vary too much.)  Called by whole waves; wave-uniform state.
struct JobSrc {
  int next, hi;  // the current chunk
  int tried;     // ranges found empty
  int chunk;     // jobs per atomic (job_chunk)
};
// Jobs a wave takes per atomic: kChunk while the launch has plenty (a
// persistent launch drains faster when no wave holds many unstarted jobs,
// but every atomic costs), fewer when it has fewer jobs than waves x kChunk
// -- the frame's last bounce iterations, where a few thousand long paths
// would otherwise queue on a few dozen waves -- down to kMinChunk.
constexpr int kMinChunk = 16;
__device__ __forceinline__ JobSrc job_src(int n) {
  const int waves = (int)(gridDim.x * (blockDim.x >> 6));
  return JobSrc{0, 0, 0, min(kChunk, max(kMinChunk, n / max(1, waves)))};
}
__device__ __forceinline__ bool job_refill(JobSrc& js, int32_t* heads, int n) {
  const int home = blockIdx.x % kWfShards;
  while (js.tried < kWfShards) {
    const int s = (home + js.tried) % kWfShards;
    const int lo_s = (int)((long long)n * s / kWfShards), hi_s = (int)((long long)n * (s + 1) / kWfShards);
    int got = 0;
    if ((threadIdx.x & 63) == 0) got = atomicAdd(&heads[s * 32], js.chunk);
    got = __builtin_amdgcn_readfirstlane(got);
    if (lo_s + got < hi_s) {
      js.next = lo_s + got;
      js.hi = min(hi_s, js.next + js.chunk);
      return true;
    }
    ++js.tried;
  }
  return false;
}

// ---------------------------------------------------------------- extend
// Persistent closest-hit traversal of the live paths (hitWorld,
// renderer.go:333-346, in the BVH form of rt_device.h closest_hit: same
// tests, same exact-t tie rule).  Wave w owns jobs [n w / W, n (w+1) / W) and
// refills idle lanes from them.  A hit leaves (sphere, root numerator) for
// shade1; a miss ends the path with the radiance it has (renderer.go:170-173).
template <bool kCount, bool kFull>
__global__ RT_TRAV_ATTR void wf_extend(const WfParams p) {
  const Dense dn = dense(p.ctl->cur_cnt);
  const int n = dn.start[kWfShards];
  if (n == 0) return;
  lds_node* lt = stage_tree(p);
  JobSrc js = job_src(n);
  bool more = true;  // wave-uniform: jobs may remain
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int* stack = wf_stack(p.stack_depth);
  const WfPaths& a = p.cur;
  const double tmin = 0.001;
  bool busy = false;
  size_t slot = 0;
  d3 o = mk(0, 0, 0), d = mk(0, 0, 0);
  double av = 0, inv_a = 0, closest = 0;
  RayQ r32{};
  float tminf = 0;
  int cur = -1, sp = 0, best_obj = -1, bidx = -1;
  for (;;) {
    const unsigned long long idle = __ballot(!busy);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull) && js.next >= js.hi)
      more = job_refill(js, p.ctl->job_head[0], n);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull)) {
      const int j = js.next + __popcll(idle & below), hi = js.hi;
      js.next = min(hi, js.next + __popcll(idle));
      if (!busy && j < hi) {
        slot = dense_at(dn, j, p.shard_cap);
        const uint32_t sid = a.sid[slot];
        bool miss = true;
        if (sid != kDeadSid && a.depth[slot] < p.max_depth) {  // traceRay's depth cut-off comes first
          cnt<kCount>(c, C_BOUNCE);
          o = ld_o(a, slot);
          d = ld_d(a, slot);
          av = len2(d);
          inv_a = approx_rcp(av);
          closest = __builtin_inf();
          best_obj = -1;
          const d3 id = inv_dir_fast(d);
          cnt<kCount>(c, C_BOX);
          if (box_hit(p.g.bvh[0], o, id, tmin, closest)) {
            r32 = ray_q(p, o, id);
            tminf = t_lo32(tmin);
            cur = bvh_code(p.g.bvh[0]);
            sp = 0;
            busy = true;
            miss = false;
          }
        }
        if (miss) {
          // the root box missed: with an opted-in sky, shade1 adds it (kSkyMiss)
          const bool sky = p.sky && sid != kDeadSid && a.depth[slot] < p.max_depth;
          p.hidx[slot] = sky ? kSkyMiss : -1;
          if (sid != kDeadSid && !sky) finish(p, sid, mk(a.lx[slot], a.ly[slot], a.lz[slot]));
        }
      }
    }
    if (__ballot(busy) == 0) {
      if (!more) break;
      continue;
    }
    if (busy) {
      descend_x<kCount, kFull>((glb_node*)p.qbvh, lt, p.lds_nodes, r32, tminf, t_hi32(closest), cur, sp, stack, c);
      if (cur != -1 && (cur & 7) != 0) {  // a leaf: the exact Sphere.Hit tests, in hittable order
        const int first = cur >> 3, count = cur & 7;
        DSphere ls[kLeafBatch];
        load_leaf(p.g.spheres, first, count, ls);
        for (int i = first; i < first + count; ++i) {
          cnt<kCount>(c, C_SPH);
          const DSphere& S = leaf_sphere(p.g.spheres, ls, first, i);
          double num;
          if (sphere_query(S, o, d, av, inv_a, tmin, closest, num)) {
            const double t = num / av;
            if (t == closest && best_obj > S.obj) continue;
            closest = t;
            bidx = i;
            best_obj = S.obj;
          }
        }
        cur = sp == 0 ? -1 : stack[--sp * 64];
      }
      if (cur == -1) {  // traversal done
        busy = false;
        if (best_obj >= 0) {
          // the hit point (HitRecord.P, sphere.go:44: t = the root / a, as
          // kept in `closest`), for shade1, the occlusion kernels and shade
          const d3 P = o + muls(d, closest);
          p.hidx[slot] = bidx;
          p.px[slot] = P.x;
          p.py[slot] = P.y;
          p.pz[slot] = P.z;
        } else if (p.sky) {  // a miss with an opted-in sky: shade1 adds it
          p.hidx[slot] = kSkyMiss;
        } else {
          p.hidx[slot] = -1;
          finish(p, a.sid[slot], mk(a.lx[slot], a.ly[slot], a.lz[slot]));
        }
      }
    }
  }
  flush_counts<kCount>(p, c, kGroupExtend);
}

// ---------------------------------------------------------------- shade1
// HitRecord of every hit (sphere.go:42-58, as in the megakernel) and one hard
// shadow ray per lit light (renderer.go:249-256,299-305) into the hard queue.
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_shade1(const WfParams p) {
  __shared__ int s_wave[kWfBlock / 64];
  __shared__ int s_base;
  const Dense dn = dense(p.ctl->cur_cnt);
  const int n = dn.start[kWfShards];
  if ((int)(blockIdx.x * kWfBlock) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int j = blockIdx.x * kWfBlock + threadIdx.x;
  size_t slot = 0;
  bool hit = false;
  d3 P = mk(0, 0, 0);
  if (j < n) {
    slot = dense_at(dn, j, p.shard_cap);
    const int hi = p.hidx[slot];
    hit = hi >= 0;
    if (hi == kSkyMiss) {  // (opt-in sky) the path ends: L + T * sky(direction)
      const WfPaths& a = p.cur;
      const d3 L = mk(a.lx[slot], a.ly[slot], a.lz[slot]), T = mk(a.tx[slot], a.ty[slot], a.tz[slot]);
      finish(p, a.sid[slot], L + mul(T, sky_color(p.sky, ld_d(a, slot))));
    }
    if (hit) {
      cnt<kCount>(c, C_SHADE);
      // (wf_extend stored the hit point; the normal and the face are
      // recomputed from it where they are used, wf_shade: the same
      // operations give the same bits, with fewer bytes through HBM)
      P = mk(p.px[slot], p.py[slot], p.pz[slot]);
    }
  }
  const int shard = blockIdx.x % kWfShards;
  uint32_t* hq = p.hardq + (size_t)shard * p.hard_cap;
  // The hard ray is first tested against the hit sphere itself: a ray that
  // leaves through the sphere (the light behind the surface, or a path
  // inside a glass sphere) is blocked by it, and an occlusion query's answer
  // does not depend on which hittable blocks it, so it is settled here
  // without a traversal (exact: the same Sphere.Hit test).
  const DSphere* S0 = hit ? &p.g.spheres[p.hidx[slot]] : nullptr;
  // lights in chunks of 32 (one bit each; any number of lights)
  for (int base = 0; base < p.nl; base += 32) {
    uint32_t lit = 0;
    if (hit) {
      const int end = min(p.nl, base + 32);
      for (int li = base; li < end; ++li) {
        d3 ldir;
        double ldist;
        light_vec(p.lights[li], P, ldir, ldist);
        uint32_t st = kUnlitBit;
        if (!(ldist < 0.001)) {
          st = 0;
          cnt<kCount>(c, C_LIGHT);
          cnt<kCount>(c, C_SHADOW);
          cnt<kCount>(c, C_SPH);
          const double a = len2(ldir);
          double num;
          if (sphere_query(*S0, P, ldir, a, approx_rcp(a), 0.001, ldist, num))
            st = kHardBit;
          else
            lit |= 1u << (li - base);
        }
        p.lstate[slot * p.nl + li] = st;
      }
    }
    int q = block_append(__popc(lit), &p.ctl->hard_cnt[shard * 32], s_wave, &s_base);
    for (uint32_t m = lit; m; m &= m - 1) hq[q++] = (uint32_t)(slot * p.nl) + (uint32_t)(base + __builtin_ctz(m));
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- occlude
// Persistent any-hit traversal of the queued shadow rays (hitWorld as used by
// calculateSmartShadow, renderer.go:305,320: is anything hit in
// [0.001, distance)?).  kSoft: the ray is normalize(lightDir + 0.1 p) of a
// queued point p (renderer.go:316-318) and a blocked ray adds 1 to its
// (path, light) count; hard: the ray is lightDir and a blocked ray sets
// kHardBit.
template <bool kCount, bool kSoft, bool kFull, bool kB4>
__device__ __forceinline__ void occlude_body(const WfParams& p) {
  const Dense dn = dense(kSoft ? p.ctl->soft_cnt : p.ctl->hard_cnt);
  const int n = dn.start[kWfShards];
  if (n == 0) return;
  lds_node* lt = kB4 ? stage_tree4(p) : stage_tree(p);
  JobSrc js = job_src(n);
  bool more = true;  // wave-uniform: jobs may remain
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int* stack = wf_stack(kB4 ? p.stack4 : p.stack_depth);
  const double tmin = 0.001;
  bool busy = false;
  uint32_t key = 0;
  d3 o = mk(0, 0, 0), d = mk(0, 0, 0);
  double av = 0, inv_a = 0, tmax = 0;
  RayQ r32{};
  float tminf = 0, tmaxf = 0;
  int cur = -1, sp = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!busy);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull) && js.next >= js.hi)
      more = job_refill(js, p.ctl->job_head[kSoft ? 2 : 1], n);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull)) {
      const int j = js.next + __popcll(idle & below), hi = js.hi;
      js.next = min(hi, js.next + __popcll(idle));
      if (!busy && j < hi) {
        const size_t at = dense_at(dn, j, kSoft ? p.soft_cap : p.hard_cap);
        uint4 e;
        if constexpr (kSoft)
          e = reinterpret_cast<const uint4*>(p.softq)[at];
        else
          e = make_uint4(p.hardq[at], 0, 0, 0);
        key = e.x;
        if constexpr (kCount) ++c.v[kSoftJobs];  // (the rays traced: flushed to the kernel's own slots only)
        const uint32_t slot = key / (uint32_t)p.nl, li = key - slot * (uint32_t)p.nl;
        o = mk(p.px[slot], p.py[slot], p.pz[slot]);
        d3 ldir;
        light_vec(p.lights[li], o, ldir, tmax);
        if constexpr (kSoft) {
          const d3 pt =
              mk(rt_bits_to_unit(e.y) * 2 - 1, rt_bits_to_unit(e.z) * 2 - 1, rt_bits_to_unit(e.w) * 2 - 1);
          d = normalize(ldir + muls(pt, 0.1));
        } else {
          d = ldir;
        }
        av = len2(d);
        inv_a = approx_rcp(av);
        const d3 id = inv_dir_fast(d);
        cnt<kCount>(c, C_BOX);
        if (box_hit(p.g.bvh[0], o, id, tmin, tmax)) {
          r32 = ray_q(p, o, id);
          tminf = t_lo32(tmin);
          tmaxf = t_hi32(tmax);
          cur = kB4 ? p.root4 : bvh_code(p.g.bvh[0]);
          sp = 0;
          busy = true;
        }
      }
    }
    if (__ballot(busy) == 0) {
      if (!more) break;
      continue;
    }
    if (busy) {
      if constexpr (kB4)
        descend4<kCount>(lt, r32, tminf, tmaxf, cur, sp, stack, c);
      else
        descend<kCount, kFull>((glb_node*)p.qbvh, lt, p.lds_nodes, r32, tminf, tmaxf, cur, sp, stack, c);
      bool blocked = false;
      if (cur != -1 && (cur & 7) != 0) {  // (a leaf; an internal node: the descent paused, descend4)
        const int first = cur >> 3, count = cur & 7;
        DSphere ls[kLeafBatch];
        load_leaf(p.g.spheres, first, count, ls);
        for (int i = first; i < first + count && !blocked; ++i) {
          cnt<kCount>(c, C_SPH);
          double num;
          blocked = sphere_query(leaf_sphere(p.g.spheres, ls, first, i), o, d, av, inv_a, tmin, tmax, num) != 0;
        }
        cur = sp == 0 ? -1 : stack[--sp * 64];
      }
      if (blocked) {
        if constexpr (kSoft)
          atomicAdd(&p.lstate[key], 1u);
        else
          p.lstate[key] = kHardBit;
      }
      if (blocked || cur == -1) busy = false;
    }
  }
  flush_counts<kCount>(p, c, kSoft ? kGroupSoft : kGroupHard);
}
template <bool kCount, bool kSoft, bool kFull>
__global__ RT_TRAV_ATTR void wf_occlude(const WfParams p) {
  occlude_body<kCount, kSoft, kFull, false>(p);
}
template <bool kCount, bool kSoft>  // over the 4-wide tree (WfParams.use4)
__global__ RT_TRAV_ATTR void wf_occlude4(const WfParams p) {
  occlude_body<kCount, kSoft, true, true>(p);
}

// ---------------------------------------------------------------- cones
// Soft shadows through shadow cones (the BVH form of the megakernel's cone
// culling, rt_kernel.hip in_cone).  calculateSmartShadow's 16 soft rays of a
// (path, light) all leave the hit point P inside the cone of half-angle
// asin(0.1) around lightDir and end at the light (renderer.go:311-320).  A
// sphere that cannot meet that cone segment cannot block any of them, so the
// blocked count over the spheres that can (the candidates) is the count over
// the scene.  wf_conegen queues every (path, light) whose hard ray is clear;
// wf_cone walks the BVH with the cone and, when at most kWfConeK spheres are
// candidates, leaves their list and kListBit in lstate; wf_softgen queues
// such a cone's stream state and accepted tries apart, and wf_listtest
// rebuilds its 16 rays and tests them against the list
// -- the same Sphere.Hit test the traversal runs -- instead
// of walking the tree.  C4 (scripts/cone_stats.py): 45 % of the clear cones
// are empty, the median cone has 1 candidate, 6 % have more than 16.
//
// Node test (binary32, on the quantized bounds).  A point X of the cone
// with projection t on the axis u lies within t tan(a) of P + t u, so on
// every axis k, lo_k - t tan(a) <= P_k + t u_k <= hi_k + t tan(a) for a box
// holding X.  With A = u_k + tau, B = u_k - tau (tau >= tan(asin 0.1)) that
// is t A >= lo_k - P_k and t B <= hi_k - P_k: two linear bounds on t per axis
// (lower or upper by the signs of A and B), intersected with [0, length].
// Like the ray's slab test (ray_q_axis), each bound is one fma of the grid
// index with its binary32 error bound folded outward, so a box the cone
// meets is never rejected.  (scripts/cone_stats.py: 67 nodes per cone walk
// against 98 with the nodes' bounding balls.)
constexpr double kTau = 0.1006;  // > tan(asin(0.1)) = 0.10050378
struct ConeQ {
  f2 ax, ay, az;        // per axis: the coefficients of the (first, second) bound
  f2 bx, by, bz;
  f2 px, py, pz;        // per axis: (second -> lower, second -> upper) penalties
  uint32_t sx, sy, sz;  // v_perm selector: which of lo / hi feeds the first bound
  float len;            // the light distance, rounded up
};
// First bound: always a lower bound.  Second: an upper bound (u_k >= tau or
// <= -tau: penalties (-3e38, 0)) or a lower bound (|u_k| < tau: (0, 3e38)).
__device__ __forceinline__ void cone_q_axis(double q0, double qd, double P, double u, f2& a, f2& b, f2& pen,
                                            uint32_t& sel, bool& ok) {
  const double A = u + kTau, B = u - kTau;
  const double iA = 1.0 / A, iB = 1.0 / B;
  const double aL = qd * iA, bL = (q0 - P) * iA;  // (lo - P) / A
  const double aH = qd * iB, bH = (q0 - P) * iB;  // (hi - P) / B
  const double eL = 2.0 * fabs(aL) + (65536.0 * fabs(aL) + fabs(bL)) * 0x1p-22;
  const double eH = 2.0 * fabs(aH) + (65536.0 * fabs(aH) + fabs(bH)) * 0x1p-22;
  const double bpL = bL - 8388608.0 * aL, bpH = bH - 8388608.0 * aH;
  double a1, b1, a2, b2;
  if (B > 0) {  // lo: lower, hi: upper
    a1 = aL, b1 = bpL - eL, a2 = aH, b2 = bpH + eH;
    sel = kSelLo;
    pen = f2{-3e38f, 0.f};
  } else if (A < 0) {  // hi: lower, lo: upper
    a1 = aH, b1 = bpH - eH, a2 = aL, b2 = bpL + eL;
    sel = kSelHi;
    pen = f2{-3e38f, 0.f};
  } else {  // both lower
    a1 = aL, b1 = bpL - eL, a2 = aH, b2 = bpH - eH;
    sel = kSelLo;
    pen = f2{0.f, 3e38f};
  }
  a = f2{(float)a1, (float)a2};
  b = f2{(float)b1, (float)b2};
  ok = ok && fabs(A) > 1e-6 && fabs(B) > 1e-6 && fabs(a1) < 1e30 && fabs(a2) < 1e30 && fabs(b1) < 1e37 &&
       fabs(b2) < 1e37;
}
// ok = false: a coefficient is not finite or too large for binary32; the
// caller then does not walk the cone (its rays are traced, exact).  (Round 3
// kept every node instead, by selects on all of ConeQ's fields; that form
// made the cone kernel 4.7x slower, 249 vs 53 ms per C4 frame, though the
// fallback never runs on C4: it changed how the kernel's code came out.)
__device__ __forceinline__ ConeQ cone_q(const WfParams& p, d3 P, d3 u, double ldist, bool& ok) {
  ConeQ k;
  ok = __builtin_isfinite(ldist);
  cone_q_axis(p.q0[0], p.qd[0], P.x, u.x, k.ax, k.bx, k.px, k.sx, ok);
  cone_q_axis(p.q0[1], p.qd[1], P.y, u.y, k.ay, k.by, k.py, k.sy, ok);
  cone_q_axis(p.q0[2], p.qd[2], P.z, u.z, k.az, k.bz, k.pz, k.sz, ok);
  k.len = (float)(ldist * (1.0 + 1e-6));
  return k;
}
__device__ __forceinline__ bool cone_node(const uint4 n, const ConeQ& k) {
  const f2 x = __builtin_elementwise_fma(q_near_far(n.x, k.sx), k.ax, k.bx);
  const f2 y = __builtin_elementwise_fma(q_near_far(n.y, k.sy), k.ay, k.by);
  const f2 z = __builtin_elementwise_fma(q_near_far(n.z, k.sz), k.az, k.bz);
  const float lx = fmaxf(x.x, x.y + k.px.x), ly = fmaxf(y.x, y.y + k.py.x), lz = fmaxf(z.x, z.y + k.pz.x);
  const float tn = fmaxf(fmaxf(lx, ly), fmaxf(lz, 0.f));
  const float tf = fminf(fminf(x.y + k.px.y, y.y + k.py.y), fminf(z.y + k.pz.y, k.len));
  return tn <= tf;
}
// A sphere: in_cone's binary64 test (the same margins), NaN kept
__device__ __forceinline__ bool cone_keeps(const DSphere& S, d3 P, d3 u, double ldist) {
  const d3 v = ld3(S.c) - P;
  const double dc2 = len2(v);
  const double dc = (double)__builtin_amdgcn_sqrtf((float)dc2);
  const double ra = fabs(S.r) * (1.0 + 1e-5) + 1e-5 * dc + 1e-12;
  const double tl = (double)__builtin_amdgcn_sqrtf((float)fmax(dc2 - ra * ra, 0.0));
  const bool miss =
      dc > ra && (dc - ra > ldist * (1.0 + 1e-5) + 1e-9 || dot(v, u) < 0.99498 * tl - 0.1 * ra - 1e-5 * dc);
  return !miss;
}

template <bool kCount, bool kFull>
__device__ __forceinline__ void cone_descend(glb_node* __restrict__ qb, lds_node* __restrict__ lt, int nlds,
                                             const ConeQ& k, int& cur, int& sp, int* stack, Counters& c) {
  while ((cur & 7) == 0) {
    uint4 L, R;
    load_pair<kFull>(qb, lt, nlds, cur >> 3, L, R);
    cnt<kCount>(c, C_BOX, 2);
    const bool hl = cone_node(L, k), hr = cone_node(R, k);
    if (hl || hr) {
      if (hl && hr) {
        stack[sp * 64] = (int)R.w;
        ++sp;
      }
      cur = hl ? (int)L.w : (int)R.w;
    } else {
      cur = sp == 0 ? -1 : stack[--sp * 64];
    }
  }
}

// The same walk over the 4-wide tree (descend4's order: the first hit child
// entered, the other hit children pushed)
template <bool kCount>
#ifndef RT_CONE_FRAC
#define RT_CONE_FRAC 4
#endif
__device__ __forceinline__ void cone_descend4(lds_node* __restrict__ lt, const ConeQ& k, int& cur, int& sp, int* stack,
                                              Counters& c) {
  const int entered = RT_CONE_FRAC > 0 ? __popcll(__ballot(true)) : 0;
  while ((cur & 7) == 0) {
    const int base = cur >> 5, nk = ((cur >> 3) & 3) + 1;  // the group's first slot and size (bvh.cpp)
    const uint4 n0 = as_uint4(lt[base]), n1 = as_uint4(lt[base + 1]), n2 = as_uint4(lt[base + 2]),
                n3 = as_uint4(lt[base + 3]);
    cnt<kCount>(c, C_BOX, nk);
    const int cs[4] = {(int)n0.w, (int)n1.w, (int)n2.w, (int)n3.w};
    const bool hs[4] = {cone_node(n0, k), cone_node(n1, k), cone_node(n2, k) && nk > 2, cone_node(n3, k) && nk > 3};
    bool taken = false;
#pragma unroll
    for (int i = 3; i >= 0; --i)
      if (hs[i]) {
        if (taken) stack[sp++ * 64] = cur;
        cur = cs[i];
        taken = true;
      }
    if (!taken) cur = sp == 0 ? -1 : stack[--sp * 64];
    if (RT_CONE_FRAC > 0 && __popcll(__ballot((cur & 7) == 0)) * RT_CONE_FRAC <= entered) break;
  }
}

// lights base + i (i < 32) of a path that are lit (wf_shade1: not within
// 0.001 of the hit point) and whose hard ray is clear; `listed`: those of
// them whose cone left a candidate list
__device__ __forceinline__ uint32_t clear_lights(const WfParams& p, size_t slot, bool hit, int base,
                                                 uint32_t* listed = nullptr, uint32_t* empty = nullptr,
                                                 uint32_t* wide = nullptr) {
  uint32_t own = 0, lst = 0, emp = 0, wid = 0;
  if (hit) {
    const int end = min(p.nl, base + 32);
    for (int li = base; li < end; ++li) {
      const uint32_t ls = p.lstate[slot * p.nl + li];
      if (!(ls & (kHardBit | kUnlitBit))) own |= 1u << (li - base);
      if (ls & kListBit) lst |= 1u << (li - base);
      if (ls & kEmptyBit) emp |= 1u << (li - base);
      if (ls & kWideBit) wid |= 1u << (li - base);
    }
  }
  if (listed) *listed = lst;
  if (empty) *empty = emp;
  if (wide) *wide = wid;
  return own;
}

// One cone job per (path, light) with a clear hard ray, into the workgroup's
// shard of the cone queue.
__global__ __launch_bounds__(kWfBlock) void wf_conegen(const WfParams p) {
  __shared__ int s_wave[kWfBlock / 64];
  __shared__ int s_base;
  const Dense dn = dense(p.ctl->cur_cnt);
  const int n = dn.start[kWfShards];
  if ((int)(blockIdx.x * kWfBlock) >= n) return;
  const int j = blockIdx.x * kWfBlock + threadIdx.x;
  size_t slot = 0;
  bool hit = false;
  if (j < n) {
    slot = dense_at(dn, j, p.shard_cap);
    hit = p.hidx[slot] >= 0;
  }
  const int shard = blockIdx.x % kWfShards;
  uint32_t* cq = p.coneq + (size_t)shard * p.hard_cap;
  for (int base = 0; base < p.nl; base += 32) {
    const uint32_t own = clear_lights(p, slot, hit, base);
    int q = block_append(__popc(own), &p.ctl->cone_cnt[shard * 32], s_wave, &s_base);
    for (uint32_t m = own; m; m &= m - 1) cq[q++] = (uint32_t)(slot * p.nl) + (uint32_t)(base + __builtin_ctz(m));
  }
}

// Persistent cone traversal of the queued cones (the job distribution and
// LDS tree of the occlusion kernels): every sphere of every leaf the cone's
// node tests reach gets cone_keeps; candidates go to the cone's list, up to
// kWfConeK (one more ends the walk: the cone's rays are traced instead).
// The hit sphere itself is left out as in cone_candidates (rt_kernel.hip)
// when the cone leaves its front face at a clear angle.
template <bool kCount, bool kFull, bool kB4>
__device__ __forceinline__ void cone_body(const WfParams& p) {
  const Dense dn = dense(p.ctl->cone_cnt);
  const int n = dn.start[kWfShards];
  if (n == 0) return;
  lds_node* lt = kB4 ? stage_tree4(p) : stage_tree(p);
  JobSrc js = job_src(n);
  bool more = true;  // wave-uniform: jobs may remain
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int lane = threadIdx.x & 63;
  const unsigned long long below = (1ull << lane) - 1ull;
  int* stack = wf_stack(kB4 ? p.stack4 : p.stack_depth);
  bool busy = false;
  uint32_t key = 0;
  d3 P = mk(0, 0, 0), u = mk(0, 0, 0);
  double ldist = 0;
  ConeQ k{};
  int excl = -1, found = 0, cur = -1, sp = 0;
  for (;;) {
    const unsigned long long idle = __ballot(!busy);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull) && js.next >= js.hi)
      more = job_refill(js, p.ctl->job_head[3], n);
    if (more && (__popcll(idle) >= kRefill || idle == ~0ull)) {
      const int j = js.next + __popcll(idle & below), hi = js.hi;
      js.next = min(hi, js.next + __popcll(idle));
      if (!busy && j < hi) {
        key = p.coneq[dense_at(dn, j, p.hard_cap)];
        const uint32_t slot = key / (uint32_t)p.nl, li = key - slot * (uint32_t)p.nl;
        P = ld_P(p, (int)slot);
        light_vec(p.lights[li], P, u, ldist);
        const DSphere& S0 = p.g.spheres[p.hidx[slot]];
        const d3 outward = divs(P - ld3(S0.c), S0.r);
        const bool self_out = dot(ld_d(p.cur, slot), outward) < 0 && dot(outward, u) >= 0.1015;
        excl = self_out ? S0.obj : -1;
        bool ok;
        k = cone_q(p, P, u, ldist, ok);
        // (a cone whose bounds cannot be evaluated is not walked: "too many
        // candidates", so its rays are traced)
        found = ok ? 0 : kWfConeWide + 1;
        cur = ok ? (kB4 ? p.root4 : bvh_code(p.g.bvh[0])) : -1;
        sp = 0;
        busy = true;
      }
    }
    if (__ballot(busy) == 0) {
      if (!more) break;
      continue;
    }
    if (busy) {
      if constexpr (kB4)
        cone_descend4<kCount>(lt, k, cur, sp, stack, c);
      else
        cone_descend<kCount, kFull>((glb_node*)p.qbvh, lt, p.lds_nodes, k, cur, sp, stack, c);
      if (cur != -1 && (cur & 7) != 0) {  // (a leaf; an internal node: the walk paused, cone_descend4)
        const int first = cur >> 3, count = cur & 7;
        DSphere ls[kLeafBatch];
        load_leaf(p.g.spheres, first, count, ls);
        int32_t* cl = p.cand + (size_t)key * kWfConeWide;
        for (int i = first; i < first + count; ++i) {
          const DSphere& S = leaf_sphere(p.g.spheres, ls, first, i);
          if (S.obj == excl && S.r > 0) continue;
          cnt<kCount>(c, C_SPH);
          if (cone_keeps(S, P, u, ldist)) {
            if (found < kWfConeWide) cl[found] = i;
            ++found;
          }
        }
        cur = found > kWfConeWide || sp == 0 ? -1 : stack[--sp * 64];
      }
      if (cur == -1) {  // walked (or too many candidates: the rays are traced)
        busy = false;
        if (found == 0) {
          p.lstate[key] = kListBit | kEmptyBit;
        } else if (found <= kWfConeK) {
          if (found < kWfConeK) p.cand[(size_t)key * kWfConeWide + found] = -1;
          p.lstate[key] = kListBit;
        } else if (found <= kWfConeWide) {
          if (found < kWfConeWide) p.cand[(size_t)key * kWfConeWide + found] = -1;
          p.lstate[key] = kWideBit;
        }
      }
    }
  }
  flush_counts<kCount>(p, c, kGroupSoft);
}
template <bool kCount, bool kFull>
__global__ RT_TRAV_ATTR void wf_cone(const WfParams p) {
  cone_body<kCount, kFull, false>(p);
}
template <bool kCount>  // over the 4-wide tree (WfParams.use4)
__global__ RT_TRAV_ATTR void wf_cone4(const WfParams p) {
  cone_body<kCount, true, true>(p);
}

// The image pixel (y W + x) and sample index of sample id `sid` (wf_regen's
// mapping): the key of its soft-shadow streams (spec v4, include/rt_rng.h)
__device__ __forceinline__ uint64_t sid_soft_key(const WfParams& p, uint32_t sid) {
  const uint32_t q = sid / (uint32_t)p.spp;
  const uint32_t lp = p.lp0 + q;
  const uint32_t smp = sid - q * (uint32_t)p.spp;
  const int lt = (int)(lp >> 10), tp = (int)(lp & 1023);
  const int tile = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
  const int x = (tile % p.tiles_x) * 32 + (tp & 31), y = (tile / p.tiles_x) * 32 + (tp >> 5);
  return rt_soft_key(p.seed_key, (uint32_t)y * (uint32_t)p.W + (uint32_t)x, smp);
}

// ---------------------------------------------------------------- softgen
// For every light whose hard ray is clear, in light order: a cone with more
// than kWfConeK candidates gets the 16 points of calculateSmartShadow's soft
// rays from its stream (rejection sampling, vector.go:132-139) as 16
// consecutive soft-queue entries, traced by wf_occlude<soft>; a listed cone
// (wf_cone) gets two entries, its stream state and accepted tries, from the
// far end of the shard's queue (list_cnt counts them), and wf_listtest
// rebuilds its points; an empty cone gets nothing (its rays cannot be
// blocked).
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_softgen(const WfParams p) {
  __shared__ int s_wave[kWfBlock / 64];
  __shared__ int s_base;
  __shared__ uint32_t s_slot[kWfBlock], s_own[kWfBlock], s_list[kWfBlock], s_empty[kWfBlock], s_wide[kWfBlock];
  const Dense dn = dense(p.ctl->cur_cnt);
  const int n = dn.start[kWfShards];
  if ((int)(blockIdx.x * kWfBlock) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int j = blockIdx.x * kWfBlock + threadIdx.x;
  size_t slot = 0;
  bool hit = false;
  if (j < n) {
    slot = dense_at(dn, j, p.shard_cap);
    hit = p.hidx[slot] >= 0;
  }
  const int shard = blockIdx.x % kWfShards;
  // the 16 points of each light of `own`: traced rays at entries q.. of the
  // shard's queue, a listed light's two entries ending before soft_cap - ql
  // (ql += 2).  Each light's points come from its own stream
  // (spec v4: (sample, depth, light), include/rt_rng.h); an empty cone's rays
  // cannot be blocked and need none, so nothing is drawn for it (the
  // counting variant walks its tries for the reference's draw count).
  auto gen = [&](size_t sl, uint32_t own, uint32_t listed, uint32_t empty, uint32_t wide, int base, int q, int ql,
                 int qw) {
    uint4* sq = reinterpret_cast<uint4*>(p.softq) + (size_t)shard * p.soft_cap;
    const uint64_t skey = sid_soft_key(p, p.cur.sid[sl]);
    const uint32_t depth = (uint32_t)p.cur.depth[sl];
    for (uint32_t m = own; m; m &= m - 1) {
      const int li = base + __builtin_ctz(m);
      const uint32_t key = (uint32_t)(sl * p.nl) + (uint32_t)li;
      const uint32_t bit = m & (0u - m);
      cnt<kCount>(c, C_SHADOW, 16);
      const bool keep = !(empty & bit);
      if (!keep && !kCount) continue;
      // (r05) a listed cone gets two entries at the far end: its stream state
      // and which of its first 64 tries were accepted; wf_listtest rebuilds
      // the points from them through the jump table.  (Both kinds run the one
      // rejection loop below: separate loops for listed and traced cones
      // diverged, 20.5 -> 25.2 ms per C4 frame.)
      // (a wide cone's two entries, the same, go to the wide queue: wf_widetest)
      const bool lst = keep && (listed & bit), wid = keep && (wide & bit), two = lst || wid;
      size_t at = 0;  // (an index, not a bumped pointer)
      if (keep && !two) {
        at = (size_t)q;
        q += 16;
      }
      rt_rng rng{rt_soft_state(skey, depth, (uint32_t)li)};
      const uint64_t x0 = rng.x;
      uint64_t mask = 0;
      for (int k = 0, t = 0; k < 16; ++t) {
        const uint32_t ux = rt_rng_next(&rng), uy = rt_rng_next(&rng), uz = rt_rng_next(&rng);
        if (!two || t < p.list_tries) cnt<kCount>(c, C_RNG, 3);  // (a listed cone's later tries: wf_listtest)
        const bool acc = unit_ball_accept(ux, uy, uz);
        if (acc && keep && !two) sq[at + k] = make_uint4(key, ux, uy, uz);
        mask |= acc && t < p.list_tries ? 1ull << (t & 63) : 0ull;
        k += acc ? 1 : 0;
      }
      if (two) {
        uint4* le = lst ? sq + (p.soft_cap - ql - 2)
                        : reinterpret_cast<uint4*>(p.wideq) + (size_t)shard * p.wide_cap + qw;
        le[0] = make_uint4(key, (uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)mask);
        le[1] = make_uint4((uint32_t)(mask >> 32), 0u, 0u, 0u);
        if (lst)
          ql += 2;
        else
          qw += 2;
      }
    }
  };
  if (p.nl <= 32) {
    // Most paths have no clear light (C4: 12 % of hard rays are clear): the
    // paths that have one are gathered to the workgroup's first lanes, so
    // the rejection sampling runs on full waves and the other waves of the
    // workgroup skip it (one path per lane either way: same draws, same order)
    uint32_t listed, empty, wide;
    const uint32_t own = clear_lights(p, slot, hit, 0, &listed, &empty, &wide);
    int total;
    const int at = block_prefix(own != 0 ? 1 : 0, s_wave, total);
    if (own) {
      s_slot[at] = (uint32_t)slot;
      s_own[at] = own;
      s_list[at] = listed;
      s_empty[at] = empty;
      s_wide[at] = wide;
    }
    __syncthreads();
    const bool work = (int)threadIdx.x < total;
    const uint32_t ws = work ? s_slot[threadIdx.x] : 0u, wo = work ? s_own[threadIdx.x] : 0u;
    const uint32_t wl = work ? s_list[threadIdx.x] : 0u, we = work ? s_empty[threadIdx.x] : 0u;
    const uint32_t ww = work ? s_wide[threadIdx.x] : 0u;
    const int q = block_append(16 * __popc(wo & ~wl & ~ww), &p.ctl->soft_cnt[shard * 32], s_wave, &s_base);
    const int ql = block_append(2 * __popc(wl & ~we), &p.ctl->list_cnt[shard * 32], s_wave, &s_base);
    const int qw = block_append(2 * __popc(ww), &p.ctl->wide_cnt[shard * 32], s_wave, &s_base);
    if (work) gen(ws, wo, wl, we, ww, 0, q, ql, qw);
    flush_counts<kCount>(p, c);
    return;
  }
  // more than 32 lights: in chunks of 32 (one bit each), in light order
  for (int base = 0; base < p.nl; base += 32) {
    uint32_t listed, empty, wide;
    const uint32_t own = clear_lights(p, slot, hit, base, &listed, &empty, &wide);
    const int q = block_append(16 * __popc(own & ~listed & ~wide), &p.ctl->soft_cnt[shard * 32], s_wave, &s_base);
    const int ql = block_append(2 * __popc(listed & ~empty), &p.ctl->list_cnt[shard * 32], s_wave, &s_base);
    const int qw = block_append(2 * __popc(wide), &p.ctl->wide_cnt[shard * 32], s_wave, &s_base);
    if (own) gen(slot, own, listed, empty, wide, base, q, ql, qw);
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- listtest
// The 16 soft rays of a listed cone against its candidates, one cone per
// thread: the ray (normalize(lightDir + 0.1 p), wf_occlude<soft>'s), the
// range [0.001, distance) and the Sphere.Hit test of the traversal, so the
// blocked count is the one the traversal would find.  Candidates four at a
// time (their loads together, then every ray still clear against them).
// (One ray per thread, the cone's 16 lanes sharing its loads and a ballot
// for the count: 41 vs 31 ms per C4 frame; rays outer, each entry read once
// and the candidates re-read from L2 per ray: 51 vs 31 ms.)
// the two entries of listed cone j at the far end of its shard (wf_softgen):
// {key, stream state lo, hi, accepted-try mask lo}, {mask hi, 0, 0, 0}
__device__ __forceinline__ const uint4* list_entry(const WfParams& p, const Dense& dn, int j) {
  const size_t at = dense_at(dn, 2 * j, p.soft_cap);
  const size_t sh = at / (size_t)p.soft_cap, off = at - sh * (size_t)p.soft_cap;
  return reinterpret_cast<const uint4*>(p.softq) + sh * (size_t)p.soft_cap + (p.soft_cap - off - 2);
}
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_listtest(const WfParams p) {
  const Dense dn = dense(p.ctl->list_cnt);  // (two entries per cone, in one shard)
  const int n = dn.start[kWfShards] / 2;
  if ((int)(blockIdx.x * kWfBlock) >= n) return;
  int j = blockIdx.x * kWfBlock + threadIdx.x;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  // the workgroup's cones ordered by their candidate groups of four (1..4),
  // so a wave's lanes loop over about as many groups each (a wave waits
  // for its longest list)
  {
    __shared__ int s_bucket[4], s_order[kWfBlock];
    if (threadIdx.x < 4) s_bucket[threadIdx.x] = 0;
    __syncthreads();
    int b = 0;
    if (j < n) {
      const uint32_t key = list_entry(p, dn, j)->x;
      // groups of four up to the one holding the list's end (-1; entries
      // past it are stale): bucket 1, 2, 3-4, 5+ groups
      const int4* cl = reinterpret_cast<const int4*>(p.cand + (size_t)key * kWfConeWide);
      int g = 1;
      while (g < kWfConeK / 4 && (cl[g - 1].x | cl[g - 1].y | cl[g - 1].z | cl[g - 1].w) >= 0) ++g;
      b = g == 1 ? 0 : (g == 2 ? 1 : (g <= 4 ? 2 : 3));
    }
    const int pos = atomicAdd(&s_bucket[b], 1);
    __syncthreads();
    int base = 0;
    for (int k = 0; k < b; ++k) base += s_bucket[k];
    s_order[base + pos] = j;
    __syncthreads();
    j = s_order[threadIdx.x];
  }
  if (j < n) {
    // (r05) the cone's 16 points, rebuilt from its stream state and the
    // tries wf_softgen accepted: try t's draws are 3t..3t+2 (the jump table
    // gives the state before draw 3t), so no rejection loop runs here; the
    // queue carries 32 B per cone instead of the 16 points' 256 B.  (If the
    // 16th point needs more than p.list_tries (64) tries, about once in 10^6
    // cones, the rest come from the sequential loop from that try; the GPU
    // tests force the limit low to exercise it.)  Kept in registers for
    // every candidate group.
    const uint4* e = list_entry(p, dn, j);
    const uint4 e0 = e[0];
    const uint32_t key = e0.x;
    const uint64_t x0 = (uint64_t)e0.y | (uint64_t)e0.z << 32;
    uint64_t mask = (uint64_t)e0.w | (uint64_t)e[1].x << 32;
    uint32_t ux[16], uy[16], uz[16];
    {
      uint64_t xt = 0;
      bool tail = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (mask != 0) {
          const int t = __builtin_ctzll(mask);
          mask &= mask - 1;
          const uint64_t s0 = state_at3(x0, p.jump, t), s1 = s0 * RT_PCG_MULT + RT_PCG_INC,
                         s2 = s1 * RT_PCG_MULT + RT_PCG_INC;
          ux[r] = rt_pcg_out(s0);
          uy[r] = rt_pcg_out(s1);
          uz[r] = rt_pcg_out(s2);
        } else {
          if (!tail) {
            xt = state_at3(x0, p.jump, p.list_tries);
            tail = true;
          }
          rt_rng rng{xt};
          for (;;) {
            const uint32_t a = rt_rng_next(&rng), b = rt_rng_next(&rng), z = rt_rng_next(&rng);
            cnt<kCount>(c, C_RNG, 3);
            if (unit_ball_accept(a, b, z)) {
              ux[r] = a;
              uy[r] = b;
              uz[r] = z;
              break;
            }
          }
          xt = rng.x;
        }
      }
    }
    const uint32_t slot = key / (uint32_t)p.nl, li = key - slot * (uint32_t)p.nl;
    const d3 o = ld_P(p, (int)slot);
    d3 ldir;
    double tmax;
    light_vec(p.lights[li], o, ldir, tmax);
    const int32_t* cl = p.cand + (size_t)key * kWfConeWide;
    uint32_t blocked = 0;  // one bit per ray
    for (int g = 0; g < kWfConeK; g += 4) {
      const int4 q4 = *reinterpret_cast<const int4*>(cl + g);
      const int id[4] = {q4.x, q4.y, q4.z, q4.w};
      bool valid[4];
      DSphere ls[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        valid[k] = id[k] >= 0 && (k == 0 || valid[k - 1]);
        ls[k] = p.g.spheres[valid[k] ? id[k] : 0];
      }
      if (!valid[0]) break;
#pragma unroll 1
      for (int r = 0; r < 16; ++r) {
        if (blocked & (1u << r)) continue;
        // (a wave-uniform index: v_movrels, no scratch)
        const d3 pt = mk(rt_bits_to_unit(ux[r]) * 2 - 1, rt_bits_to_unit(uy[r]) * 2 - 1, rt_bits_to_unit(uz[r]) * 2 - 1);
        const d3 d = normalize(ldir + muls(pt, 0.1));
        const double av = len2(d), inv_a = approx_rcp(av);
        bool b = false;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (valid[k] && !b) {
            cnt<kCount>(c, C_SPH);
            double num;
            b = sphere_query(ls[k], o, d, av, inv_a, 0.001, tmax, num) != 0;
          }
        blocked |= b ? 1u << r : 0u;
      }
      if (!valid[3]) break;
    }
    p.lstate[key] = (uint32_t)__popc(blocked);
  }
  flush_counts<kCount>(p, c, kGroupSoft);
}

// ---------------------------------------------------------------- widetest
// (r05) The 16 soft rays of a wide cone (kWfConeK < candidates <=
// kWfConeWide) against its list, one ray per lane: 16 lanes per cone, four
// cones per wave, each lane looping over the cone's candidates (the same
// sphere for the 16 lanes: one broadcast load) with the traversal's ray,
// range and Sphere.Hit test, so the blocked count is the traversal's.  Such
// a cone's rays were traced through the BVH before (wf_occlude<soft>, in
// the densest parts of the scene).  Lane r rebuilds point r from the cone's
// stream state and accepted-try mask (wf_softgen), as wf_listtest does; a
// point past the mask continues the sequential loop.  Persistent: the grid
// loops over the cones.
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_widetest(const WfParams p) {
  const Dense dn = dense(p.ctl->wide_cnt);  // (two entries per cone, in one shard)
  const int n = dn.start[kWfShards] / 2;
  if ((int)(blockIdx.x * (kWfBlock / 16)) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int lane = (int)(threadIdx.x & 63), r = lane & 15;
  const int groups = (int)gridDim.x * (kWfBlock / 16);
  for (int j = (int)(blockIdx.x * (kWfBlock / 16) + threadIdx.x / 16); j < n; j += groups) {
    const size_t at = dense_at(dn, 2 * j, p.wide_cap);
    const uint4* e = reinterpret_cast<const uint4*>(p.wideq) + at;
    const uint4 e0 = e[0];
    const uint32_t key = e0.x;
    const uint64_t x0 = (uint64_t)e0.y | (uint64_t)e0.z << 32;
    const uint64_t mask = (uint64_t)e0.w | (uint64_t)e[1].x << 32;
    uint32_t ux = 0, uy = 0, uz = 0;
    const int na = __popcll(mask);
    if (r < na) {  // the r-th accepted try among the mask's
      uint64_t m = mask;
      for (int i = 0; i < r; ++i) m &= m - 1;
      const uint64_t s0 = state_at3(x0, p.jump, __builtin_ctzll(m)), s1 = s0 * RT_PCG_MULT + RT_PCG_INC,
                     s2 = s1 * RT_PCG_MULT + RT_PCG_INC;
      ux = rt_pcg_out(s0);
      uy = rt_pcg_out(s1);
      uz = rt_pcg_out(s2);
    } else {  // past the mask: the sequential loop from try p.list_tries (lane 15 counts its draws)
      rt_rng rng{state_at3(x0, p.jump, p.list_tries)};
      for (int k = na;;) {
        const uint32_t a = rt_rng_next(&rng), b = rt_rng_next(&rng), z = rt_rng_next(&rng);
        if (r == 15) cnt<kCount>(c, C_RNG, 3);
        if (unit_ball_accept(a, b, z)) {
          if (k == r) {
            ux = a;
            uy = b;
            uz = z;
            break;
          }
          ++k;
        }
      }
    }
    const uint32_t slot = key / (uint32_t)p.nl, li = key - slot * (uint32_t)p.nl;
    const d3 o = ld_P(p, (int)slot);
    d3 ldir;
    double tmax;
    light_vec(p.lights[li], o, ldir, tmax);
    const d3 pt = mk(rt_bits_to_unit(ux) * 2 - 1, rt_bits_to_unit(uy) * 2 - 1, rt_bits_to_unit(uz) * 2 - 1);
    const d3 d = normalize(ldir + muls(pt, 0.1));
    const double av = len2(d), inv_a = approx_rcp(av);
    const int32_t* cl = p.cand + (size_t)key * kWfConeWide;
    bool blocked = false;
    // candidates four at a time: their ids and spheres loaded together (the
    // same for the cone's 16 lanes), then tested in list order
    for (int g = 0; g < kWfConeWide; g += 4) {
      const int4 q4 = *reinterpret_cast<const int4*>(cl + g);
      const int id[4] = {q4.x, q4.y, q4.z, q4.w};
      bool valid[4];
      DSphere ls[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        valid[k] = id[k] >= 0 && (k == 0 || valid[k - 1]);
        ls[k] = p.g.spheres[valid[k] ? id[k] : 0];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (valid[k] && !blocked) {
          cnt<kCount>(c, C_SPH);
          double num;
          blocked = sphere_query(ls[k], o, d, av, inv_a, 0.001, tmax, num) != 0;
        }
      if (!valid[3]) break;
#if RT_WIDE_EXIT
      if (((__ballot(blocked) >> (lane & 48)) & 0xFFFFull) == 0xFFFFull) break;  // all 16 blocked
#endif
    }
    const unsigned long long bm = __ballot(blocked);
    if (r == 0) p.lstate[key] = (uint32_t)__popcll((bm >> (lane & 48)) & 0xFFFFull);
  }
  flush_counts<kCount>(p, c, kGroupSoft);
}

// ---------------------------------------------------------------- shade
// calculateDirectLighting (renderer.go:229-297) with the shadow results,
// Material.Scatter and the traceRay combination (renderer.go:181-226).
// Finished paths write their sample's radiance; survivors are appended to the
// workgroup's shard of the next path array.
template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_shade(const WfParams p) {
  __shared__ int s_wave[kWfBlock / 64];
  __shared__ int s_base;
  const Dense dn = dense(p.ctl->cur_cnt);
  const int n = dn.start[kWfShards];
  if ((int)(blockIdx.x * kWfBlock) >= n) return;
  Counters c;
  if constexpr (kCount)
    for (int k = 0; k < 9; ++k) c.v[k] = 0;
  const int j = blockIdx.x * kWfBlock + threadIdx.x;
  bool cont = false;
  d3 P = mk(0, 0, 0), nd = mk(0, 0, 0), T = mk(0, 0, 0), L = mk(0, 0, 0);
  rt_rng rng{0};
  uint32_t sid = 0;
  int depth = 0;
  if (j < n) {
    const size_t slot = dense_at(dn, j, p.shard_cap);
    if (p.hidx[slot] >= 0) {
      const WfPaths& a = p.cur;
      P = mk(p.px[slot], p.py[slot], p.pz[slot]);
      const d3 d = ld_d(a, slot);
      // HitRecord (sphere.go:42-58): the outward normal at P, flipped to face the ray
      const DSphere& S0 = p.g.spheres[p.hidx[slot]];
      const d3 outward = divs(P - ld3(S0.c), S0.r);
      const bool front = dot(d, outward) < 0;
      const d3 N = front ? outward : neg(outward);
      const DMat* __restrict__ m = p.mats + S0.mat;
      T = mk(a.tx[slot], a.ty[slot], a.tz[slot]);
      L = mk(a.lx[slot], a.ly[slot], a.lz[slot]);
      rng.x = a.rng[slot];
      sid = a.sid[slot];
      depth = a.depth[slot];
      d3 D = mk(m->ambient, m->ambient, m->ambient);
      for (int li = 0; li < p.nl; ++li) {
        const DLight& Lt = p.lights[li];
        d3 ldir;
        double ldist;
        light_vec(Lt, P, ldir, ldist);
        if (!(ldist < 0.001)) {
          const uint32_t ls = p.lstate[slot * p.nl + li];
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
              const int spw = m->spec_pow;
              double si = spw == 64 ? pow_n<64>(hc) : (spw == 48 ? pow_n<48>(hc) : pow_n<32>(hc));
              D = D + muls(ld3(Lt.color), si * intensity * sf * metallic * 3.0);
            }
          }
        }
      }
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
  }
  const int shard = blockIdx.x % kWfShards;
  const int q = block_append(cont ? 1 : 0, &p.ctl->next_cnt[shard * 32], s_wave, &s_base);
  if (cont) store_path(p.next, (size_t)shard * p.shard_cap + q, P, nd, T, L, rng.x, sid, depth);
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- regen
// New samples for the free slots of the next array: shard s takes the
// samples [next + free_0 + .. + free_{s-1}, ...) into its slots after its
// survivors, in order (a pixel's samples are consecutive, so neighbouring
// lanes trace neighbouring camera rays).  Out-of-image pixels of edge tiles
// become dead slots (kDeadSid).  Deterministic: no atomics.
struct RegenPlan {
  long long first[kWfShards];  // first new sample of shard s
  int take[kWfShards];         // new samples of shard s
  long long taken;             // all shards
};
__device__ __forceinline__ RegenPlan regen_plan(const WfCtl* ctl, int shard_cap) {
  RegenPlan r;
  long long pos = (long long)ctl->next_sample;
  const long long total = (long long)ctl->total;
#pragma unroll
  for (int s = 0; s < kWfShards; ++s) {
    const long long fr = shard_cap - ctl->next_cnt[s * 32];
    const long long t = min(fr, max(0ll, total - pos));
    r.first[s] = pos;
    r.take[s] = (int)t;
    pos += t;
  }
  r.taken = pos - (long long)ctl->next_sample;
  return r;
}

template <bool kCount>
__global__ __launch_bounds__(kWfBlock) void wf_regen(const WfParams p) {
  const int t = blockIdx.x * kWfBlock + threadIdx.x;  // over kWfShards * shard_cap slots
  const int s = min(t / p.shard_cap, kWfShards - 1), local = t - s * p.shard_cap;
  const int have = p.ctl->next_cnt[s * 32];
  Counters c;
  if constexpr (kCount)
    for (int i = 0; i < 9; ++i) c.v[i] = 0;
  if (local >= have && local < p.shard_cap) {
    const RegenPlan rp = regen_plan(p.ctl, p.shard_cap);
    int take = 0;
    long long first = 0;
#pragma unroll
    for (int k = 0; k < kWfShards; ++k)
      if (k == s) {
        take = rp.take[k];
        first = rp.first[k];
      }
    const int k = local - have;
    if (k < take) {
      const uint32_t sid = (uint32_t)(first + k);
      const uint32_t q = sid / (uint32_t)p.spp;
      const uint32_t lp = p.lp0 + q;
      const int smp = (int)(sid - q * (uint32_t)p.spp);
      const int lt = (int)(lp >> 10), tp = (int)(lp & 1023);
      const int tile = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
      const int x = (tile % p.tiles_x) * 32 + (tp & 31), y = (tile / p.tiles_x) * 32 + (tp >> 5);
      const size_t slot = (size_t)s * p.shard_cap + local;
      if (tile >= p.ntiles || x >= p.W || y >= p.H) {
        p.next.sid[slot] = kDeadSid;
      } else {
        cnt<kCount>(c, C_CAM);
        const CamK ck = make_cam(p.seed_key, p.W, p.H, p.aspect, p.cam[0], p.cam[1], p.cam[2]);
        rt_rng rng;
        d3 o, d;
        camera_ray_c<kCount>(ck, x, y, smp, rng, o, d, c);
        store_path(p.next, slot, o, d, mk(1, 1, 1), mk(0, 0, 0), rng.x, sid, 0);
      }
    }
  }
  flush_counts<kCount>(p, c);
}

// ---------------------------------------------------------------- book
// The next array becomes current; queues reset; the loop state for the host.
__global__ void wf_book(const WfParams p) {
  if (threadIdx.x != 0) return;
  WfCtl* ctl = p.ctl;
  const RegenPlan rp = regen_plan(ctl, p.shard_cap);
  int live = 0;
#pragma unroll
  for (int s = 0; s < kWfShards; ++s) {
    const int nc = ctl->next_cnt[s * 32] + rp.take[s];
    ctl->cur_cnt[s * 32] = nc;
    ctl->next_cnt[s * 32] = 0;
    ctl->hard_cnt[s * 32] = 0;
    ctl->soft_cnt[s * 32] = 0;
    ctl->cone_cnt[s * 32] = 0;
    ctl->list_cnt[s * 32] = 0;
    ctl->wide_cnt[s * 32] = 0;
    ctl->job_head[3][s * 32] = 0;
    ctl->job_head[0][s * 32] = 0;
    ctl->job_head[1][s * 32] = 0;
    ctl->job_head[2][s * 32] = 0;
    live += nc;
  }
  ctl->next_sample += rp.taken;
  ctl->live = live;
  ctl->dry = ctl->next_sample >= ctl->total ? 1 : 0;
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
  const int tile = p.tile_list ? p.tile_list[lt] : p.rank + lt * p.world;
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
// persistent kernels: as many workgroups as fit on the device at once
template <typename K>
static int resident_grid(K kernel, int block, size_t shmem) {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
  // (the attribute is a permission: set to the whole LDS once, it never has
  // to change, so renderers of other scene shapes on the same device cannot
  // lower it under a launch of this one)
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            kLdsBytes);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, shmem) != hipSuccess || per < 1) per = 1;
  return cus * per;
}

static size_t trav_shmem(const WfParams& p) {
  return (size_t)p.trav_block * p.stack_depth * sizeof(int) + (size_t)p.lds_nodes * sizeof(uint4);
}

int wf_lds_nodes(int stack_depth, int nodes, int block, int wgs_per_cu) {
  const long long room =
      ((long long)kLdsBytes / std::max(1, wgs_per_cu) - (long long)block * stack_depth * (long long)sizeof(int)) /
      (long long)sizeof(uint4);
  if (room >= nodes) return nodes;
  if (room < 1) return 0;
  return (int)(room % 2 ? room : room - 1);
}

// (prof: events recorded at the kernel boundaries of a profiled context,
// rt_context_profile; ev[k] opens kernel class k, ev[k + 1] closes it)
static inline void mark(const hipEvent_t* ev, int k, hipStream_t st) {
  if (ev) (void)hipEventRecord(ev[k], st);
}

template <bool kCount>
static int enqueue_regen_book(const WfParams& p, hipStream_t st, const hipEvent_t* ev) {
  const int slots = kWfShards * p.shard_cap;
  // (once every sample has started, regen has nothing to do)
  if (!p.dry) hipLaunchKernelGGL((wf_regen<kCount>), dim3((slots + kWfBlock - 1) / kWfBlock), dim3(kWfBlock), 0, st, p);
  hipLaunchKernelGGL(wf_book, dim3(1), dim3(64), 0, st, p);
  mark(ev, kWfRegen + 1, st);
  return (int)hipGetLastError();
}

// the traversal kernels of one bounce: closest hit, hard and soft occlusion
template <bool kCount, bool kFull>
static void enqueue_trav(const WfParams& p, hipStream_t st, int which) {
  const dim3 bt(p.trav_block);
  const size_t sh = trav_shmem(p);
  // resident grids per (device, LDS bytes, workgroup size): an rt_renderer
  // drives its devices from one thread each (rt_multi.cpp), and contexts of
  // different scenes may share a device
  struct Grids {
    int ext = 0, occ_h = 0, occ_s = 0, cone = 0;
  };
  if (p.use4 && which != 0) {  // occlusion and cone walks over the 4-wide tree
    const size_t sh4 = (size_t)p.trav_block * p.stack4 * sizeof(int) + (size_t)p.nodes4 * sizeof(uint4);
    static std::mutex mu4;
    static std::map<std::tuple<int, size_t, int>, Grids> cache4;
    int dev = 0;
    (void)hipGetDevice(&dev);
    Grids g;
    {
      std::lock_guard<std::mutex> lock(mu4);
      const auto key = std::make_tuple(dev, sh4, p.trav_block);
      auto it = cache4.find(key);
      if (it == cache4.end()) {
        Grids c;
        c.occ_h = resident_grid(wf_occlude4<kCount, false>, p.trav_block, sh4);
        c.occ_s = resident_grid(wf_occlude4<kCount, true>, p.trav_block, sh4);
        c.cone = resident_grid(wf_cone4<kCount>, p.trav_block, sh4);
        it = cache4.emplace(key, c).first;
      }
      g = it->second;
    }
    if (which == 1) hipLaunchKernelGGL((wf_occlude4<kCount, false>), dim3(g.occ_h), bt, sh4, st, p);
    if (which == 2) hipLaunchKernelGGL((wf_occlude4<kCount, true>), dim3(g.occ_s), bt, sh4, st, p);
    if (which == 3) hipLaunchKernelGGL((wf_cone4<kCount>), dim3(g.cone), bt, sh4, st, p);
    return;
  }
  static std::mutex mu;
  static std::map<std::tuple<int, size_t, int>, Grids> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  Grids g;
  {
    std::lock_guard<std::mutex> lock(mu);
    const auto key = std::make_tuple(dev, sh, p.trav_block);
    auto it = cache.find(key);
    if (it == cache.end()) {
      Grids c;
      c.ext = resident_grid(wf_extend<kCount, kFull>, p.trav_block, sh);
      c.occ_h = resident_grid(wf_occlude<kCount, false, kFull>, p.trav_block, sh);
      c.occ_s = resident_grid(wf_occlude<kCount, true, kFull>, p.trav_block, sh);
      c.cone = resident_grid(wf_cone<kCount, kFull>, p.trav_block, sh);
      it = cache.emplace(key, c).first;
    }
    g = it->second;
  }
  if (which == 0) hipLaunchKernelGGL((wf_extend<kCount, kFull>), dim3(g.ext), bt, sh, st, p);
  if (which == 1) hipLaunchKernelGGL((wf_occlude<kCount, false, kFull>), dim3(g.occ_h), bt, sh, st, p);
  if (which == 2) hipLaunchKernelGGL((wf_occlude<kCount, true, kFull>), dim3(g.occ_s), bt, sh, st, p);
  if (which == 3) hipLaunchKernelGGL((wf_cone<kCount, kFull>), dim3(g.cone), bt, sh, st, p);
}

template <bool kCount>
static int enqueue_bounce(const WfParams& p, hipStream_t st, const hipEvent_t* ev) {
  const dim3 b(kWfBlock);
  // dense kernels: one thread per live path, at most one per slot; while the
  // last paths drain, the host's bound keeps tens of thousands of empty
  // workgroups out of each launch
  const long long live = std::min<long long>((long long)kWfShards * p.shard_cap, std::max(p.live_bound, 1));
  const dim3 gd((unsigned)((live + kWfBlock - 1) / kWfBlock));
  const bool full = p.lds_nodes >= p.bvh_nodes;
  auto trav = [&](int which) {
    if (full)
      enqueue_trav<kCount, true>(p, st, which);
    else
      enqueue_trav<kCount, false>(p, st, which);
  };
  mark(ev, kWfExtend, st);
  trav(0);
  mark(ev, kWfShade1, st);
  hipLaunchKernelGGL((wf_shade1<kCount>), gd, b, 0, st, p);
  mark(ev, kWfHard, st);
  if (p.nl > 0) trav(1);
  mark(ev, kWfCone, st);
  if (p.nl > 0 && p.soft) {
    hipLaunchKernelGGL(wf_conegen, gd, b, 0, st, p);
    trav(3);
  }
  mark(ev, kWfSoftgen, st);
  if (p.nl > 0 && p.soft) hipLaunchKernelGGL((wf_softgen<kCount>), gd, b, 0, st, p);
  mark(ev, kWfList, st);
  if (p.nl > 0 && p.soft) {  // (at most one listed cone per path and light)
    const long long cones = live * p.nl;
    hipLaunchKernelGGL((wf_listtest<kCount>), dim3((unsigned)((cones + kWfBlock - 1) / kWfBlock)), b, 0, st, p);
    // wide cones: a persistent grid (16 lanes per cone; far fewer cones)
    const long long wblocks = std::min<long long>((cones + kWfBlock / 16 - 1) / (kWfBlock / 16), 4096);
    hipLaunchKernelGGL((wf_widetest<kCount>), dim3((unsigned)wblocks), b, 0, st, p);
  }
  mark(ev, kWfSoft, st);
  if (p.nl > 0 && p.soft) trav(2);
  mark(ev, kWfShade, st);
  hipLaunchKernelGGL((wf_shade<kCount>), gd, b, 0, st, p);
  mark(ev, kWfRegen, st);
  return enqueue_regen_book<kCount>(p, st, ev);
}

// first == true: the arrays are empty; only regen + book (the first samples)
int wf_launch_bounce(const WfParams& p, bool first, bool count, void* stream, const void* prof) {
  hipStream_t st = (hipStream_t)stream;
  const hipEvent_t* ev = (const hipEvent_t*)prof;
  if (first) {
    mark(ev, kWfRegen, st);
    return count ? enqueue_regen_book<true>(p, st, ev) : enqueue_regen_book<false>(p, st, ev);
  }
  return count ? enqueue_bounce<true>(p, st, ev) : enqueue_bounce<false>(p, st, ev);
}

// (see preload_render_kernels)
int preload_wf_kernels() {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(wf_book));
}

int wf_launch_resolve(const WfParams& p, int npix, void* stream) {
  if (npix <= 0) return hipSuccess;
  hipLaunchKernelGGL(wf_resolve, dim3((npix + kWfBlock - 1) / kWfBlock), dim3(kWfBlock), 0, (hipStream_t)stream, p,
                     npix);
  return (int)hipGetLastError();
}


// Cross-lane reads from inactive lanes counted by this file's kernels in an
// RT_CHECK_XLANE build (rt_device.h); -1 in a normal build.  reset: zero it.
long long xlane_faults_wavefront(bool reset) {
#ifdef RT_CHECK_XLANE
  unsigned long long v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_xlane_faults), sizeof v) != hipSuccess) return -2;
  if (reset) {
    const unsigned long long z = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_xlane_faults), &z, sizeof z) != hipSuccess) return -2;
  }
  return (long long)v;
#else
  (void)reset;
  return -1;
#endif
}

}  // namespace rtgo
