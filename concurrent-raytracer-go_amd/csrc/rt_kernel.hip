// rt_kernel.hip — gfx950 (CDNA4) kernels of the renderer core.
//
// One launch renders every 32x32 tile (createRenderTasks,
// internal/renderer/renderer.go:398-436) that this rank owns.  Design
// (DESIGN.md §4):
//   the host cuts this rank's tiles into work BLOCKS (pixels of one tile x
//     a range of their samples, schedule.cpp), sized and ordered heaviest
//     first from a one-sample pilot render; one one-wave workgroup renders
//     one block;
//   a block runs in three phases (render_kernel below): every camera sample
//     of the block's live pixels gets its closest hit (misses end at once);
//     the hit samples form a list that the wave drains through a ring of LDS
//     radiance slots, a lane without a path taking the next entry, so
//     traceRay (renderer.go:165-227, unrolled) runs on dense waves even when
//     almost every camera ray misses; finished entries are summed per pixel
//     in sample order (tracePixel, renderer.go:150-163), divided by spp,
//     tone-mapped (toneMap, renderer.go:348-367) and written once (float3
//     linear radiance + RGBA8);
//   per bounce and light, the 16 jittered shadow rays (calculateSmartShadow,
//     renderer.go:299-331) are produced in a wave-converged section: rays of
//     many owner lanes go through an LDS queue and are traced on full waves
//     (soft_queue); when only a few lanes need them, all 64 lanes evaluate
//     one owner's rejection tries in parallel (PCG jump-ahead,
//     include/rt_rng.h, soft_coop) -- same draws, same rays, same result as
//     the sequential loop; when few lanes still run paths, the idle lanes
//     split the closest-hit and cone scans of the others (wide mode).
// Large sphere scenes (a BVH) take the wavefront path instead
// (rt_wavefront.hip) unless rt_tuning.path asks for the megakernel.
// Small linear-scan scenes are staged into LDS by every workgroup; large
// sphere scenes use a BVH (bvh.cpp) with per-lane LDS stacks.  Primitives
// that provably cannot be hit (tile frustum / shadow cone tests with wide
// margins) are skipped; everything else gets the reference's exact test.
// All path arithmetic is binary64 in the reference's order, compiled with
// -ffp-contract=off, so every decision (hit / miss, root choice, rejection
// test, reflect vs refract) is bit-identical to the oracle's.  Divisions that
// only feed range tests are filtered by a reciprocal multiply with a 2^-40
// relative margin; the exact IEEE division runs whenever the filter cannot
// decide.
#include <hip/hip_runtime.h>

#include "../../include/rt_rng.h"
#include "rt_device.h"
#include "rt_internal.h"

// waves per SIMD of render_kernel: measured best of 2/3/4 (4 spills the FP64 path state)
#ifndef RT_WAVES_PER_SIMD
#define RT_WAVES_PER_SIMD 3
#endif
// cooperative soft shadows when at most this many lanes need them (measured
// best of 0/2/4/8 in round 1; 4 and 16 within noise in round 2)
#ifndef RT_COOP_MAX
#define RT_COOP_MAX 8
#endif
constexpr int kCoopMax = RT_COOP_MAX;
// soft_queue: the owners still drawing finish cooperatively once at most
// this many are left (measured best of 0/1/2/4, r03)
#ifndef RT_SQ_TAIL
#define RT_SQ_TAIL 2
#endif
constexpr int kSqTail = RT_SQ_TAIL;
// soft_queue: rejection tries per pass of its loop (measured best of 1..6
// within the LDS budget, r03)
#ifndef RT_SQ_TRIES
#define RT_SQ_TRIES 2
#endif
constexpr int kSqTries = RT_SQ_TRIES;
// The lone-path form (solo_path): off by default since r05.
// Under RNG spec v4 a lone bounce is cheap, and the form no longer shortens
// anything (K = 20 frames 229.7 k vs 231.7 k Mrays/s without it, six rounds;
// one frame 0.574 vs 0.571 ms), while its call frames left ~47 MB of dirty
// scratch per one-frame launch (74.7 vs 18.6 MB of HBM traffic).  The
// cross-lane checking build compiles it in (Makefile xlane), so it stays
// tested; RT_SOLO=1 restores it.  (measurement switch: cone helpers off)
#ifndef RT_SOLO
#define RT_SOLO 0
#endif
#ifndef RT_CONE_HELPERS  // (not RT_CONE_WIDE: rt_internal.h's candidate-list width)
#define RT_CONE_HELPERS 1
#endif

namespace rtgo {

// The lane id through a volatile move: an LDS address derived from it is
// computed where it is used instead of being kept live through the bounce
// loop (live across the lone-path call, such values are spilled to scratch
// once per wave: the one-frame launch's bulk HBM writes)
__device__ __forceinline__ int lane_now() {  // (one-wave workgroups: the lane is threadIdx.x)
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
// Set bits of a wave mask below the calling lane (v_mbcnt): no 64-bit
// per-lane "below" mask has to stay live (it was spilled to scratch)
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ------------------------------------------------------------ culling
// Shadow-cone culling (linear-scan scenes with <= 64 spheres and <= 64
// triangles).  calculateSmartShadow's rays all leave the hit point P inside
// the cone around ldir of half-angle asin(0.1) (|RandomVec3InUnitSphere *
// 0.1| < 0.1, renderer.go:316-317) and end at the light (tMax = distance).
// A primitive whose bounding sphere cannot meet that cone segment can never
// be hit by the hard ray or by any of the 16 soft rays, so it is left out of
// their tests; everything else gets the exact Sphere.Hit / Triangle.Hit
// test, so occlusion results are unchanged.  Margins (~1e-7 relative) are
// eight orders of magnitude above binary64 rounding.
//
// The two square roots are single-precision hardware roots (v_sqrt_f32 of
// the binary64 value rounded to float: relative error < 2e-7, far inside
// the 1e-5 relative margins below).  A culling test only has to be
// conservative, not exact: float overflow gives dc = inf (kept), underflow
// gives dc = 0 (kept).  No early exits, so the compiler can batch the
// loads of consecutive spheres.
__device__ __forceinline__ bool in_cone(const double* cc, double r, d3 P, d3 ldir, double ldist) {
  const d3 v = ld3(cc) - P;
  const double dc2 = len2(v);
  const double dc = (double)__builtin_amdgcn_sqrtf((float)dc2);
  const double ra = fabs(r) * KC(1.0 + 1e-5) + KC(1e-5) * dc + KC(1e-12);  // inflated radius
  const bool inside = dc <= ra;                                           // P inside / on it
  const bool beyond = dc - ra > ldist * KC(1.0 + 1e-5) + KC(1e-9);      // beyond the light
  // angle(v, ldir) <= alpha + beta, sin(alpha) = 0.1, sin(beta) = ra/dc:
  // v.ldir >= dc*cos(alpha+beta) = cos(alpha)*sqrt(dc^2-ra^2) - 0.1*ra
  const double tl = (double)__builtin_amdgcn_sqrtf((float)fmax(dc2 - ra * ra, 0.0));
  const bool meets = dot(v, ldir) >= KC(0.99498) * tl - KC(0.1) * ra - KC(1e-5) * dc;
  return inside || (!beyond && meets);
}

// `self` is the hittable that was hit.  When the hit is on its OUTSIDE and
// every cone direction leaves the surface by a clear angle (N.ldir >= 0.1015
// > sin(alpha), N the normal facing the ray's side), a convex hittable
// (sphere of positive radius, or createCube's box) cannot be hit again at
// t >= 0.001.  A hit from inside is never left out: the shadow ray has to
// cross the object.  "Outside" per kind:
//   sphere: FrontFace (sphere.go:42-48 takes the true outward normal);
//   cube:   FrontFace != "its normals point in" (DBox.front_out): createCube
//           winds them inward, so FrontFace there means a hit from inside.
__device__ __forceinline__ bool box_self_out(const DBox& B, bool front) { return (int)front == B.front_out; }

__device__ __forceinline__ Cand cone_candidates(const Geo& p, d3 P, d3 N, bool front, int self, d3 ldir,
                                                double ldist) {
  const bool leaves = dot(N, ldir) >= KC(0.1015);
  const bool sphere_out = front && leaves;
  Cand m{0ull, 0ull};
  for (int i = 0; i < p.ns; ++i) {
    const DSphere& S = p.spheres[i];
    if (sphere_out && S.obj == self && S.r > 0) continue;
    if (in_cone(S.c, S.r, P, ldir, ldist)) m.s |= 1ull << i;
  }
  // triangles by cube: one cone test against the bounding sphere of the
  // cube's box admits its 12 triangles (their exact tests follow per ray)
  for (int j = 0; j < p.nb; ++j) {
    const DBox& B = p.boxes[j];
    if (leaves && B.obj == self && box_self_out(B, front)) continue;
    if (in_cone(B.bc, B.br, P, ldir, ldist)) m.t |= 0xFFFull << B.first;
  }
  return m;
}

// hitWorld(shadowRay, 0.001, dist) restricted to the candidates.
template <bool kCount>
__device__ __forceinline__ bool any_hit_masked(const Geo& p, d3 o, d3 d, double tmax, Cand m, Counters& c) {
  if (m.t) {  // a cube whose box the ray misses cannot be hit: drop its 12 triangles
    const d3 id = inv_dir(d);
    for (int j = 0; j < p.nb; ++j) {
      const DBox& B = p.boxes[j];
      const unsigned long long g = 0xFFFull << B.first;
      if ((m.t & g) && !ray_box(B, o, id, 0.001, tmax)) m.t &= ~g;
    }
  }
  if (m.s) {  // (most camera rays have no candidate at all)
    const double a = len2(d);
    const double inv_a = approx_rcp(a);
    for (unsigned long long b = m.s; b; b &= b - 1) {
      const int i = __builtin_ctzll(b);
      cnt<kCount>(c, C_SPH);
      double num;
      if (sphere_query(p.spheres[i], o, d, a, inv_a, 0.001, tmax, num)) return true;
    }
  }
  for (unsigned long long b = m.t; b; b &= b - 1) {
    const int i = __builtin_ctzll(b);
    cnt<kCount>(c, C_TRI);
    double t, u, v;
    if (tri_test(p.tris[i], o, d, 0.001, tmax, t, u, v)) return true;
  }
  return false;
}

// Occlusion of one shadow ray: candidates when culling is on, else all.
template <bool kCount>
__device__ __forceinline__ bool shadow_blocked(const Geo& p, bool masks, d3 o, d3 d, double tmax, Cand m,
                                               int* stack, Counters& c) {
  if (masks) return (m.s | m.t) != 0 && any_hit_masked<kCount>(p, o, d, tmax, m, c);
  return any_hit<kCount>(p, o, d, tmax, stack, c);
}

// ------------------------------------------------------------ wide mode
// When few lanes of a wave still run paths (the end of a block, where one
// long path sets the launch's critical path), the idle lanes help: every
// lane that needs a query (an "owner", at most 16) gets a group of
// S = 64 / next_pow2(owners) helper lanes, which split the primitive scan
// (primitive i goes to helper i mod S) and merge their results.  Only for
// sphere-only linear-scan scenes (no triangles): the merges below are exact
// for spheres.  wide_groups: the owner table (LDS), this lane's owner and its
// index within the group; S is returned.
__device__ __forceinline__ int wide_groups(bool need, unsigned long long qmask, int nq, int* owner_tab, int& ow,
                                           int& k, bool& helper) {
  const int lane = (int)(threadIdx.x & 63);
  const int S = nq <= 4 ? 16 : (nq <= 8 ? 8 : 4);
  if (need) owner_tab[lanes_below(qmask)] = lane;
  __syncthreads();
  const int grp = lane / S;
  k = lane - grp * S;
  helper = grp < nq;
  ow = helper ? owner_tab[grp] : lane;
  __syncthreads();  // the table is reused by the next call
  return S;
}

// hitWorld's closest hit over the spheres (the scene has no triangles), with
// helpers.  Each helper scans its spheres in hittable order with the
// sequential rule; the group then keeps the smallest t, and of equal t the
// larger hittable index (what the sequential scan ends with: a tie replaces
// the current hit unless its index is larger).  Exact for finite rays; an
// owner with a non-finite ray (or a = 0) is flagged in `fallback` and scans
// on its own.  Returns found for owner lanes.
template <bool kCount>
__device__ __forceinline__ bool closest_wide(const Geo& g, bool need, unsigned long long qmask, int nq, d3 o, d3 d,
                                             HitSel& hs, bool& fallback, Counters& c) {
  __shared__ int owner_tab[16];
  const int lane = (int)(threadIdx.x & 63);
  int ow, k;
  bool helper;
  const int S = wide_groups(need, qmask, nq, owner_tab, ow, k, helper);
  const d3 ro = mk(__shfl(o.x, ow), __shfl(o.y, ow), __shfl(o.z, ow));
  const d3 rd = mk(__shfl(d.x, ow), __shfl(d.y, ow), __shfl(d.z, ow));
  const double a = len2(rd);
  const double inv_a = approx_rcp(a);
  double bt = __builtin_inf(), bnum = 0;
  int bobj = -1, bidx = -1;
  bool found = false;
  if (helper) {
    for (int i = k; i < g.ns; i += S) {
      cnt<kCount>(c, C_SPH);
      const DSphere& Sp = g.spheres[i];
      double num;
      if (sphere_query(Sp, ro, rd, a, inv_a, 0.001, bt, num)) {
        const double t = num / a;
        if (t == bt && bobj > Sp.obj) continue;
        bt = t;
        bnum = num;
        bidx = i;
        bobj = Sp.obj;
        found = true;
      }
    }
  }
  for (int off = S >> 1; off >= 1; off >>= 1) {  // within the group (aligned to S)
    const double t2 = __shfl_xor(bt, off), n2 = __shfl_xor(bnum, off);
    const int o2 = __shfl_xor(bobj, off), i2 = __shfl_xor(bidx, off), f2 = __shfl_xor((int)found, off);
    if (f2 && (!found || t2 < bt || (t2 == bt && o2 > bobj))) {
      bt = t2;
      bnum = n2;
      bobj = o2;
      bidx = i2;
      found = true;
    }
  }
  const int lead = need ? lanes_below(qmask) * S : lane;
  const double fnum = __shfl(bnum, lead);
  const int fidx = __shfl(bidx, lead), ffound = __shfl((int)found, lead);
  fallback = need && !(__builtin_isfinite(o.x + o.y + o.z) && a > 0 && __builtin_isfinite(__shfl(a, lead)));
  hs.num = fnum;
  hs.idx = fidx;
  hs.is_tri = 0;
  return ffound != 0;
}

// cone_candidates (spheres only) with helpers: each helper tests its
// spheres, the group ORs the bits.  Same tests, same mask.
__device__ __forceinline__ unsigned long long cone_wide(const Geo& g, bool need, unsigned long long qmask, int nq,
                                                        d3 P, d3 N, bool front, int self, d3 ldir, double ldist) {
  __shared__ int owner_tab2[16];
  const int lane = (int)(threadIdx.x & 63);
  int ow, k;
  bool helper;
  const int S = wide_groups(need, qmask, nq, owner_tab2, ow, k, helper);
  const d3 Po = mk(__shfl(P.x, ow), __shfl(P.y, ow), __shfl(P.z, ow));
  const d3 Lo = mk(__shfl(ldir.x, ow), __shfl(ldir.y, ow), __shfl(ldir.z, ow));
  const double dist = __shfl(ldist, ow);
  const bool self_out = __shfl((int)(front && dot(N, ldir) >= KC(0.1015)), ow) != 0;
  const int selfo = __shfl(self, ow);
  unsigned long long m = 0;
  if (helper) {
    for (int i = k; i < g.ns; i += S) {
      const DSphere& Sp = g.spheres[i];
      if (self_out && Sp.obj == selfo && Sp.r > 0) continue;
      if (in_cone(Sp.c, Sp.r, Po, Lo, dist)) m |= 1ull << i;
    }
  }
  for (int off = S >> 1; off >= 1; off >>= 1) m |= __shfl_xor(m, off);
  const int lead = need ? lanes_below(qmask) * S : lane;
  return __shfl(m, lead);
}

// ------------------------------------------------------------ inert lights
// (r05) A lit light whose shadow rays cannot change the shading: cos =
// Max(0, N.L) is 0, so calculateDirectLighting's intensity is 0 * I / d^2 =
// +0 and each term it adds is (finite) * 0 * shadowFactor * ... = +-0, and
// adding +-0 to D, which has no zero component, leaves D's bits unchanged --
// whether the term is added (shadow factor > 0) or not (= 0).  Finite means:
// the light's intensity and colour, the material's albedo, metallic and
// diffuse strength (the specular power is of a unit or zero half vector:
// Vec3.Normalize keeps zero, vector.go:61-67, so it is finite).  Such a
// light's hard and soft
// shadow rays are not traced (their result is not observable) and its soft
// points are not drawn (spec v4).  `D` is the ambient plus the terms of the
// lights before this one.
__device__ __forceinline__ bool light_inert(const DMat* m, const DLight& Lt, d3 N, d3 ldir, d3 D) {
  return gmax0(dot(N, ldir)) == 0.0 && D.x != 0.0 && D.y != 0.0 && D.z != 0.0 && __builtin_isfinite(Lt.intensity) &&
         __builtin_isfinite(Lt.color[0] + Lt.color[1] + Lt.color[2]) &&
         __builtin_isfinite(m->albedo[0] + m->albedo[1] + m->albedo[2]) && __builtin_isfinite(m->metallic) &&
         __builtin_isfinite(m->diffuse_strength);
}

// ------------------------------------------------------------ soft shadows
// Cooperative form for ONE owner lane, executed by the whole (converged)
// wave: lane h evaluates rejection try h of the owner's stream (draws
// 3h..3h+2 via the PCG jump table), a ballot picks the first `need`
// accepted tries in order, those lanes trace their rays, and the owner's
// stream advances by exactly the draws the sequential loop would consume.
// All arguments are wave-uniform (the owner's values, read from its lane).
struct CoopOut {
  uint64_t x;  // the owner's stream state after its 16 points
  int unocc;   // unoccluded rays
  int tries;   // rejection tries consumed
};
template <bool kCount>
__device__ __forceinline__ CoopOut soft_coop(const Geo p, bool masks, bool trace, d3 P, d3 ldir, double ldist, Cand cm, uint64_t x,
                             const uint64_t* jump, int* stack, Counters& c) {
  const int lane = (int)(threadIdx.x & 63);
  int need = 16, unocc = 0, tries = 0;
  while (need > 0) {
    const uint64_t x0 = state_at3(x, jump, lane), x1 = x0 * RT_PCG_MULT + RT_PCG_INC,
                   x2 = x1 * RT_PCG_MULT + RT_PCG_INC;
    const uint32_t o0 = rt_pcg_out(x0), o1 = rt_pcg_out(x1), o2 = rt_pcg_out(x2);
    const bool acc = unit_ball_accept(o0, o1, o2);
    const unsigned long long am = __ballot(acc);
    const int rank = lanes_below(am);
    const bool chosen = acc && rank < need;
    const unsigned long long chm = __ballot(chosen);
    const int nch = __popcll(chm);
    // tries consumed: up to and including the last chosen one
    const int used = nch == need ? 64 - __clzll(chm) : 64;
    bool occ = false;
    if (chosen && trace)
      occ = shadow_blocked<kCount>(p, masks, P, normalize(ldir + muls(unit_ball_point(o0, o1, o2), 0.1)), ldist, cm,
                                   stack, c);
    unocc += nch - __popcll(__ballot(chosen && occ));
    need -= nch;
    tries += used;
    x = state_at3(x, jump, used);
  }
  return CoopOut{x, unocc, tries};
}

// Queue form for many owners (more than kCoopMax lanes need soft
// shadows for this light), executed by the whole converged wave.  Each
// owner runs its own rejection tries on its own stream, in order (the same
// draws as 16 calls of RandomVec3InUnitSphere); an accepted point is
// appended to an LDS queue as its three raw 32-bit draws and the owner's
// lane.  Whenever 64 points are queued, every lane takes one, rebuilds the
// point from the raw draws, reads the owner's hit point, light direction,
// distance and candidates across lanes, and traces the jittered ray.  The
// sequential form traced a ray in nearly every try step at about half the
// lanes; here the tries run alone and the rays run on full waves.  The
// result is a count of unoccluded rays, so the order in which rays are
// traced does not change it.  Returns the owner's count (0 elsewhere).
template <bool kCount>
__device__ __forceinline__ int soft_queue(const Geo& p, bool masks, bool need_soft, bool trace, d3 P, d3 ldir,
                                          double ldist, Cand cm, rt_rng& rng, const uint64_t* jump, int* stack,
                                          Counters& c) {
  // queued points: raw draws x, y, z, owner lane (a ring).  It holds what
  // a pass can leave: < 64 points not yet traced, 64 per try of the pass and
  // 16 per owner of the cooperative tail (256 or more entries; a power of 2
  // up to 256, so the index is a mask there)
  constexpr int kRingNeed = 64 * kSqTries + 64 + 16 * kSqTail;
  constexpr unsigned kRing = kRingNeed <= 256 ? 256u : (unsigned)kRingNeed;
  __shared__ uint4 sq[kRing];
  __shared__ int sq_unocc[64];  // per owner: unoccluded rays
  const int lane = lane_now() & 63;
  sq_unocc[lane] = 0;
  int need = need_soft ? 16 : 0, free_rays = 0;  // free_rays: points of an owner with nothing to trace
  int head = 0, tail = 0;  // wave-uniform ring positions
  for (;;) {
    // kSqTries tries per pass: the later tries are drawn ahead and each
    // is consumed only when the owner still needs a point after the ones
    // before it (so the stream advances by exactly the draws the sequential
    // loop takes).
    constexpr int K = kSqTries;
    bool acc[K];
    uint32_t u[K][3];
#pragma unroll
    for (int t = 0; t < K; ++t) {
      acc[t] = false;
      u[t][0] = u[t][1] = u[t][2] = 0;
    }
    if (need > 0) {
      rt_rng r = rng;
#pragma unroll
      for (int t = 0; t < K; ++t) {
        u[t][0] = rt_rng_next(&r);
        u[t][1] = rt_rng_next(&r);
        u[t][2] = rt_rng_next(&r);
        if (need > 0) {
          rng = r;
          cnt<kCount>(c, C_RNG, 3);
          if (unit_ball_accept(u[t][0], u[t][1], u[t][2])) {
            --need;
            cnt<kCount>(c, C_SHADOW);
            if (trace) acc[t] = true;  // only rays that can be blocked are queued
            else ++free_rays;
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const unsigned long long am = __ballot(acc[t]);
      if (acc[t]) sq[(unsigned)(tail + lanes_below(am)) % kRing] = make_uint4(u[t][0], u[t][1], u[t][2], (uint32_t)lane);
      tail += __popcll(am);
    }
    if constexpr (kSqTail > 0) {
      // The last few owners still drawing finish cooperatively, one at a
      // time: lane h evaluates try h of the owner's stream (jump table), as
      // in soft_coop; the first `need` accepted tries are its points, queued
      // in try order, and the stream advances past the last one taken.  The
      // wave no longer loops on its unluckiest owners' tries one by one.
      // (at most 16 points per owner: the ring holds them, see kRing)
      const unsigned long long rem = __ballot(need > 0);
      if (rem != 0 && __popcll(rem) <= kSqTail) {
        for (unsigned long long b = rem; b; b &= b - 1) {
          const int ow = __builtin_ctzll(b);
          int nd = __builtin_amdgcn_readlane(need, ow);
          const bool tr = __builtin_amdgcn_readlane(trace ? 1 : 0, ow) != 0;
          uint64_t x = rl64(rng.x, ow);
          int got = 0, tries = 0;
          while (nd > 0) {
            const uint64_t x0 = state_at3(x, jump, lane), x1 = x0 * RT_PCG_MULT + RT_PCG_INC,
                           x2 = x1 * RT_PCG_MULT + RT_PCG_INC;
            const uint32_t o0 = rt_pcg_out(x0), o1 = rt_pcg_out(x1), o2 = rt_pcg_out(x2);
            const bool acc = unit_ball_accept(o0, o1, o2);
            const unsigned long long am = __ballot(acc);
            const bool chosen = acc && lanes_below(am) < nd;
            const unsigned long long chm = __ballot(chosen);
            const int nch = __popcll(chm);
            const int used = nch == nd ? 64 - __clzll(chm) : 64;
            if (tr) {
              if (chosen) sq[(unsigned)(tail + lanes_below(chm)) % kRing] = make_uint4(o0, o1, o2, (uint32_t)ow);
              tail += nch;
            }
            got += nch;
            nd -= nch;
            tries += used;
            x = state_at3(x, jump, used);
          }
          if (lane == ow) {
            rng.x = x;
            need = 0;
            if (!tr) free_rays += got;
            cnt<kCount>(c, C_RNG, 3ull * tries);
            cnt<kCount>(c, C_SHADOW, got);
          }
        }
      }
    }
    const bool more = __ballot(need > 0) != 0;
    while (tail - head >= 64 || (!more && tail > head)) {
      __syncthreads();
      const int n = min(64, tail - head);
      const uint4 e = sq[(unsigned)(head + lane) % kRing];
      const int ow = lane < n ? (int)e.w : lane;
      // the owner's ray inputs, read across lanes (every lane takes part)
      const d3 Po = mk(__shfl(P.x, ow), __shfl(P.y, ow), __shfl(P.z, ow));
      const d3 Lo = mk(__shfl(ldir.x, ow), __shfl(ldir.y, ow), __shfl(ldir.z, ow));
      const double dist = __shfl(ldist, ow);
      const Cand co{__shfl(cm.s, ow), p.nt ? __shfl(cm.t, ow) : 0ull};  // (no triangles: cm.t is 0)
      if (lane < n) {
        const d3 pt = mk(rt_bits_to_unit(e.x) * 2 - 1, rt_bits_to_unit(e.y) * 2 - 1, rt_bits_to_unit(e.z) * 2 - 1);
        if (!shadow_blocked<kCount>(p, masks, Po, normalize(Lo + muls(pt, 0.1)), dist, co, stack, c))
          atomicAdd(&sq_unocc[ow], 1);
      }
      head += n;
      __syncthreads();
    }
    if (!more && head == tail) break;
  }
  __syncthreads();
  return need_soft ? sq_unocc[lane] + free_rays : 0;
}


// ------------------------------------------------------------ kernel
// Kernel parameters that only the sample set-up and the epilogue need are
// re-read from the kernarg segment through a laundered pointer at each use
// (scalar-cache loads) instead of being held in SGPRs across the bounce
// loop: the loop's SGPR pressure otherwise spills uniform values into VGPR
// lanes and reloads them inside the intersection loops.
typedef const __attribute__((address_space(4))) KParams* KArg;  // constant (kernarg) address space
__device__ __forceinline__ KArg fresh() {
  // KParams is the kernel's only argument: it sits at offset 0 of the kernarg segment
  KArg k = (KArg)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(k));
  return k;
}

// This main workgroup's index: the grid's, less the tail helpers placed
// before it (KParams.tail_pos; launch_render)
__device__ __forceinline__ unsigned main_wg(KArg k) {
  const unsigned b = blockIdx.x;
  return (k->tail != nullptr && b >= (unsigned)k->tail_pos) ? b - (unsigned)k->tail_helpers : b;
}
// The launch's frame and block of this workgroup (KParams.nframes)
__device__ __forceinline__ int frame_of(KArg k) {
  return k->nframes > 1 ? (int)(main_wg(k) % (unsigned)k->nframes) : 0;
}
__device__ __forceinline__ int block_of(KArg k) {
  return k->nframes > 1 ? (int)(main_wg(k) / (unsigned)k->nframes) : (int)main_wg(k);
}
// a split pixel's radiance row / hit-bit words / sub-block counter in this frame's copy
__device__ __forceinline__ size_t split_index(KArg k, int slot) {
  return (size_t)frame_of(k) * (size_t)k->nsplit + (size_t)slot;
}

// ------------------------------------------------------------ work blocks
// A BLOCK is np consecutive row-major pixels of one 32x32 tile with all
// their spp samples: NB = np*spp sample ids, pixel-major (id = p*spp + s).
// One workgroup renders one block.  The host lists the blocks in its tile
// dispatch order (tiles sorted by estimated cost) and makes them small on
// tiles with geometry (schedule.cpp build_blocks).
struct BlockLoc {
  int lt, tile, tx, ty;  // local tile, global tile, tile coords
  int p0, np;            // first pixel (row-major in the tile), pixel count
  int s0, ns;            // samples [s0, s0+ns) of each pixel (all spp unless split)
  int slot, nsub;        // split pixel: its radiance slot row and number of sub-blocks (slot < 0: not split)
  bool black;            // kBlockBlack: no camera ray of the tile can hit anything
  unsigned long long ms, mt;  // primary masks: union over the block's pixels (fill_block_masks)
  unsigned long long live;    // its pixels whose own primary masks are not empty
};
__device__ __forceinline__ BlockLoc block_loc(KArg k, int b) {
  BlockLoc r;
  const int4 e = reinterpret_cast<const int4*>(k->blocks)[4 * b];
  const int4 f = reinterpret_cast<const int4*>(k->blocks)[4 * b + 1];
  const int4 g = reinterpret_cast<const int4*>(k->blocks)[4 * b + 2];
  const int4 l = reinterpret_cast<const int4*>(k->blocks)[4 * b + 3];
  r.ms = (unsigned long long)(uint32_t)g.x | ((unsigned long long)(uint32_t)g.y << 32);
  r.mt = (unsigned long long)(uint32_t)g.z | ((unsigned long long)(uint32_t)g.w << 32);
  r.live = (unsigned long long)(uint32_t)l.x | ((unsigned long long)(uint32_t)l.y << 32);
  r.lt = e.x;
  r.p0 = e.y;
  r.np = e.z;
  r.s0 = e.w;
  r.ns = f.x;
  r.slot = f.y;
  r.nsub = f.z;
  r.black = (f.w & kBlockBlack) != 0;
  r.tile = l.z;  // the block's global tile (sched_blocks: strided or a partition's list)
  r.tx = r.tile % k->tiles_x;
  r.ty = r.tile / k->tiles_x;
  return r;
}

// The scene view and switches of one phase of the bounce loop, re-read
// per phase (see fresh()).  Staged scenes address the LDS copy.
struct Hot {
  Geo g;
  const DMat* mats;
  const DLight* lights;
  const uint64_t* jump;
  int nl, max_depth;
  bool recursive, soft, masks;
};
extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];
template <bool kStage>
__device__ __forceinline__ Hot hot(KArg k) {
  Hot h;
  h.g = Geo{k->spheres, k->tris, k->boxes, k->bvh, k->ns, k->nt, k->use_bvh, k->nb};
  h.mats = k->mats;
  h.lights = k->lights;
  h.jump = k->jump;
  if constexpr (kStage) {
    const unsigned char* base = reinterpret_cast<const unsigned char*>(k->stage_src);
    h.g.spheres = reinterpret_cast<const DSphere*>(dyn_lds + (reinterpret_cast<const unsigned char*>(k->spheres) - base));
    h.g.tris = reinterpret_cast<const DTri*>(dyn_lds + (reinterpret_cast<const unsigned char*>(k->tris) - base));
    h.g.boxes = reinterpret_cast<const DBox*>(dyn_lds + (reinterpret_cast<const unsigned char*>(k->boxes) - base));
    h.mats = reinterpret_cast<const DMat*>(dyn_lds + (reinterpret_cast<const unsigned char*>(k->mats) - base));
    h.lights = reinterpret_cast<const DLight*>(dyn_lds + (reinterpret_cast<const unsigned char*>(k->lights) - base));
    const long jo = reinterpret_cast<const unsigned char*>(k->jump) - base;
    if (jo < k->stage_bytes) h.jump = reinterpret_cast<const uint64_t*>(dyn_lds + jo);
    // staged scenes are linear-scan scenes (set_scene stages only without a
    // BVH): the staged kernels carry no BVH traversal code at all
    h.g.use_bvh = 0;
  }
  h.nl = k->nl;
  h.max_depth = k->max_depth;
  h.recursive = k->recursive != 0;
  h.soft = k->soft != 0;
  h.masks = !h.g.use_bvh && h.g.ns <= 64 && h.g.nt <= 64;  // shadow-cone culling available
  return h;
}
template <bool kStage>
__device__ __forceinline__ Hot hot() {
  return hot<kStage>(fresh());
}

// Camera ray of sample s of pixel (x, y): tracePixel's jitter
// (renderer.go:155-156, the first two draws of the stream) and getRay
// (renderer.go:377-390).  Leaves `rng` after those two draws.  CamK holds
// the launch-uniform inputs; phase 1 loads it once per block (SGPRs), the
// shading loop rebuilds it from the kernarg segment where it needs it.
__device__ __forceinline__ CamK cam_k(KArg k) {
  return make_cam(k->frame_key[frame_of(k)], k->W, k->H, k->aspect, k->cam[0], k->cam[1], k->cam[2]);
}
template <bool kCount>
__device__ __forceinline__ void camera_ray(KArg k, int x, int y, int s, rt_rng& rng, d3& o, d3& d, Counters& c) {
  camera_ray_c<kCount>(cam_k(k), x, y, s, rng, o, d, c);
}

// ------------------------------------------------------------ solo paths
// When a single path is left running in a wave (the end of a block, where
// a long metal-metal interreflection sets the launch's critical path), the
// idle lanes join it: every lane holds the path's state and computes the
// same binary64 values (the serial parts need no cross-lane traffic), while
// the loops over primitives run in parallel, one primitive per lane, with
// exact merges:
//   closest hit - every lane tests its primitives over [0.001, +inf); the
//     hits are then replayed in hittable scan order with hitWorld's rule
//     (accept t <= closest; an equal t only for a hittable index not below
//     the current one).  A root that Sphere.Hit rejects against a smaller
//     tMax is larger than that tMax, and so is the other root, so the replay
//     accepts exactly what the sequential scan accepts (renderer.go:333-346);
//   shadow cones and the hard shadow ray - a ballot of per-primitive tests
//     (an occlusion query has no order);
//   soft shadows - soft_coop (already wave-wide for one owner).
// The path runs to its end; then the main loop takes over again.  Linear-
// scan scenes with at most 64 spheres and 64 triangles (the staged scenes);
// the counting and pilot variants keep the per-lane loop.  (Lone bounce,
// 2 lights with soft shadows: 9.8 -> 6.1 us, scripts/latency_probe.py.
// Two paths in 32-lane groups, same scheme with shuffles, measured slower:
// headline 0.82 vs 0.775 ms, the group form's registers spill.)
__device__ __forceinline__ bool solo_closest(const Geo& g, d3 o, d3 d, HitSel& hs) {
  const int lane = (int)(threadIdx.x & 63);
  const double a = len2(d);
  const double inv_a = approx_rcp(a);
  double closest = __builtin_inf();
  int best_obj = -1;
  bool found = false;
  // lane i tests sphere i, then triangle i; the hits are replayed in
  // hittable scan order (spheres before triangles)
#pragma unroll
  for (int tri = 0; tri < 2; ++tri) {
    double t = 0, nm = 0, u = 0, v = 0;
    bool f;
    int myobj = 0;  // (the lane's hittable index, read with its primitive: the replay takes it by readlane)
    if (!tri) {
      f = false;
      if (lane < g.ns) {
        const DSphere& S = g.spheres[lane];
        myobj = S.obj;
        f = sphere_query(S, o, d, a, inv_a, 0.001, __builtin_inf(), nm) != 0;
      }
      if (f) t = nm / a;
    } else {
      f = false;
      if (lane < g.nt) {
        myobj = g.tris[lane].obj;
        f = tri_test(g.tris[lane], o, d, 0.001, __builtin_inf(), t, u, v);
      }
    }
    for (unsigned long long b = __ballot(f); b; b &= b - 1) {
      const int i = __builtin_ctzll(b);
      const double ti = rld(t, i);
      const int obj = (int)rl32((uint32_t)myobj, i);
      if (closest < ti || (ti == closest && best_obj > obj)) continue;
      closest = ti;
      best_obj = obj;
      hs.num = tri ? ti : rld(nm, i);
      if (tri) {
        hs.u = rld(u, i);
        hs.v = rld(v, i);
      }
      hs.idx = i;
      hs.is_tri = tri;
      found = true;
    }
  }
  return found;
}

// ---- parallel direct lighting of a lone path (solo_lights)
// The tries of a bounce's soft-shadow streams, evaluated ahead: try k of the
// stream whose state is x uses draws 3k, 3k+1, 3k+2 (RandomVec3InUnitSphere,
// vector.go:132-139); lane h holds try h of light 0's stream (a) and of light
// 1's (b) (spec v4, include/rt_rng.h: each (sample, bounce, light) has a
// stream of its own).  A light whose hard ray is clear takes the first 16
// accepted tries of its stream, so all lights' soft rays are known once the
// hard rays are, and can be traced at once.
struct SoloTries {
  uint32_t a0, a1, a2, b0, b1, b2;  // the draws of try h of stream a, of stream b
  unsigned long long ma, mb;        // accepted tries 0..63 of each (wave-uniform)
};
__device__ __forceinline__ SoloTries solo_tries(uint64_t xa, uint64_t xb, uint64_t jA, uint64_t jC) {
  SoloTries t;
  uint64_t s = jA * xa + jC;  // state before draw 3h of stream a
  t.a0 = rt_pcg_out(s);
  s = s * RT_PCG_MULT + RT_PCG_INC;
  t.a1 = rt_pcg_out(s);
  s = s * RT_PCG_MULT + RT_PCG_INC;
  t.a2 = rt_pcg_out(s);
  s = jA * xb + jC;  // ... of stream b
  t.b0 = rt_pcg_out(s);
  s = s * RT_PCG_MULT + RT_PCG_INC;
  t.b1 = rt_pcg_out(s);
  s = s * RT_PCG_MULT + RT_PCG_INC;
  t.b2 = rt_pcg_out(s);
  t.ma = __ballot(unit_ball_accept(t.a0, t.a1, t.a2));
  t.mb = __ballot(unit_ball_accept(t.b0, t.b1, t.b2));
  return t;
}
// The index after the 16th accepted try of each stream's 64 (-1: fewer):
// every lane ranks its tries among the accepted ones (v_mbcnt) and two
// ballots find the 16th of each
__device__ __forceinline__ void solo_take16(const SoloTries& t, int& ia, int& ib) {
  const int lane = (int)(threadIdx.x & 63);
  const bool aa = (t.ma >> lane) & 1ull, ab = (t.mb >> lane) & 1ull;
  const unsigned long long a16 = __ballot(aa && lanes_below(t.ma) + 1 == 16);
  const unsigned long long b16 = __ballot(ab && lanes_below(t.mb) + 1 == 16);
  ia = a16 ? __builtin_ctzll(a16) + 1 : -1;
  ib = b16 ? __builtin_ctzll(b16) + 1 : -1;
}

// RT_WG_TIMING builds: s_memtime clocks of a lone path's bounce by section
// (solo_clk[k], wave-uniform; scripts/latency_probe.py PROBE_SECTIONS):
// 0 loop top + closest hit, 1 hit record, 2 stream tries + light vectors +
// cones + hard rays, 3 soft rays, 4 lighting terms, 5 scatter, 6 bounces,
// 7 entries;
// SOLO_S(k), k >= 8: clocks from the start of the current section to that
// point of it (the parallel-lights form: 8 tries, 9 light vectors, 10 their
// shuffles, 11 cones + hard rays + ballots; 12 the soft rays of tries
// 0..63, 13 of tries 64..127; 14 the lighting terms before the sum)
#ifdef RT_WG_TIMING
__shared__ unsigned long long solo_clk[16];
#define SOLO_T(k)                                          \
  do {                                                     \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    solo_clk[k] += now_ - solo_t0;                         \
    solo_t0 = now_;                                        \
  } while (0)
#define SOLO_S(k)                                                           \
  do {                                                                      \
    solo_clk[k] += __builtin_amdgcn_s_memtime() - solo_t0;                  \
  } while (0)
#else
#define SOLO_T(k) \
  do {            \
  } while (0)
#define SOLO_S(k) \
  do {            \
  } while (0)
#endif

// The path of lane `ow`, run to its end by the whole wave: its radiance.
// A real call (RT_SOLO_CALL, the default): its registers then do not add to
// the shade loop's, whose per-iteration scratch spills they caused when it
// was inlined.  A callee has no kernarg segment pointer of
// its own -- __builtin_amdgcn_kernarg_segment_ptr() lowers to a null pointer
// outside a kernel entry point, which is what made round 4's non-inlined
// variant fault on its first parameter load -- so the kernel passes it in
// (`karg`) and every per-bounce read launders that copy (launder()).
#ifndef RT_SOLO_CALL
#define RT_SOLO_CALL 0
#endif
#if RT_SOLO_CALL
#define RT_SOLO_ATTR __noinline__
#else
#define RT_SOLO_ATTR __forceinline__
#endif
__device__ __forceinline__ KArg launder(KArg k) {
  // (a call's arguments arrive in VGPRs: made wave-uniform first)
  const uint64_t v = (uint64_t)(uintptr_t)k;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  KArg r = (KArg)(uintptr_t)(((uint64_t)hi << 32) | lo);
  asm volatile("" : "+s"(r));
  return r;
}
template <bool kSky>
__device__ RT_SOLO_ATTR d3 solo_path(KArg karg, int ow, d3 o, d3 d, d3 T, d3 L, uint64_t rx, int depth,
                                     uint64_t skey, int* stack, int* dep_out = nullptr) {
  const int lane = (int)(threadIdx.x & 63);
  o = rl3(o, ow);
  d = rl3(d, ow);
  T = rl3(T, ow);
  L = rl3(L, ow);
  rt_rng rng{rl64(rx, ow)};
  depth = (int)rl32((uint32_t)depth, ow);
  Counters c;
#ifdef RT_WG_TIMING
  unsigned long long solo_t0 = __builtin_amdgcn_s_memtime();
#endif
  // the parallel lighting form (solo_lights): sphere-only scenes with one or
  // two lights, a (light, sphere) pair per lane
  bool par;
  // jump coefficients of try `lane` (solo_tries), held in VGPRs for the
  // lone path's bounces: no memory access per bounce
  uint64_t jA, jC;
  {
    const Hot h0 = hot<true>(launder(karg));
    par = h0.g.nt == 0 && h0.nl >= 1 && h0.nl <= 2 && h0.nl * h0.g.ns <= 64;
    jA = h0.jump[2 * lane];
    jC = h0.jump[2 * lane + 1];
  }
#ifdef RT_WG_TIMING
  solo_clk[7] += 1;
#endif
  for (;;) {
    const Hot h = hot<true>(launder(karg));
    const Geo& g = h.g;
    if (depth >= h.max_depth) {  // traceRay depth cut-off: contributes 0
      if (dep_out) *dep_out = depth;
      return L;
    }
#ifdef RT_WG_TIMING
    solo_clk[6] += 1;
#endif
    // (1) closest hit (hitWorld, renderer.go:170)
    HitSel hs;
    const bool found = solo_closest(g, o, d, hs);
    SOLO_T(0);
    if (!found) {  // miss -> black (or the opted-in sky)
      if constexpr (kSky) L = L + mul(T, sky_color(launder(karg)->sky, d));
      if (dep_out) *dep_out = depth + 1;
      return L;
    }
    d3 P, N;
    bool front;
    int mi, self;
    if (!hs.is_tri) {  // sphere.go:42-58
      const DSphere& S0 = g.spheres[hs.idx];
      const double t = hs.num / len2(d);
      P = o + muls(d, t);
      d3 outward = divs(P - ld3(S0.c), S0.r);
      front = dot(d, outward) < 0;
      N = front ? outward : neg(outward);
      mi = S0.mat;
      self = S0.obj;
    } else {  // triangle.go:68-81
      const DTri& T0 = g.tris[hs.idx];
      P = o + muls(d, hs.num);
      double w = 1.0 - hs.u - hs.v;
      d3 n = ld3(T0.n);
      N = normalize((muls(n, w) + muls(n, hs.u)) + muls(n, hs.v));
      front = dot(d, N) < 0;
      if (!front) N = neg(N);
      mi = T0.mat;
      self = T0.obj;
    }
    SOLO_T(1);
    // (2) calculateDirectLighting (renderer.go:229-297)
    const DMat* __restrict__ m = h.mats + mi;
    d3 D = mk(m->ambient, m->ambient, m->ambient);
    if (par) {
      // every light at once: lane li (< nl) its light vector; lane
      // li * ns + s the pair (light li, sphere s) for the shadow cone and the
      // hard ray; then all lights' soft rays from the tries; then the
      // lighting terms per lane li, added to D in light order (the same
      // operations and sums as the loop below, so the same bits)
      const int nl = h.nl, ns = g.ns;
      SoloTries tr{};
      if (h.soft) tr = solo_tries(rt_soft_state(skey, (uint32_t)depth, 0u), rt_soft_state(skey, (uint32_t)depth, 1u), jA, jC);
      SOLO_S(8);
      d3 lvd = mk(0, 0, 0);
      double lvl = 0;
      // the lighting terms' parts that do not depend on the shadows (lane
      // li < nl, light li): diffuse_strength * intensity and si * intensity,
      // the left operands of calculateDirectLighting's products, computed
      // here so their square roots and divisions overlap the light vector's
      // (the same operations in the same order: the same bits)
      double di = 0, sii = 0;
      const double metallic = m->metallic;
      if (lane < nl) {
        const d3 lv = ld3(h.lights[lane].pos) - P;
        const d3 view = normalize(neg(P));  // (independent of the light: interleaves with lv's chain)
        lvl = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
        lvd = lvl == 0 ? mk(0, 0, 0) : divs(lv, lvl);
        const double cos_t = gmax0(dot(N, lvd));
        const double intensity = cos_t * h.lights[lane].intensity / (lvl * lvl);
        di = m->diffuse_strength * intensity;
        if (metallic > 0.5) {
          const d3 half = normalize(lvd + view);
          const double hc = gmax0(dot(N, half));
          const int sp = m->spec_pow;
          const double si = sp == 64 ? pow_n<64>(hc) : (sp == 48 ? pow_n<48>(hc) : pow_n<32>(hc));
          sii = si * intensity;
        }
      }
      // (light values move across lanes by shuffles where they are used: held
      // as wave-uniform values they would take SGPRs the bounce loop needs)
      const unsigned long long litm = __ballot(lane < nl && !(lvl < 0.001));
      SOLO_S(9);
      const int lj = lane >= ns ? 1 : 0, sj = lane - lj * ns;  // this lane's pair
      const d3 ldj = mk(__shfl(lvd.x, lj), __shfl(lvd.y, lj), __shfl(lvd.z, lj));
      const double dlj = __shfl(lvl, lj);
      SOLO_S(10);
      bool cone = false, blk = false;
      if (lane < nl * ns && ((litm >> lj) & 1ull)) {
        const DSphere& S = g.spheres[sj];
        const bool self_out = front && dot(N, ldj) >= KC(0.1015);
        cone = !(self_out && S.obj == self && S.r > 0) && in_cone(S.c, S.r, P, ldj, dlj);
        // the hard ray against every sphere, as hitWorld does, independent
        // of the cone test so the two chains overlap (a sphere outside the
        // cone cannot be hit: the same answer as testing the candidates only)
        const double a = len2(ldj);
        double num;
        blk = sphere_query(S, P, ldj, a, approx_rcp(a), 0.001, dlj, num) != 0;
      }
      const unsigned long long cones = __ballot(cone), blks = __ballot(blk);
      SOLO_S(11);
      const unsigned long long sm = ns >= 64 ? ~0ull : (1ull << ns) - 1ull;
      const unsigned long long cm0 = cones & sm, cm1 = (cones >> ns) & sm;
      const bool lit0 = litm & 1ull, lit1 = (litm >> 1) & 1ull;
      const bool occ0 = (blks & sm) != 0, occ1 = ((blks >> ns) & sm) != 0;
      const bool need0 = lit0 && !occ0 && h.soft, need1 = lit1 && !occ1 && h.soft;
      // soft rays: each light takes the first 16 accepted tries of its own
      // stream (spec v4; a light without soft rays draws nothing)
      int i16a = -1, i16b = -1;
      solo_take16(tr, i16a, i16b);
      const int e0 = need0 ? i16a : 0, e1 = need1 ? i16b : 0;
      SOLO_T(2);
      int un0 = 16, un1 = 16;
      if (e0 >= 0 && e1 >= 0) {
        int cnt0 = 0, cnt1 = 0;
#pragma unroll
        for (int half = 0; half < 2; ++half) {  // light 0 (stream a), then light 1 (stream b)
          if (half == 1 && !need1) break;
          if (half == 0 && !need0) continue;
          const bool acc = ((half ? tr.mb : tr.ma) >> lane) & 1ull;
          const bool in = lane < (half ? e1 : e0);
          const d3 lD = mk(__shfl(lvd.x, half), __shfl(lvd.y, half), __shfl(lvd.z, half));
          const double lT = __shfl(lvl, half);
          bool occ = false;
          if (acc && in) {
            const d3 pt = half ? unit_ball_point(tr.b0, tr.b1, tr.b2) : unit_ball_point(tr.a0, tr.a1, tr.a2);
            const d3 sd = normalize(lD + muls(pt, 0.1));
            const double a = len2(sd);
            const double ia = approx_rcp(a);
            // (every candidate, no early exit: their loads issue together)
            for (unsigned long long b = half ? cm1 : cm0; b; b &= b - 1) {
              double num;
              occ = (sphere_query(g.spheres[__builtin_ctzll(b)], P, sd, a, ia, 0.001, lT, num) != 0) || occ;
            }
          }
          (half ? cnt1 : cnt0) = __popcll(__ballot(acc && in && !occ));
          if (half == 0) SOLO_S(12);
        }
        SOLO_S(13);
        un0 = cnt0;
        un1 = cnt1;
      } else {
        // (64 tries of a stream did not hold 16 points: that light's soft
        // rays cooperatively from its stream, as below)
        for (int li = 0; li < 2; ++li) {
          if (!(li ? need1 : need0)) continue;
          const Cand cl{li ? cm1 : cm0, 0ull};
          const CoopOut r = soft_coop<false>(g, true, cl.s != 0, P, rl3(lvd, li), rld(lvl, li), cl,
                                             rt_soft_state(skey, (uint32_t)depth, (uint32_t)li), h.jump, stack, c);
          (li ? un1 : un0) = r.unocc;
        }
      }
      SOLO_T(3);
      // the lighting terms of light lane (< nl), then D in light order
      d3 tdif = mk(0, 0, 0), tspec = mk(0, 0, 0);
      if (lane < nl) {
        const bool occ = lane ? occ1 : occ0;
        const int un = lane ? un1 : un0;
        const double sf = occ ? 0.0 : (h.soft ? (double)un / 16.0 : 1.0);  // shadowSum / 16
        tdif = muls(ld3(m->albedo), di * sf);
        if (metallic > 0.5) tspec = muls(ld3(h.lights[lane].color), sii * sf * metallic * 3.0);
      }
      SOLO_S(14);
#pragma unroll
      for (int li = 0; li < 2; ++li) {
        if (li >= nl) break;
        const bool lit = li ? lit1 : lit0, occ = li ? occ1 : occ0;
        const int un = li ? un1 : un0;
        const double sf = occ ? 0.0 : (h.soft ? (double)un / 16.0 : 1.0);
        if (lit && sf > 0.0) {
          D = D + rl3(tdif, li);
          if (metallic > 0.5) D = D + rl3(tspec, li);
        }
      }
      SOLO_T(4);
    } else
    for (int li = 0; li < h.nl; ++li) {
      const DLight& Lt = h.lights[li];
      const d3 lv = ld3(Lt.pos) - P;
      const double ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
      const d3 ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
      if (ldist < 0.001) continue;  // renderer.go:252-254
      // the shadow cone's candidates, one primitive per lane (cone_candidates)
      const bool leaves = dot(N, ldir) >= KC(0.1015);
      bool cs = false, cb = false;
      if (lane < g.ns) {
        const DSphere& S = g.spheres[lane];
        cs = !(front && leaves && S.obj == self && S.r > 0) && in_cone(S.c, S.r, P, ldir, ldist);
      }
      if (lane < g.nb) {  // (nb <= 5: 12 triangles per cube)
        const DBox& B = g.boxes[lane];
        cb = !(leaves && B.obj == self && box_self_out(B, front)) && in_cone(B.bc, B.br, P, ldir, ldist);
      }
      Cand cm{__ballot(cs), 0ull};
      for (unsigned long long b = __ballot(cb); b; b &= b - 1) cm.t |= 0xFFFull << g.boxes[__builtin_ctzll(b)].first;
      // the hard shadow ray (renderer.go:305), the candidates in parallel
      bool blk = false;
      if ((cm.s >> lane) & 1ull) {
        const double a = len2(ldir);
        double num;
        blk = sphere_query(g.spheres[lane], P, ldir, a, approx_rcp(a), 0.001, ldist, num) != 0;
      }
      if ((cm.t >> lane) & 1ull) {
        double t, u, v;
        blk = blk || tri_test(g.tris[lane], P, ldir, 0.001, ldist, t, u, v);
      }
      const bool occl = __ballot(blk) != 0;
      int unocc = 0;
      if (!occl && h.soft) {
        // the 16 soft rays (renderer.go:311-327), not traced for an inert light
        const bool trace = (cm.s | cm.t) != 0 && !light_inert(m, Lt, N, ldir, D);
        // (spec v4: the points come from the light's own stream; rays that
        // cannot be blocked need none of them)
        if (trace) {
          const CoopOut r = soft_coop<false>(g, true, true, P, ldir, ldist, cm,
                                             rt_soft_state(skey, (uint32_t)depth, (uint32_t)li), h.jump, stack, c);
          unocc = r.unocc;
        } else {
          unocc = 16;
        }
      }
      const double sf = occl ? 0.0 : (h.soft ? (double)unocc / 16.0 : 1.0);  // shadowSum / 16
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
    // (3) Material.Scatter and the traceRay combination (renderer.go:181-226)
    const d3 E = ld3(m->emit);
    const Scat sc = scatter<false>(m, d, N, front, rng, c);
    SOLO_T(5);
    if (!sc.ok) {
      if (dep_out) *dep_out = depth + 1;
      return L + mul(T, E + D);
    }
    L = L + mul(T, E + muls(D, m->dw));
    if (!h.recursive || depth + 1 >= h.max_depth) {
      if (dep_out) *dep_out = depth + 1;
      return L;
    }
    T = mul(T, muls(sc.A, m->rw));
    o = P;
    d = sc.nd;
    depth += 1;
  }
}

// Render kernel: one wave (64 lanes) per block, three phases.  A one-wave
// workgroup needs no barriers and leaves the CU as soon as its own work is
// done (4-wave workgroups held their slots until their slowest wave ended).
//   1 VISIBILITY - the lanes generate the block's NB camera rays (NB/64
//       each) and ask only "does it hit anything?" (an any-hit query over
//       [0.001, +inf), with the tile's frustum candidates).  A miss is black
//       (renderer.go:170-173) and is finished; a hit sets the sample's bit.
//       At 800x600x100 97% of the camera rays end here.
//   2 SHADE - the hit samples, ascending, form a list that the wave drains
//       through a ring of kRound LDS radiance slots: a lane without a path
//       takes the next entry, rebuilds its camera ray and runs the path
//       (traceRay, renderer.go:165-227, unrolled: closest hit, direct
//       lighting with hard + soft shadows, scatter) to its end, storing the
//       radiance in the entry's slot.  Shading runs on dense waves instead
//       of on the ~3% of lanes whose camera ray hit.  Soft shadows of the
//       few paths still running at the end run cooperatively (soft_coop).
//   3 RESOLVE - whenever the ring is full, every pixel adds the finished
//       entries before the earliest running path to its running sum, in
//       sample order (misses add +0: the same sum as tracePixel,
//       renderer.go:150-163, bit for bit); at the end the sum is divided by
//       spp, tone-mapped (renderer.go:348-367) and written once (float3
//       linear + RGBA8).
constexpr int kRound = 128;  // list entries shaded per round (LDS radiance slots)
// second closest-hit pass of a shade iteration (render_kernel): taken when at
// least this many lanes are free after the first (0: never).  Measured (r05,
// K = 100 throughput, two rounds each): never 148.8 k, 4 155.6 k, 8 156.2 k,
// 16 157.5 k Mrays/s; one frame at a time unchanged (0.74-0.75 ms)
#ifndef RT_REFILL2_MIN
#define RT_REFILL2_MIN 16
#endif
constexpr int kRefill2Min = RT_REFILL2_MIN;

// ---- tail helpers (TailCtl in rt_internal.h)
// Device-scope hand-offs on MI355X (MI355X_MICROARCH.md, inter-workgroup
// visibility): the 8 XCDs' L2 caches are not coherent with each other, and an
// agent-scope release fence writes back the whole XCD L2's dirty lines
// (buffer_wbl2: microseconds, and tens of them when many waves fence at
// once).  The tail protocol hands its data over WITHOUT fences, in the
// guide's "8-B agent atomics both sides" form: every byte a helper or a
// block hands over (a queued path, a row's samples, bits and header) is
// stored write-through with relaxed agent-scope atomic stores (st_wt*, sc1),
// the storing wave drains them (s_waitcnt vmcnt(0)), and only then stores
// the flag or adds to the counter that signals them; the consumer polls the
// flag or takes the counter's returned value and reads every handed-over
// byte with relaxed agent-scope atomic loads (ld_wt*, sc1).  Counters that
// every block touches are sharded (TailCtl.done), and the export's gate
// reads before it adds.  (Measured on the headline frame: a __threadfence
// at every block's end, or 2 atomics per draining iteration on one line,
// made the launch 2-3x slower.)
__device__ __forceinline__ unsigned int ld_rlx(const unsigned int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void st_wt64(void* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt32(void* p, uint32_t v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wtd(double* p, double v) { st_wt64(p, __builtin_bit_cast(uint64_t, v)); }
__device__ __forceinline__ uint64_t ld_wt64(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_wt32(const void* p) {
  return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wtd(const double* p) { return __builtin_bit_cast(double, ld_wt64(p)); }
// One pixel's mean, tone map (renderer.go:348-367) and write, as the epilogue
// writes it: sum / spp (DivScalar(float64(samples))), float3 + RGBA8.
__device__ __forceinline__ void store_pixel(KArg k, int fr, size_t oi, double sx, double sy, double sz) {
  const double n = (double)k->spp_total;
  const double mx = sx / n, my = sy / n, mz = sz / n;
  float* const ol = k->frame_lin[fr];
  uint8_t* const orgba = k->frame_rgba[fr];
  if (ol) {
    ol[oi * 3 + 0] = (float)mx;
    ol[oi * 3 + 1] = (float)my;
    ol[oi * 3 + 2] = (float)mz;
  }
  if (orgba) *reinterpret_cast<uint32_t*>(orgba + oi * 4) = tonemap_rgba8(mx, my, mz);
}
// Samples [k0, n) of a per-sample radiance row added to `a` (lanes 0..2:
// channel `lane`) in sample order, a sample whose hit bit is clear adding +0
// (a miss: traceRay's black, renderer.go:170-173, summed as tracePixel sums,
// renderer.go:150-163).  The whole wave loads each chunk of kRound samples
// into `buf` (LDS); lanes 0..2 then add it in order.
// (kWT: the row was handed over write-through: every load of it is sc1)
template <bool kWT>
__device__ __forceinline__ double row_sum(double (*buf)[3], const double* row, const uint32_t* hw, int k0, int n,
                                          double a, int lane) {
  for (int c0 = k0; c0 < n; c0 += kRound) {
    const int cn = min(kRound, n - c0);
    for (int i = lane; i < cn; i += 64) {
      const int s = c0 + i;
      const bool hit = ((kWT ? ld_wt32(hw + (s >> 5)) : hw[s >> 5]) >> (s & 31)) & 1u;
      buf[i][0] = hit ? (kWT ? ld_wtd(row + 3 * s + 0) : row[3 * s + 0]) : 0.0;
      buf[i][1] = hit ? (kWT ? ld_wtd(row + 3 * s + 1) : row[3 * s + 1]) : 0.0;
      buf[i][2] = hit ? (kWT ? ld_wtd(row + 3 * s + 2) : row[3 * s + 2]) : 0.0;
    }
    __syncthreads();
    if (lane < 3)
      for (int i = 0; i < cn; ++i) a += buf[i][lane];
    __syncthreads();
  }
  return a;
}

// A tail helper: one of the one-wave workgroups past the grid's main blocks.
// It takes exported paths off the queue and runs each to its end with the
// whole wave (solo_path), delivers its radiance to the row of its pixel and,
// when it is the pixel's last contributor, sums the row and writes the
// pixel.  It leaves once every main block has finished and the queue is
// empty (main blocks never wait for a helper, so that always comes); the last
// helper to leave zeroes the control block for the context's next launch.
__device__ __forceinline__ void tail_helper(KArg karg, int* stack, double (*buf)[3]) {
  const int lane = (int)(threadIdx.x & 63);
  const KArg k0 = launder(karg);
  TailCtl* const ctl = k0->tail;
  const unsigned int epoch = k0->tail_epoch, cap = (unsigned int)k0->tail_cap, main_wgs = (unsigned int)k0->num_wgs;
  if (lane == 0) atomicAdd(ctl->gate, 1ull << 32);  // one more helper
  const unsigned long long t_born = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_idle = t_born;
  int polls = 0;
#ifdef RT_WG_TIMING
  unsigned long long dbg_first = 0, dbg_paths = 0, dbg_solo = 0, dbg_last = 0, dbg_last_d0 = 0, dbg_last_d1 = 0,
                     dbg_bounces = 0;
#endif
  for (;;) {
    int idx = -1;
    if (lane == 0) {
      for (;;) {
        const unsigned int t = min(ld_rlx(ctl->tail), cap), h = ld_rlx(ctl->head);
        if (h >= t) break;
        if (atomicCAS(ctl->head, h, h + 1u) == h) {
          idx = (int)h;
          break;
        }
      }
    }
    idx = __builtin_amdgcn_readfirstlane(idx);
    if (idx < 0) {
      // every main block finished (the sharded counters, one per lane; read
      // every 32nd idle poll)?  Then nothing more can be queued: leave once
      // the queue is empty
      if ((++polls & 31) == 0) {
        unsigned int dn = lane < kTailShards ? ld_rlx(&ctl->done[lane * 32]) : 0u;
        for (int off = 32; off >= 1; off >>= 1) dn += __shfl_xor(dn, off);
        if (__builtin_amdgcn_readfirstlane(dn) >= main_wgs) {
          const unsigned int h = ld_rlx(ctl->head), t = min(ld_rlx(ctl->tail), cap);
          if (__builtin_amdgcn_readfirstlane(h >= t ? 1 : 0)) break;
          continue;
        }
      }
      // (a bound that is never expected to bite: main blocks are at most a
      // 1024-sample block each; a stuck helper must not hang the device)
      if (__builtin_amdgcn_s_memrealtime() - t_idle > 1000000000ull) {  // 10 s at 100 MHz
        if (lane == 0) atomicOr(&ctl->err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(96);  // (~2.6 us between polls: idle helpers must not crowd the lines they poll)
      continue;
    }
    // the entry was reserved by a block that writes it at once
    bool ready = true;
    for (const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
         __hip_atomic_load(&k0->tail_ready[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch;) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 1000000000ull) {  // (never expected: 10 s)
        ready = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!__builtin_amdgcn_readfirstlane(ready ? 1 : 0)) {
      if (lane == 0) atomicOr(&ctl->err, 2u);
      break;
    }
    // the record: written through by its exporter, drained before the flag
    const unsigned long long t_path = __builtin_amdgcn_s_memrealtime();
    const TailPath* q = k0->tail_q + idx;
    const d3 o = mk(ld_wtd(q->o), ld_wtd(q->o + 1), ld_wtd(q->o + 2)), d = mk(ld_wtd(q->d), ld_wtd(q->d + 1), ld_wtd(q->d + 2));
    const d3 T = mk(ld_wtd(q->T), ld_wtd(q->T + 1), ld_wtd(q->T + 2)), L0 = mk(ld_wtd(q->L), ld_wtd(q->L + 1), ld_wtd(q->L + 2));
    const uint64_t rx = ld_wt64(&q->rng), sk = ld_wt64(&q->skey);
    const int depth = (int)ld_wt32(&q->depth), sample = (int)ld_wt32(&q->sample), kind = (int)ld_wt32(&q->kind),
              row = (int)ld_wt32(&q->row), nsub = (int)ld_wt32(&q->nsub), fr = (int)ld_wt32(&q->frame);
    const int64_t oi = (int64_t)ld_wt64(&q->oi);
    int dep_end = depth;
    const d3 L = solo_path<false>(karg, 0, o, d, T, L0, rx, depth, sk, stack, &dep_end);
    const KArg k = launder(karg);
#ifdef RT_WG_TIMING
    if (!dbg_first) dbg_first = t_path;
    dbg_paths += 1;
    dbg_solo += __builtin_amdgcn_s_memrealtime() - t_path;
    dbg_last = t_path;
    dbg_last_d0 = (unsigned long long)depth;
    dbg_last_d1 = (unsigned long long)dep_end;
    dbg_bounces += (unsigned long long)(dep_end - depth);
#endif
    const int spp = k->spp_total, bw = (spp + 31) >> 5;
    int last = 0;
    if (lane == 0) {
      atomicAdd(&ctl->solo_ticks, (unsigned int)(__builtin_amdgcn_s_memrealtime() - t_path));
      atomicAdd(&ctl->paths_done, 1u);
      // the sample, written through and drained before the counter
      if (kind == kTailRow) {
        double* r = k->tail_rows + ((size_t)row * spp + sample) * 3;
        st_wtd(r, L.x);
        st_wtd(r + 1, L.y);
        st_wtd(r + 2, L.z);
        atomicOr(k->tail_bits + (size_t)row * bw + (sample >> 5), 1u << (sample & 31));
        wt_drain();
        last = atomicSub(&k->tail_hdr[row].counter, 1) == 1 ? 1 : 0;
      } else {
        double* r = k->split_rad + ((size_t)row * spp + sample) * 3;
        st_wtd(r, L.x);
        st_wtd(r + 1, L.y);
        st_wtd(r + 2, L.z);
        atomicOr(k->split_hits + (size_t)row * bw + (sample >> 5), 1u << (sample & 31));
        wt_drain();
        last = atomicAdd(&k->split_cnt[row], 1) == nsub - 1 ? 1 : 0;
      }
      atomicAdd(ctl->gate, ~0ull);  // one exported path fewer in flight (-1 on the low half)
    }
    last = __builtin_amdgcn_readfirstlane(last);
    if (last) {
      // the pixel's last contributor: its row in sample order, then the pixel
      // (every byte of the row read sc1: written through or by atomics)
      double a;
      int pfr = fr;
      size_t poi = (size_t)oi;
      if (kind == kTailRow) {
        const TailRow* hd = k->tail_hdr + row;
        a = lane < 3 ? ld_wtd(hd->prefix + lane) : 0.0;
        a = row_sum<true>(buf, k->tail_rows + (size_t)row * spp * 3, k->tail_bits + (size_t)row * bw,
                          (int)ld_wt32(&hd->k0), spp, a, lane);
        pfr = (int)ld_wt32(&hd->frame);
        poi = (size_t)ld_wt64(&hd->oi);
      } else {
        uint32_t* hw = k->split_hits + (size_t)row * bw;
        a = row_sum<true>(buf, k->split_rad + (size_t)row * spp * 3, hw, 0, spp, 0.0, lane);
        // the slot's hit bits and counter are left zeroed for the next launch
        for (int i = lane; i < bw; i += 64) hw[i] = 0u;
        if (lane == 0) k->split_cnt[row] = 0;
      }
      const double sx = rld(a, 0), sy = rld(a, 1), sz = rld(a, 2);
      if (lane == 0) store_pixel(k, pfr, poi, sx, sy, sz);
    }
    t_idle = __builtin_amdgcn_s_memrealtime();
  }
  int gone = 0;
#ifdef RT_WG_TIMING
  if (k0->dbg && lane == 0) {  // a helper's record: start, first path, end, paths, their ticks; [14] = -1
    unsigned long long* r = k0->dbg + (size_t)blockIdx.x * kDbgStride;
    r[0] = t_born;
    r[1] = dbg_first;
    r[2] = __builtin_amdgcn_s_memrealtime();
    r[3] = dbg_solo;
    r[4] = dbg_last;     // the last path's start,
    r[5] = dbg_last_d0;  // its depth when exported,
    r[6] = dbg_last_d1;  // and at its end
    r[7] = dbg_paths;
    r[8] = dbg_bounces;
    r[14] = ~0ull;
  }
#endif
  if (lane == 0) {
    atomicAdd(&ctl->helper_ticks, (unsigned int)(__builtin_amdgcn_s_memrealtime() - t_born));
    atomicAdd(ctl->gate, ~0ull << 32);  // one helper fewer (-2^32)
    gone = (int)atomicAdd(ctl->helpers_gone, 1u);
  }
  if (__builtin_amdgcn_readfirstlane(gone) + 1 == k0->tail_helpers) {
    // every helper and every main block is done: ready for the next launch
    if (lane < kTailShards) ctl->done[lane * 32] = 0u;
    if (lane == 0) {
      ctl->tail[0] = 0;
      ctl->head[0] = 0;
      ctl->gate[0] = 0;
      ctl->rows_used[0] = 0;
      ctl->helpers_gone[0] = 0;
    }
  }
}

template <bool kCount, bool kStage, bool kPilot, bool kSky, bool kTailT>
__device__ __forceinline__ void render_body(const KParams& pk) {
  __shared__ uint32_t hbits[kMaxBlockSamples / 32];  // hit samples of the block
  __shared__ int hoff[kMaxBlockSamples / 32 + 1];    // list offset of each bit word; [words] = #hits
  __shared__ double slot[kRound][3];                 // radiance of the round's entries
  __shared__ double psum[64][3];                     // per pixel: running sum over samples
  __shared__ uint8_t lpix[64];                       // phase 1: the block's live pixels
  __shared__ uint64_t skey[64];                      // per lane: its path's soft-shadow key (rt_soft_key, spec v4)
  // dynamic LDS (dyn_lds): [staged scene prefix (kStage)][BVH stack (stack_depth x 64 ints)]
  // tail helpers: render_kernel_tail exports a block's last
  // few long paths to the helpers past its main blocks.  The product kernel
  // has none of that code (compiled in but unused it cost 2-3 % one frame,
  // 1.5 % batched: r06 A/B)
  constexpr bool kTail = kTailT && kStage && !kCount && !kPilot && !kSky;

  const int lane = threadIdx.x;
  int* stack = reinterpret_cast<int*>(dyn_lds + pk.stack_off) + lane;
  if constexpr (kTail) {
    if (pk.tail != nullptr && blockIdx.x - (unsigned)pk.tail_pos < (unsigned)pk.tail_helpers) {
      // a tail helper (launch_render adds them only with pk.tail set)
      const uint4* __restrict__ src = reinterpret_cast<const uint4*>(pk.stage_src);
      uint4* dst = reinterpret_cast<uint4*>(dyn_lds);
      for (int i = lane; i < pk.stage_bytes / 16; i += 64) dst[i] = src[i];
      __syncthreads();
      tail_helper(fresh(), stack, slot);
      return;
    }
  }
  // a row pixel (tail helpers): its dynamic row and first row sample (-1: none)
  __shared__ int prow[kTail ? 64 : 1];
  __shared__ short pk0[kTail ? 64 : 1];
  __shared__ uint32_t xm[kTail ? kRound / 32 : 1];  // ring slots whose path was exported
  if constexpr (kTail) {
    prow[lane] = -1;
    if (lane < kRound / 32) xm[lane] = 0u;
  }
  const BlockLoc blk = block_loc(fresh(), block_of(fresh()));
  // a black block (up to 64 pixels x spp samples) sets no hit bits
  const int nwords = blk.black ? 0 : (blk.np * blk.ns + 31) >> 5;
  if (lane < nwords) hbits[lane] = 0;
  {
    // a later sample pass continues each pixel's running sum (acc_mode bit 0)
    double a0 = 0, a1 = 0, a2 = 0;
    if ((pk.acc_mode & 1) && blk.slot < 0 && lane < blk.np && blk.p0 + lane < 1024) {
      const double* a = pk.acc + ((size_t)blk.lt * 1024 + blk.p0 + lane) * 3;
      a0 = a[0];
      a1 = a[1];
      a2 = a[2];
    }
    psum[lane][0] = a0;
    psum[lane][1] = a1;
    psum[lane][2] = a2;
  }
  if constexpr (kStage) {
    // LDS-staged scene primitives: spheres | triangles | boxes | materials |
    // lights [| jump table] (one contiguous prefix of the device scene buffer), so the
    // divergent per-lane reads of the shadow / scatter code hit LDS instead
    // of L1/L2 (measured: 55% of wave time in memory waits without it)
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(pk.stage_src);
    uint4* dst = reinterpret_cast<uint4*>(dyn_lds);
    for (int i = lane; i < pk.stage_bytes / 16; i += 64) dst[i] = src[i];
  }
  __syncthreads();

  Counters c, culled;
  if constexpr (kCount) {
    for (int i = 0; i < kCounters; ++i) c.v[i] = culled.v[i] = 0;
  }
#ifdef RT_WG_TIMING
  if (lane < 16) solo_clk[lane] = 0;
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long dbg_iter = 0;
  // wave-uniform section clocks (s_memtime): hit, lighting, soft; phase 1 (visibility)
  unsigned long long dbg_hit = 0, dbg_light = 0, dbg_soft = 0, dbg_vis = 0;
  // cone + hard shadow, scatter, lane-iterations alive, coop owners served, soft_seq passes
  unsigned long long dbg_hard = 0, dbg_scat = 0, dbg_alive = 0, dbg_coop = 0, dbg_seq = 0;
  // shade-iteration clocks and counts by live lanes: 1, 2, 3-4, 5-8, > 8
  unsigned long long dbg_bclk[5] = {0, 0, 0, 0, 0}, dbg_bcnt[5] = {0, 0, 0, 0, 0}, dbg_bts = 0;
  int dbg_bprev = -1;
  const unsigned long long tv0 = __builtin_amdgcn_s_memtime();
#endif
  const Cand all{~0ull, ~0ull};

  // ---- phase 1: visibility of the block's camera rays
  {
    // everything the loop needs is loaded once, before it (wave-uniform:
    // SGPRs); re-reading the kernarg segment inside the loop put scalar
    // load round trips on every iteration
    KArg k = fresh();
    const BlockLoc loc = block_loc(k, block_of(k));
    const int NB = loc.np * loc.ns, ns = loc.ns;
    // primary-ray frustum culling (host-computed per pixel, schedule.cpp):
    // only primitives whose bounding sphere meets the cone of a pixel's
    // camera rays can be hit by them.  A pixel with no candidate is black
    // (every sample misses, renderer.go:170-173, and adds +0): its samples
    // are not traced.  The others are tested against the union of the
    // block's pixel masks.  (The counting variant walks every sample, so the
    // path counts stay the reference's.)
    Cand prim = all;
    unsigned long long pxlive = loc.np >= 64 ? ~0ull : (1ull << loc.np) - 1ull;
    if (k->tile_masks) {
      prim = Cand{loc.ms, loc.mt};
      pxlive = loc.live;
    }
    // compact list of the live pixels (block-local indices)
    if (lane < loc.np && ((pxlive >> lane) & 1ull)) lpix[lanes_below(pxlive)] = (uint8_t)lane;
    __syncthreads();
    const int nlive = __popcll(pxlive);
    const CamK ck = cam_k(k);
    const int W = k->W, H = k->H;
    // traceRay's depth cut-off comes first: with max_depth <= 0 every sample is black
    const bool live = loc.tile < k->ntiles, trace = k->max_depth > 0;
    const int x0 = loc.tx * 32, y0 = loc.ty * 32, p0 = loc.p0, s0 = loc.s0, sbase = k->sample_base;
    const Hot h = hot<kStage>();
    // id / ns by a multiply-high with m = floor((2^32 - 1) / ns) + 1: exact
    // for id, ns < 2^16 (NB <= kMaxBlockSamples); ns == 1 has no 32-bit m
    const uint32_t mdiv = ns > 1 ? 0xFFFFFFFFu / (uint32_t)ns + 1u : 0u;
    // A black block's tile has empty primary masks: every camera ray misses
    // (renderer.go:170-173), every sample is +0, so nothing is traced.  The
    // counting variant still walks its samples for the path counts (its
    // queries have no candidates: no hit bit is ever set).
    const int NL = kCount ? NB : (loc.black ? 0 : nlive * ns);
    // with an opted-in sky a miss returns the sky (not +0): every camera
    // sample is shaded (no culling applies: the host disables the masks)
    constexpr bool sky = kSky;
    for (int j = lane; j < NL; j += 64) {
      // j -> (pixel, sample): every sample of the block (kCount) or of its
      // live pixels, in order
      const int pj = ns > 1 ? (int)__umulhi((uint32_t)j, mdiv) : j, sl = j - pj * ns;
      const int p = kCount ? pj : (int)lpix[pj], s = s0 + sl, id = p * ns + sl;
      const int tp = p0 + p;
      const int x = x0 + (tp & 31), y = y0 + (tp >> 5);
      // (kCount) this sample's counts; a sample the product never traces (a
      // black block, or a pixel without primary candidates) also goes to
      // `culled`, so the executed work is the difference (rt_counts.culled)
      Counters cs;
      if constexpr (kCount)
        for (int i = 0; i < kCounters; ++i) cs.v[i] = 0;
      [&] {
        if (tp >= 1024 || !live || x >= W || y >= H) return;
        cnt<kCount>(cs, C_CAM);
        rt_rng rng;
        d3 o, d;
        camera_ray_c<kCount>(ck, x, y, sbase + s, rng, o, d, cs);
        if (!trace) return;
        cnt<kCount>(cs, C_BOUNCE);
        // hit or miss is all this phase needs: an any-hit query over
        // [0.001, +inf) decides exactly what hitWorld's closest hit would
        const bool hit = sky || (h.masks ? any_hit_masked<kCount>(h.g, o, d, __builtin_inf(), prim, cs)
                                         : any_hit<kCount>(h.g, o, d, __builtin_inf(), stack, cs));
        if (hit) atomicOr(&hbits[id >> 5], 1u << (id & 31));
      }();
      if constexpr (kCount) {
        const bool traced = !loc.black && ((pxlive >> p) & 1ull);
        for (int i = 0; i < kCounters; ++i) {
          c.v[i] += cs.v[i];
          if (!traced) culled.v[i] += cs.v[i];
        }
      }
    }
  }
  __syncthreads();
  // ---- the hit list: ascending sample ids (the <= 32 bit words scanned across the wave)
  {
    const int cw = lane < nwords ? __popc(hbits[lane]) : 0;
    int incl = cw;  // inclusive scan over the wave (Hillis-Steele)
    for (int off = 1; off < 64; off <<= 1) {
      const int t = __shfl_up(incl, off);
      if (lane >= off) incl += t;
    }
    if (lane < nwords) hoff[lane] = incl - cw;
    if (lane == 63) hoff[nwords] = incl;
  }
  __syncthreads();
  const int nh = hoff[nwords];
  // sample id (pixel * ns + sample - s0) of hit-list entry e < nh: the bit
  // word holding it (the last word whose list offset is <= e, by binary
  // search over hoff), then the (e - offset)-th set bit of that word.  No
  // materialized list: its 2 KB of LDS cost occupancy.
  auto entry_id = [&](int e) -> int {
    int w = 0;
    for (int step = 16; step; step >>= 1)
      if (w + step < nwords && hoff[w + step] <= e) w += step;
    uint32_t word = hbits[w];
    int k = e - hoff[w], pos = 0;
    for (int sh = 16; sh; sh >>= 1) {
      const int n = __popc(word & ((1u << sh) - 1u));
      if (k >= n) {
        k -= n;
        word >>= sh;
        pos += sh;
      }
    }
    return w * 32 + pos;
  };
#ifdef RT_WG_TIMING
  dbg_vis = __builtin_amdgcn_s_memtime() - tv0;
#endif

  // ---- phases 2 + 3: shade the hit list through a RING of kRound radiance
  // slots (entry e -> slot e % kRound).  Paths finish out of order; the
  // per-pixel sums are taken in entry order (= sample order) by
  // resolve_entries once every entry before the earliest path still running
  // has finished.  A long path therefore holds only its own slot: the other
  // lanes keep taking entries until the ring is full (a barrier per batch of
  // kRound entries made every batch wait for its longest path).
  static_assert((kRound & (kRound - 1)) == 0, "kRound must be a power of two");
  // adds entries [a, b) (all finished) to their pixels' sums in order; a
  // split pixel's block stores them in its radiance slot row instead
  auto resolve_entries = [&](int a, int b) {
    // the lane id laundered through a volatile move: keeps this rarely run
    // code's lane-dependent addresses from being hoisted out of the shading
    // loop (they would occupy registers, or scratch, for the whole loop)
    int lane;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"((int)threadIdx.x));
    if (blk.slot >= 0) {
      KArg k = fresh();
      double* row = k->split_rad + split_index(k, blk.slot) * k->spp * 3;
      uint32_t* hw = k->split_hits + split_index(k, blk.slot) * ((k->spp + 31) >> 5);
      for (int e = a + lane; e < b; e += 64) {
        const int s = blk.s0 + entry_id(e);  // one pixel: id = sample - s0
        const int q = e & (kRound - 1);
        if constexpr (kTail) {
          if ((xm[q >> 5] >> (q & 31)) & 1u) continue;  // exported: its helper writes the sample
        }
        if constexpr (kTail) {  // (written through: read sc1 by the pixel's last contributor, maybe a helper)
          st_wtd(row + 3 * s + 0, slot[q][0]);
          st_wtd(row + 3 * s + 1, slot[q][1]);
          st_wtd(row + 3 * s + 2, slot[q][2]);
        } else {  // (combined in L2, written back by the release fence below)
          row[3 * s + 0] = slot[q][0];
          row[3 * s + 1] = slot[q][1];
          row[3 * s + 2] = slot[q][2];
        }
        atomicOr(hw + (s >> 5), 1u << (s & 31));
      }
    } else {
      const int P = blk.np, spp = blk.ns;
      if (lane < P) {
        const int a0 = lane * spp, a1 = a0 + spp;
        int e0 = hoff[a0 >> 5] + __popc(hbits[a0 >> 5] & ((1u << (a0 & 31)) - 1u));
        int e1 = (a1 >> 5) < nwords ? hoff[a1 >> 5] + __popc(hbits[a1 >> 5] & ((1u << (a1 & 31)) - 1u)) : nh;
        e0 = max(e0, a);
        e1 = min(e1, b);
        bool rowed = false;
        if constexpr (kTail) rowed = prow[lane] >= 0;
        if (rowed) {
          // a pixel with exported paths (tail helpers): samples before its
          // first exported one go to its running sum as below, the later
          // ones (the exported ones aside: their helpers write them) to its
          // row, which the pixel's last contributor sums in order
          KArg k = fresh();
          const int r = prow[lane], k0 = pk0[lane], bw = (k->spp_total + 31) >> 5;
          double* row = k->tail_rows + (size_t)r * k->spp_total * 3;
          uint32_t* hw = k->tail_bits + (size_t)r * bw;
          double ax = psum[lane][0], ay = psum[lane][1], az = psum[lane][2];
          for (int e = e0; e < e1; ++e) {
            const int q = e & (kRound - 1);
            if ((xm[q >> 5] >> (q & 31)) & 1u) continue;
            const int sl = entry_id(e) - a0;
            if (sl < k0) {
              ax += slot[q][0];
              ay += slot[q][1];
              az += slot[q][2];
            } else {  // (written through: the row's last contributor reads it sc1)
              st_wtd(row + 3 * sl + 0, slot[q][0]);
              st_wtd(row + 3 * sl + 1, slot[q][1]);
              st_wtd(row + 3 * sl + 2, slot[q][2]);
              atomicOr(hw + (sl >> 5), 1u << (sl & 31));
            }
          }
          psum[lane][0] = ax;
          psum[lane][1] = ay;
          psum[lane][2] = az;
        } else if (e0 < e1) {
          double ax = psum[lane][0], ay = psum[lane][1], az = psum[lane][2];
          for (int e = e0; e < e1; ++e) {
            const int q = e & (kRound - 1);
            ax += slot[q][0];
            ay += slot[q][1];
            az += slot[q][2];
          }
          psum[lane][0] = ax;
          psum[lane][1] = ay;
          psum[lane][2] = az;
        }
      }
    }
  };
  if (nh > 0) {
    d3 o = mk(0, 0, 0), d = mk(0, 0, 0), T = mk(1, 1, 1);
    rt_rng rng{0};
    int depth = 0, entry = 0;
    bool alive = false;
    int next = 0, resolved = 0;  // wave-uniform: next entry to start; entries [0, resolved) summed
    int drain_it = 0;            // (tail helpers) iterations since every entry started
    // The path's radiance L lives in its entry's ring slot (the slot is the
    // path's own until it finishes, and resolve_entries reads it only then):
    // read and written once per bounce, in VGPRs it held 6 registers through
    // the lighting section and pushed the loop into scratch spills
    // (scratch 40 -> 28 B/lane; headline 0.79 -> 0.775 ms).  Macros: the
    // same accessors as lambdas came out with 40 B/lane of scratch again.
#define path_L() mk(slot[entry & (kRound - 1)][0], slot[entry & (kRound - 1)][1], slot[entry & (kRound - 1)][2])
#define set_path_L(v)                    \
  do {                                   \
    const d3 v_ = (v);                   \
    const int q_ = entry & (kRound - 1); \
    slot[q_][0] = v_.x;                  \
    slot[q_][1] = v_.y;                  \
    slot[q_][2] = v_.z;                  \
  } while (0)
    for (;;) {
      // (1) closest hit (hitWorld, renderer.go:170), in up to two passes: a
      // lane whose ray missed (or reached the depth cut-off) finishes at once
      // and, while other lanes go on to light their hits, takes the next
      // entry (its camera ray hits: phase 1 found a hit for it) and runs that
      // closest hit in a second pass -- so lighting and scatter, the bulk of
      // an iteration, run on the lanes of both passes' hits instead of
      // idling every lane whose ray missed (57 % of the headline's traced
      // rays hit: the lighting used to run on ~60 % of the lanes)
      bool shade = false, front = false, fin = false;
      d3 P = mk(0, 0, 0), N = mk(0, 0, 0);
      int mi = 0, self = -1;
      HitSel hs;
      int outer = 0;  // 1: continue the shade loop, 2: leave it
#ifdef RT_WG_TIMING
      unsigned long long ts0 = 0;
#endif
      for (int pass = 0;; ++pass) {
        const unsigned long long freem = __ballot(!alive);
        int limit = min(nh, resolved + kRound);
        if (freem != 0 && next == limit && next < nh) {
          // the ring is full and lanes are idle: sum every entry before the
          // earliest one still running (a wave-wide min over the live lanes)
          // (swizzles within each half-wave, then the two halves' lane 0)
          int lo = alive ? entry : next;
          lo = min(lo, __builtin_amdgcn_ds_swizzle(lo, 0x1F | (16 << 10)));
          lo = min(lo, __builtin_amdgcn_ds_swizzle(lo, 0x1F | (8 << 10)));
          lo = min(lo, __builtin_amdgcn_ds_swizzle(lo, 0x1F | (4 << 10)));
          lo = min(lo, __builtin_amdgcn_ds_swizzle(lo, 0x1F | (2 << 10)));
          lo = min(lo, __builtin_amdgcn_ds_swizzle(lo, 0x1F | (1 << 10)));
          lo = min(__builtin_amdgcn_readlane(lo, 0), __builtin_amdgcn_readlane(lo, 32));
          if (lo > resolved) {
            __syncthreads();
            resolve_entries(resolved, lo);
            __syncthreads();
            if constexpr (kTail) {
              // the resolved entries' ring slots take new entries now: their
              // exported marks go (slot s is in [resolved, lo) mod kRound iff
              // (s - resolved) mod kRound < lo - resolved)
              if (lane < kRound / 32) {
                uint32_t m = 0;
                for (int j = 0; j < 32; ++j)
                  m |= (uint32_t)(((32 * lane + j - resolved) & (kRound - 1)) < lo - resolved) << j;
                xm[lane] &= ~m;
              }
            }
            resolved = lo;
            limit = min(nh, resolved + kRound);
          }
        }
        // lanes without a path take the next entries, in lane order
        const int e = next + lanes_below(freem);
        if (!alive && e < limit) {
          KArg k = fresh();
          const BlockLoc loc = block_loc(k, block_of(k));
          const int id = entry_id(e), ns = loc.ns;
          const int p = id / ns, s = k->sample_base + loc.s0 + id - p * ns;
          const int tp = loc.p0 + p;
          Counters nc;  // phase 1 counted this camera ray and its draws
          const int px = loc.tx * 32 + (tp & 31), py = loc.ty * 32 + (tp >> 5);
          camera_ray<false>(k, px, py, s, rng, o, d, nc);
          skey[lane_now()] = rt_soft_key(k->frame_key[frame_of(k)], (uint32_t)py * (uint32_t)k->W + (uint32_t)px, (uint32_t)s);
          entry = e;
          T = mk(1, 1, 1);
          set_path_L(mk(0, 0, 0));
          depth = 0;
          alive = true;
        }
        next = min(limit, next + __popcll(freem));
        if (pass == 0) {
          if (__ballot(alive) == 0) {  // wave-uniform
            outer = next >= nh ? 2 : 1;  // every entry done / ring full of finished entries: resolve, then refill
            break;
          }
#ifdef RT_WG_TIMING
          ++dbg_iter;
          dbg_alive += __popcll(__ballot(alive));
          {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            if (dbg_bprev >= 0) dbg_bclk[dbg_bprev] += now - dbg_bts;
            const int nal = __popcll(__ballot(alive));
            dbg_bprev = nal == 1 ? 0 : (nal == 2 ? 1 : (nal <= 4 ? 2 : (nal <= 8 ? 3 : 4)));
            dbg_bcnt[dbg_bprev] += 1;
            dbg_bts = now;
          }
          if (dbg_iter % 4 == 0 && dbg_iter / 4 < 16 && lane == 0 && fresh()->dbg)
            fresh()->dbg[(size_t)blockIdx.x * kDbgStride + 16 + dbg_iter / 4] = __builtin_amdgcn_s_memrealtime();
          ts0 = __builtin_amdgcn_s_memtime();
#endif
          if constexpr (kTail) {
            // Tail helpers: every entry has started and at
            // most tail_kmax paths are left, each tail_dmin bounces deep or
            // more -- the block's drain.  Each goes to a helper wave (while
            // one is free), which runs it alone at solo latency; its radiance
            // reaches the pixel through the pixel's row (resolve_entries, the
            // epilogue), the same sum in the same order.
            // (every tail_every-th iteration of the drain, 4 by default: the gate read is a memory round
            // trip on the lone paths' chain, and a drain shorter than that
            // gains nothing from a helper)
            // The block's drain: every entry has started.  (Exporting at ring
            // stalls too -- the ring full behind a long path, whose export lets
            // the lanes take new entries -- measured slower: one frame 0.555 ->
            // 0.620 ms at 64 helpers; more, shorter paths queue for the helpers
            // ahead of the long ones.  The resolve below supports it: rows are
            // filled mid-loop and exported ring slots are unmarked on reuse.)
            if (next >= nh && (++drain_it & fresh()->tail_every_mask) == 0 && fresh()->tail != nullptr) {
              const unsigned long long am = __ballot(alive);
              if (__popcll(am) <= fresh()->tail_kmax) {
                for (unsigned long long em = __ballot(alive && depth >= fresh()->tail_dmin); em; em &= em - 1) {
                  const int ow = __builtin_ctzll(em);
                  const unsigned long long t_x = __builtin_amdgcn_s_memrealtime();
                  KArg k = fresh();
                  TailCtl* ctl = k->tail;
                  int idx = -1;
                  // a helper for it (paths in flight < live helpers: the gate word is
                  // read first, so draining waves do not add to it in vain) and a
                  // queue entry
                  if (lane == 0) {
                    const unsigned long long g0 = __hip_atomic_load(ctl->gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)g0 < (uint32_t)(g0 >> 32)) {
                      const unsigned long long g = atomicAdd(ctl->gate, 1ull);
                      if ((uint32_t)g < (uint32_t)(g >> 32)) {
                        const unsigned int t = atomicAdd(ctl->tail, 1u);
                        if (t < (unsigned int)k->tail_cap) idx = (int)t;  // (entries past the cap are never taken)
                      }
                      if (idx < 0) atomicAdd(ctl->gate, ~0ull);
                    }
                  }
                  idx = __builtin_amdgcn_readfirstlane(idx);
                  // (all the handed-over bytes below are written through: st_wt*)
                  if (idx < 0) break;  // (no helper free: the paths stay here)
                  const int e = (int)rl32((uint32_t)entry, ow);
                  const BlockLoc loc = block_loc(k, block_of(k));
                  const int id = entry_id(e), ns = loc.ns;
                  const int p = id / ns, sl = id - p * ns;
                  const int tp = loc.p0 + p;
                  const int px = loc.tx * 32 + (tp & 31), py = loc.ty * 32 + (tp >> 5);
                  const int64_t oi = k->layout == RT_LAYOUT_IMAGE ? (int64_t)py * k->W + px
                                                                  : (int64_t)loc.lt * 1024 + tp;
                  int kind, row, sample;
                  if (loc.slot >= 0) {  // a split pixel: its split row (its counter owes one more finisher)
                    kind = kTailSplit;
                    row = (int)split_index(k, loc.slot);
                    sample = loc.s0 + sl;
                    if (lane == 0) atomicSub(&k->split_cnt[row], 1);
                  } else {
                    kind = kTailRow;
                    sample = sl;
                    int r = prow[p];
                    if (r < 0) {  // the pixel's dynamic row (one row per export at most: rows_used < cap)
                      if (lane == 0) r = (int)atomicAdd(ctl->rows_used, 1u);
                      r = __builtin_amdgcn_readfirstlane(r);
                      const int bw = (k->spp_total + 31) >> 5;
                      for (int w = lane; w < bw; w += 64) st_wt32(k->tail_bits + (size_t)r * bw + w, 0u);
                      if (lane == 0) {
                        TailRow* hd = k->tail_hdr + r;
                        st_wt32(&hd->counter, 2u);  // the block's own share (given back in its epilogue) + this path
                        st_wt32(&hd->k0, (uint32_t)sl);
                        st_wt32(&hd->frame, (uint32_t)frame_of(k));
                        st_wt64(&hd->oi, (uint64_t)oi);
                        prow[p] = r;
                        pk0[p] = (short)sl;
                      }
                    } else if (lane == 0) {
                      pk0[p] = (short)min((int)pk0[p], sl);
                      atomicAdd(&k->tail_hdr[r].counter, 1);  // one more path owes the row a sample
                    }
                    row = r;
                  }
                  if (lane == ow) {
                    TailPath* q = k->tail_q + idx;
                    const int qs = e & (kRound - 1);
                    st_wtd(q->o, o.x); st_wtd(q->o + 1, o.y); st_wtd(q->o + 2, o.z);
                    st_wtd(q->d, d.x); st_wtd(q->d + 1, d.y); st_wtd(q->d + 2, d.z);
                    st_wtd(q->T, T.x); st_wtd(q->T + 1, T.y); st_wtd(q->T + 2, T.z);
                    st_wtd(q->L, slot[qs][0]); st_wtd(q->L + 1, slot[qs][1]); st_wtd(q->L + 2, slot[qs][2]);
                    st_wt64(&q->rng, rng.x);
                    st_wt64(&q->skey, skey[ow]);
                    st_wt32(&q->depth, (uint32_t)depth);
                    st_wt32(&q->sample, (uint32_t)sample);
                    st_wt32(&q->kind, (uint32_t)kind);
                    st_wt32(&q->row, (uint32_t)row);
                    st_wt32(&q->nsub, (uint32_t)loc.nsub);
                    st_wt32(&q->frame, (uint32_t)frame_of(k));
                    st_wt64(&q->oi, (uint64_t)oi);
                    alive = false;
                  }
                  if (lane == 0) {
                    const int qs = e & (kRound - 1);
                    xm[qs >> 5] |= 1u << (qs & 31);
                    atomicAdd(&ctl->exported, 1u);
                  }
                  wt_drain();  // every lane's write-through stores, then the flag
                  if (lane == ow) __hip_atomic_store(&k->tail_ready[idx], k->tail_epoch, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                  if (lane == 0) atomicAdd(&ctl->export_ticks, (unsigned int)(__builtin_amdgcn_s_memrealtime() - t_x));
                }
                if (__ballot(alive) == 0) {  // every path left went to a helper
                  outer = next >= nh ? 2 : 1;  // done / the ring moves on: resolve, then refill
                  break;
                }
              }
            }
          }
          if constexpr (kStage && !kCount && !kPilot && RT_SOLO) {
            // one path left (no free lane found an entry to start): the whole
            // wave runs it to its end (solo_path)
            const unsigned long long am = __ballot(alive);
            // (two or three paths run one after the other this way measured
            // slower: 0.79 / 0.93 vs 0.78 ms)
            if (__popcll(am) == 1 && hot<kStage>().masks) {
              const d3 Lr = solo_path<kSky>(fresh(), __builtin_ctzll(am), o, d, T, path_L(), rng.x, depth,
                                          skey[__builtin_ctzll(am)], stack);
              if (lane == __builtin_ctzll(am)) {
                const int q = entry & (kRound - 1);
                slot[q][0] = Lr.x;
                slot[q][1] = Lr.y;
                slot[q][2] = Lr.z;
                alive = false;
              }
              outer = 1;
              break;
            }
          }
        }  // pass 0

        bool wide_q = false, wide_found = false, wide_fb = false;
        if constexpr (kStage) {  // wave-uniform: few paths left -> helpers
          const Hot h = hot<kStage>();
          const bool need = alive && !shade && depth < h.max_depth;
          const unsigned long long qm = __ballot(need);
          const int nq = __popcll(qm);
          // (from 16 spheres on: below that the group set-up and merge cost more
          // than the short scan they split; measured on the 5-sphere scene)
          if (h.g.nt == 0 && h.g.ns >= 16 && nq > 0 && nq <= 16) {
            // (kCount: helpers count their sphere tests, primary queries included)
            wide_found = closest_wide<kCount>(h.g, need, qm, nq, o, d, hs, wide_fb, c);
            wide_q = true;
          }
        }
        if (alive && !shade) {
          const Hot h = hot<kStage>();
          const Geo& gg = h.g;
          bool done = depth >= h.max_depth;  // traceRay depth cut-off: contributes 0
          bool missed = false;
          if (!done) {
            if (kCount && depth == 0) {  // phase 1 counted the primary query
              Counters nc;
              done = (wide_q && !wide_fb) ? !wide_found : !closest_hit<false>(gg, o, d, hs, stack, all, nc);
            } else {
              cnt<kCount>(c, C_BOUNCE);
              done = (wide_q && !wide_fb) ? !wide_found
                                          : !closest_hit<kCount>(gg, o, d, hs, stack, all, c);  // miss -> black
            }
            missed = done;
          }
          if (done) {
            if constexpr (kSky) {  // an opted-in sky instead of black (rt_settings.sky)
              if (missed) set_path_L(path_L() + mul(T, sky_color(fresh()->sky, d)));
            }
            if constexpr (kPilot) {  // a measuring render: the pixel's longest path and its bounces
              KArg k = fresh();
              const BlockLoc loc = block_loc(k, block_of(k));
              const size_t px = (size_t)loc.lt * 1024 + loc.p0 + entry_id(entry) / loc.ns;
              atomicMax(k->work_max + px, (unsigned)depth + 1u);
              atomicAdd(k->work_sum + px, (unsigned)depth + 1u);
            }
            alive = false;  // finished: its radiance is in its slot, the lane is free for the second pass
          } else {
            shade = true;
            cnt<kCount>(c, C_SHADE);
            // HitRecord of the closest primitive (sphere.go:42-58, triangle.go:68-81)
            if (!hs.is_tri) {
              const DSphere& S0 = gg.spheres[hs.idx];
              const double t = hs.num / len2(d);
              P = o + muls(d, t);
              d3 outward = divs(P - ld3(S0.c), S0.r);
              front = dot(d, outward) < 0;
              N = front ? outward : neg(outward);
              mi = S0.mat;
              self = S0.obj;
            } else {
              const DTri& T0 = gg.tris[hs.idx];
              P = o + muls(d, hs.num);
              double w = 1.0 - hs.u - hs.v;
              d3 n = ld3(T0.n);
              N = normalize((muls(n, w) + muls(n, hs.u)) + muls(n, hs.v));
              front = dot(d, N) < 0;
              if (!front) N = neg(N);
              mi = T0.mat;
              self = T0.obj;
            }
          }
        }
        // a second pass when enough lanes are free and entries are left
        if (pass > 0 || kRefill2Min <= 0 || __popcll(__ballot(!alive)) < kRefill2Min || next >= nh) break;
      }  // passes
      if (outer == 1) continue;
      if (outer == 2) break;

#ifdef RT_WG_TIMING
      const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
      dbg_hit += ts1 - ts0;
#endif

      if (__ballot(shade) != 0) {
        // (2) calculateDirectLighting (renderer.go:229-297), light by light
        const Hot h = hot<kStage>();
        const Geo& gg = h.g;
        const bool masks = h.masks, soft = h.soft;
        const DMat* __restrict__ m = h.mats + mi;
        d3 D = mk(0, 0, 0);
        if (shade) D = mk(m->ambient, m->ambient, m->ambient);
        for (int li = 0; li < h.nl; ++li) {
          const DLight& Lt = h.lights[li];
          d3 ldir = mk(0, 0, 0);
          double ldist = 0;
          Cand cm{0ull, 0ull};
          bool lit = false, occl = false;
#ifdef RT_WG_TIMING
          const unsigned long long th0 = __builtin_amdgcn_s_memtime();
#endif
          if (shade) {
            d3 lv = ld3(Lt.pos) - P;
            ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
            ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
            lit = !(ldist < 0.001);
            if (lit) {
              cnt<kCount>(c, C_LIGHT);
              cnt<kCount>(c, C_SHADOW);
            }
          }
          // (r05) an inert light (light_inert): its shadow rays are not
          // traced (the counting variant traces them, for the reference's
          // counts, and books them as culled)
          const bool dark = shade && lit && light_inert(m, Lt, N, ldir, D);
          const bool hard = shade && lit && (kCount || !dark);
          bool wide_c = false;
          if constexpr (kStage) {  // few lit hit points: the cone tests with helpers
            if (masks && gg.nt == 0 && RT_CONE_HELPERS) {
              const unsigned long long cq = __ballot(hard);
              const int ncq = __popcll(cq);
              if (ncq > 0 && ncq <= 16) {
                const unsigned long long ms = cone_wide(gg, hard, cq, ncq, P, N, front, self, ldir, ldist);
                if (hard) cm = Cand{ms, 0ull};
                wide_c = true;
              }
            }
          }
          if (hard) {
            if (masks && !wide_c) cm = cone_candidates(gg, P, N, front, self, ldir, ldist);
            if constexpr (kCount) {
              const unsigned long long s0 = c.v[C_SPH], t0 = c.v[C_TRI];
              occl = shadow_blocked<kCount>(gg, masks, P, ldir, ldist, cm, stack, c);  // hard shadow ray
              if (dark) {
                culled.v[C_SHADOW] += 1;
                culled.v[C_SPH] += c.v[C_SPH] - s0;
                culled.v[C_TRI] += c.v[C_TRI] - t0;
              }
            } else {
              occl = shadow_blocked<kCount>(gg, masks, P, ldir, ldist, cm, stack, c);  // hard shadow ray
            }
          }
#ifdef RT_WG_TIMING
          dbg_hard += __builtin_amdgcn_s_memtime() - th0;
#endif
          const bool need_soft = lit && !occl && soft;
          // the 16 soft rays are traced unless their shadow cone is empty or
          // the light is inert (dark: the shading is the same whatever they hit)
          const bool trace = (!masks || (cm.s | cm.t) != 0) && !dark;
          int unocc = 0;
          // Spec v4 (include/rt_rng.h): the 16 points come from the stream of
          // (sample, depth, light), not from the path's.  A lane whose rays
          // cannot be blocked (empty shadow cone, or dark) needs none of them:
          // all 16 are unoccluded, nothing is drawn.  (The counting variant
          // still walks their tries, for the reference's draw count, and
          // books them as culled: executed work is the difference.)
          const bool free_soft = need_soft && !trace;
          if (free_soft) {
            unocc = 16;
            if constexpr (kCount) {
              rt_rng fr{rt_soft_state(skey[lane_now()], (uint32_t)depth, (uint32_t)li)};
              unsigned long long tries = 0;
              for (int got = 0; got < 16; ++tries) {
                const uint32_t ux = rt_rng_next(&fr), uy = rt_rng_next(&fr), uz = rt_rng_next(&fr);
                got += unit_ball_accept(ux, uy, uz) ? 1 : 0;
              }
              cnt<kCount>(c, C_SHADOW, 16);
              cnt<kCount>(c, C_RNG, 3ull * tries);
              culled.v[C_SHADOW] += 16;
              culled.v[C_RNG] += 3ull * tries;
            }
          }
          const bool traced_soft = need_soft && trace;
          rt_rng srng{traced_soft ? rt_soft_state(skey[lane_now()], (uint32_t)depth, (uint32_t)li) : 0ull};
          // soft shadows: wave-converged decision between the two forms
          const unsigned long long owners = __ballot(traced_soft);
#ifdef RT_WG_TIMING
          const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
#endif
          if (owners != 0) {
#ifdef RT_WG_TIMING
            if (__popcll(owners) <= kCoopMax) dbg_coop += __popcll(owners); else ++dbg_seq;
#endif
            // cooperative soft shadows when at most kCoopMax lanes need them
            if (__popcll(owners) <= kCoopMax) {
              for (unsigned long long b = owners; b; b &= b - 1) {
                const int ow = __builtin_ctzll(b);
                const CoopOut r = soft_coop<kCount>(
                    gg, masks, true, inv3(rl3(P, ow)), inv3(rl3(ldir, ow)),
                    inv(rld(ldist, ow)), Cand{rl64(cm.s, ow), rl64(cm.t, ow)}, rl64(srng.x, ow), h.jump, stack, c);
                if (lane == ow) {
                  unocc = r.unocc;
                  cnt<kCount>(c, C_SHADOW, 16);
                  cnt<kCount>(c, C_RNG, 3ull * r.tries);
                }
              }
            } else {
              const int uq = soft_queue<kCount>(gg, masks, traced_soft, true, P, ldir, ldist, cm, srng, h.jump, stack, c);
              if (traced_soft) unocc = uq;  // (a free lane keeps its 16)
            }
          }
#ifdef RT_WG_TIMING
          dbg_soft += __builtin_amdgcn_s_memtime() - ts2;
#endif
          if (lit) {
            const double sf = occl ? 0.0 : (soft ? (double)unocc / 16.0 : 1.0);  // shadowSum / 16
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
#ifdef RT_WG_TIMING
        dbg_light += __builtin_amdgcn_s_memtime() - ts1;
#endif
        // (3) Material.Scatter and the traceRay combination (renderer.go:181-226)
#ifdef RT_WG_TIMING
        const unsigned long long tc0 = __builtin_amdgcn_s_memtime();
#endif
        if (shade) {
          d3 E = ld3(m->emit);
          const Scat sc = scatter<kCount>(m, d, N, front, rng, c);
          if (!sc.ok) {
            set_path_L(path_L() + mul(T, E + D));
            fin = true;
          } else {
            set_path_L(path_L() + mul(T, E + muls(D, m->dw)));
            fin = !h.recursive || depth + 1 >= h.max_depth;
            if (!fin) {
              T = mul(T, muls(sc.A, m->rw));
              o = P;
              d = sc.nd;
              depth += 1;
            }
          }
        }
#ifdef RT_WG_TIMING
        dbg_scat += __builtin_amdgcn_s_memtime() - tc0;
#endif
      }
      if (fin) {  // the path's radiance goes to its entry's ring slot
        if constexpr (kPilot) {  // a measuring render: the pixel's longest path and its bounces
          KArg k = fresh();
          const BlockLoc loc = block_loc(k, block_of(k));
          const size_t px = (size_t)loc.lt * 1024 + loc.p0 + entry_id(entry) / loc.ns;
          atomicMax(k->work_max + px, (unsigned)depth + 1u);
          atomicAdd(k->work_sum + px, (unsigned)depth + 1u);
        }
        alive = false;  // (its radiance is in its slot already)
      }
    }
    __syncthreads();
    resolve_entries(resolved, nh);
    __syncthreads();
  }
#undef path_L
#undef set_path_L
#ifdef RT_WG_TIMING
  const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
  if (dbg_bprev >= 0) dbg_bclk[dbg_bprev] += __builtin_amdgcn_s_memtime() - dbg_bts;
#endif

  // ---- phase 3 (final): mean, tone map, one write per pixel
  KArg k = fresh();
  // the lane id laundered (see resolve_entries): the LDS addresses of this
  // epilogue are computed here, not kept live (spilled) from the prologue
  int lane3;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lane3) : "v"((int)threadIdx.x));
  bool resolve = true;
  if (blk.slot >= 0) {
    // a split pixel: the last of its sub-blocks to finish sums the hit
    // samples of the slot row in sample order (misses add +0) and writes it
    // Tail kernel: its row samples were written through, drained before the
    // counter, and the last contributor reads the row sc1 (the tail
    // helpers' hand-off, above).  Product kernel: plain stores, a release
    // fence before the counter and an acquire fence after it (the same
    // time, r06 A/B, and the row's samples reach HBM as whole lines: the
    // write-through form wrote 3.8 MB more per headline frame)
    if constexpr (kTail)
      wt_drain();
    else
      __threadfence();
    int old = 0;
    if (lane3 == 0) old = atomicAdd(&k->split_cnt[split_index(k, blk.slot)], 1);
    old = __builtin_amdgcn_readfirstlane(old);
    resolve = old == blk.nsub - 1;
    if (resolve) {
      if constexpr (!kTail) __threadfence();
      const double* row = k->split_rad + split_index(k, blk.slot) * k->spp * 3;
      uint32_t* hw = k->split_hits + split_index(k, blk.slot) * ((k->spp + 31) >> 5);
      // chunks of kRound samples: all lanes load (in parallel) into the LDS
      // slots, misses as +0, then one lane per channel adds them in order
      double a = 0;  // (a later sample pass continues the running sum)
      if ((k->acc_mode & 1) && lane3 < 3) a = k->acc[((size_t)blk.lt * 1024 + blk.p0) * 3 + lane3];
      a = row_sum<kTail>(slot, row, hw, 0, k->spp, a, lane3);
      if (lane3 < 3) psum[0][lane3] = a;
      // the slot's hit bits and counter are left zeroed for the next launch
      // (the host clears them only when it builds a schedule: no memset per frame)
      for (int i = lane3; i < ((k->spp + 31) >> 5); i += 64) hw[i] = 0u;
      if (lane3 == 0) k->split_cnt[split_index(k, blk.slot)] = 0;
      __syncthreads();
    }
  }
  if (resolve) {
    const BlockLoc loc = block_loc(k, block_of(k));
    const int p = lane3;
    const int tp = loc.p0 + p;
    const int x = loc.tx * 32 + (tp & 31), y = loc.ty * 32 + (tp >> 5);
    bool rowed = false;  // (tail helpers: the pixel's row writes it, below)
    if constexpr (kTail) rowed = prow[p] >= 0;
    if (rowed) {
    } else if ((k->acc_mode & 2) && p < loc.np && tp < 1024) {  // not the last sample pass: keep the running sum
      double* a = k->acc + ((size_t)loc.lt * 1024 + tp) * 3;
      a[0] = psum[p][0];
      a[1] = psum[p][1];
      a[2] = psum[p][2];
    } else if (p < loc.np && tp < 1024 && loc.tile < k->ntiles && x < k->W && y < k->H) {
      const double n = (double)k->spp_total;
      const double mx = psum[p][0] / n, my = psum[p][1] / n, mz = psum[p][2] / n;  // DivScalar(float64(samples))
      const size_t oi = k->layout == RT_LAYOUT_IMAGE ? (size_t)y * k->W + x : (size_t)loc.lt * 1024 + (size_t)tp;
      const int fr = frame_of(k);
      float* const ol = k->frame_lin[fr];
      uint8_t* const orgba = k->frame_rgba[fr];
      if (ol) {
        ol[oi * 3 + 0] = (float)mx;
        ol[oi * 3 + 1] = (float)my;
        ol[oi * 3 + 2] = (float)mz;
      }
      if (orgba) {
        *reinterpret_cast<uint32_t*>(orgba + oi * 4) = tonemap_rgba8(mx, my, mz);
      }
    }
  }
  if constexpr (kTail) {
    // pixels with exported paths: the block gives back its share of each
    // row (the running sum of the samples before the row's first one), and
    // the row's last contributor sums it and writes the pixel
    if (k->tail != nullptr && blk.slot < 0) {
      int last = 0;
      if (prow[lane3] >= 0) {
        TailRow* hd = k->tail_hdr + prow[lane3];
        st_wtd(hd->prefix, psum[lane3][0]);
        st_wtd(hd->prefix + 1, psum[lane3][1]);
        st_wtd(hd->prefix + 2, psum[lane3][2]);
        st_wt32(&hd->k0, (uint32_t)pk0[lane3]);
      }
      wt_drain();  // (the resolve's row samples too) before the counter
      if (prow[lane3] >= 0) last = atomicSub(&k->tail_hdr[prow[lane3]].counter, 1) == 1 ? 1 : 0;
      for (unsigned long long b = __ballot(last); b; b &= b - 1) {
        const int r = prow[__builtin_ctzll(b)], spp = k->spp_total, bw = (spp + 31) >> 5;
        const TailRow* hd = k->tail_hdr + r;
        double a = lane3 < 3 ? ld_wtd(hd->prefix + lane3) : 0.0;
        a = row_sum<true>(slot, k->tail_rows + (size_t)r * spp * 3, k->tail_bits + (size_t)r * bw, (int)ld_wt32(&hd->k0),
                          spp, a, lane3);
        const double sx = rld(a, 0), sy = rld(a, 1), sz = rld(a, 2);
        if (lane3 == 0) store_pixel(k, (int)ld_wt32(&hd->frame), (size_t)ld_wt64(&hd->oi), sx, sy, sz);
      }
    }
  }
  if constexpr (kCount) {
    for (int i = 0; i < 2 * kCounters; ++i) {
      // wave reduction, then one atomic per counter
      unsigned long long v = i < kCounters ? c.v[i] : culled.v[i - kCounters];
      for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
      if (lane3 == 0) atomicAdd(&k->counts[i], v);
    }
  }
#ifdef RT_WG_TIMING
  if (k->dbg && lane3 == 0) {
    unsigned long long* r = k->dbg + (size_t)blockIdx.x * kDbgStride;
    r[0] = t_start;
    r[1] = t_loop;
    r[2] = __builtin_amdgcn_s_memrealtime();
    r[3] = dbg_hit;
    r[4] = dbg_light;
    r[5] = dbg_soft;
    r[6] = dbg_vis;
    r[7] = dbg_iter;
    r[8] = dbg_hard;
    r[9] = dbg_scat;
    r[10] = dbg_alive;
    r[11] = dbg_coop;
    r[12] = dbg_seq;
    r[13] = (unsigned long long)blk.np * 65536ull + (unsigned long long)blk.ns;
    r[14] = (unsigned long long)(blk.slot + 1);
    for (int i = 0; i < 5; ++i) {
      r[32 + i] = dbg_bclk[i];
      r[37 + i] = dbg_bcnt[i];
    }
    if (solo_clk[6])  // a lone path ran: its section clocks replace the iteration stamps
      for (int i = 0; i < 16; ++i) r[16 + i] = solo_clk[i];
    r[42] = solo_clk[6];  // lone-path bounces (0: none ran)
    r[43] = solo_clk[7];  // entries into solo_path
  }
#endif
  if constexpr (kTail) {
    if (k->tail != nullptr) {
      // this main block is done: it queues nothing more (no fence: its queue
      // reservations were returning atomics, complete before this one)
      if (lane3 == 0) atomicAdd(&k->tail->done[(blockIdx.x % kTailShards) * 32], 1u);
    }
  }
}
template <bool kCount, bool kStage, bool kPilot, bool kSky>
__global__ __launch_bounds__(64, RT_WAVES_PER_SIMD) void render_kernel(const KParams pk) {
  render_body<kCount, kStage, kPilot, kSky, false>(pk);
}
// the staged product render with tail helpers (rt_tuning.tail_helpers > 0)
__global__ __launch_bounds__(64, RT_WAVES_PER_SIMD) void render_kernel_tail(const KParams pk) {
  render_body<false, true, false, false, true>(pk);
}

// Gathered shares [world][share_bytes] (each: [max_local][1024] float3, then
// [max_local][1024] RGBA8 at rgba_off) -> W*H images.  One thread per image
// pixel, so the image writes are coalesced; a tile row's 32 pixels read 384
// contiguous bytes of its share.
__global__ __launch_bounds__(256) void unpack_kernel(int W, int H, int world, int tiles_x,
                                                     const uint8_t* __restrict__ g, size_t share_bytes,
                                                     size_t rgba_off, float* __restrict__ ol,
                                                     uint8_t* __restrict__ orgba) {
  const long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (long long)W * H) return;
  const int y = (int)(o / W), x = (int)(o - (long long)y * W);
  const int t = (y >> 5) * tiles_x + (x >> 5);
  const int r = t % world, lt = t / world;
  const size_t pi = (size_t)lt * 1024 + (size_t)((y & 31) * 32 + (x & 31));
  const uint8_t* share = g + (size_t)r * share_bytes;
  if (ol) {
    const float* pl = reinterpret_cast<const float*>(share) + pi * 3;
    ol[o * 3 + 0] = pl[0];
    ol[o * 3 + 1] = pl[1];
    ol[o * 3 + 2] = pl[2];
  }
  if (orgba)
    *reinterpret_cast<uint32_t*>(orgba + o * 4) = *reinterpret_cast<const uint32_t*>(share + rgba_off + pi * 4);
}

// The same scatter for a partition: slot[t] = {owner rank, local tile}; frame
// blockIdx.y of nframes, gathered as [world][nframes][share], written to
// [nframes][W*H] images.
__global__ __launch_bounds__(256) void unpack_map_kernel(int W, int H, int tiles_x, int nframes,
                                                         const int2* __restrict__ slot, const uint8_t* __restrict__ g,
                                                         size_t share_bytes, size_t rgba_off, float* __restrict__ ol,
                                                         uint8_t* __restrict__ orgba) {
  const long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (long long)W * H) return;
  const int f = blockIdx.y;
  const long long oo = (long long)f * W * H + o;
  const int y = (int)(o / W), x = (int)(o - (long long)y * W);
  const int2 rl = slot[(y >> 5) * tiles_x + (x >> 5)];
  const size_t pi = (size_t)rl.y * 1024 + (size_t)((y & 31) * 32 + (x & 31));
  const uint8_t* share = g + ((size_t)rl.x * nframes + f) * share_bytes;
  if (ol) {
    const float* pl = reinterpret_cast<const float*>(share) + pi * 3;
    ol[oo * 3 + 0] = pl[0];
    ol[oo * 3 + 1] = pl[1];
    ol[oo * 3 + 2] = pl[2];
  }
  if (orgba)
    *reinterpret_cast<uint32_t*>(orgba + oo * 4) = *reinterpret_cast<const uint32_t*>(share + rgba_off + pi * 4);
}

size_t render_shmem(const KParams& p) {
  return (size_t)p.stack_off + (p.use_bvh ? sizeof(int) * p.stack_depth * 64 : 0);
}

// Loads this file's code object onto the current device now: with HIP's lazy
// loading it would otherwise be loaded inside the first render launch
// (rt_context_create calls it once per device and process).
int preload_render_kernels() {
  hipFuncAttributes a;
  return (int)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(render_kernel<false, true, false, false>));
}

// The runtime's first-use set-up, on `stream`, so that it happens in the
// constructor (NewParallelRenderer, main.go:46-47) instead of inside the
// first Render (profiles/r04_cli_trace.json, a fresh `raytracer` process;
// scripts/copy_probe.hip):
//   - an empty launch (kernel argument pool);
//   - a launch with private (scratch) memory: the first kernel that needs
//     scratch makes the runtime allocate the device's scratch pool (the
//     first render launch started 1.26 ms after it was enqueued); 512 B per
//     lane covers every render kernel variant (<= 328 B);
//   - copies each way through pageable and pinned memory, and device->host
//     copies queued behind a kernel that is still running: the first time a
//     process's copy has to wait for a running kernel it starts ~8-9 ms after
//     the kernel ends (the CLI's image download; scripts/copy_probe.hip:
//     later ones start at once, 0.16 ms for 8 MB).  warm_busy runs ~0.2 ms
//     so the copies are queued while it still runs.
//     (Render itself copies only from an idle stream, rt_renderer_render.)
__global__ void warm_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] = 0;
}
__global__ void warm_scratch(int* p, int n) {
  volatile int a[128];  // (volatile: kept in private memory)
  for (int i = 0; i < 128; ++i) a[i] = i * n + (int)threadIdx.x;
  if (p && n < 0) p[threadIdx.x] = a[(threadIdx.x * 7) & 127];
}
__global__ void warm_busy(float* p, int iters) {
  float v = (float)threadIdx.x;
  for (int k = 0; k < iters; ++k) v = v * 0.999f + 1.0f;  // a dependent chain: ~4 clocks per step
  if (p && v < 0.f) p[threadIdx.x] = v;
}
int warm_device(void* stream, void* dev_buf, void* host_pinned, void* host_pageable, size_t bytes) {
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(warm_kernel, dim3(1), dim3(64), 0, st, (int*)dev_buf);
  hipLaunchKernelGGL(warm_scratch, dim3(1), dim3(64), 0, st, (int*)dev_buf, 1);
  static thread_local unsigned char host[4096];
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(dev_buf, host, sizeof host, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(host, dev_buf, sizeof host, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dev_buf, host_pinned, bytes, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(dev_buf, host_pageable, bytes, hipMemcpyHostToDevice, st);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {  // behind a kernel: into pageable, then pinned memory
    hipLaunchKernelGGL(warm_busy, dim3(1), dim3(64), 0, st, (float*)dev_buf, 10000);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(k ? host_pinned : host_pageable, dev_buf, bytes, hipMemcpyDeviceToHost, st);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return (int)e;
}

int launch_render(const KParams& pin, bool count, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (pin.num_wgs <= 0) return hipSuccess;
  KParams p = pin;
  if (p.nframes <= 1) {  // one frame: entry 0 from the single-frame fields
    p.nframes = 1;
    p.frame_key[0] = p.seed_key;
    p.frame_lin[0] = p.out_linear;
    p.frame_rgba[0] = p.out_rgba;
  }
  const size_t shmem = render_shmem(p);
  const bool stage = p.stage_bytes > 0;
  // tail helpers: render_kernel_tail exports paths;
  // tail_helpers one-wave workgroups follow its num_wgs main blocks
  const bool tail = p.tail && stage && !count && !p.sky && !p.work_max && p.acc_mode == 0 && p.tail_helpers > 0;
  if (!tail) p.tail = nullptr;
  const dim3 g(p.num_wgs + (tail ? p.tail_helpers : 0)), b(64);
  // (the opted-in sky has instantiations of its own: its code would cost the
  // others registers; the pilot and the counting variant ignore it -- path
  // lengths and counts do not depend on what a miss returns)
  if (count && p.sky) {
    // counts with an opted-in sky: the image comes from the sky variant, the
    // counts from a second, output-less launch of the counting variant (it
    // leaves the split rows zeroed like any launch and neither reads nor
    // writes the sample-pass sums)
    KParams q = p;
    q.counts = nullptr;
    const int e = launch_render(q, false, stream);
    if (e != hipSuccess) return e;
    q = p;
    q.sky = nullptr;
    q.out_linear = nullptr;
    q.out_rgba = nullptr;
    q.acc = nullptr;
    q.acc_mode = 0;
    return launch_render(q, true, stream);
  }
  if (p.work_max) {  // a measuring render (pilot or first frame): its own instantiation (and kernel name)
    if (stage)
      hipLaunchKernelGGL((render_kernel<false, true, true, false>), g, b, shmem, st, p);
    else
      hipLaunchKernelGGL((render_kernel<false, false, true, false>), g, b, shmem, st, p);
  } else if (count && stage) {
    hipLaunchKernelGGL((render_kernel<true, true, false, false>), g, b, shmem, st, p);
  } else if (count) {
    hipLaunchKernelGGL((render_kernel<true, false, false, false>), g, b, shmem, st, p);
  } else if (p.sky && stage) {
    hipLaunchKernelGGL((render_kernel<false, true, false, true>), g, b, shmem, st, p);
  } else if (p.sky) {
    hipLaunchKernelGGL((render_kernel<false, false, false, true>), g, b, shmem, st, p);
  } else if (stage && tail) {
    hipLaunchKernelGGL(render_kernel_tail, g, b, shmem, st, p);
  } else if (stage) {
    hipLaunchKernelGGL((render_kernel<false, true, false, false>), g, b, shmem, st, p);
  } else {
    hipLaunchKernelGGL((render_kernel<false, false, false, false>), g, b, shmem, st, p);
  }
  return (int)hipGetLastError();
}

// The image to pinned host memory, written by the GPU itself (16 B per lane,
// coalesced): the first Render of a renderer, where a copy-engine transfer
// started 7-15 ms late in a fresh process (rt_renderer_render).
__global__ __launch_bounds__(256) void download_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
int launch_download(const void* d_src, void* h_dst_mapped, size_t bytes, void* stream) {
  if (bytes == 0) return hipSuccess;
  if ((bytes & 15) || ((uintptr_t)d_src & 15) || ((uintptr_t)h_dst_mapped & 15)) return hipErrorInvalidValue;
  const size_t n16 = bytes / 16;
  const unsigned grid = (unsigned)((n16 + 255) / 256 < 2048 ? (n16 + 255) / 256 : 2048);
  hipLaunchKernelGGL(download_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const uint4*)d_src,
                     (uint4*)h_dst_mapped, n16);
  return (int)hipGetLastError();
}

// s_memrealtime counts at 100 MHz: the wave sleeps until `ticks` have passed
// since it started (a bounded wait: it always ends)
__global__ void spin_kernel(unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
int launch_spin(double ms, void* stream) {
  const double t = ms < 60000.0 ? ms : 60000.0;  // at most a minute
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (unsigned long long)(t * 1e5));
  return (int)hipGetLastError();
}

int launch_unpack(int32_t W, int32_t H, int32_t world, const void* gathered, size_t share_bytes, size_t rgba_off,
                  float* ol, uint8_t* orgba, void* stream) {
  const long long total = (long long)W * H;
  if (total <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, W, H, world, (W + 31) / 32,
                     (const uint8_t*)gathered, share_bytes, rgba_off, ol, orgba);
  return (int)hipGetLastError();
}

int launch_unpack_map(int32_t W, int32_t H, int32_t nframes, const int32_t* slot, const void* gathered,
                      size_t share_bytes, size_t rgba_off, float* ol, uint8_t* orgba, void* stream) {
  const long long total = (long long)W * H;
  if (total <= 0 || nframes <= 0) return hipSuccess;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(unpack_map_kernel, dim3(blocks, nframes), dim3(256), 0, (hipStream_t)stream, W, H, (W + 31) / 32,
                     nframes, reinterpret_cast<const int2*>(slot), (const uint8_t*)gathered, share_bytes, rgba_off, ol,
                     orgba);
  return (int)hipGetLastError();
}


// Cross-lane reads from inactive lanes counted by this file's kernels in an
// RT_CHECK_XLANE build (rt_device.h); -1 in a normal build.  reset: zero it.
long long xlane_faults_kernel(bool reset) {
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
