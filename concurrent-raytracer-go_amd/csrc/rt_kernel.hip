// rt_kernel.hip — gfx950 (CDNA4) kernels of the renderer core.
//
// One launch renders every 32x32 tile (createRenderTasks,
// internal/renderer/renderer.go:398-436) that this rank owns.  Mapping
// (DESIGN.md §Kernels):
//   workgroup (256 lanes = 4 wave64) = P consecutive row-major pixels of a
//     tile x S sample slices (P = 256/S, S chosen by the host, ~spp/2);
//   lane (p, q) traces samples q, q+S, q+2S, ... of pixel p with a
//     persistent, iterative bounce loop (traceRay, renderer.go:165-227,
//     unrolled): a lane whose path ends immediately regenerates its next
//     camera sample, so paths of different length keep the lanes busy;
//   a wave therefore holds the samples of one or two pixels — near-identical
//     rays, so the branchy shading code stays coherent;
//   the S slice sums of a pixel are reduced in LDS in slice order, divided by
//     spp, tone-mapped (toneMap, renderer.go:348-367) and written once:
//     float3 linear radiance + RGBA8.
// Scene data for linear-scan scenes is read with wave-uniform addresses, so
// it lives in SGPRs via the scalar cache (zero LDS bank cycles, no VGPRs).
// Large sphere scenes use a BVH (bvh.cpp) traversed with a per-lane stack in
// LDS.  All arithmetic is binary64 in the reference's order, compiled with
// -ffp-contract=off, so every decision (hit / miss, root choice, rejection
// test, reflect vs refract) is bit-identical to the oracle's.  Divisions that
// only feed range tests are filtered by a reciprocal multiply with a 2^-40
// relative error margin; the exact IEEE division runs whenever the filter
// cannot decide, so the filtered decision always equals Go's.
#include <hip/hip_runtime.h>

#include "../../include/rt_rng.h"
#include "rt_internal.h"

#ifndef RT_WAVES_PER_SIMD
#define RT_WAVES_PER_SIMD 3  // measured best of 2/3/4 (4 spills the FP64 path state)
#endif

namespace rtgo {

// ------------------------------------------------------------ Vec3 (vector.go)
struct d3 {
  double x, y, z;
};
__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ d3 mul(d3 a, d3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ d3 muls(d3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ d3 divs(d3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ d3 neg(d3 a) { return mk(a.x * -1, a.y * -1, a.z * -1); }  // MulScalar(-1)
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ d3 cross(d3 a, d3 b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double len2(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
__device__ __forceinline__ d3 normalize(d3 a) {  // Vec3.Normalize: zero stays zero
  double l = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  if (l == 0) return mk(0, 0, 0);
  return divs(a, l);
}
__device__ __forceinline__ d3 reflect(d3 v, d3 n) { return v - muls(n, 2 * dot(v, n)); }
__device__ __forceinline__ d3 refract(d3 v, d3 n, double eta) {  // vector.go:81-96
  double ct = dot(v, n);
  if (ct > 0) {
    n = neg(n);
    eta = 1 / eta;
    ct = -ct;
  }
  double s2 = eta * eta * (1 - ct * ct);
  if (s2 > 1) return reflect(v, n);
  double c2 = sqrt(1 - s2);
  return muls(v, eta) - muls(n, eta * ct + c2);
}
__device__ __forceinline__ d3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

// Go math.Max / math.Min where one operand is a constant (every use on the
// path): NaN propagates, Max(0, -0) = +0.
__device__ __forceinline__ double gmax0(double y) { return !(y <= 0.0) ? y : 0.0; }   // Max(0, y)
__device__ __forceinline__ double gmin1_first(double y) { return (1.0 < y) ? 1.0 : y; }  // Min(1, y)
__device__ __forceinline__ double gmin_x1(double x) { return !(x >= 1.0) ? x : 1.0; }   // Min(x, 1)
__device__ __forceinline__ double clamp01(double v) { return gmax0(gmin1_first(v)); }  // Max(0, Min(1, v))

// Go math.Pow(x, n) for a positive integer n: Go multiplies by repeated
// squaring (pow.go); frexp/ldexp only rescale by powers of two, so for
// normal-range values these products round identically.
template <int N>
__device__ __forceinline__ double pow_n(double x) {
  double a = 1.0;
  double x1 = x;
#pragma unroll
  for (int i = N; i != 0; i >>= 1) {
    if (i & 1) a = a * x1;
    if (i >> 1) x1 = x1 * x1;
  }
  return a;
}
// Go's uint8(float64) on amd64 (CVTTSD2SQ, then low byte): NaN -> 0.
__device__ __forceinline__ uint32_t go_u8(double f) {
  if (__builtin_isnan(f)) return 0;
  return (uint32_t)(uint8_t)(int64_t)f;
}
// Pow(x, 1/2.2) with Go's special cases (x<0 -> NaN, 0 -> 0, 1 -> 1).
__device__ __forceinline__ double pow_gamma(double x, double y) {
  if (x == 1) return 1;
  if (__builtin_isnan(x)) return x;
  if (x == 0) return 0;
  if (__builtin_isinf(x)) return x > 0 ? x : __builtin_inf();
  if (x < 0) return __builtin_nan("");
  return exp(y * log(x));
}

struct Counters {
  unsigned long long v[9];
};
enum { C_CAM = 0, C_BOUNCE, C_SHADOW, C_SPH, C_TRI, C_BOX, C_SHADE, C_LIGHT, C_RNG };

template <bool kCount>
__device__ __forceinline__ void cnt(Counters& c, int i) {
  if constexpr (kCount) c.v[i] += 1;
}

template <bool kCount>
__device__ __forceinline__ double draw(rt_rng& r, Counters& c) {
  cnt<kCount>(c, C_RNG);
  return rt_rng_draw(&r);
}

// RandomVec3InUnitSphere, vector.go:132-139.
template <bool kCount>
__device__ __forceinline__ d3 rand_in_unit_sphere(rt_rng& r, Counters& c) {
  for (;;) {
    double x = draw<kCount>(r, c);
    double y = draw<kCount>(r, c);
    double z = draw<kCount>(r, c);
    d3 p = mk(x * 2 - 1, y * 2 - 1, z * 2 - 1);
    if (len2(p) < 1) return p;
  }
}

// ------------------------------------------------------------ intersection
// 1/a to ~2^-50 (v_rcp_f64 + one Newton step): only feeds root_out's
// filter, whose 2^-40 margin absorbs the error.
__device__ __forceinline__ double approx_rcp(double a) {
  const double r0 = __builtin_amdgcn_rcp(a);
  const double e = __builtin_fma(-a, r0, 1.0);
  return __builtin_fma(r0, e, r0);
}

// Is root = num / a outside [tmin, tmax] (Go: `root < tMin || tMax < root`)?
// Decided from num * inv_a when the 2^-40 margin settles it, else by the
// exact quotient — so the answer always equals the reference's.
__device__ __forceinline__ bool root_out(double num, double a, double inv_a, double tmin, double tmax) {
  const double r = num * inv_a;
  const double e = fabs(r) * 0x1p-40;
  if (r + e < tmin || r - e > tmax) return true;    // surely outside
  if (r - e >= tmin && r + e <= tmax) return false;  // surely inside
  const double q = num / a;                          // undecided / NaN / inf: exact
  return q < tmin || tmax < q;
}

// Sphere.Hit (sphere.go:22-40) as a range query: which root Go accepts.
// Returns 0 = miss, 1 = first root, 2 = second root.
__device__ __forceinline__ int sphere_query(const DSphere& S, d3 o, d3 d, double a, double inv_a, double tmin,
                                            double tmax, double& num) {
  double ocx = o.x - S.c[0], ocy = o.y - S.c[1], ocz = o.z - S.c[2];
  double hb = ocx * d.x + ocy * d.y + ocz * d.z;
  double c = (ocx * ocx + ocy * ocy + ocz * ocz) - S.r2;
  double disc = hb * hb - a * c;
  if (disc < 0) return 0;
  double sq = sqrt(disc);
  double n1 = -hb - sq;
  if (!root_out(n1, a, inv_a, tmin, tmax)) {
    num = n1;
    return 1;
  }
  double n2 = -hb + sq;
  if (!root_out(n2, a, inv_a, tmin, tmax)) {
    num = n2;
    return 2;
  }
  return 0;
}

// Triangle.Hit acceptance (triangle.go:36-66).
__device__ __forceinline__ bool tri_test(const DTri& T, d3 o, d3 d, double tmin, double tmax, double& t,
                                         double& uo, double& vo) {
  d3 e1 = ld3(T.e1), e2 = ld3(T.e2);
  d3 h = cross(d, e2);
  double a = dot(e1, h);
  if (a > -1e-6 && a < 1e-6) return false;
  double f = 1.0 / a;
  d3 s = o - ld3(T.v0);
  double u = f * dot(s, h);
  if (u < 0.0 || u > 1.0) return false;
  d3 q = cross(s, e1);
  double v = f * dot(d, q);
  if (v < 0.0 || u + v > 1.0) return false;
  double tv = f * dot(e2, q);
  if (tv < tmin || tv > tmax) return false;
  t = tv;
  uo = u;
  vo = v;
  return true;
}

// ------------------------------------------------------------ BVH traversal
constexpr int kStack = 40;  // per-lane LDS stack depth (binned SAH over 10k spheres: depth ~ 20-30)

// Conservative slab test of a float box against [tmin, tnear_max].
__device__ __forceinline__ bool box_hit(const DBVHNode& n, d3 o, d3 id, double tmin, double tmax) {
  double tx0 = ((double)n.lo[0] - o.x) * id.x, tx1 = ((double)n.hi[0] - o.x) * id.x;
  double ty0 = ((double)n.lo[1] - o.y) * id.y, ty1 = ((double)n.hi[1] - o.y) * id.y;
  double tz0 = ((double)n.lo[2] - o.z) * id.z, tz1 = ((double)n.hi[2] - o.z) * id.z;
  double tn = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmax(fmin(tz0, tz1), tmin));
  double tf = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmin(fmax(tz0, tz1), tmax));
  // margins: the box is padded by >= 1 float ulp; allow 1e-9 relative slack
  return tn <= tf + fabs(tf) * 1e-9 + 1e-12;
}

__device__ __forceinline__ d3 inv_dir(d3 d) {
  // zero components get a huge finite inverse: no 0*inf NaN in the slabs
  return mk(1.0 / (d.x != 0 ? d.x : 1e-300), 1.0 / (d.y != 0 ? d.y : 1e-300), 1.0 / (d.z != 0 ? d.z : 1e-300));
}

struct Cand {
  unsigned long long s, t;  // bit i: sphere i / triangle i may be hit (linear scenes, <= 64 each)
};

struct HitSel {
  double num;  // chosen root numerator (t = num / a) for spheres, t for triangles
  double u, v;
  int idx;     // primitive index
  int is_tri;
};

// hitWorld closest hit, renderer.go:333-346.  Linear scan in hittable order
// (spheres before triangles; an exact-t tie is resolved by hittable index so
// the later hittable wins, as in Go), or BVH traversal with the same rule.
template <bool kCount>
__device__ __forceinline__ bool closest_hit(const KParams& p, d3 o, d3 d, HitSel& hs, int* stack, Cand m,
                                            Counters& c) {
  const double tmin = 0.001;
  double closest = __builtin_inf();
  bool found = false;
  int best_obj = -1;
  const double a = len2(d);
  const double inv_a = approx_rcp(a);
  if (p.use_bvh) {
    const d3 id = inv_dir(d);
    int sp = 0;
    int node = 0;
    for (;;) {
      const DBVHNode n = p.bvh[node];
      cnt<kCount>(c, C_BOX);
      if (box_hit(n, o, id, tmin, closest)) {
        if (n.count == 0) {
          stack[sp * 64] = n.left_or_first + 1;
          ++sp;
          node = n.left_or_first;
          continue;
        }
        for (int i = n.left_or_first; i < n.left_or_first + n.count; ++i) {
          cnt<kCount>(c, C_SPH);
          const DSphere& S = p.spheres[i];
          double num;
          if (sphere_query(S, o, d, a, inv_a, tmin, closest, num)) {
            const double t = num / a;
            if (t == closest && best_obj > S.obj) continue;
            closest = t;
            hs.num = num;
            hs.idx = i;
            hs.is_tri = 0;
            best_obj = S.obj;
            found = true;
          }
        }
      }
      if (sp == 0) break;
      --sp;
      node = stack[sp * 64];
    }
    return found;
  }
  // candidate masks (primary rays: the workgroup's frustum culling; all ones
  // otherwise) are wave-uniform, so the skips are scalar branches
  const bool use_m = p.ns <= 64 && p.nt <= 64;
  for (int i = 0; i < p.ns; ++i) {
    if (use_m && !((m.s >> i) & 1)) continue;
    cnt<kCount>(c, C_SPH);
    const DSphere& S = p.spheres[i];
    double num;
    if (sphere_query(S, o, d, a, inv_a, tmin, closest, num)) {
      const double t = num / a;
      if (t == closest && best_obj > S.obj) continue;
      closest = t;
      hs.num = num;
      hs.idx = i;
      hs.is_tri = 0;
      best_obj = S.obj;
      found = true;
    }
  }
  for (int i = 0; i < p.nt; ++i) {
    if (use_m && !((m.t >> i) & 1)) continue;
    cnt<kCount>(c, C_TRI);
    const DTri& T = p.tris[i];
    double t, u, v;
    if (tri_test(T, o, d, tmin, closest, t, u, v)) {
      if (t == closest && best_obj > T.obj) continue;
      closest = t;
      hs.num = t;
      hs.u = u;
      hs.v = v;
      hs.idx = i;
      hs.is_tri = 1;
      best_obj = T.obj;
      found = true;
    }
  }
  return found;
}

// hitWorld used as an occlusion query (calculateSmartShadow only asks
// whether any hittable is hit in [tmin, tmax], renderer.go:305,320).
template <bool kCount>
__device__ __forceinline__ bool any_hit(const KParams& p, d3 o, d3 d, double tmax, int* stack, Counters& c) {
  const double tmin = 0.001;
  const double a = len2(d);
  const double inv_a = approx_rcp(a);
  if (p.use_bvh) {
    const d3 id = inv_dir(d);
    int sp = 0;
    int node = 0;
    for (;;) {
      const DBVHNode n = p.bvh[node];
      cnt<kCount>(c, C_BOX);
      if (box_hit(n, o, id, tmin, tmax)) {
        if (n.count == 0) {
          stack[sp * 64] = n.left_or_first + 1;
          ++sp;
          node = n.left_or_first;
          continue;
        }
        for (int i = n.left_or_first; i < n.left_or_first + n.count; ++i) {
          cnt<kCount>(c, C_SPH);
          double num;
          if (sphere_query(p.spheres[i], o, d, a, inv_a, tmin, tmax, num)) return true;
        }
      }
      if (sp == 0) break;
      --sp;
      node = stack[sp * 64];
    }
    return false;
  }
  for (int i = 0; i < p.ns; ++i) {
    cnt<kCount>(c, C_SPH);
    double num;
    if (sphere_query(p.spheres[i], o, d, a, inv_a, tmin, tmax, num)) return true;
  }
  for (int i = 0; i < p.nt; ++i) {
    cnt<kCount>(c, C_TRI);
    double t, u, v;
    if (tri_test(p.tris[i], o, d, tmin, tmax, t, u, v)) return true;
  }
  return false;
}

// ------------------------------------------------------------ shading
// Shadow-cone culling (linear-scan scenes with <= 64 spheres and <= 64
// triangles).  calculateSmartShadow's rays all leave the hit point P inside
// the cone around ldir of half-angle asin(0.1) (|RandomVec3InUnitSphere *
// 0.1| < 0.1, renderer.go:316-317) and end at the light (tMax = distance).
// A primitive whose bounding sphere cannot meet that cone segment can never
// be hit by the hard ray or by any of the 16 soft rays, so it is left out of
// their tests; everything else gets the exact Sphere.Hit / Triangle.Hit
// test, so occlusion results are unchanged.  Margins (~1e-7 relative) are
// eight orders of magnitude above binary64 rounding.
// Does the cone (apex, unit axis, half-angle with cosine cos_t / sine sin_t)
// meet the sphere (cc, r)?  Conservative: the radius is inflated by ~1e-7.
__device__ __forceinline__ bool cone_meets_sphere(const double* cc, double r, d3 apex, d3 axis, double cos_t,
                                                  double sin_t) {
  const d3 v = ld3(cc) - apex;
  const double dc2 = len2(v);
  const double dc = sqrt(dc2);
  const double ra = fabs(r) * (1.0 + 1e-7) + 1e-7 * dc + 1e-12;
  if (dc <= ra) return true;
  const double tl = sqrt(fmax(dc2 - ra * ra, 0.0));
  // angle(v, axis) <= theta + beta  <=>  v.axis >= cos_t*tl - sin_t*ra
  return dot(v, axis) >= cos_t * (1.0 - 1e-9) * tl - (sin_t + 1e-9) * ra - 1e-7 * dc;
}

__device__ __forceinline__ bool in_cone(const double* cc, double r, d3 P, d3 ldir, double ldist) {
  const d3 v = ld3(cc) - P;
  const double dc2 = len2(v);
  const double dc = sqrt(dc2);
  const double ra = fabs(r) * (1.0 + 1e-7) + 1e-7 * dc + 1e-12;  // inflated radius
  if (dc <= ra) return true;                                       // P inside / on it
  if (dc - ra > ldist * (1.0 + 1e-7) + 1e-9) return false;         // beyond the light
  // angle(v, ldir) <= alpha + beta, sin(alpha) = 0.1, sin(beta) = ra/dc:
  // v.ldir >= dc*cos(alpha+beta) = cos(alpha)*sqrt(dc^2-ra^2) - 0.1*ra
  const double tl = sqrt(fmax(dc2 - ra * ra, 0.0));
  return dot(v, ldir) >= 0.99498 * tl - 0.1 * ra - 1e-7 * dc;
}

// `self` is the hittable that was hit.  When the hit is on its outside
// (front face) and every cone direction leaves the surface by a clear angle
// (N.ldir >= 0.1015 > sin(alpha)), a convex hittable (sphere of positive
// radius, or createCube's box) cannot be hit again at t >= 0.001.
__device__ __forceinline__ Cand cone_candidates(const KParams& p, d3 P, d3 N, bool front, int self, d3 ldir,
                                                double ldist) {
  const bool self_out = front && dot(N, ldir) >= 0.1015;
  Cand m{0ull, 0ull};
  for (int i = 0; i < p.ns; ++i) {
    const DSphere& S = p.spheres[i];
    if (self_out && S.obj == self && S.r > 0) continue;
    if (in_cone(S.c, S.r, P, ldir, ldist)) m.s |= 1ull << i;
  }
  for (int i = 0; i < p.nt; ++i) {
    const DTri& T = p.tris[i];
    if (self_out && T.obj == self) continue;
    if (in_cone(T.bc, T.br, P, ldir, ldist)) m.t |= 1ull << i;
  }
  return m;
}

// hitWorld(shadowRay, 0.001, dist) restricted to the candidates.
template <bool kCount>
__device__ __forceinline__ bool any_hit_masked(const KParams& p, d3 o, d3 d, double tmax, Cand m, Counters& c) {
  const double a = len2(d);
  const double inv_a = approx_rcp(a);
  for (unsigned long long b = m.s; b; b &= b - 1) {
    const int i = __builtin_ctzll(b);
    cnt<kCount>(c, C_SPH);
    double num;
    if (sphere_query(p.spheres[i], o, d, a, inv_a, 0.001, tmax, num)) return true;
  }
  for (unsigned long long b = m.t; b; b &= b - 1) {
    const int i = __builtin_ctzll(b);
    cnt<kCount>(c, C_TRI);
    double t, u, v;
    if (tri_test(p.tris[i], o, d, 0.001, tmax, t, u, v)) return true;
  }
  return false;
}

// calculateDirectLighting (renderer.go:229-297) with calculateSmartShadow
// (renderer.go:299-331) inlined.  The 16 soft rays of a light are produced
// by ONE loop over rejection tries (3 draws each, the same draws in the same
// order as 16 calls of RandomVec3InUnitSphere): a wave then runs ~max over
// lanes of the total tries (~43) instead of 16 x the max tries per point
// (~7), and the ray of an accepted point is traced right away.
template <bool kCount>
__device__ __forceinline__ d3 direct_lighting(const KParams& p, const DMat* __restrict__ m, d3 P, d3 N, bool front,
                                              int self, rt_rng& rng, int* stack, Counters& c,
                                              unsigned long long (&dt)[3]) {
  const double amb = m->ambient;
  d3 total = mk(amb, amb, amb);
  const bool masks = !p.use_bvh && p.ns <= 64 && p.nt <= 64;
  for (int li = 0; li < p.nl; ++li) {
    const DLight& L = p.lights[li];
    d3 lv = ld3(L.pos) - P;
    double ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
    d3 ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
    if (ldist < 0.001) continue;
    cnt<kCount>(c, C_LIGHT);
    cnt<kCount>(c, C_SHADOW);
    Cand cm{~0ull, ~0ull};
    bool occluded;
    if (masks) {
#ifdef RT_WG_TIMING
      const unsigned long long u0 = __builtin_amdgcn_s_memtime();
#endif
      cm = cone_candidates(p, P, N, front, self, ldir, ldist);
#ifdef RT_WG_TIMING
      const unsigned long long u1 = __builtin_amdgcn_s_memtime();
      dt[0] += u1 - u0;
#endif
      occluded = (cm.s | cm.t) != 0 && any_hit_masked<kCount>(p, P, ldir, ldist, cm, c);
#ifdef RT_WG_TIMING
      dt[1] += __builtin_amdgcn_s_memtime() - u1;
#endif
    } else {
      occluded = any_hit<kCount>(p, P, ldir, ldist, stack, c);
    }
    double sf;
    if (occluded) {
      sf = 0.0;
    } else if (p.soft) {
#ifdef RT_WG_TIMING
      const unsigned long long u2 = __builtin_amdgcn_s_memtime();
#endif
      const bool trace = !masks || (cm.s | cm.t) != 0;
      int need = 16, unocc = 0;
      while (need > 0) {
        const double x = draw<kCount>(rng, c);
        const double y = draw<kCount>(rng, c);
        const double z = draw<kCount>(rng, c);
        const d3 pt = mk(x * 2 - 1, y * 2 - 1, z * 2 - 1);
        if (len2(pt) < 1) {
          --need;
          cnt<kCount>(c, C_SHADOW);
          bool occ = false;
          if (trace) {
            const d3 sdir = normalize(ldir + muls(pt, 0.1));
            occ = masks ? any_hit_masked<kCount>(p, P, sdir, ldist, cm, c)
                        : any_hit<kCount>(p, P, sdir, ldist, stack, c);
          }
          unocc += occ ? 0 : 1;
        }
      }
      sf = (double)unocc / 16.0;  // shadowSum (a count of 1.0s) / 16
#ifdef RT_WG_TIMING
      dt[2] += __builtin_amdgcn_s_memtime() - u2;
#endif
    } else {
      sf = 1.0;
    }
    if (sf > 0.0) {
      const double metallic = m->metallic;
      double cos_t = gmax0(dot(N, ldir));
      double intensity = cos_t * L.intensity / (ldist * ldist);
      total = total + muls(ld3(m->albedo), m->diffuse_strength * intensity * sf);
      if (metallic > 0.5) {
        d3 view = normalize(neg(P));
        d3 half = normalize(ldir + view);
        double hc = gmax0(dot(N, half));
        const int sp = m->spec_pow;
        double si = sp == 64 ? pow_n<64>(hc) : (sp == 48 ? pow_n<48>(hc) : pow_n<32>(hc));
        total = total + muls(ld3(L.color), si * intensity * sf * metallic * 3.0);
      }
    }
  }
  return total;
}

// Material.Scatter for the 7 JSON-reachable materials.  Single exit, result
// by value (out-parameters on divergent paths were demoted to scratch).
struct Scat {
  d3 nd, A;
  bool ok;
};
template <bool kCount>
__device__ __forceinline__ Scat scatter(const DMat* __restrict__ m, d3 d, d3 N, bool front, rt_rng& rng,
                                        Counters& c) {
  const int kind = m->kind;
  Scat r;
  r.ok = kind != RT_MAT_DIFFUSELIGHT;  // DiffuseLight does not scatter, material.go:296-298
  r.A = ld3(m->color);                 // Lambertian/Glass colour, Dielectric (1,1,1) (make_mat)
  r.nd = mk(0, 0, 0);
  if (kind == RT_MAT_LAMBERTIAN) {  // material.go:26-35
    d3 sd = N + rand_in_unit_sphere<kCount>(rng, c);
    if (fabs(sd.x) < 1e-8 && fabs(sd.y) < 1e-8 && fabs(sd.z) < 1e-8) sd = N;
    r.nd = normalize(sd);
  } else if (kind == RT_MAT_GLASS || kind == RT_MAT_DIELECTRIC) {  // advanced_materials.go:21-46
    const double ior = m->ior;
    double ratio = front ? 1.0 / ior : ior;
    d3 u = normalize(d);
    double ct = gmin_x1(dot(neg(u), N));
    double st = sqrt(1.0 - ct * ct);
    bool refl = ratio * st > 1.0;  // cannotRefract
    if (!refl) {                   // Go's || short-circuit: the draw happens only here
      double r0 = (1 - ratio) / (1 + ratio);
      r0 = r0 * r0;
      double R = r0 + (1 - r0) * pow_n<5>(1 - ct);
      refl = R > draw<kCount>(rng, c);
    }
    r.nd = refl ? reflect(u, N) : refract(u, N, ratio);
  } else if (r.ok) {
    // Metal (material.go:75-113), Shiny (:169-189), PerfectMirror
    // (advanced_materials.go:125-151): mirror direction, optional perturbation
    d3 refl = reflect(d, N);
    if (m->rough_draw) {
      d3 pert = muls(rand_in_unit_sphere<kCount>(rng, c), m->roughness);
      refl = normalize(refl + pert);
    }
    const double f0 = m->f0;
    const double f = f0 + (1.0 - f0) * pow_n<5>(1.0 - fabs(dot(d, N)));
    const d3 col = r.A;
    // Metal/Shiny blend factor fs; PerfectMirror: Go constant-folds
    // (1.0 - 0.9) exactly to float64(0.1), i.e. col*0.1 + f*0.9
    const double fs = m->fs;
    const double wc = kind == RT_MAT_PERFECTMIRROR ? 0.1 : 1.0 - fs;
    const double wf = kind == RT_MAT_PERFECTMIRROR ? 0.9 : fs;
    d3 ea = mk(col.x * wc + f * wf, col.y * wc + f * wf, col.z * wc + f * wf);
    if (kind == RT_MAT_METAL) {
      ea = mk(clamp01(ea.x), clamp01(ea.y), clamp01(ea.z));
      if (m->blend_metal) {
        const double mf = m->mf;
        ea = mk(ea.x * (1.0 - mf) + f * mf, ea.y * (1.0 - mf) + f * mf, ea.z * (1.0 - mf) + f * mf);
      }
    } else if (kind == RT_MAT_SHINY) {
      ea = mk(gmin1_first(ea.x), gmin1_first(ea.y), gmin1_first(ea.z));
    }
    r.A = ea;
    r.nd = refl;
  }
  return r;
}

// ------------------------------------------------------------ kernel
template <bool kCount, bool kStage>
__global__ __launch_bounds__(256, RT_WAVES_PER_SIMD) void render_kernel(const KParams pk) {
  __shared__ double red[3][256];
  __shared__ unsigned long long cred[9];
  // dynamic LDS: [staged scene (kStage)][BVH stacks (kStack x 256 ints, lane-interleaved)]
  extern __shared__ __attribute__((aligned(16))) unsigned char dyn_lds[];

  const int tid = threadIdx.x;
  KParams p = pk;
  if constexpr (kStage) {
    // LDS-staged scene primitives: spheres | triangles | materials | lights
    // (one contiguous prefix of the device scene buffer), so the divergent
    // per-lane primitive reads of the shadow and scatter code hit LDS
    // (~64 cycles) instead of L1/L2 (measured: 55% of wave time in waits)
    const uint4* __restrict__ src = reinterpret_cast<const uint4*>(pk.stage_src);
    uint4* dst = reinterpret_cast<uint4*>(dyn_lds);
    for (int i = tid; i < pk.stage_bytes / 16; i += 256) dst[i] = src[i];
    const unsigned char* base = reinterpret_cast<const unsigned char*>(pk.stage_src);
    p.spheres = reinterpret_cast<const DSphere*>(dyn_lds + (reinterpret_cast<const unsigned char*>(pk.spheres) - base));
    p.tris = reinterpret_cast<const DTri*>(dyn_lds + (reinterpret_cast<const unsigned char*>(pk.tris) - base));
    p.mats = reinterpret_cast<const DMat*>(dyn_lds + (reinterpret_cast<const unsigned char*>(pk.mats) - base));
    p.lights = reinterpret_cast<const DLight*>(dyn_lds + (reinterpret_cast<const unsigned char*>(pk.lights) - base));
    __syncthreads();
  }
  const int S = p.slices;
  const int P = p.pix_per_wg;
  const int wg = blockIdx.x;
  // dispatch order: the host sorts this rank's tiles by estimated cost, so
  // long multi-bounce paths start first instead of trailing the launch
  const int slot = wg / p.blocks_per_tile;
  const int blk = wg - slot * p.blocks_per_tile;
  const int lt = p.tile_order ? p.tile_order[slot] : slot;  // local tile index
  const int tile = p.rank + lt * p.world;
  const int tx = tile % p.tiles_x, ty = tile / p.tiles_x;
  const int pix = tid / S;  // pixel within the block
  const int q = tid - pix * S;  // sample slice
  const int tp = blk * P + pix;  // row-major pixel index within the 32x32 tile
  const int lx = tp & 31, ly = tp >> 5;
  const int x = tx * 32 + lx, y = ty * 32 + ly;
  const bool valid = pix < P && tp < 1024 && tile < p.ntiles && x < p.W && y < p.H;
  int* stack = reinterpret_cast<int*>(dyn_lds + p.stack_off) + (tid >> 6) * (kStack * 64) + (tid & 63);

  Counters c;
  if constexpr (kCount) {
    for (int i = 0; i < 9; ++i) c.v[i] = 0;
    if (tid < 9) cred[tid] = 0;
  }
#ifdef RT_WG_TIMING
  const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
  unsigned long long dbg_hit = 0, dbg_light = 0, dbg_scat = 0, dbg_iter = 0;
#endif
  unsigned long long dbg_t[3] = {0, 0, 0};  // timing builds: candidates / hard shadow / soft loop

  const uint32_t pixel = (uint32_t)y * (uint32_t)p.W + (uint32_t)x;
  const double W = (double)p.W, H = (double)p.H;
  // getRay constants (renderer.go:377-390): lowerLeftCorner = origin -
  // horizontal/2 - vertical/2 - (0,0,focal)
  const double vw = 2.0 * p.aspect;
  const double llcx = p.cam[0] - vw / 2, llcy = p.cam[1] - 1.0, llcz = p.cam[2] - 1.0;

  // primary-ray frustum culling (host-computed per tile, schedule.cpp): only
  // primitives whose bounding sphere meets the cone of the tile's camera
  // rays are scanned for depth-0 hits.  Every sample still generates and
  // traces its ray; provably-missed primitives are skipped, like a BVH.
  const Cand all{~0ull, ~0ull};
  Cand prim = all;
  if (p.tile_masks) {
    prim.s = p.tile_masks[2 * lt];
    prim.t = p.tile_masks[2 * lt + 1];
  }

  double sx = 0, sy = 0, sz = 0;  // this lane's sample sum
  d3 o = mk(0, 0, 0), d = mk(0, 0, 0), T = mk(1, 1, 1), L = mk(0, 0, 0);
  rt_rng rng{0, 0, 0, 0};
  int depth = 0;
  int s = q;
  bool alive = false;

  for (;;) {
    if (!alive) {
      if (!valid || s >= p.spp) break;
      rt_rng_init(&rng, p.seed_key, pixel, (uint32_t)s);
      s += S;
      cnt<kCount>(c, C_CAM);
      double u = ((double)x + draw<kCount>(rng, c)) / W;
      double v = ((double)y + draw<kCount>(rng, c)) / H;
      o = mk(p.cam[0], p.cam[1], p.cam[2]);
      d = mk(((llcx + vw * u) + 0.0) - o.x, ((llcy + 0.0) + 2.0 * v) - o.y, ((llcz + 0.0) + 0.0) - o.z);
      T = mk(1, 1, 1);
      L = mk(0, 0, 0);
      depth = 0;
      alive = true;
    }
    bool done = depth >= p.max_depth;  // traceRay depth cut-off: contributes 0
    HitSel hs;
#ifdef RT_WG_TIMING
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
    ++dbg_iter;
#endif
    if (!done) {
      cnt<kCount>(c, C_BOUNCE);
      done = !closest_hit<kCount>(p, o, d, hs, stack, depth == 0 ? prim : all, c);  // miss -> black
    }
#ifdef RT_WG_TIMING
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
    dbg_hit += ts1 - ts0;
#endif
    if (done) {
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    cnt<kCount>(c, C_SHADE);
    // HitRecord of the closest primitive (sphere.go:42-58, triangle.go:68-81)
    d3 P, N;
    bool front;
    int mi, self;
    if (!hs.is_tri) {
      const DSphere& S0 = p.spheres[hs.idx];
      const double t = hs.num / len2(d);
      P = o + muls(d, t);
      d3 outward = divs(P - ld3(S0.c), S0.r);
      front = dot(d, outward) < 0;
      N = front ? outward : neg(outward);
      mi = S0.mat;
      self = S0.obj;
    } else {
      const DTri& T0 = p.tris[hs.idx];
      P = o + muls(d, hs.num);
      double w = 1.0 - hs.u - hs.v;
      d3 n = ld3(T0.n);
      N = normalize((muls(n, w) + muls(n, hs.u)) + muls(n, hs.v));
      front = dot(d, N) < 0;
      if (!front) N = neg(N);
      mi = T0.mat;
      self = T0.obj;
    }
    const DMat* __restrict__ m = p.mats + mi;
#ifdef RT_WG_TIMING
    const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
#endif
    d3 D = direct_lighting<kCount>(p, m, P, N, front, self, rng, stack, c, dbg_t);
#ifdef RT_WG_TIMING
    const unsigned long long ts3 = __builtin_amdgcn_s_memtime();
    dbg_light += ts3 - ts2;
#endif
    d3 E = ld3(m->emit);
    const Scat sc = scatter<kCount>(m, d, N, front, rng, c);
#ifdef RT_WG_TIMING
    dbg_scat += __builtin_amdgcn_s_memtime() - ts3;
#endif
    if (!sc.ok) {
      L = L + mul(T, E + D);
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    L = L + mul(T, E + muls(D, m->dw));
    if (!p.recursive || depth + 1 >= p.max_depth) {
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    T = mul(T, muls(sc.A, m->rw));
    o = P;
    d = sc.nd;
    depth += 1;
  }

#ifdef RT_WG_TIMING
  const unsigned long long t_loop = __builtin_amdgcn_s_memrealtime();
#endif
  // ---- reduce the S slices of each pixel in slice order
  red[0][tid] = sx;
  red[1][tid] = sy;
  red[2][tid] = sz;
  if constexpr (kCount) {
    __syncthreads();
    for (int i = 0; i < 9; ++i) atomicAdd(&cred[i], c.v[i]);
  }
  // pairwise tree over the S slices of each pixel (fixed order: the result
  // depends only on the samples, never on timing or the GPU count)
  for (int n = S; n > 1;) {
    const int h = (n + 1) >> 1;
    __syncthreads();
    if (pix < P && q < n - h) {
      red[0][tid] += red[0][tid + h];
      red[1][tid] += red[1][tid + h];
      red[2][tid] += red[2][tid + h];
    }
    n = h;
  }
  __syncthreads();
  if (tid < P) {
    const int tp2 = blk * P + tid;
    const int lx2 = tp2 & 31, ly2 = tp2 >> 5;
    const int x2 = tx * 32 + lx2, y2 = ty * 32 + ly2;
    if (tp2 < 1024 && tile < p.ntiles && x2 < p.W && y2 < p.H) {
      const int base = tid * S;
      const double ax = red[0][base], ay = red[1][base], az = red[2][base];
      const double n = (double)p.spp;
      const double mx = ax / n, my = ay / n, mz = az / n;  // DivScalar(float64(samples))
      size_t oi;
      if (p.layout == RT_LAYOUT_IMAGE)
        oi = (size_t)y2 * p.W + x2;
      else
        oi = (size_t)lt * 1024 + (size_t)tp2;
      if (p.out_linear) {
        p.out_linear[oi * 3 + 0] = (float)mx;
        p.out_linear[oi * 3 + 1] = (float)my;
        p.out_linear[oi * 3 + 2] = (float)mz;
      }
      if (p.out_rgba) {
        // toneMap (renderer.go:348-367) then Vec3.ToRGB (vector.go:106-109)
        const double g = 1.0 / 2.2;
        const double tx_ = clamp01(pow_gamma(1.0 - exp(-(mx * 1.0)), g));
        const double ty_ = clamp01(pow_gamma(1.0 - exp(-(my * 1.0)), g));
        const double tz_ = clamp01(pow_gamma(1.0 - exp(-(mz * 1.0)), g));
        const uint32_t px4 = go_u8(clamp01(tx_) * 255) | (go_u8(clamp01(ty_) * 255) << 8) |
                             (go_u8(clamp01(tz_) * 255) << 16) | (255u << 24);
        *reinterpret_cast<uint32_t*>(p.out_rgba + oi * 4) = px4;
      }
    }
  }
  if constexpr (kCount) {
    __syncthreads();
    if (tid < 9) atomicAdd(&p.counts[tid], cred[tid]);
  }
#ifdef RT_WG_TIMING
  for (int off = 32; off > 0; off >>= 1) {  // wave max of the per-lane section times
    dbg_hit = max(dbg_hit, (unsigned long long)__shfl_xor(dbg_hit, off));
    dbg_light = max(dbg_light, (unsigned long long)__shfl_xor(dbg_light, off));
    dbg_scat = max(dbg_scat, (unsigned long long)__shfl_xor(dbg_scat, off));
    dbg_iter = max(dbg_iter, (unsigned long long)__shfl_xor(dbg_iter, off));
    for (int k = 0; k < 3; ++k) dbg_t[k] = max(dbg_t[k], (unsigned long long)__shfl_xor(dbg_t[k], off));
  }
  if (p.dbg && (tid & 63) == 0) {
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    unsigned long long* r = p.dbg + ((size_t)wg * 4 + (tid >> 6)) * 8;
    r[0] = t_start;
    r[1] = t_loop;
    r[2] = __builtin_amdgcn_s_memrealtime();
    r[3] = ((unsigned long long)xcc << 32) | hw;
    r[4] = dbg_hit;
    r[5] = dbg_light;
    r[6] = dbg_scat;
    r[7] = dbg_iter;
    r[4] = dbg_t[0];  // repurposed: candidates
    r[6] = dbg_t[2];  // soft loop (hard shadow = light - both)
    r[5] = dbg_light;
  }
#endif
}

// Gathered [world][max_local][1024] packed tiles -> W*H image.
__global__ __launch_bounds__(256) void unpack_kernel(int W, int H, int world, int max_local, int tiles_x,
                                                     int ntiles, const float* __restrict__ pl,
                                                     const uint8_t* __restrict__ pr, float* __restrict__ ol,
                                                     uint8_t* __restrict__ orgba) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // over world*max_local*1024
  const long long total = (long long)world * max_local * 1024;
  if (i >= total) return;
  const int r = (int)(i / ((long long)max_local * 1024));
  const int rem = (int)(i - (long long)r * max_local * 1024);
  const int lt = rem / 1024, pi = rem % 1024;
  const int t = r + lt * world;
  if (t >= ntiles) return;
  const int x = (t % tiles_x) * 32 + pi % 32, y = (t / tiles_x) * 32 + pi / 32;
  if (x >= W || y >= H) return;
  const size_t o = (size_t)y * W + x;
  if (ol && pl) {
    ol[o * 3 + 0] = pl[i * 3 + 0];
    ol[o * 3 + 1] = pl[i * 3 + 1];
    ol[o * 3 + 2] = pl[i * 3 + 2];
  }
  if (orgba && pr) *reinterpret_cast<uint32_t*>(orgba + o * 4) = *reinterpret_cast<const uint32_t*>(pr + i * 4);
}

int launch_render(const KParams& p, bool count, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (p.num_wgs <= 0) return hipSuccess;
  const size_t shmem = (size_t)p.stack_off + (p.use_bvh ? sizeof(int) * kStack * 256 : 0);
  const bool stage = p.stage_bytes > 0;
  if (count && stage)
    hipLaunchKernelGGL((render_kernel<true, true>), dim3(p.num_wgs), dim3(256), shmem, st, p);
  else if (count)
    hipLaunchKernelGGL((render_kernel<true, false>), dim3(p.num_wgs), dim3(256), shmem, st, p);
  else if (stage)
    hipLaunchKernelGGL((render_kernel<false, true>), dim3(p.num_wgs), dim3(256), shmem, st, p);
  else
    hipLaunchKernelGGL((render_kernel<false, false>), dim3(p.num_wgs), dim3(256), shmem, st, p);
  return (int)hipGetLastError();
}

int launch_unpack(int32_t W, int32_t H, int32_t world, int32_t max_local, const float* pl, const uint8_t* pr,
                  float* ol, uint8_t* orgba, void* stream) {
  const long long total = (long long)world * max_local * 1024;
  if (total <= 0) return hipSuccess;
  const int tiles_x = (W + 31) / 32, ntiles = tiles_x * ((H + 31) / 32);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, W, H, world, max_local,
                     tiles_x, ntiles, pl, pr, ol, orgba);
  return (int)hipGetLastError();
}

}  // namespace rtgo
