// rt_device.h — device code shared by the gfx950 kernels of the renderer
// core: the megakernel (rt_kernel.hip) and the wavefront path for BVH scenes
// (rt_wavefront.hip).  Vec3 arithmetic (internal/math/vector.go), Go's math
// semantics, the intersection tests (Sphere.Hit, Triangle.Hit), BVH
// traversal, and Material.Scatter — all binary64 in the reference's order
// (built with -ffp-contract=off), so every kernel that uses them makes the
// oracle's decisions bit for bit.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/rt_rng.h"
#include "rt_internal.h"

// Cross-lane reads belong in CONVERGED code.  __shfl (ds_bpermute) from a
// lane that is inactive at the read returns no data, so an owner's state
// read inside an owner-only branch silently becomes 0: a rejected r03
// soft-shadow variant hung that way (a stream restarted from state 0 every
// round and never accepted a point).  The checking build
// (`make xlane`, -DRT_CHECK_XLANE) routes every __shfl of the kernels through
// rt_checked_shfl, which counts reads whose source lane is inactive; the GPU
// test suite renders with it and requires zero (tests/test_gpu_xlane.py).
#ifdef RT_CHECK_XLANE
namespace rtgo {
__device__ unsigned long long g_xlane_faults;  // (one per translation unit: see xlane_faults_*)
}
template <typename T>
__device__ __forceinline__ T rt_checked_shfl(T v, int src, int width = 64) {
  const unsigned long long ex = __builtin_amdgcn_read_exec();
  const int lane = (int)(threadIdx.x & 63);
  const int from = (lane & ~(width - 1)) + (src & (width - 1));
  if (!((ex >> (from & 63)) & 1ull)) atomicAdd(&rtgo::g_xlane_faults, 1ull);
  return __shfl(v, src, width);
}
#define __shfl(...) rt_checked_shfl(__VA_ARGS__)
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

// A binary64 constant materialised at its use (two s_mov_b32) rather than
// hoisted into an SGPR pair for the whole kernel: the bounce loop is
// SGPR-bound, and hoisted constants push loop state into VGPR-lane spills.
constexpr uint64_t bits(double v) { return __builtin_bit_cast(uint64_t, v); }
template <uint64_t B>
__device__ __forceinline__ double kconst() {
  uint32_t lo, hi;
  asm volatile("s_mov_b32 %0, %2\n\ts_mov_b32 %1, %3"
               : "=s"(lo), "=s"(hi)
               : "i"((uint32_t)B), "i"((uint32_t)(B >> 32)));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
#define KC(v) kconst<bits(v)>()

// ------------------------------------------------------------ lane helpers
__device__ __forceinline__ uint32_t rl32(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  return ((uint64_t)rl32((uint32_t)(v >> 32), lane) << 32) | rl32((uint32_t)v, lane);
}
__device__ __forceinline__ double rld(double v, int lane) {
  return __builtin_bit_cast(double, rl64(__builtin_bit_cast(uint64_t, v), lane));
}
__device__ __forceinline__ d3 rl3(d3 v, int lane) { return mk(rld(v.x, lane), rld(v.y, lane), rld(v.z, lane)); }
// keep a (uniform) value in VGPRs: the SGPR file is the scarce one in the bounce loop
__device__ __forceinline__ double inv(double v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ d3 inv3(d3 v) { return mk(inv(v.x), inv(v.y), inv(v.z)); }

struct Counters {
  unsigned long long v[9];
};
enum { C_CAM = 0, C_BOUNCE, C_SHADOW, C_SPH, C_TRI, C_BOX, C_SHADE, C_LIGHT, C_RNG };

template <bool kCount>
__device__ __forceinline__ void cnt(Counters& c, int i, unsigned long long n = 1) {
  if constexpr (kCount) c.v[i] += n;
}

template <bool kCount>
__device__ __forceinline__ double draw(rt_rng& r, Counters& c) {
  cnt<kCount>(c, C_RNG);
  return rt_rng_draw(&r);
}

// State before draw 3h of a stream whose state is x: x_3h = A_3h x + C_3h
// (jump table entry h, in LDS); draws 3h+1, 3h+2 follow by plain steps.
__device__ __forceinline__ uint64_t state_at3(uint64_t x, const uint64_t* jump, int h) {
  return jump[2 * h] * x + jump[2 * h + 1];
}

// RandomVec3InUnitSphere, vector.go:132-139.
// RandomVec3InUnitSphere (internal/math/vector.go:132-139) from three raw
// draws: p = 2 RandomFloat() - 1 per axis, accepted when LengthSquared() < 1.
// The point is exact in binary64 (u = x 2^-32 has 32 significant bits, so
// 2u - 1 does not round); only the binary64 sum of squares rounds.
__device__ __forceinline__ d3 unit_ball_point(uint32_t ux, uint32_t uy, uint32_t uz) {
  return mk(rt_bits_to_unit(ux) * 2 - 1, rt_bits_to_unit(uy) * 2 - 1, rt_bits_to_unit(uz) * 2 - 1);
}
// The acceptance decision, screened in binary32: each coordinate is within
// 2^-22 of the exact 2u - 1 (the draw rounded to 24 bits, one fma rounding),
// so the float sum of squares is within 2^-19 of the exact one and the
// binary64 sum within 2^-50.  Below 1 - 2^-16 the binary64 test accepts,
// above 1 + 2^-16 it rejects; in between (a shell holding ~4e-5 of the
// tries) the reference's binary64 arithmetic decides.  Same answer, a
// fraction of the binary64 operations.
__device__ __forceinline__ bool unit_ball_accept(uint32_t ux, uint32_t uy, uint32_t uz) {
  const float fx = __builtin_fmaf((float)ux, 0x1p-31f, -1.f), fy = __builtin_fmaf((float)uy, 0x1p-31f, -1.f),
              fz = __builtin_fmaf((float)uz, 0x1p-31f, -1.f);
  const float l = __builtin_fmaf(fz, fz, __builtin_fmaf(fy, fy, fx * fx));
  if (l < 1.f - 0x1p-16f) return true;
  if (l > 1.f + 0x1p-16f) return false;
  return len2(unit_ball_point(ux, uy, uz)) < 1;
}

template <bool kCount>
__device__ __forceinline__ d3 rand_in_unit_sphere(rt_rng& r, Counters& c) {
  for (;;) {
    const uint32_t ux = rt_rng_next(&r), uy = rt_rng_next(&r), uz = rt_rng_next(&r);
    cnt<kCount>(c, C_RNG, 3);
    if (unit_ball_accept(ux, uy, uz)) return unit_ball_point(ux, uy, uz);
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

// Conservative slab test of a float box against [tmin, tmax].
__device__ __forceinline__ bool box_hit(const DBVHNode& n, d3 o, d3 id, double tmin, double tmax) {
  double tx0 = ((double)n.lo[0] - o.x) * id.x, tx1 = ((double)n.hi[0] - o.x) * id.x;
  double ty0 = ((double)n.lo[1] - o.y) * id.y, ty1 = ((double)n.hi[1] - o.y) * id.y;
  double tz0 = ((double)n.lo[2] - o.z) * id.z, tz1 = ((double)n.hi[2] - o.z) * id.z;
  double tn = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmax(fmin(tz0, tz1), tmin));
  double tf = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmin(fmax(tz0, tz1), tmax));
  // margins: the box is padded by >= 1 float ulp; allow 1e-9 relative slack
  return tn <= tf + fabs(tf) * KC(1e-9) + KC(1e-12);
}

// The ray in binary32 for the slab tests below the root: origin rounded to
// float (error <= 2^-24 |o| per axis, covered by the boxes' padding,
// bvh.cpp), inverse direction rounded and clamped to 1e30 (inv_dir's 1e300
// for a zero component stays a huge finite value, no 0 * inf).
struct Ray32 {
  float ox, oy, oz, ix, iy, iz;
};
__device__ __forceinline__ Ray32 ray32(d3 o, d3 id) {
  return Ray32{(float)o.x, (float)o.y, (float)o.z, (float)fmin(fmax(id.x, -1e30), 1e30),
               (float)fmin(fmax(id.y, -1e30), 1e30), (float)fmin(fmax(id.z, -1e30), 1e30)};
}
// a [tmin, tmax] window widened for binary32 (both are >= 0)
__device__ __forceinline__ float t_lo32(double t) { return (float)(t * (1.0 - 0x1p-20)); }
__device__ __forceinline__ float t_hi32(double t) { return (float)(t * (1.0 + 0x1p-20)); }
// binary32 slab test of a child box, conservative: the products carry
// < 2^-21 relative error, the slack below is 2^-20 of the interval ends;
// also returns the entry distance (child ordering)
__device__ __forceinline__ bool box_hit32(const DBVHNode& n, const Ray32& r, float tmin, float tmax, float& tn) {
  const float tx0 = (n.lo[0] - r.ox) * r.ix, tx1 = (n.hi[0] - r.ox) * r.ix;
  const float ty0 = (n.lo[1] - r.oy) * r.iy, ty1 = (n.hi[1] - r.oy) * r.iy;
  const float tz0 = (n.lo[2] - r.oz) * r.iz, tz1 = (n.hi[2] - r.oz) * r.iz;
  tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
  const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
  return tn <= tf + (fabsf(tn) + fabsf(tf)) * 0x1p-20f;
}
// BVH traversal state: a node is (first << 3) | count, count 0 = internal
// node whose children are the adjacent records first, first + 1 (bvh.cpp),
// count 1..4 = leaf of spheres [first, first + count).  Children are tested
// together, from the one 64-B load of their two records; the nearer one hit
// is entered and the other pushed, so the per-lane LDS stack holds ready
// node codes and a pop needs no memory access.
__device__ __forceinline__ int bvh_code(const DBVHNode& n) { return (n.left_or_first << 3) | n.count; }

__device__ __forceinline__ d3 inv_dir(d3 d) {
  // zero components get a huge finite inverse: no 0*inf NaN in the slabs
  return mk(1.0 / (d.x != 0 ? d.x : 1e-300), 1.0 / (d.y != 0 ? d.y : 1e-300), 1.0 / (d.z != 0 ? d.z : 1e-300));
}
// The same through approx_rcp (v_rcp_f64 + one Newton step: relative error
// near 2^-50): the slab tests that use it (box_hit's 1e-9 relative slack,
// the quantized test's 2^-22 bound, rt_wavefront.hip ray_q_axis) only need
// a conservative inverse, and it spares three IEEE divisions per ray.
__device__ __forceinline__ d3 inv_dir_fast(d3 d) {
  return mk(approx_rcp(d.x != 0 ? d.x : 1e-300), approx_rcp(d.y != 0 ? d.y : 1e-300),
            approx_rcp(d.z != 0 ? d.z : 1e-300));
}


// Can the ray meet the (padded) box within [tmin, tmax]?  Conservative:
// slab test with the same slack as box_hit; `id` from inv_dir().
__device__ __forceinline__ bool ray_box(const DBox& b, d3 o, d3 id, double tmin, double tmax) {
  const double tx0 = (b.lo[0] - o.x) * id.x, tx1 = (b.hi[0] - o.x) * id.x;
  const double ty0 = (b.lo[1] - o.y) * id.y, ty1 = (b.hi[1] - o.y) * id.y;
  const double tz0 = (b.lo[2] - o.z) * id.z, tz1 = (b.hi[2] - o.z) * id.z;
  const double tn = fmax(fmax(fmin(tx0, tx1), fmin(ty0, ty1)), fmax(fmin(tz0, tz1), tmin));
  const double tf = fmin(fmin(fmax(tx0, tx1), fmax(ty0, ty1)), fmin(fmax(tz0, tz1), tmax));
  return tn <= tf + fabs(tf) * KC(1e-9) + KC(1e-12);
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
__device__ __forceinline__ bool closest_hit(const Geo& p, d3 o, d3 d, HitSel& hs, int* stack, Cand m,
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
    cnt<kCount>(c, C_BOX);
    const DBVHNode root = p.bvh[0];
    if (!box_hit(root, o, id, tmin, closest)) return false;
    const Ray32 r32 = ray32(o, id);
    const float tminf = t_lo32(tmin);
    // while-while (Aila & Laine): lanes descend internal nodes together,
    // then test their leaves together; -1 = traversal finished
    int cur = bvh_code(root);
    while (cur != -1) {
      while ((cur & 7) == 0) {
        const int first = cur >> 3;
        const DBVHNode L = p.bvh[first], R = p.bvh[first + 1];
        cnt<kCount>(c, C_BOX, 2);
        float tl, tr;
        const float tmaxf = t_hi32(closest);
        const bool hl = box_hit32(L, r32, tminf, tmaxf, tl), hr = box_hit32(R, r32, tminf, tmaxf, tr);
        if (hl || hr) {
          const bool lfirst = hl && (!hr || tl <= tr);
          if (hl && hr) {
            stack[sp * 64] = lfirst ? bvh_code(R) : bvh_code(L);
            ++sp;
          }
          cur = lfirst ? bvh_code(L) : bvh_code(R);
        } else {
          cur = sp == 0 ? -1 : stack[--sp * 64];
        }
      }
      if (cur == -1) break;
      const int first = cur >> 3, count = cur & 7;
      for (int i = first; i < first + count; ++i) {
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
      cur = sp == 0 ? -1 : stack[--sp * 64];
    }
    return found;
  }
  // candidate masks (primary rays: the tile's frustum culling; all ones
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
  // triangles cube by cube, in hittable order: a cube whose box the ray
  // misses within [tmin, closest] cannot hold an accepted hit
  const d3 id = inv_dir(d);
  for (int j = 0; j < p.nb; ++j) {
    const DBox& B = p.boxes[j];
    if (use_m && !((m.t >> B.first) & 0xFFFull)) continue;
    if (!ray_box(B, o, id, tmin, closest)) continue;
    for (int i = B.first; i < B.first + B.count; ++i) {
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
  }
  return found;
}

// hitWorld used as an occlusion query over everything (BVH or large linear
// scenes): calculateSmartShadow only asks whether any hittable is hit in
// [tmin, tmax] (renderer.go:305,320).
template <bool kCount>
__device__ __forceinline__ bool any_hit(const Geo& p, d3 o, d3 d, double tmax, int* stack, Counters& c) {
  const double tmin = 0.001;
  const double a = len2(d);
  const double inv_a = approx_rcp(a);
  if (p.use_bvh) {
    const d3 id = inv_dir(d);
    int sp = 0;
    cnt<kCount>(c, C_BOX);
    const DBVHNode root = p.bvh[0];
    if (!box_hit(root, o, id, tmin, tmax)) return false;
    const Ray32 r32 = ray32(o, id);
    const float tminf = t_lo32(tmin), tmaxf = t_hi32(tmax);
    int cur = bvh_code(root);  // while-while, as in closest_hit
    while (cur != -1) {
      while ((cur & 7) == 0) {
        const int first = cur >> 3;
        const DBVHNode L = p.bvh[first], R = p.bvh[first + 1];
        cnt<kCount>(c, C_BOX, 2);
        float tl, tr;
        const bool hl = box_hit32(L, r32, tminf, tmaxf, tl), hr = box_hit32(R, r32, tminf, tmaxf, tr);
        if (hl || hr) {
          const bool lfirst = hl && (!hr || tl <= tr);
          if (hl && hr) {
            stack[sp * 64] = lfirst ? bvh_code(R) : bvh_code(L);
            ++sp;
          }
          cur = lfirst ? bvh_code(L) : bvh_code(R);
        } else {
          cur = sp == 0 ? -1 : stack[--sp * 64];
        }
      }
      if (cur == -1) break;
      const int first = cur >> 3, count = cur & 7;
      for (int i = first; i < first + count; ++i) {
        cnt<kCount>(c, C_SPH);
        double num;
        if (sphere_query(p.spheres[i], o, d, a, inv_a, tmin, tmax, num)) return true;
      }
      cur = sp == 0 ? -1 : stack[--sp * 64];
    }
    return false;
  }
  for (int i = 0; i < p.ns; ++i) {
    cnt<kCount>(c, C_SPH);
    double num;
    if (sphere_query(p.spheres[i], o, d, a, inv_a, tmin, tmax, num)) return true;
  }
  const d3 id = inv_dir(d);
  for (int j = 0; j < p.nb; ++j) {
    const DBox& B = p.boxes[j];
    if (!ray_box(B, o, id, tmin, tmax)) continue;
    for (int i = B.first; i < B.first + B.count; ++i) {
      cnt<kCount>(c, C_TRI);
      double t, u, v;
      if (tri_test(p.tris[i], o, d, tmin, tmax, t, u, v)) return true;
    }
  }
  return false;
}

// ------------------------------------------------------------ scatter
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

// ------------------------------------------------------------ camera
// Launch-uniform inputs of the camera rays (getRay, renderer.go:377-390).
struct CamK {
  uint64_t key;
  uint32_t W;
  double dW, dH, vw, llcx, llcy, llcz, ox, oy, oz;
  double rW, rH;  // refined reciprocals of dW, dH (div_by)
};
// The compiler's binary64 division n / d is v_div_scale (n and d), v_rcp_f64,
// two Newton steps on the reciprocal, q = n*r, the residual fma, v_div_fmas
// and v_div_fixup.  For the camera jitter n = x + rand is in [0, W) with
// rand a multiple of 2^-32 (so n is 0 or at least 2^-32) and d = W or H is
// an integer in [1, 2^16]: v_div_scale scales nothing, v_div_fmas is a plain
// fma and v_div_fixup returns its input, so the sequence is the three
// operations below with the reciprocal refinement done once per block, and
// the quotient is the IEEE one bit for bit (validate_settings bounds W, H).
__device__ __forceinline__ double refined_rcp(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double div_by(double n, double d, double r) {
  const double q = n * r;
  return __builtin_fma(__builtin_fma(-d, q, n), r, q);
}
template <bool kCount>
__device__ __forceinline__ void camera_ray_c(const CamK& ck, int x, int y, int s, rt_rng& rng, d3& o, d3& d,
                                             Counters& c) {
  rt_rng_init(&rng, ck.key, (uint32_t)y * ck.W + (uint32_t)x, (uint32_t)s);
  const double u = div_by((double)x + draw<kCount>(rng, c), ck.dW, ck.rW);
  const double v = div_by((double)y + draw<kCount>(rng, c), ck.dH, ck.rH);
  o = mk(ck.ox, ck.oy, ck.oz);
  d = mk(((ck.llcx + ck.vw * u) + 0.0) - o.x, ((ck.llcy + 0.0) + 2.0 * v) - o.y, ((ck.llcz + 0.0) + 0.0) - o.z);
}

__device__ __forceinline__ CamK make_cam(uint64_t seed_key, int W, int H, double aspect, double cx, double cy,
                                         double cz) {
  CamK r;
  r.key = seed_key;
  r.W = (uint32_t)W;
  r.dW = (double)W;
  r.dH = (double)H;
  r.rW = refined_rcp(r.dW);
  r.rH = refined_rcp(r.dH);
  // lowerLeftCorner = origin - horizontal/2 - vertical/2 - (0,0,focal)
  r.vw = 2.0 * aspect;
  r.llcx = cx - r.vw / 2;
  r.llcy = cy - 1.0;
  r.llcz = cz - 1.0;
  r.ox = cx;
  r.oy = cy;
  r.oz = cz;
  return r;
}

// ------------------------------------------------------------ pixel output
// toneMap (renderer.go:348-367) then Vec3.ToRGB (vector.go:106-109) of a
// pixel's mean radiance: opaque RGBA8.
// Go's math.Max / math.Min (NaN propagates; +0 > -0).
__device__ __forceinline__ double go_max2(double x, double y) {
  if (__builtin_isinf(x) && x > 0) return x;
  if (__builtin_isinf(y) && y > 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return __builtin_signbit(x) ? y : x;
  return x > y ? x : y;
}
__device__ __forceinline__ double go_min2(double x, double y) {
  if (__builtin_isinf(x) && x < 0) return x;
  if (__builtin_isinf(y) && y < 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return __builtin_signbit(x) ? x : y;
  return x < y ? x : y;
}

// AtmosphereConfig.GetSkyColor (internal/atmosphere/atmosphere.go:100-135),
// binary64 in its order; its undefined FastVec3* helpers are the Vec3
// methods (vector.go): Normalize (0 for a zero vector), a.Lerp(b, t) =
// a + (b - a) * t, Dot, MulScalar; Max / Min with Go's NaN rules; Clamp(0.1, 0.98).
__device__ __forceinline__ d3 sky_lerp(d3 a, d3 b, double t) { return a + muls(b - a, t); }
// (inlined: a call in the bounce loop would impose the call ABI's register
// split on the whole kernel; this code only runs on a miss with a sky)
__device__ __forceinline__ d3 sky_color(const DSky* __restrict__ a, d3 dir) {
  const d3 u = normalize(dir);
  const double t = 0.5 * (u.y + 1.0);
  d3 sky = sky_lerp(ld3(a->bottom), ld3(a->top), t);
  const double depth = go_max2(0.0, u.y);
  const double atmospheric = exp(-depth * a->depth);
  const d3 scattering = sky_lerp(ld3(a->rayleigh), ld3(a->mie), atmospheric);
  sky = sky_lerp(sky, scattering, 0.25);
  const double sun_dot = dot(u, ld3(a->sun_dir));
  if (sun_dot > (1.0 - a->sun_size)) {
    double si = pow((sun_dot - (1.0 - a->sun_size)) / a->sun_size, 1.5);
    si = go_min2(si, 1.0);
    sky = sky_lerp(sky, ld3(a->sun_color), si * a->sun_intensity * 0.9);
  }
  double tf = a->time_of_day;
  if (tf > 0.5) tf = 1.0 - tf;
  tf *= 2.0;
  const double darkness = 1.0 - tf * 0.3;
  sky = muls(sky, darkness);
  if (a->fog_density > 0.0) sky = sky_lerp(ld3(a->fog_color), sky, exp(-a->fog_density));
  return mk(go_max2(0.1, go_min2(0.98, sky.x)), go_max2(0.1, go_min2(0.98, sky.y)),
            go_max2(0.1, go_min2(0.98, sky.z)));
}

__device__ __forceinline__ uint32_t tonemap_rgba8(double mx, double my, double mz) {
  const double g = 1.0 / 2.2;
  const double tx_ = clamp01(pow_gamma(1.0 - exp(-(mx * 1.0)), g));
  const double ty_ = clamp01(pow_gamma(1.0 - exp(-(my * 1.0)), g));
  const double tz_ = clamp01(pow_gamma(1.0 - exp(-(mz * 1.0)), g));
  return go_u8(clamp01(tx_) * 255) | (go_u8(clamp01(ty_) * 255) << 8) | (go_u8(clamp01(tz_) * 255) << 16) |
         (255u << 24);
}

}  // namespace rtgo
