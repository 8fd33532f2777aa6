// rt_kernel.hip — gfx950 (CDNA4) kernels of the renderer core.
//
// One launch renders every 32x32 tile (createRenderTasks,
// internal/renderer/renderer.go:398-436) that this rank owns.  Mapping
// (DESIGN.md §Kernels):
//   workgroup (256 lanes = 4 wave64) = one block of P pixels inside a tile
//                                     x S sample slices, P*S = 256;
//   lane = (pixel p, slice q) and traces samples q, q+S, q+2S, ... of its
//          pixel one after the other with a persistent, iterative bounce loop
//          (traceRay, renderer.go:165-227, unrolled): a lane whose path ends
//          immediately regenerates the next camera sample, so paths of
//          different length keep the wave's lanes busy instead of idling
//          until the longest path of the wave ends (ray compaction at the
//          lane level);
//   the S slice sums of a pixel are reduced in LDS in fixed slice order,
//   divided by spp, tone-mapped (toneMap, renderer.go:348-367) and written
//   once: float3 linear radiance + RGBA8.
// Scene data for linear-scan scenes is read with wave-uniform addresses, so
// it lives in SGPRs via the scalar cache (better than LDS: zero bank cycles,
// no VGPRs).  All arithmetic is binary64 in the reference's order; the file
// is compiled with -ffp-contract=off so results match the oracle bit for bit
// except for the sum order over samples and exp/log in the tone map.
#include <hip/hip_runtime.h>

#include "../../include/rt_rng.h"
#include "rt_internal.h"

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
    n = muls(n, -1);
    eta = 1 / eta;
    ct = -ct;
  }
  double s2 = eta * eta * (1 - ct * ct);
  if (s2 > 1) return reflect(v, n);
  double c2 = sqrt(1 - s2);
  return muls(v, eta) - muls(n, eta * ct + c2);
}
__device__ __forceinline__ d3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

// Go math.Max / math.Min (NaN-propagating, signed-zero aware).
__device__ __forceinline__ double gmax(double x, double y) {
  if (__builtin_isinf(x) && x > 0) return x;
  if (__builtin_isinf(y) && y > 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return __builtin_signbit(x) ? y : x;
  return x > y ? x : y;
}
__device__ __forceinline__ double gmin(double x, double y) {
  if (__builtin_isinf(x) && x < 0) return x;
  if (__builtin_isinf(y) && y < 0) return y;
  if (__builtin_isnan(x) || __builtin_isnan(y)) return __builtin_nan("");
  if (x == 0 && x == y) return __builtin_signbit(x) ? x : y;
  return x < y ? x : y;
}
// Go math.Pow(x, n) for a positive integer n: Go multiplies by repeated
// squaring (pow.go); frexp/ldexp only rescale by powers of two, so for
// normal-range values the products below round identically.
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
__device__ __forceinline__ double pow_spec(double x, int n) {
  if (n == 64) return pow_n<64>(x);
  if (n == 48) return pow_n<48>(x);
  return pow_n<32>(x);
}
// Go's uint8(float64) on amd64 (CVTTSD2SQ, then low byte): NaN -> 0.
__device__ __forceinline__ uint8_t go_u8(double f) {
  if (__builtin_isnan(f)) return 0;
  return (uint8_t)(int64_t)f;
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
__device__ __forceinline__ void cnt(Counters& c, int i, unsigned long long n = 1) {
  if constexpr (kCount) c.v[i] += n;
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
// Sphere.Hit root selection (sphere.go:22-40); returns the accepted root or
// a negative "miss" signal through `ok`.
__device__ __forceinline__ bool sphere_root(const DSphere& S, d3 o, d3 d, double a, double tmin, double tmax,
                                            double& t) {
  double ocx = o.x - S.c[0], ocy = o.y - S.c[1], ocz = o.z - S.c[2];
  double hb = ocx * d.x + ocy * d.y + ocz * d.z;
  double c = (ocx * ocx + ocy * ocy + ocz * ocz) - S.r * S.r;
  double disc = hb * hb - a * c;
  if (disc < 0) return false;
  double sq = sqrt(disc);
  double root = (-hb - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-hb + sq) / a;
    if (root < tmin || tmax < root) return false;
  }
  t = root;
  return true;
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

struct HitSel {
  double t, u, v;
  int idx;     // primitive index
  int is_tri;
};

// hitWorld closest hit, renderer.go:333-346 (linear scan in hittable order;
// spheres are scanned before triangles, exact t ties resolved by hittable
// index so the later hittable wins as in Go).
template <bool kCount>
__device__ __forceinline__ bool closest_hit(const KParams& p, d3 o, d3 d, double tmin, HitSel& hs,
                                            Counters& c) {
  double closest = __builtin_inf();
  bool found = false;
  int best_obj = -1;
  double a = len2(d);
  const DSphere* __restrict__ sp = p.spheres;
  for (int i = 0; i < p.ns; ++i) {
    cnt<kCount>(c, C_SPH);
    double t;
    if (sphere_root(sp[i], o, d, a, tmin, closest, t)) {
      closest = t;
      hs.t = t;
      hs.idx = i;
      hs.is_tri = 0;
      best_obj = sp[i].obj;
      found = true;
    }
  }
  const DTri* __restrict__ tp = p.tris;
  for (int i = 0; i < p.nt; ++i) {
    cnt<kCount>(c, C_TRI);
    double t, u, v;
    if (tri_test(tp[i], o, d, tmin, closest, t, u, v)) {
      if (t == closest && best_obj > tp[i].obj) continue;
      closest = t;
      hs.t = t;
      hs.u = u;
      hs.v = v;
      hs.idx = i;
      hs.is_tri = 1;
      best_obj = tp[i].obj;
      found = true;
    }
  }
  return found;
}

// hitWorld used as an occlusion query (calculateSmartShadow only asks
// whether any hittable is hit in [tmin, tmax], renderer.go:305,320).
template <bool kCount>
__device__ __forceinline__ bool any_hit(const KParams& p, d3 o, d3 d, double tmin, double tmax, Counters& c) {
  double a = len2(d);
  const DSphere* __restrict__ sp = p.spheres;
  for (int i = 0; i < p.ns; ++i) {
    cnt<kCount>(c, C_SPH);
    double t;
    if (sphere_root(sp[i], o, d, a, tmin, tmax, t)) return true;
  }
  const DTri* __restrict__ tp = p.tris;
  for (int i = 0; i < p.nt; ++i) {
    cnt<kCount>(c, C_TRI);
    double t, u, v;
    if (tri_test(tp[i], o, d, tmin, tmax, t, u, v)) return true;
  }
  return false;
}

// ------------------------------------------------------------ shading
// calculateDirectLighting (renderer.go:229-297) with calculateSmartShadow
// (renderer.go:299-331) inlined.
template <bool kCount>
__device__ __forceinline__ d3 direct_lighting(const KParams& p, const DMat& m, d3 P, d3 N, rt_rng& rng,
                                              Counters& c) {
  d3 total = mk(m.ambient, m.ambient, m.ambient);
  d3 albedo = ld3(m.albedo);
  const double metallic = m.metallic;
  for (int li = 0; li < p.nl; ++li) {
    const DLight& L = p.lights[li];
    d3 lv = ld3(L.pos) - P;
    double ldist = sqrt(lv.x * lv.x + lv.y * lv.y + lv.z * lv.z);
    d3 ldir = ldist == 0 ? mk(0, 0, 0) : divs(lv, ldist);
    if (ldist < 0.001) continue;
    cnt<kCount>(c, C_LIGHT);
    cnt<kCount>(c, C_SHADOW);
    double sf;
    if (any_hit<kCount>(p, P, ldir, 0.001, ldist, c)) {
      sf = 0.0;
    } else if (p.soft) {
      double sum = 0.0;
      for (int i = 0; i < 16; ++i) {
        d3 off = muls(rand_in_unit_sphere<kCount>(rng, c), 0.1);
        d3 sdir = normalize(ldir + off);
        cnt<kCount>(c, C_SHADOW);
        if (!any_hit<kCount>(p, P, sdir, 0.001, ldist, c)) sum += 1.0;
      }
      sf = sum / 16.0;
    } else {
      sf = 1.0;
    }
    if (sf > 0.0) {
      double cos_t = gmax(0, dot(N, ldir));
      double intensity = cos_t * L.intensity / (ldist * ldist);
      total = total + muls(albedo, m.diffuse_strength * intensity * sf);
      if (metallic > 0.5) {
        d3 view = normalize(muls(P, -1));
        d3 half = normalize(ldir + view);
        double si = pow_spec(gmax(0, dot(N, half)), m.spec_pow);
        total = total + muls(ld3(L.color), si * intensity * sf * metallic * 3.0);
      }
    }
  }
  return total;
}

// Material.Scatter for the 7 JSON-reachable materials.
template <bool kCount>
__device__ __forceinline__ bool scatter(const DMat& m, d3 d, d3 P, d3 N, bool front, rt_rng& rng, d3& nd,
                                        d3& A, Counters& c) {
  const int kind = m.kind;
  if (kind == RT_MAT_DIFFUSELIGHT) return false;  // material.go:296-298
  if (kind == RT_MAT_LAMBERTIAN) {                // material.go:26-35
    d3 sd = N + rand_in_unit_sphere<kCount>(rng, c);
    if (fabs(sd.x) < 1e-8 && fabs(sd.y) < 1e-8 && fabs(sd.z) < 1e-8) sd = N;
    nd = normalize(sd);
    A = ld3(m.color);
    return true;
  }
  if (kind == RT_MAT_GLASS || kind == RT_MAT_DIELECTRIC) {  // advanced_materials.go:21-46
    A = kind == RT_MAT_GLASS ? ld3(m.color) : mk(1.0, 1.0, 1.0);
    double ratio = front ? 1.0 / m.ior : m.ior;
    d3 u = normalize(d);
    double ct = gmin(dot(muls(u, -1), N), 1.0);
    double st = sqrt(1.0 - ct * ct);
    bool cannot = ratio * st > 1.0;
    bool refl = cannot;
    if (!cannot) {  // Go's || short-circuit: the draw happens only here
      double r0 = (1 - ratio) / (1 + ratio);
      r0 = r0 * r0;
      double R = r0 + (1 - r0) * pow_n<5>(1 - ct);
      refl = R > draw<kCount>(rng, c);
    }
    nd = refl ? reflect(u, N) : refract(u, N, ratio);
    return true;
  }
  // Metal (material.go:75-113), Shiny (:169-189), PerfectMirror
  // (advanced_materials.go:125-151): mirror direction, optional perturbation
  d3 refl = reflect(d, N);
  if (m.rough_draw) {
    d3 pert = muls(rand_in_unit_sphere<kCount>(rng, c), m.roughness);
    refl = normalize(refl + pert);
  }
  double cos_t = fabs(dot(d, N));
  double f = m.f0 + (1.0 - m.f0) * pow_n<5>(1.0 - cos_t);
  d3 col = ld3(m.color);
  if (kind == RT_MAT_METAL) {
    const double fs = m.fs;
    d3 ea = mk(col.x * (1.0 - fs) + f * fs, col.y * (1.0 - fs) + f * fs, col.z * (1.0 - fs) + f * fs);
    ea = mk(gmax(0.0, gmin(1.0, ea.x)), gmax(0.0, gmin(1.0, ea.y)), gmax(0.0, gmin(1.0, ea.z)));
    if (m.blend_metal) {
      const double mf = m.mf;
      ea = mk(ea.x * (1.0 - mf) + f * mf, ea.y * (1.0 - mf) + f * mf, ea.z * (1.0 - mf) + f * mf);
    }
    A = ea;
  } else if (kind == RT_MAT_SHINY) {
    const double fs = m.fs;
    A = mk(gmin(1.0, col.x * (1.0 - fs) + f * fs), gmin(1.0, col.y * (1.0 - fs) + f * fs),
           gmin(1.0, col.z * (1.0 - fs) + f * fs));
  } else {  // PerfectMirror
    // Go constant-folds (1.0 - 0.9) exactly to float64(0.1)
    A = mk(col.x * 0.1 + f * 0.9, col.y * 0.1 + f * 0.9, col.z * 0.1 + f * 0.9);
  }
  nd = refl;
  return true;
}

// ------------------------------------------------------------ kernel
template <bool kCount>
__global__ __launch_bounds__(256) void render_kernel(const KParams p) {
  __shared__ double red[3][256];
  __shared__ unsigned long long cred[9];

  const int tid = threadIdx.x;
  const int P = p.pix_per_wg;
  const int S = p.slices;
  const int blocks_per_tile = 1024 / P;
  const int wg = blockIdx.x;
  const int lt = wg / blocks_per_tile;  // local tile index
  const int sub = wg - lt * blocks_per_tile;
  const int tile = p.rank + lt * p.world;
  const int tx = tile % p.tiles_x, ty = tile / p.tiles_x;
  const int bpr = 32 / p.blk_w;  // blocks per tile row
  const int bx = sub % bpr, by = sub / bpr;
  const int pix = tid % P;  // pixel within the block
  const int q = tid / P;    // sample slice
  const int lx = bx * p.blk_w + pix % p.blk_w;
  const int ly = by * p.blk_h + pix / p.blk_w;
  const int x = tx * 32 + lx, y = ty * 32 + ly;
  const bool valid = tile < p.ntiles && x < p.W && y < p.H;

  Counters c;
  if constexpr (kCount) {
    for (int i = 0; i < 9; ++i) c.v[i] = 0;
    if (tid < 9) cred[tid] = 0;
  }

  const uint32_t pixel = (uint32_t)y * (uint32_t)p.W + (uint32_t)x;
  const d3 cam = mk(p.cam[0], p.cam[1], p.cam[2]);
  // getRay constants (renderer.go:377-390)
  const double vw = 2.0 * p.aspect;
  const d3 llc = mk(cam.x - vw / 2, cam.y - 1.0, cam.z - 1.0);

  double sx = 0, sy = 0, sz = 0;  // this lane's sample sum
  d3 o = cam, d = mk(0, 0, 0), T = mk(1, 1, 1), L = mk(0, 0, 0);
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
      double u = ((double)x + draw<kCount>(rng, c)) / (double)p.W;
      double v = ((double)y + draw<kCount>(rng, c)) / (double)p.H;
      o = cam;
      d = mk(((llc.x + vw * u) + 0.0) - cam.x, ((llc.y + 0.0) + 2.0 * v) - cam.y, ((llc.z + 0.0) + 0.0) - cam.z);
      T = mk(1, 1, 1);
      L = mk(0, 0, 0);
      depth = 0;
      alive = true;
    }
    if (depth >= p.max_depth) {  // traceRay depth cut-off: contributes 0
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    HitSel hs;
    cnt<kCount>(c, C_BOUNCE);
    if (!closest_hit<kCount>(p, o, d, 0.001, hs, c)) {  // miss -> black
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    cnt<kCount>(c, C_SHADE);
    // HitRecord of the closest primitive (sphere.go:42-58, triangle.go:68-81)
    d3 P = o + muls(d, hs.t);
    d3 N;
    bool front;
    int mi;
    if (!hs.is_tri) {
      const DSphere& S0 = p.spheres[hs.idx];
      d3 outward = divs(P - ld3(S0.c), S0.r);
      front = dot(d, outward) < 0;
      N = front ? outward : muls(outward, -1);
      mi = S0.mat;
    } else {
      const DTri& T0 = p.tris[hs.idx];
      double w = 1.0 - hs.u - hs.v;
      d3 n = ld3(T0.n);
      N = normalize((muls(n, w) + muls(n, hs.u)) + muls(n, hs.v));
      front = dot(d, N) < 0;
      if (!front) N = muls(N, -1);
      mi = T0.mat;
    }
    const DMat& m = p.mats[mi];
    d3 E = ld3(m.emit);
    d3 D = direct_lighting<kCount>(p, m, P, N, rng, c);
    d3 nd, A;
    if (!scatter<kCount>(m, d, P, N, front, rng, nd, A, c)) {
      d3 ed = E + D;
      L = L + mul(T, ed);
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    d3 ed = E + muls(D, m.dw);
    L = L + mul(T, ed);
    if (!p.recursive || depth + 1 >= p.max_depth) {
      sx += L.x;
      sy += L.y;
      sz += L.z;
      alive = false;
      continue;
    }
    T = mul(T, muls(A, m.rw));
    o = P;
    d = nd;
    depth += 1;
  }

  // ---- reduce the S slices of each pixel in fixed order
  red[0][tid] = sx;
  red[1][tid] = sy;
  red[2][tid] = sz;
  if constexpr (kCount) {
    __syncthreads();
    for (int i = 0; i < 9; ++i) atomicAdd(&cred[i], c.v[i]);
  }
  __syncthreads();
  if (tid < P && valid) {
    double tx3 = 0, ty3 = 0, tz3 = 0;
    for (int k = 0; k < S; ++k) {
      tx3 += red[0][k * P + tid];
      ty3 += red[1][k * P + tid];
      tz3 += red[2][k * P + tid];
    }
    const double n = (double)p.spp;
    double mean[3] = {tx3 / n, ty3 / n, tz3 / n};
    size_t oi;
    if (p.layout == RT_LAYOUT_IMAGE)
      oi = (size_t)y * p.W + x;
    else
      oi = (size_t)lt * 1024 + (size_t)ly * 32 + lx;
    if (p.out_linear) {
      p.out_linear[oi * 3 + 0] = (float)mean[0];
      p.out_linear[oi * 3 + 1] = (float)mean[1];
      p.out_linear[oi * 3 + 2] = (float)mean[2];
    }
    if (p.out_rgba) {
      // toneMap (renderer.go:348-367) then Vec3.ToRGB (vector.go:106-109)
      const double g = 1.0 / 2.2;
      uint8_t b[3];
      for (int k = 0; k < 3; ++k) {
        double v = mean[k] * 1.0;
        v = 1.0 - exp(-v);
        v = pow_gamma(v, g);
        v = gmax(0.0, gmin(1.0, v));
        v = gmax(0.0, gmin(1.0, v));
        b[k] = go_u8(v * 255);
      }
      uchar4 px4 = make_uchar4(b[0], b[1], b[2], 255);
      *reinterpret_cast<uchar4*>(p.out_rgba + oi * 4) = px4;
    }
  }
  if constexpr (kCount) {
    __syncthreads();
    if (tid < 9) atomicAdd(&p.counts[tid], cred[tid]);
  }
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
  if (orgba && pr) *reinterpret_cast<uchar4*>(orgba + o * 4) = *reinterpret_cast<const uchar4*>(pr + i * 4);
}

int launch_render(const KParams& p, bool count, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (p.num_wgs <= 0) return hipSuccess;
  if (count)
    hipLaunchKernelGGL(render_kernel<true>, dim3(p.num_wgs), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(render_kernel<false>, dim3(p.num_wgs), dim3(256), 0, st, p);
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
