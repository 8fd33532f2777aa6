/*
 * oracle.c — CPU restatement of the reference's per-pixel ray-trace hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  This file restates, in plain C
 * and in the reference's own evaluation order, the Go code of
 *   internal/renderer/renderer.go:67-390   (Render, tracePixel, traceRay,
 *                                            calculateDirectLighting,
 *                                            calculateSmartShadow, hitWorld,
 *                                            toneMap, getRay, tiles)
 *   internal/geometry/sphere.go:22-59, triangle.go:13-88
 *   internal/scene/scene.go:59-209          (hittables, createCube, Mesh.Hit)
 *   internal/material/material.go:9-318, advanced_materials.go:9-171
 *   internal/math/vector.go:9-197, random.go:8-30
 * and Go's math.Pow / Max / Min semantics (Go standard library, go 1.24.5,
 * src/math/pow.go, dim.go — no third-party code is involved, go.mod:1-3).
 * Arithmetic is binary64 with no contraction (built with -ffp-contract=off):
 * Go on amd64 does not fuse multiply-adds.  Recursion is kept as in Go.
 * The only deliberate change is the random stream (include/rt_rng.h).
 */
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt_rng.h"

/* ------------------------------------------------------------ Go math */

static int is_odd_int(double x) {
  /* math.isOddInt (pow.go) */
  if (fabs(x) >= 9007199254740992.0) return 0; /* 1<<53: all even */
  double xi;
  double xf = modf(x, &xi);
  return xf == 0 && ((int64_t)xi & 1) == 1;
}

double oracle_go_pow(double x, double y) {
  /* math.Pow special cases, in Go's order */
  if (y == 0 || x == 1) return 1;
  if (y == 1) return x;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0) {
    if (y < 0) {
      if (signbit(x) && is_odd_int(y)) return -INFINITY;
      return INFINITY;
    }
    if (y > 0) {
      if (signbit(x) && is_odd_int(y)) return x;
      return 0;
    }
  }
  if (isinf(y)) {
    if (x == -1) return 1;
    if ((fabs(x) < 1) == (y > 0)) return 0;
    return INFINITY;
  }
  if (isinf(x)) {
    if (x < 0) return oracle_go_pow(1 / x, -y);
    if (y < 0) return 0;
    if (y > 0) return INFINITY;
  }
  if (y == 0.5) return sqrt(x);
  if (y == -0.5) return 1 / sqrt(x);

  double yi;
  double yf = modf(fabs(y), &yi);
  if (yf != 0 && x < 0) return NAN;
  if (yi >= 9223372036854775808.0) {
    if (x == -1) return 1;
    if ((fabs(x) < 1) == (y > 0)) return 0;
    return INFINITY;
  }
  /* ans = a1 * 2**ae */
  double a1 = 1.0;
  int64_t ae = 0;
  if (yf != 0) {
    if (yf > 0.5) {
      yf--;
      yi++;
    }
    a1 = exp(yf * log(x));
  }
  /* ans *= x**yi by repeated squaring (mantissa / exponent kept apart) */
  int xe_i;
  double x1 = frexp(x, &xe_i);
  int64_t xe = xe_i;
  for (int64_t i = (int64_t)yi; i != 0; i >>= 1) {
    if (xe < -(1 << 12) || (1 << 12) < xe) {
      ae += xe;
      break;
    }
    if ((i & 1) == 1) {
      a1 *= x1;
      ae += xe;
    }
    x1 *= x1;
    xe *= 2; /* Go's xe <<= 1 on a negative int (two's complement); a left shift of a negative value is UB in C */
    if (x1 < .5) {
      x1 += x1;
      xe--;
    }
  }
  if (y < 0) {
    a1 = 1 / a1;
    ae = -ae;
  }
  if (ae > 100000) ae = 100000;
  if (ae < -100000) ae = -100000;
  return ldexp(a1, (int)ae);
}

double oracle_go_max(double x, double y) {
  if ((isinf(x) && x > 0) || (isinf(y) && y > 0)) return INFINITY;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? y : x;
  return x > y ? x : y;
}

double oracle_go_min(double x, double y) {
  if ((isinf(x) && x < 0) || (isinf(y) && y < 0)) return -INFINITY;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}

/* ------------------------------------------------------------ Vec3 */

typedef struct {
  double x, y, z;
} vec3;

static inline vec3 V(double x, double y, double z) {
  vec3 r = {x, y, z};
  return r;
}
static inline vec3 vadd(vec3 a, vec3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 vsub(vec3 a, vec3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 vmul(vec3 a, vec3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 vmuls(vec3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }
static inline vec3 vdivs(vec3 a, double s) { return V(a.x / s, a.y / s, a.z / s); }
static inline double vdot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline vec3 vcross(vec3 a, vec3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline double vlen2(vec3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
static inline double vlen(vec3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static inline vec3 vnorm(vec3 a) {
  double l = vlen(a);
  if (l == 0) return V(0, 0, 0);
  return vdivs(a, l);
}
static inline vec3 vreflect(vec3 v, vec3 n) { return vsub(v, vmuls(n, 2 * vdot(v, n))); }
static vec3 vrefract(vec3 v, vec3 n, double eta) {
  double cos_t = vdot(v, n);
  if (cos_t > 0) {
    n = vmuls(n, -1);
    eta = 1 / eta;
    cos_t = -cos_t;
  }
  double sin2 = eta * eta * (1 - cos_t * cos_t);
  if (sin2 > 1) return vreflect(v, n);
  double cos2 = sqrt(1 - sin2);
  return vsub(vmuls(v, eta), vmuls(n, eta * cos_t + cos2));
}
static inline vec3 vclamp(vec3 v, double lo, double hi) {
  return V(oracle_go_max(lo, oracle_go_min(hi, v.x)), oracle_go_max(lo, oracle_go_min(hi, v.y)),
           oracle_go_max(lo, oracle_go_min(hi, v.z)));
}
static inline int vnear_zero(vec3 v) {
  const double s = 1e-8;
  return fabs(v.x) < s && fabs(v.y) < s && fabs(v.z) < s;
}
static inline vec3 varr(const double* a) { return V(a[0], a[1], a[2]); }

/* ------------------------------------------------------------ counts */

typedef struct {
  uint64_t camera_rays, bounce_rays, shadow_rays, sphere_tests, triangle_tests, shade_events, light_evals,
      rng_draws;
} ocounts;

typedef struct {
  rt_rng rng;
  ocounts* c;
  uint64_t soft_key;  /* rt_soft_key of the sample (spec v4: its soft-shadow streams) */
} ostream;

static inline double rnd(ostream* s) {
  s->c->rng_draws++;
  return rt_rng_draw(&s->rng);
}

/* vector.go:124-139 */
static vec3 random_in_unit_sphere(ostream* s) {
  for (;;) {
    double x = rnd(s), y = rnd(s), z = rnd(s);
    vec3 p = vsub(vmuls(V(x, y, z), 2), V(1, 1, 1));
    if (vlen2(p) < 1) return p;
  }
}

/* ------------------------------------------------------------ scene */

typedef struct {
  int kind;
  vec3 color; /* albedo / emit */
  double roughness, metallic, specular, ior;
} omat;

typedef struct {
  vec3 v[3], n[3];
} otri;

typedef struct {
  int type; /* RT_OBJ_* */
  vec3 center;
  double radius;
  otri tris[12];
  const omat* mat;
} ohittable;

typedef struct {
  ohittable* objs;
  int n;
  omat* mats;
  vec3* lpos;
  vec3* lcolor;
  double* lint;
  int nl;
  vec3 cam_pos;
  double aspect;
  int max_depth, samples, recursive, soft;
  uint64_t seed_key;
  int W, H;
  int sky; /* RT_SKY_*: 0 = a miss is black (renderer.go:170-173) */
  /* CPU-baseline variant only (oracle_render_ex use_bvh): a sphere BVH */
  struct obvh_node* bvh;
  int* bvh_prims; /* hittable index per leaf slot */
  /* oracle_path_lengths only: bounces (traceRay calls) of every sample's
   * path, [pixel y*W+x][sample], clamped at 255; NULL otherwise */
  uint8_t* path_len;
} oscene;

/* ------------------------------------------------------------ sky (opt-in)
 * AtmosphereConfig (internal/atmosphere/atmosphere.go:8-26) and its presets
 * NewDefaultAtmosphere / NewWhiteAtmosphere / NewSunsetAtmosphere /
 * NewNightAtmosphere (atmosphere.go:28-98), index RT_SKY_* - 1. */
typedef struct {
  vec3 top, bottom, sun_dir, sun_color;
  double sun_intensity, sun_size;
  vec3 rayleigh, mie;
  double depth, fog_density;
  vec3 fog_color;
  double haze, time_of_day;
} osky;

static const osky kSkyPresets[4] = {
    {{0.6, 0.8, 1.0}, {0.9, 0.95, 1.0}, {0.0, 0.8, -0.6}, {1.0, 0.98, 0.95}, 1.2, 0.015, {0.6, 0.8, 1.0},
     {1.0, 0.98, 0.95}, 0.3, 0.0, {0.9, 0.92, 0.95}, 0.05, 0.6},
    {{0.98, 0.98, 1.0}, {0.92, 0.92, 0.95}, {0.0, 0.8, -0.6}, {1.0, 0.99, 0.97}, 0.8, 0.012, {0.9, 0.9, 0.95},
     {0.95, 0.95, 0.98}, 0.2, 0.0, {0.95, 0.95, 0.98}, 0.02, 0.6},
    {{1.0, 0.4, 0.2}, {1.0, 0.8, 0.6}, {0.0, 0.3, -0.9}, {1.0, 0.6, 0.3}, 1.2, 0.03, {1.0, 0.4, 0.2},
     {1.0, 0.8, 0.6}, 0.8, 0.1, {1.0, 0.8, 0.6}, 0.3, 0.8},
    {{0.1, 0.1, 0.3}, {0.2, 0.2, 0.4}, {0.0, -0.7, -0.7}, {0.8, 0.8, 1.0}, 0.3, 0.005, {0.1, 0.1, 0.3},
     {0.8, 0.8, 1.0}, 0.2, 0.0, {0.1, 0.1, 0.2}, 0.0, 0.0},
};

/* FastVec3Lerp(a, b, t): undefined in the reference; taken as a.Lerp(b, t) =
 * a.Add(b.Sub(a).MulScalar(t)) (vector.go:116-118), like FastLerp
 * (advanced_math.go:84-86). */
static vec3 sky_lerp(vec3 a, vec3 b, double t) { return vadd(a, vmuls(vsub(b, a), t)); }

/* GetSkyColor, atmosphere.go:100-135 (FastVec3Normalize/Dot/MulScalar taken
 * as Normalize, Dot, MulScalar). */
vec3 oracle_sky_color_v(int sky, vec3 dir) {
  const osky* a = &kSkyPresets[sky - 1];
  vec3 u = vnorm(dir);
  double t = 0.5 * (u.y + 1.0);
  vec3 c = sky_lerp(a->bottom, a->top, t);
  double depth = oracle_go_max(0.0, u.y);
  double atmospheric = exp(-depth * a->depth);
  vec3 scattering = sky_lerp(a->rayleigh, a->mie, atmospheric);
  c = sky_lerp(c, scattering, 0.25);
  double sun_dot = vdot(u, a->sun_dir);
  if (sun_dot > (1.0 - a->sun_size)) {
    double si = oracle_go_pow((sun_dot - (1.0 - a->sun_size)) / a->sun_size, 1.5);
    si = oracle_go_min(si, 1.0);
    c = sky_lerp(c, a->sun_color, si * a->sun_intensity * 0.9);
  }
  double tf = a->time_of_day;
  if (tf > 0.5) tf = 1.0 - tf;
  tf *= 2.0;
  double darkness = 1.0 - tf * 0.3;
  c = vmuls(c, darkness);
  if (a->fog_density > 0.0) c = sky_lerp(a->fog_color, c, exp(-a->fog_density));
  return vclamp(c, 0.1, 0.98);
}

void oracle_sky_color(int sky, const double dir[3], double out[3]) {
  vec3 c = oracle_sky_color_v(sky, V(dir[0], dir[1], dir[2]));
  out[0] = c.x;
  out[1] = c.y;
  out[2] = c.z;
}

typedef struct {
  double t;
  vec3 p, n;
  int front;
  const omat* mat;
} hitrec;

typedef struct {
  vec3 o, d;
} oray;

/* material constructors: NewLambertian/NewMetal/... (material.go,
 * advanced_materials.go) with their Min(x, 1.0) clamps */
static omat make_material(const rt_material* m) {
  omat r;
  memset(&r, 0, sizeof r);
  r.kind = m->kind;
  r.color = varr(m->color);
  switch (m->kind) {
    case RT_MAT_METAL:
    case RT_MAT_SHINY:
      r.roughness = oracle_go_min(m->roughness, 1.0);
      r.metallic = oracle_go_min(m->metallic, 1.0);
      r.specular = oracle_go_min(m->specular, 1.0);
      r.ior = 1.5;
      break;
    case RT_MAT_PERFECTMIRROR:
      r.roughness = oracle_go_min(m->roughness, 1.0);
      r.ior = 2.0;
      break;
    case RT_MAT_GLASS:
    case RT_MAT_DIELECTRIC:
      r.ior = m->refraction_index;
      break;
    default:
      break;
  }
  return r;
}

/* Material.GetAlbedo */
static vec3 mat_albedo(const omat* m) {
  switch (m->kind) {
    case RT_MAT_DIELECTRIC: return V(1, 1, 1);
    case RT_MAT_DIFFUSELIGHT: return V(0, 0, 0);
    default: return m->color;
  }
}
/* Material.GetMetallic */
static double mat_metallic(const omat* m) {
  switch (m->kind) {
    case RT_MAT_METAL:
    case RT_MAT_SHINY: return m->metallic;
    case RT_MAT_PERFECTMIRROR: return 1.0;
    default: return 0.0;
  }
}
/* Material.Emitted */
static vec3 mat_emitted(const omat* m) { return m->kind == RT_MAT_DIFFUSELIGHT ? m->color : V(0, 0, 0); }

/* material.go:115-129 (Metal/Shiny calculateFresnel; f0 per channel equal) */
static vec3 schlick3(double ior, double cos_t) {
  double f0 = oracle_go_pow((ior - 1.0) / (ior + 1.0), 2.0);
  double s = f0 + (1.0 - f0) * oracle_go_pow(1.0 - cos_t, 5);
  return V(s, s, s);
}

/* material.go:282-286 */
static double reflectance(double cosine, double ref_idx) {
  double r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1 - r0) * oracle_go_pow(1 - cosine, 5);
}

/* Material.Scatter — returns scattered flag */
static int mat_scatter(const omat* m, oray in, const hitrec* h, ostream* s, oray* out, vec3* atten) {
  switch (m->kind) {
    case RT_MAT_METAL: { /* material.go:75-113 */
      vec3 refl = vreflect(in.d, h->n);
      if (m->roughness > 0.001) {
        vec3 pert = vmuls(random_in_unit_sphere(s), m->roughness);
        refl = vnorm(vadd(refl, pert));
      }
      vec3 albedo = m->color;
      double cos_t = fabs(vdot(in.d, h->n));
      vec3 f = schlick3(m->ior, cos_t);
      double fs = 0.6 + m->metallic * 0.4;
      vec3 ea = V(albedo.x * (1.0 - fs) + f.x * fs, albedo.y * (1.0 - fs) + f.y * fs,
                  albedo.z * (1.0 - fs) + f.z * fs);
      ea = V(oracle_go_max(0.0, oracle_go_min(1.0, ea.x)), oracle_go_max(0.0, oracle_go_min(1.0, ea.y)),
             oracle_go_max(0.0, oracle_go_min(1.0, ea.z)));
      if (m->metallic > 0.8) {
        double mf = 0.4 + m->metallic * 0.5;
        ea = V(ea.x * (1.0 - mf) + f.x * mf, ea.y * (1.0 - mf) + f.y * mf, ea.z * (1.0 - mf) + f.z * mf);
      }
      out->o = h->p;
      out->d = refl;
      *atten = ea;
      return 1;
    }
    case RT_MAT_SHINY: { /* material.go:169-189 */
      vec3 refl = vreflect(in.d, h->n);
      if (m->roughness > 0) {
        refl = vadd(refl, vmuls(random_in_unit_sphere(s), m->roughness));
        refl = vnorm(refl);
      }
      double cos_t = fabs(vdot(in.d, h->n));
      vec3 f = schlick3(m->ior, cos_t);
      double fs = 0.4 + m->specular * 0.4;
      vec3 ea = V(oracle_go_min(1.0, m->color.x * (1.0 - fs) + f.x * fs),
                  oracle_go_min(1.0, m->color.y * (1.0 - fs) + f.y * fs),
                  oracle_go_min(1.0, m->color.z * (1.0 - fs) + f.z * fs));
      out->o = h->p;
      out->d = refl;
      *atten = ea;
      return 1;
    }
    case RT_MAT_PERFECTMIRROR: { /* advanced_materials.go:125-151 */
      vec3 refl = vreflect(in.d, h->n);
      if (m->roughness > 0.001) {
        vec3 pert = vmuls(random_in_unit_sphere(s), m->roughness);
        refl = vnorm(vadd(refl, pert));
      }
      double cos_t = fabs(vdot(in.d, h->n));
      double f0 = oracle_go_pow((m->ior - 1.0) / (m->ior + 1.0), 2.0);
      double sch = f0 + (1.0 - f0) * oracle_go_pow(1.0 - cos_t, 5);
      /* Go folds the untyped constant (1.0 - 0.9) exactly: it is float64(0.1),
       * not the C double difference 0.09999999999999998 */
      const double one_minus_09 = 0.1;
      vec3 ec = V(m->color.x * one_minus_09 + sch * 0.9, m->color.y * one_minus_09 + sch * 0.9,
                  m->color.z * one_minus_09 + sch * 0.9);
      out->o = h->p;
      out->d = refl;
      *atten = ec;
      return 1;
    }
    case RT_MAT_GLASS:
    case RT_MAT_DIELECTRIC: { /* advanced_materials.go:21-46; material.go:235-260 */
      vec3 att = m->kind == RT_MAT_GLASS ? m->color : V(1.0, 1.0, 1.0);
      double ratio = h->front ? 1.0 / m->ior : m->ior;
      vec3 u = vnorm(in.d);
      double cos_t = oracle_go_min(vdot(vmuls(u, -1), h->n), 1.0);
      double sin_t = sqrt(1.0 - cos_t * cos_t);
      int cannot = ratio * sin_t > 1.0;
      vec3 dir;
      /* Go's || short-circuits: the draw happens only if !cannot */
      if (cannot || reflectance(cos_t, ratio) > rnd(s))
        dir = vreflect(u, h->n);
      else
        dir = vrefract(u, h->n, ratio);
      out->o = h->p;
      out->d = dir;
      *atten = att;
      return 1;
    }
    case RT_MAT_DIFFUSELIGHT: /* material.go:296-298 */
      return 0;
    default: { /* RT_MAT_LAMBERTIAN, material.go:26-35 */
      vec3 sd = vadd(h->n, random_in_unit_sphere(s));
      if (vnear_zero(sd)) sd = h->n;
      sd = vnorm(sd);
      out->o = h->p;
      out->d = sd;
      *atten = m->color;
      return 1;
    }
  }
}

/* ------------------------------------------------------------ geometry */

/* sphere.go:22-59 */
static int sphere_hit(const ohittable* sp, oray r, double tmin, double tmax, hitrec* rec) {
  vec3 oc = vsub(r.o, sp->center);
  double a = vlen2(r.d);
  double half_b = vdot(oc, r.d);
  double c = vlen2(oc) - sp->radius * sp->radius;
  double disc = half_b * half_b - a * c;
  if (disc < 0) return 0;
  double sq = sqrt(disc);
  double root = (-half_b - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-half_b + sq) / a;
    if (root < tmin || tmax < root) return 0;
  }
  double t = root;
  vec3 p = vadd(r.o, vmuls(r.d, t));
  vec3 outward = vdivs(vsub(p, sp->center), sp->radius);
  int front = vdot(r.d, outward) < 0;
  rec->t = t;
  rec->p = p;
  rec->n = front ? outward : vmuls(outward, -1);
  rec->front = front;
  rec->mat = sp->mat;
  return 1;
}

/* triangle.go:36-88 */
static int triangle_hit(const otri* tr, const omat* mat, oray r, double tmin, double tmax, hitrec* rec) {
  vec3 e1 = vsub(tr->v[1], tr->v[0]);
  vec3 e2 = vsub(tr->v[2], tr->v[0]);
  vec3 h = vcross(r.d, e2);
  double a = vdot(e1, h);
  if (a > -1e-6 && a < 1e-6) return 0;
  double f = 1.0 / a;
  vec3 s = vsub(r.o, tr->v[0]);
  double u = f * vdot(s, h);
  if (u < 0.0 || u > 1.0) return 0;
  vec3 q = vcross(s, e1);
  double v = f * vdot(r.d, q);
  if (v < 0.0 || u + v > 1.0) return 0;
  double t = f * vdot(e2, q);
  if (t < tmin || t > tmax) return 0;
  vec3 p = vadd(r.o, vmuls(r.d, t));
  double w = 1.0 - u - v;
  vec3 n = vnorm(vadd(vadd(vmuls(tr->n[0], w), vmuls(tr->n[1], u)), vmuls(tr->n[2], v)));
  int front = vdot(r.d, n) < 0;
  if (!front) n = vmuls(n, -1);
  rec->t = t;
  rec->p = p;
  rec->n = n;
  rec->front = front;
  rec->mat = mat;
  return 1;
}

/* NewTriangle, triangle.go:13-34 */
static otri make_triangle(vec3 v0, vec3 v1, vec3 v2) {
  otri t;
  t.v[0] = v0;
  t.v[1] = v1;
  t.v[2] = v2;
  vec3 n = vnorm(vcross(vsub(v1, v0), vsub(v2, v0)));
  t.n[0] = t.n[1] = t.n[2] = n;
  return t;
}

/* createCube, scene.go:150-190 */
static void make_cube(vec3 pos, vec3 size, otri out[12]) {
  vec3 hs = vdivs(size, 2.0);
  vec3 vert[8] = {
      vadd(pos, V(-hs.x, -hs.y, -hs.z)), vadd(pos, V(hs.x, -hs.y, -hs.z)), vadd(pos, V(hs.x, hs.y, -hs.z)),
      vadd(pos, V(-hs.x, hs.y, -hs.z)),  vadd(pos, V(-hs.x, -hs.y, hs.z)), vadd(pos, V(hs.x, -hs.y, hs.z)),
      vadd(pos, V(hs.x, hs.y, hs.z)),    vadd(pos, V(-hs.x, hs.y, hs.z)),
  };
  static const int faces[6][4] = {{0, 1, 2, 3}, {1, 5, 6, 2}, {5, 4, 7, 6}, {4, 0, 3, 7}, {3, 2, 6, 7}, {4, 5, 1, 0}};
  for (int f = 0; f < 6; f++) {
    vec3 v0 = vert[faces[f][0]], v1 = vert[faces[f][1]], v2 = vert[faces[f][2]], v3 = vert[faces[f][3]];
    out[2 * f] = make_triangle(v0, v1, v2);
    out[2 * f + 1] = make_triangle(v0, v2, v3);
  }
}

/* ------------------------------------------------------------ CPU BVH
 * NOT the reference: the reference scans every hittable (renderer.go:333-346).
 * This median-split sphere BVH exists only for bench.py's secondary CPU
 * baseline of the 10k-sphere configs ("cpu_ref with the
 * build's BVH"), so the GPU speedup's algorithmic share is visible.  It
 * returns the linear scan's closest hit: boxes are padded and tested with a
 * slack, every sphere in a box the ray meets gets the exact Sphere.Hit, and
 * equal t resolve to the larger hittable index as in the scan (the root a
 * sphere contributes does not depend on the scan order: a root rejected
 * against a smaller tMax is larger than it, and so is the other root). */
typedef struct obvh_node {
  double lo[3], hi[3];
  int first, count; /* count 0: internal node, children first and first + 1 */
} obvh_node;

typedef struct {
  obvh_node* nodes;
  int n, cap;
} obvh_build;

static int bvh_axis;
static const oscene* bvh_sc;
static int bvh_cmp(const void* a, const void* b) {
  double ca = (&bvh_sc->objs[*(const int*)a].center.x)[bvh_axis];
  double cb = (&bvh_sc->objs[*(const int*)b].center.x)[bvh_axis];
  return ca < cb ? -1 : (ca > cb ? 1 : 0);
}

static void bvh_bounds(const oscene* sc, const int* prims, int n, double lo[3], double hi[3]) {
  for (int k = 0; k < 3; k++) {
    lo[k] = INFINITY;
    hi[k] = -INFINITY;
  }
  for (int i = 0; i < n; i++) {
    const ohittable* h = &sc->objs[prims[i]];
    const double* c = &h->center.x;
    double r = fabs(h->radius);
    for (int k = 0; k < 3; k++) {
      double pad = 1e-9 * (fabs(c[k]) + r) + 1e-12;
      if (c[k] - r - pad < lo[k]) lo[k] = c[k] - r - pad;
      if (c[k] + r + pad > hi[k]) hi[k] = c[k] + r + pad;
    }
  }
}

/* node `at` covers prims[0, n): split at the median of the longest axis */
static void bvh_split(obvh_build* b, const oscene* sc, int* prims, int base, int n, int at) {
  obvh_node* nd = &b->nodes[at];
  bvh_bounds(sc, prims + base, n, nd->lo, nd->hi);
  if (n <= 4) {
    nd->first = base;
    nd->count = n;
    return;
  }
  int axis = 0;
  for (int k = 1; k < 3; k++)
    if (nd->hi[k] - nd->lo[k] > nd->hi[axis] - nd->lo[axis]) axis = k;
  bvh_axis = axis;
  bvh_sc = sc;
  qsort(prims + base, (size_t)n, sizeof(int), bvh_cmp);
  const int child = b->n;
  b->n += 2;
  nd->first = child;
  nd->count = 0;
  bvh_split(b, sc, prims, base, n / 2, child);
  bvh_split(b, sc, prims, base + n / 2, n - n / 2, child + 1);
}

static double slab_enter(const obvh_node* nd, oray r, const double* inv, double tmin, double tmax) {
  double tn = tmin, tf = tmax;
  for (int k = 0; k < 3; k++) {
    const double o = (&r.o.x)[k];
    double t0 = (nd->lo[k] - o) * inv[k], t1 = (nd->hi[k] - o) * inv[k];
    if (t0 > t1) {
      double t = t0;
      t0 = t1;
      t1 = t;
    }
    if (t0 > tn) tn = t0;
    if (t1 < tf) tf = t1;
  }
  return tn <= tf + fabs(tf) * 1e-9 + 1e-12 ? tn : INFINITY;
}

/* closest hit (any = 0) or any hit (any = 1) in [tmin, tmax] through the BVH */
static int hit_world_bvh(const oscene* sc, oray r, double tmin, double tmax, hitrec* out, int any) {
  double inv[3];
  for (int k = 0; k < 3; k++) {
    const double d = (&r.d.x)[k];
    inv[k] = 1.0 / (d != 0 ? d : 1e-300);
  }
  int stack[64], sp = 0, found = 0, best = -1;
  double closest = tmax;
  hitrec rec;
  if (slab_enter(&sc->bvh[0], r, inv, tmin, closest) == INFINITY) return 0;
  int cur = 0;
  for (;;) {
    const obvh_node* nd = &sc->bvh[cur];
    if (nd->count == 0) {
      const double tl = slab_enter(&sc->bvh[nd->first], r, inv, tmin, closest);
      const double tr = slab_enter(&sc->bvh[nd->first + 1], r, inv, tmin, closest);
      if (tl != INFINITY || tr != INFINITY) {
        const int lfirst = tl <= tr;
        if (tl != INFINITY && tr != INFINITY && sp < 64) stack[sp++] = lfirst ? nd->first + 1 : nd->first;
        cur = lfirst ? nd->first : nd->first + 1;
        continue;
      }
    } else {
      for (int i = nd->first; i < nd->first + nd->count; i++) {
        const int hi = sc->bvh_prims[i];
        if (!sphere_hit(&sc->objs[hi], r, tmin, closest, &rec)) continue;
        if (any) return 1;
        if (rec.t == closest && found && best > hi) continue;
        closest = rec.t;
        best = hi;
        *out = rec;
        found = 1;
      }
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
  return found;
}

static void bvh_make(oscene* sc) {
  for (int i = 0; i < sc->n; i++)
    if (sc->objs[i].type != RT_OBJ_SPHERE || !isfinite(sc->objs[i].radius)) return;  /* spheres only */
  if (sc->n < 2) return;
  obvh_build b;
  b.cap = 2 * sc->n + 1;
  b.nodes = (obvh_node*)calloc((size_t)b.cap, sizeof(obvh_node));
  b.n = 1;
  sc->bvh_prims = (int*)malloc(sizeof(int) * (size_t)sc->n);
  for (int i = 0; i < sc->n; i++) sc->bvh_prims[i] = i;
  bvh_split(&b, sc, sc->bvh_prims, 0, sc->n, 0);
  sc->bvh = b.nodes;
}

/* hitWorld, renderer.go:333-346 (+ Mesh.Hit, scene.go:196-209) */
static int hit_world(const oscene* sc, oray r, double tmin, double tmax, hitrec* out, ocounts* c) {
  if (sc->bvh) return hit_world_bvh(sc, r, tmin, tmax, out, 0);
  int found = 0;
  double closest = tmax;
  hitrec rec;
  for (int i = 0; i < sc->n; i++) {
    const ohittable* h = &sc->objs[i];
    if (h->type == RT_OBJ_SPHERE) {
      c->sphere_tests++;
      if (sphere_hit(h, r, tmin, closest, &rec)) {
        closest = rec.t;
        *out = rec;
        found = 1;
      }
    } else {
      /* Mesh.Hit: closest over its triangles, within [tmin, closest] */
      int mfound = 0;
      double mclosest = closest;
      hitrec mrec;
      for (int k = 0; k < 12; k++) {
        c->triangle_tests++;
        if (triangle_hit(&h->tris[k], h->mat, r, tmin, mclosest, &rec)) {
          mclosest = rec.t;
          mrec = rec;
          mfound = 1;
        }
      }
      if (mfound) {
        closest = mrec.t;
        *out = mrec;
        found = 1;
      }
    }
  }
  return found;
}

/* ------------------------------------------------------------ renderer */

/* calculateSmartShadow, renderer.go:299-331.  Its 16 RandomVec3InUnitSphere
 * points draw from the (sample, depth, light) soft-shadow stream of spec v4
 * (include/rt_rng.h), not from the sample's stream. */
static double smart_shadow(const oscene* sc, const hitrec* h, int li, int depth, ostream* s) {
  vec3 ldir = vnorm(vsub(sc->lpos[li], h->p));
  double ldist = vlen(vsub(sc->lpos[li], h->p));
  oray sr = {h->p, ldir};
  hitrec tmp;
  s->c->shadow_rays++;
  if (sc->bvh ? hit_world_bvh(sc, sr, 0.001, ldist, &tmp, 1) : hit_world(sc, sr, 0.001, ldist, &tmp, s->c))
    return 0.0;
  if (sc->soft) {
    double sum = 0.0;
    ostream ps;  /* the points' stream (its draws are counted with the sample's) */
    ps.rng.x = rt_soft_state(s->soft_key, (uint32_t)depth, (uint32_t)li);
    ps.c = s->c;
    ps.soft_key = s->soft_key;
    for (int i = 0; i < 16; i++) {
      vec3 off = vmuls(random_in_unit_sphere(&ps), 0.1);
      vec3 sdir = vnorm(vadd(ldir, off));
      oray ss = {h->p, sdir};
      s->c->shadow_rays++;
      if (!(sc->bvh ? hit_world_bvh(sc, ss, 0.001, ldist, &tmp, 1) : hit_world(sc, ss, 0.001, ldist, &tmp, s->c)))
        sum += 1.0;
    }
    return sum / (double)16;
  }
  return 1.0;
}

/* calculateDirectLighting, renderer.go:229-297 */
static vec3 direct_lighting(const oscene* sc, const hitrec* h, int depth, ostream* s) {
  vec3 total = V(0, 0, 0);
  const omat* m = h->mat;
  vec3 albedo = mat_albedo(m);
  double metallic = mat_metallic(m);
  double amb = 0.1;
  if (metallic > 0.9)
    amb = 0.05;
  else if (metallic > 0.7)
    amb = 0.07;
  else if (metallic > 0.5)
    amb = 0.08;
  total = vadd(total, V(amb, amb, amb));
  for (int li = 0; li < sc->nl; li++) {
    vec3 ldir = vnorm(vsub(sc->lpos[li], h->p));
    double ldist = vlen(vsub(sc->lpos[li], h->p));
    if (ldist < 0.001) continue;
    s->c->light_evals++;
    double sf = smart_shadow(sc, h, li, depth, s);
    if (sf > 0.0) {
      double cos_t = oracle_go_max(0, vdot(h->n, ldir));
      double intensity = cos_t * sc->lint[li] / (ldist * ldist);
      double ds = 0.25;
      if (metallic > 0.95)
        ds = 0.05;
      else if (metallic > 0.9)
        ds = 0.08;
      else if (metallic > 0.8)
        ds = 0.12;
      else if (metallic > 0.7)
        ds = 0.15;
      else if (metallic > 0.5)
        ds = 0.2;
      total = vadd(total, vmuls(albedo, ds * intensity * sf));
      if (metallic > 0.5) {
        vec3 view = vnorm(vmuls(h->p, -1));
        vec3 half = vnorm(vadd(ldir, view));
        double sp = 32.0;
        if (metallic > 0.9)
          sp = 64.0;
        else if (metallic > 0.8)
          sp = 48.0;
        double si = oracle_go_pow(oracle_go_max(0, vdot(h->n, half)), sp);
        total = vadd(total, vmuls(sc->lcolor[li], si * intensity * sf * metallic * 3.0));
      }
    }
  }
  return total;
}

/* traceRay, renderer.go:165-227 */
static vec3 trace_ray(const oscene* sc, oray r, int depth, ostream* s) {
  if (depth >= sc->max_depth) return V(0, 0, 0);
  hitrec h;
  s->c->bounce_rays++;
  if (!hit_world(sc, r, 0.001, INFINITY, &h, s->c))  /* black, or an opted-in sky (rt_settings.sky) */
    return sc->sky ? oracle_sky_color_v(sc->sky, r.d) : V(0.0, 0.0, 0.0);
  const omat* m = h.mat;
  s->c->shade_events++;
  vec3 emitted = mat_emitted(m);
  vec3 direct = direct_lighting(sc, &h, depth, s);
  oray scattered;
  vec3 att;
  if (!mat_scatter(m, r, &h, s, &scattered, &att)) return vadd(emitted, direct);
  vec3 refl = V(0, 0, 0);
  if (sc->recursive) refl = trace_ray(sc, scattered, depth + 1, s);
  double metallic = mat_metallic(m);
  double rw, dw;
  if (metallic > 0.95) {
    rw = 0.85; dw = 0.15;
  } else if (metallic > 0.9) {
    rw = 0.8; dw = 0.2;
  } else if (metallic > 0.8) {
    rw = 0.75; dw = 0.25;
  } else if (metallic > 0.7) {
    rw = 0.7; dw = 0.3;
  } else if (metallic > 0.5) {
    rw = 0.6; dw = 0.4;
  } else if (metallic > 0.2) {
    rw = 0.4; dw = 0.6;
  } else {
    return vadd(vadd(emitted, direct), vmul(att, refl));
  }
  return vadd(vadd(emitted, vmuls(direct, dw)), vmuls(vmul(att, refl), rw));
}

/* getRay, renderer.go:377-390 */
static oray get_ray(const oscene* sc, double u, double v) {
  double vh = 2.0;
  double vw = vh * sc->aspect;
  double focal = 1.0;
  vec3 origin = sc->cam_pos;
  vec3 horizontal = V(vw, 0, 0);
  vec3 vertical = V(0, vh, 0);
  vec3 llc = vsub(vsub(vsub(origin, vdivs(horizontal, 2)), vdivs(vertical, 2)), V(0, 0, focal));
  vec3 dir = vsub(vadd(vadd(llc, vmuls(horizontal, u)), vmuls(vertical, v)), origin);
  oray r = {origin, dir};
  return r;
}

/* tracePixel, renderer.go:150-163 */
static vec3 trace_pixel(const oscene* sc, int x, int y, ocounts* c) {
  vec3 color = V(0, 0, 0);
  uint32_t pixel = (uint32_t)y * (uint32_t)sc->W + (uint32_t)x;
  for (int smp = 0; smp < sc->samples; smp++) {
    ostream st;
    st.c = c;
    rt_rng_init(&st.rng, sc->seed_key, pixel, (uint32_t)smp);
    st.soft_key = rt_soft_key(sc->seed_key, pixel, (uint32_t)smp);
    c->camera_rays++;
    double u = ((double)x + rnd(&st)) / (double)sc->W;
    double v = ((double)y + rnd(&st)) / (double)sc->H;
    oray r = get_ray(sc, u, v);
    const uint64_t b0 = c->bounce_rays;
    color = vadd(color, trace_ray(sc, r, 0, &st));
    if (sc->path_len) {
      const uint64_t n = c->bounce_rays - b0;
      sc->path_len[(size_t)pixel * (size_t)sc->samples + (size_t)smp] = (uint8_t)(n > 255 ? 255 : n);
    }
  }
  return vdivs(color, (double)sc->samples);
}

/* toneMap, renderer.go:348-367 */
void oracle_tonemap(const double in[3], double out[3]) {
  double exposure = 1.0, gamma = 2.2;
  vec3 c = vmuls(varr(in), exposure);
  c.x = 1.0 - exp(-c.x);
  c.y = 1.0 - exp(-c.y);
  c.z = 1.0 - exp(-c.z);
  c.x = oracle_go_pow(c.x, 1.0 / gamma);
  c.y = oracle_go_pow(c.y, 1.0 / gamma);
  c.z = oracle_go_pow(c.z, 1.0 / gamma);
  c.x = oracle_go_max(0.0, oracle_go_min(1.0, c.x));
  c.y = oracle_go_max(0.0, oracle_go_min(1.0, c.y));
  c.z = oracle_go_max(0.0, oracle_go_min(1.0, c.z));
  out[0] = c.x;
  out[1] = c.y;
  out[2] = c.z;
}

/* Go's uint8(float64): amd64 CVTTSD2SQ then truncation to 8 bits; NaN and
 * out-of-range give 0x8000000000000000 -> 0. */
static uint8_t go_uint8(double f) {
  if (isnan(f) || f >= 9.2233720368547758e18 || f < -9.2233720368547758e18) return 0;
  return (uint8_t)(int64_t)f;
}

/* Vec3.ToRGB, vector.go:106-109 */
void oracle_to_rgb(const double in[3], uint8_t out[3]) {
  vec3 c = vclamp(varr(in), 0, 1);
  out[0] = go_uint8(c.x * 255);
  out[1] = go_uint8(c.y * 255);
  out[2] = go_uint8(c.z * 255);
}

/* ------------------------------------------------------------ threads */

typedef struct {
  const oscene* sc;
  int tiles_x, tiles_y, ntiles;
  int rank, world, max_tiles;
  int next; /* next local tile index (row-major tile order) */
  pthread_mutex_t mu;
  double* out_linear;
  uint8_t* out_rgba;
  ocounts total;
} ojob;

static void* worker(void* arg) {
  ojob* job = (ojob*)arg;
  ocounts c;
  memset(&c, 0, sizeof c);
  const oscene* sc = job->sc;
  for (;;) {
    pthread_mutex_lock(&job->mu);
    int lt = job->next++;
    pthread_mutex_unlock(&job->mu);
    int t = job->rank + lt * job->world;
    if (t >= job->ntiles || (job->max_tiles >= 0 && lt >= job->max_tiles)) break;
    int tx = t % job->tiles_x, ty = t / job->tiles_x;
    int x0 = tx * 32, y0 = ty * 32;
    int x1 = x0 + 32 > sc->W ? sc->W : x0 + 32;
    int y1 = y0 + 32 > sc->H ? sc->H : y0 + 32;
    for (int y = y0; y < y1; y++)
      for (int x = x0; x < x1; x++) {
        vec3 col = trace_pixel(sc, x, y, &c);
        size_t pi = (size_t)y * sc->W + x;
        if (job->out_linear) {
          job->out_linear[pi * 3 + 0] = col.x;
          job->out_linear[pi * 3 + 1] = col.y;
          job->out_linear[pi * 3 + 2] = col.z;
        }
        if (job->out_rgba) {
          double in[3] = {col.x, col.y, col.z}, tm[3];
          uint8_t rgb[3];
          oracle_tonemap(in, tm);
          oracle_to_rgb(tm, rgb);
          job->out_rgba[pi * 4 + 0] = rgb[0];
          job->out_rgba[pi * 4 + 1] = rgb[1];
          job->out_rgba[pi * 4 + 2] = rgb[2];
          job->out_rgba[pi * 4 + 3] = 255;
        }
      }
  }
  pthread_mutex_lock(&job->mu);
  job->total.camera_rays += c.camera_rays;
  job->total.bounce_rays += c.bounce_rays;
  job->total.shadow_rays += c.shadow_rays;
  job->total.sphere_tests += c.sphere_tests;
  job->total.triangle_tests += c.triangle_tests;
  job->total.shade_events += c.shade_events;
  job->total.light_evals += c.light_evals;
  job->total.rng_draws += c.rng_draws;
  pthread_mutex_unlock(&job->mu);
  return NULL;
}

int oracle_render(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* st, int32_t rank,
                  int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear, uint8_t* out_rgba,
                  rt_counts* counts) {
  return oracle_render_ex(scene, width, height, st, rank, world, nthreads, max_tiles, out_linear, out_rgba, counts,
                          0);
}

static int render_impl(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* st, int32_t rank,
                       int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear, uint8_t* out_rgba,
                       rt_counts* counts, int32_t use_bvh, uint8_t* path_len);

int oracle_render_ex(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* st, int32_t rank,
                     int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear, uint8_t* out_rgba,
                     rt_counts* counts, int32_t use_bvh) {
  return render_impl(scene, width, height, st, rank, world, nthreads, max_tiles, out_linear, out_rgba, counts, use_bvh,
                     NULL);
}

int oracle_path_lengths(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* st,
                        int32_t nthreads, uint8_t* out) {
  if (!out) return RT_E_INVALID;
  return render_impl(scene, width, height, st, 0, 1, nthreads, -1, NULL, NULL, NULL, 0, out);
}

static int render_impl(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* st, int32_t rank,
                       int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear, uint8_t* out_rgba,
                       rt_counts* counts, int32_t use_bvh, uint8_t* path_len) {
  if (!scene || !st || width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world) return RT_E_INVALID;
  if (scene->num_objects < 0 || scene->num_lights < 0) return RT_E_INVALID;
  if (nthreads < 1) nthreads = 1;
  oscene sc;
  memset(&sc, 0, sizeof sc);
  sc.n = scene->num_objects;
  sc.objs = (ohittable*)calloc(sc.n > 0 ? sc.n : 1, sizeof(ohittable));
  sc.mats = (omat*)calloc(sc.n > 0 ? sc.n : 1, sizeof(omat));
  sc.nl = scene->num_lights;
  sc.lpos = (vec3*)calloc(sc.nl > 0 ? sc.nl : 1, sizeof(vec3));
  sc.lcolor = (vec3*)calloc(sc.nl > 0 ? sc.nl : 1, sizeof(vec3));
  sc.lint = (double*)calloc(sc.nl > 0 ? sc.nl : 1, sizeof(double));
  for (int i = 0; i < sc.n; i++) {
    const rt_object* o = &scene->objects[i];
    sc.mats[i] = make_material(&o->material);
    ohittable* h = &sc.objs[i];
    h->type = o->type;
    h->mat = &sc.mats[i];
    if (o->type == RT_OBJ_SPHERE) {
      h->center = varr(o->position);
      h->radius = o->radius;
    } else {
      make_cube(varr(o->position), varr(o->size), h->tris);
    }
  }
  for (int i = 0; i < sc.nl; i++) {
    sc.lpos[i] = varr(scene->lights[i].position);
    sc.lcolor[i] = varr(scene->lights[i].color);
    sc.lint[i] = scene->lights[i].intensity;
  }
  sc.cam_pos = varr(scene->camera.position);
  sc.aspect = scene->camera.aspect_ratio;
  sc.max_depth = st->max_depth;
  sc.sky = st->sky;
  sc.samples = st->samples;
  sc.recursive = st->recursive_reflections != 0;
  sc.soft = st->soft_shadows != 0;
  sc.seed_key = rt_rng_seed_key(st->seed);
  sc.W = width;
  sc.H = height;
  sc.path_len = path_len;
  if (use_bvh) bvh_make(&sc);

  ojob job;
  memset(&job, 0, sizeof job);
  job.sc = &sc;
  job.tiles_x = (width + 31) / 32;
  job.tiles_y = (height + 31) / 32;
  job.ntiles = job.tiles_x * job.tiles_y;
  job.rank = rank;
  job.world = world;
  job.max_tiles = max_tiles;
  job.out_linear = out_linear;
  job.out_rgba = out_rgba;
  pthread_mutex_init(&job.mu, NULL);
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int i = 0; i < nthreads; i++) pthread_create(&th[i], NULL, worker, &job);
  for (int i = 0; i < nthreads; i++) pthread_join(th[i], NULL);
  pthread_mutex_destroy(&job.mu);
  free(th);
  if (counts) {
    memset(counts, 0, sizeof *counts);
    counts->camera_rays = job.total.camera_rays;
    counts->bounce_rays = job.total.bounce_rays;
    counts->shadow_rays = job.total.shadow_rays;
    counts->sphere_tests = job.total.sphere_tests;
    counts->triangle_tests = job.total.triangle_tests;
    counts->shade_events = job.total.shade_events;
    counts->light_evals = job.total.light_evals;
    counts->rng_draws = job.total.rng_draws;
  }
  free(sc.bvh);
  free(sc.bvh_prims);
  free(sc.objs);
  free(sc.mats);
  free(sc.lpos);
  free(sc.lcolor);
  free(sc.lint);
  return RT_OK;
}

/* ------------------------------------------------------------ unit hooks */

void oracle_vec_op(int op, const double a[3], const double b[3], double eta, double out[3]) {
  vec3 A = varr(a), B = varr(b), R = V(0, 0, 0);
  switch (op) {
    case 0: R = vadd(A, B); break;
    case 1: R = vsub(A, B); break;
    case 2: R = vmul(A, B); break;
    case 3: R = vcross(A, B); break;
    case 4: R = vnorm(A); break;
    case 5: R = vreflect(A, B); break;
    case 6: R = vrefract(A, B, eta); break;
    case 7: R = vclamp(A, 0, 1); break;
    default: break;
  }
  out[0] = R.x;
  out[1] = R.y;
  out[2] = R.z;
}
double oracle_vec_dot(const double a[3], const double b[3]) { return vdot(varr(a), varr(b)); }
double oracle_vec_length(const double a[3]) { return vlen(varr(a)); }

static void rec_out(const hitrec* h, double rec[8]) {
  rec[0] = h->t;
  rec[1] = h->p.x;
  rec[2] = h->p.y;
  rec[3] = h->p.z;
  rec[4] = h->n.x;
  rec[5] = h->n.y;
  rec[6] = h->n.z;
  rec[7] = h->front;
}

int oracle_sphere_hit(const double center[3], double radius, const double o[3], const double d[3], double tmin,
                      double tmax, double rec[8]) {
  ohittable sp;
  memset(&sp, 0, sizeof sp);
  sp.center = varr(center);
  sp.radius = radius;
  oray r = {varr(o), varr(d)};
  hitrec h;
  if (!sphere_hit(&sp, r, tmin, tmax, &h)) return 0;
  rec_out(&h, rec);
  return 1;
}

int oracle_triangle_hit(const double v0[3], const double v1[3], const double v2[3], const double o[3],
                        const double d[3], double tmin, double tmax, double rec[8]) {
  otri t = make_triangle(varr(v0), varr(v1), varr(v2));
  oray r = {varr(o), varr(d)};
  hitrec h;
  if (!triangle_hit(&t, NULL, r, tmin, tmax, &h)) return 0;
  rec_out(&h, rec);
  return 1;
}

int oracle_scatter(const rt_material* m, const double ray_o[3], const double ray_d[3], const double rec[8],
                   uint64_t seed, uint32_t pixel, uint32_t sample, int32_t skip, double out[6], int32_t* draws) {
  omat om = make_material(m);
  ocounts c;
  memset(&c, 0, sizeof c);
  ostream st;
  st.c = &c;
  st.soft_key = 0;
  rt_rng_init(&st.rng, rt_rng_seed_key(seed), pixel, sample);
  for (int i = 0; i < skip; i++) rt_rng_draw(&st.rng);
  hitrec h;
  h.t = rec[0];
  h.p = V(rec[1], rec[2], rec[3]);
  h.n = V(rec[4], rec[5], rec[6]);
  h.front = rec[7] != 0;
  h.mat = &om;
  oray in = {varr(ray_o), varr(ray_d)}, sc;
  vec3 att = V(0, 0, 0);
  sc.o = sc.d = V(0, 0, 0);
  int ok = mat_scatter(&om, in, &h, &st, &sc, &att);
  out[0] = sc.d.x;
  out[1] = sc.d.y;
  out[2] = sc.d.z;
  out[3] = att.x;
  out[4] = att.y;
  out[5] = att.z;
  if (draws) *draws = (int32_t)c.rng_draws;
  return ok;
}

void oracle_rng_draws(uint64_t seed, uint32_t pixel, uint32_t sample, int32_t n, double* out, uint64_t* raw) {
  rt_rng r;
  rt_rng_init(&r, rt_rng_seed_key(seed), pixel, sample);
  for (int i = 0; i < n; i++) {
    uint64_t x = rt_rng_next(&r);
    if (raw) raw[i] = x;
    if (out) out[i] = rt_bits_to_unit(x);
  }
}

/* The 16 soft-shadow points of (pixel, sample, depth, light) as smart_shadow
 * draws them (spec v4), and the rejection tries they took. */
void oracle_soft_points(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t depth, uint32_t light, double out[48],
                        int32_t* tries) {
  ocounts c;
  memset(&c, 0, sizeof c);
  ostream ps;
  ps.c = &c;
  ps.soft_key = rt_soft_key(rt_rng_seed_key(seed), pixel, sample);
  ps.rng.x = rt_soft_state(ps.soft_key, depth, light);
  for (int i = 0; i < 16; i++) {
    const vec3 p = random_in_unit_sphere(&ps);
    out[3 * i + 0] = p.x;
    out[3 * i + 1] = p.y;
    out[3 * i + 2] = p.z;
  }
  if (tries) *tries = (int32_t)(c.rng_draws / 3);
}

void oracle_cube_triangles(const double position[3], const double size[3], double out[108]) {
  otri t[12];
  make_cube(varr(position), varr(size), t);
  for (int i = 0; i < 12; i++)
    for (int k = 0; k < 3; k++) {
      out[i * 9 + k * 3 + 0] = t[i].v[k].x;
      out[i * 9 + k * 3 + 1] = t[i].v[k].y;
      out[i * 9 + k * 3 + 2] = t[i].v[k].z;
    }
}
