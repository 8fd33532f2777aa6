// scene_flat.cpp — GetHittables + createCube + the material constructors
// (internal/scene/scene.go:59-190, internal/material/*.go) as flat device
// records (rt_scene_dev.h), the opt-in sky presets, and the host-only entry
// points of the ABI (settings defaults, tile arithmetic).  No HIP calls, so
// the sanitizer build (tests/c/Makefile) links it directly.
//
// Compiled with -ffp-contract=off: the precomputations (cube vertices,
// triangle edges and normals, material tables) must equal the values the
// reference computes per test.
#include <math.h>
#include <string.h>

#include "rt_internal.h"

namespace rtgo {

// ---------------------------------------------------------------- Go math
static double go_min(double x, double y) {
  if ((isinf(x) && x < 0) || (isinf(y) && y < 0)) return -INFINITY;
  if (isnan(x) || isnan(y)) return NAN;
  if (x == 0 && x == y) return signbit(x) ? x : y;
  return x < y ? x : y;
}

struct v3 {
  double x, y, z;
};
static v3 mk(double x, double y, double z) { return v3{x, y, z}; }
static v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 divs(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
static v3 cross(v3 a, v3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static v3 normalize(v3 a) {
  double l = sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
  if (l == 0) return mk(0, 0, 0);
  return divs(a, l);
}
static v3 arr(const double* p) { return mk(p[0], p[1], p[2]); }
static void put(double* d, v3 v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

// Material constructors (material.go:22-73,159-167,231-233,292-294;
// advanced_materials.go:14-19,117-123) and the metallic tables the renderer
// derives from GetMetallic (renderer.go:193-226,236-246,262-287).
static DMat make_mat(const rt_material& m) {
  DMat d;
  memset(&d, 0, sizeof d);
  d.kind = m.kind;
  put(d.color, arr(m.color));
  double metallic = 0.0;
  switch (m.kind) {
    case RT_MAT_METAL:
    case RT_MAT_SHINY:
      d.roughness = go_min(m.roughness, 1.0);
      metallic = go_min(m.metallic, 1.0);
      d.ior = 1.5;
      put(d.albedo, arr(m.color));
      if (m.kind == RT_MAT_METAL) {
        d.rough_draw = d.roughness > 0.001;
        d.fs = 0.6 + metallic * 0.4;
        d.mf = 0.4 + metallic * 0.5;
        d.blend_metal = metallic > 0.8;
      } else {
        d.rough_draw = d.roughness > 0;
        d.fs = 0.4 + go_min(m.specular, 1.0) * 0.4;
      }
      break;
    case RT_MAT_PERFECTMIRROR:
      d.roughness = go_min(m.roughness, 1.0);
      d.rough_draw = d.roughness > 0.001;
      metallic = 1.0;
      d.ior = 2.0;
      put(d.albedo, arr(m.color));
      break;
    case RT_MAT_GLASS:
      d.ior = m.refraction_index;
      put(d.albedo, arr(m.color));
      break;
    case RT_MAT_DIELECTRIC:  // attenuation and GetAlbedo are (1,1,1), material.go:236,266-268
      d.ior = m.refraction_index;
      put(d.color, mk(1.0, 1.0, 1.0));
      put(d.albedo, mk(1.0, 1.0, 1.0));
      break;
    case RT_MAT_DIFFUSELIGHT:
      put(d.emit, arr(m.color));
      break;
    default:  // lambertian
      d.kind = RT_MAT_LAMBERTIAN;
      put(d.albedo, arr(m.color));
      break;
  }
  d.metallic = metallic;
  {  // Schlick f0 = Pow((IOR-1)/(IOR+1), 2) — Go's Pow(x,2) rounds as x*x
    double r = (d.ior - 1.0) / (d.ior + 1.0);
    d.f0 = r * r;
  }
  d.ambient = 0.1;
  if (metallic > 0.9)
    d.ambient = 0.05;
  else if (metallic > 0.7)
    d.ambient = 0.07;
  else if (metallic > 0.5)
    d.ambient = 0.08;
  d.diffuse_strength = 0.25;
  if (metallic > 0.95)
    d.diffuse_strength = 0.05;
  else if (metallic > 0.9)
    d.diffuse_strength = 0.08;
  else if (metallic > 0.8)
    d.diffuse_strength = 0.12;
  else if (metallic > 0.7)
    d.diffuse_strength = 0.15;
  else if (metallic > 0.5)
    d.diffuse_strength = 0.2;
  d.spec_pow = metallic > 0.9 ? 64 : (metallic > 0.8 ? 48 : 32);
  if (metallic > 0.95) {
    d.rw = 0.85; d.dw = 0.15;
  } else if (metallic > 0.9) {
    d.rw = 0.8; d.dw = 0.2;
  } else if (metallic > 0.8) {
    d.rw = 0.75; d.dw = 0.25;
  } else if (metallic > 0.7) {
    d.rw = 0.7; d.dw = 0.3;
  } else if (metallic > 0.5) {
    d.rw = 0.6; d.dw = 0.4;
  } else if (metallic > 0.2) {
    d.rw = 0.4; d.dw = 0.6;
  } else {
    d.rw = 1.0; d.dw = 1.0;
  }
  return d;
}

static void push_tri(FlatScene* fs, v3 v0, v3 v1, v3 v2, int mat, int obj) {
  DTri t;
  memset(&t, 0, sizeof t);
  v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  put(t.v0, v0);
  put(t.e1, e1);
  put(t.e2, e2);
  put(t.n, normalize(cross(e1, e2)));  // NewTriangle, triangle.go:13-34
  // bounding sphere for the shadow-cone culling (rt_kernel.hip); any
  // rounding here is covered by the kernel's inflation margins
  const v3 bc = divs(add(add(v0, v1), v2), 3.0);
  double br = 0;
  for (v3 v : {v0, v1, v2}) {
    v3 dv = sub(v, bc);
    br = fmax(br, sqrt(dv.x * dv.x + dv.y * dv.y + dv.z * dv.z));
  }
  put(t.bc, bc);
  t.br = br;
  t.mat = mat;
  t.obj = obj;
  fs->tris.push_back(t);
}

void sky_presets(DSky out[kSkies]) {
  memset(out, 0, sizeof(DSky) * kSkies);
  struct P {
    double top[3], bottom[3], sun_dir[3], sun_color[3], sun_intensity, sun_size, rayleigh[3], mie[3], depth, fog,
        fog_color[3], haze, tod;
  };
  // NewDefaultAtmosphere, NewWhiteAtmosphere, NewSunsetAtmosphere,
  // NewNightAtmosphere (atmosphere.go:28-98); HazeIntensity is unused by GetSkyColor
  static const P presets[kSkies] = {
      {{0.6, 0.8, 1.0}, {0.9, 0.95, 1.0}, {0.0, 0.8, -0.6}, {1.0, 0.98, 0.95}, 1.2, 0.015, {0.6, 0.8, 1.0},
       {1.0, 0.98, 0.95}, 0.3, 0.0, {0.9, 0.92, 0.95}, 0.05, 0.6},
      {{0.98, 0.98, 1.0}, {0.92, 0.92, 0.95}, {0.0, 0.8, -0.6}, {1.0, 0.99, 0.97}, 0.8, 0.012, {0.9, 0.9, 0.95},
       {0.95, 0.95, 0.98}, 0.2, 0.0, {0.95, 0.95, 0.98}, 0.02, 0.6},
      {{1.0, 0.4, 0.2}, {1.0, 0.8, 0.6}, {0.0, 0.3, -0.9}, {1.0, 0.6, 0.3}, 1.2, 0.03, {1.0, 0.4, 0.2},
       {1.0, 0.8, 0.6}, 0.8, 0.1, {1.0, 0.8, 0.6}, 0.3, 0.8},
      {{0.1, 0.1, 0.3}, {0.2, 0.2, 0.4}, {0.0, -0.7, -0.7}, {0.8, 0.8, 1.0}, 0.3, 0.005, {0.1, 0.1, 0.3},
       {0.8, 0.8, 1.0}, 0.2, 0.0, {0.1, 0.1, 0.2}, 0.0, 0.0},
  };
  for (int i = 0; i < kSkies; ++i) {
    const P& p = presets[i];
    DSky& d = out[i];
    memcpy(d.top, p.top, sizeof d.top);
    memcpy(d.bottom, p.bottom, sizeof d.bottom);
    memcpy(d.sun_dir, p.sun_dir, sizeof d.sun_dir);
    memcpy(d.sun_color, p.sun_color, sizeof d.sun_color);
    d.sun_intensity = p.sun_intensity;
    d.sun_size = p.sun_size;
    memcpy(d.rayleigh, p.rayleigh, sizeof d.rayleigh);
    memcpy(d.mie, p.mie, sizeof d.mie);
    d.depth = p.depth;
    d.fog_density = p.fog;
    memcpy(d.fog_color, p.fog_color, sizeof d.fog_color);
    d.time_of_day = p.tod;
  }
}

void flatten_scene(const rt_scene& s, FlatScene* fs) {
  *fs = FlatScene();
  for (int i = 0; i < s.num_objects; ++i) {
    const rt_object& o = s.objects[i];
    const int mat = (int)fs->mats.size();
    fs->mats.push_back(make_mat(o.material));
    if (o.type == RT_OBJ_SPHERE) {
      DSphere sp;
      memset(&sp, 0, sizeof sp);
      put(sp.c, arr(o.position));
      sp.r = o.radius;
      sp.r2 = o.radius * o.radius;
      sp.mat = mat;
      sp.obj = i;
      fs->spheres.push_back(sp);
    } else {  // createCube, scene.go:150-190
      v3 pos = arr(o.position);
      v3 h = divs(arr(o.size), 2.0);
      v3 v[8] = {add(pos, mk(-h.x, -h.y, -h.z)), add(pos, mk(h.x, -h.y, -h.z)), add(pos, mk(h.x, h.y, -h.z)),
                 add(pos, mk(-h.x, h.y, -h.z)),  add(pos, mk(-h.x, -h.y, h.z)), add(pos, mk(h.x, -h.y, h.z)),
                 add(pos, mk(h.x, h.y, h.z)),    add(pos, mk(-h.x, h.y, h.z))};
      static const int faces[6][4] = {{0, 1, 2, 3}, {1, 5, 6, 2}, {5, 4, 7, 6},
                                      {4, 0, 3, 7}, {3, 2, 6, 7}, {4, 5, 1, 0}};
      DBox b;
      memset(&b, 0, sizeof b);
      b.first = (int32_t)fs->tris.size();
      b.count = 12;
      b.obj = i;
      for (int f = 0; f < 6; ++f) {
        push_tri(fs, v[faces[f][0]], v[faces[f][1]], v[faces[f][2]], mat, i);
        push_tri(fs, v[faces[f][0]], v[faces[f][2]], v[faces[f][3]], mat, i);
      }
      // the box of the 8 corners, padded outward (culling only; the
      // triangle tests stay exact)
      for (int a = 0; a < 3; ++a) {
        double lo = INFINITY, hi = -INFINITY;
        for (const v3& q : v) {
          const double c = a == 0 ? q.x : (a == 1 ? q.y : q.z);
          lo = fmin(lo, c);
          hi = fmax(hi, c);
        }
        const double pad = (fmax(fabs(lo), fabs(hi)) + (hi - lo)) * 1e-9 + 1e-12;
        b.lo[a] = lo - pad;
        b.hi[a] = hi + pad;
      }
      double r2 = 0;
      for (int a = 0; a < 3; ++a) {
        b.bc[a] = 0.5 * (b.lo[a] + b.hi[a]);
        r2 += (b.hi[a] - b.bc[a]) * (b.hi[a] - b.bc[a]);
      }
      b.br = sqrt(r2) * (1.0 + 1e-12);  // covers the padded box (the kernel adds its own margins)
      // the winding of createCube's face table (scene.go:164-171): normals
      // inward for a positive size product, outward for a negative one
      // (DBox.front_out).  A size difference that rounds away in a vertex
      // makes the box flat in that axis (its other faces zero-area, normal 0),
      // where leaving the plane never returns, whichever side is "out".
      const double vol = h.x * h.y * h.z;
      b.front_out = vol > 0 && isfinite(vol) ? 0 : (vol < 0 && isfinite(vol) ? 1 : -1);
      fs->boxes.push_back(b);
    }
  }
  for (int i = 0; i < s.num_lights; ++i) {
    DLight l;
    memset(&l, 0, sizeof l);
    put(l.pos, arr(s.lights[i].position));
    put(l.color, arr(s.lights[i].color));
    l.intensity = s.lights[i].intensity;
    fs->lights.push_back(l);
  }
  put(fs->cam_pos, arr(s.camera.position));
  fs->aspect = s.camera.aspect_ratio;
  fs->objects = s.num_objects;
}

}  // namespace rtgo

extern "C" {

void rt_settings_default(rt_settings* s) {
  if (!s) return;
  memset(s, 0, sizeof *s);
  // NewParallelRenderer defaults, renderer.go:54-65
  s->samples = 100;
  s->max_depth = 50;
  s->anti_aliasing = 1;
  s->recursive_reflections = 1;
  s->soft_shadows = 1;
  s->depth_of_field = 0;
  s->num_workers = 1;
  s->num_devices = 1;
  s->seed = 1;
}

void rt_tuning_default(rt_tuning* t) {
  if (!t) return;
  memset(t, 0, sizeof *t);
  t->path = RT_PATH_AUTO;
  t->pilot = 1;
  t->frustum = 1;
  t->stage = 1;
  t->wf_lds_nodes = -1;
  // a pilot path is followed for 12 bounces at most: every longer path is
  // "heavy" alike (split, dispatched first), and the pilot's own tail is one
  // 12-bounce path instead of a 50-bounce one (C2 first frame 1.39 -> 1.07 ms,
  // the main launch unchanged; scripts/first_frame_probe.py)
  t->pilot_depth = 12;
  // measured re-cuts are exact but do not shorten the launch: its tail is
  // the chains of the longest paths, not the block sizes (C2 0.80 pilot-only
  // vs 0.84 ms measured, C3 0.59 vs 0.56; scripts/tuning_sweep.py)
  t->measure = 0;
  // tail helpers: 64 at the end of the launch; drains
  // checked every 4th iteration, paths of >= 2 bounces, <= 4 left (the 0s)
  t->tail_helpers = -1;  // measured a net loss on the headline frame
}

int32_t rt_num_tiles(int32_t w, int32_t h) {
  if (w <= 0 || h <= 0) return 0;
  return ((w + 31) / 32) * ((h + 31) / 32);
}

int32_t rt_tiles_for_rank(int32_t w, int32_t h, int32_t rank, int32_t world) {
  int32_t n = rt_num_tiles(w, h);
  if (world < 1 || rank < 0 || rank >= world || rank >= n) return 0;
  return (n - rank + world - 1) / world;
}

}  // extern "C"
