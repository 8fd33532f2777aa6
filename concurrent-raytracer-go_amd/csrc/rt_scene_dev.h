// rt_scene_dev.h — flattened, device-resident scene layout (HBM).
//
// Produced on the host by flatten_scene() (rt_api.cpp) from the boundary's
// rt_scene (objects-level, like scene.Scene, internal/scene/scene.go:12-16)
// and read by the gfx950 kernels (rt_kernel.hip).  Everything the reference
// recomputes per test but which depends only on the scene is precomputed
// here with the reference's own expressions, so the values are bit-identical:
//   - triangle edges v1-v0, v2-v0 (triangle.go:37-38) and the face normal
//     normalize(edge1 x edge2) (NewTriangle, triangle.go:13-34);
//   - the material constructors' clamps (material.go:65-73, ...) and the
//     per-metallic tables of calculateDirectLighting / traceRay
//     (renderer.go:193-226, 236-246, 262-287).
// Small scenes are scanned linearly with wave-uniform (scalar-cache) loads;
// large sphere scenes use the BVH (bvh.cpp) whose nodes follow the arrays.
#pragma once
#include <stdint.h>

namespace rtgo {

struct alignas(16) DSphere {  // 48 B
  double c[3];
  double r;
  double r2;    // r*r, the value Sphere.Hit computes per test (sphere.go:26)
  int32_t mat;
  int32_t obj;  // hittable index (tie order)
};

struct alignas(16) DTri {  // 144 B
  double v0[3];
  double e1[3];  // v1 - v0
  double e2[3];  // v2 - v0
  double n[3];   // face normal = Normals[0..2]
  double bc[3];  // bounding sphere (culling only): centroid ...
  double br;     // ... and the largest vertex distance
  int32_t mat;
  int32_t obj;
  int32_t pad[2];
};

// Axis-aligned box of one cube's 12 triangles (createCube, scene.go:150-190,
// builds an axis-aligned box), padded outward by ~1e-9 relative: culling
// only -- a ray that misses it cannot hit any of its triangles.
struct alignas(16) DBox {  // 96 B
  double lo[3];
  double hi[3];
  double bc[3];   // bounding sphere of the box (shadow-cone culling)
  double br;
  int32_t first;  // first triangle (12 consecutive)
  int32_t count;
  int32_t obj;
  // What FrontFace (triangle.go:70-73) means on this cube's triangles.
  // createCube's face table winds every normal INTO the box when
  // size.x*size.y*size.z > 0, so a front-face hit comes from inside (0); an
  // odd number of negative size components mirrors the box and its normals
  // point out (1: front = outside); a zero or non-finite product: unknown
  // (-1, the hit cube is never left out of its own shadow rays).
  int32_t front_out;
};

// Material kinds: RT_MAT_* of rt_api.h.
struct alignas(16) DMat {  // 192 B
  int32_t kind;
  int32_t spec_pow;        // 64 / 48 / 32 (renderer.go:282-287), used iff metallic > 0.5
  int32_t rough_draw;      // scatter draws a unit-sphere point
  int32_t blend_metal;     // Metal: metallic > 0.8 second blend
  double color[3];         // Metal/Shiny albedo, PerfectMirror/Glass color, DiffuseLight emit
  double albedo[3];        // GetAlbedo() for direct lighting
  double emit[3];          // Emitted()
  double roughness;
  double metallic;         // GetMetallic()
  double ior;              // Glass/Dielectric refraction index; Metal/Shiny/PM: Fresnel IOR
  double f0;               // Schlick f0 = Pow((IOR-1)/(IOR+1), 2)
  double fs;               // Metal 0.6+0.4m, Shiny 0.4+0.4spec
  double mf;               // Metal 0.4+0.5m
  double ambient;          // renderer.go:236-243
  double diffuse_strength; // renderer.go:262-273
  double dw, rw;           // traceRay direct / reflection weights (1,1 when metallic <= 0.2)
  double pad;
};

struct alignas(16) DLight {  // 64 B
  double pos[3];
  double color[3];
  double intensity;
  double pad;
};

// An AtmosphereConfig preset (internal/atmosphere/atmosphere.go:8-98): the
// radiance of a ray that hits nothing when a sky is opted in (rt_settings.sky).
struct alignas(16) DSky {  // 240 B
  double top[3], bottom[3];     // SkyColorTop, SkyColorBottom
  double sun_dir[3], sun_color[3];
  double sun_intensity, sun_size;
  double rayleigh[3], mie[3];   // RayleighScattering, MieScattering
  double depth;                 // AtmosphericDepth
  double fog_density;
  double fog_color[3];
  double time_of_day;
  double pad;
};

// BVH node over spheres (binned SAH, built on host).  Bounds are float,
// rounded outward so a box never excludes a sphere point; leaves reference
// [first, first+count) of the BVH-ordered sphere array.
struct alignas(16) DBVHNode {  // 32 B
  float lo[3];
  int32_t left_or_first;  // internal: index of left child (right = left+1); leaf: first sphere
  float hi[3];
  int32_t count;          // 0 = internal node
};

// The same BVH with 16-bit quantized bounds (the wavefront kernels,
// rt_wavefront.hip): bounds are grid indices q (coordinate = q0 + q * qd per
// axis, FlatScene), rounded outward; 16 B per node, a child pair in one
// 32-B load.  w[0] = lo.x | lo.y << 16, w[1] = lo.z | hi.x << 16,
// w[2] = hi.y | hi.z << 16, w[3] = traversal code (first << 3 | count).
struct alignas(16) DQNode {  // 16 B
  uint32_t w[4];
};

}  // namespace rtgo
