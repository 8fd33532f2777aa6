/*
 * oracle.h — CPU restatement of the reference's per-pixel ray-trace path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so, and only as the checker
 * (or the timed CPU baseline) — never as the product path.  The product is
 * concurrent-raytracer-go_amd/ (librtgo.so), which fails loudly without a GPU.
 *
 * Parity pinning: the reference is Go and no Go toolchain exists here
 * (SURVEY.md §0.8), so oracle/_ref cannot be built.  The oracle is pinned by
 * the reference's own known answers (internal/math/vector_test.go:8-105,
 * math_benchmarks_test.go:126-165) plus hand-derived known answers from the
 * Go formulas (tests/test_oracle_known_answers.py).  Whole-image renderer
 * results have no reference golden: "parity unpinned" beyond
 * those unit pins — see DESIGN.md §Oracle.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Render the tiles t with t % world == rank (world = 1: all tiles) exactly as
 * (*ParallelRenderer).Render does (renderer.go:67-163), on `nthreads`
 * worker threads pulling 32x32 tiles in row-major order
 * (createRenderTasks, renderer.go:398-436).  out_linear: W*H*3 doubles
 * (mean radiance, Go image row order), out_rgba: W*H*4; either may be NULL.
 * Pixels of tiles not rendered are left untouched.  counts may be NULL.
 * max_tiles >= 0 limits the number of tiles rendered (CPU-baseline sample). */
int oracle_render(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* settings,
                  int32_t rank, int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear,
                  uint8_t* out_rgba, rt_counts* counts);

/* The same with use_bvh = 1: a sphere BVH and any-hit shadow rays instead of
 * the reference's linear scans, for bench.py's secondary CPU baseline of the
 * 10k-sphere configs -- NOT the reference's algorithm; same
 * image (tests/test_oracle_render.py).  Scenes with cubes scan linearly. */
int oracle_render_ex(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* settings,
                     int32_t rank, int32_t world, int32_t nthreads, int32_t max_tiles, double* out_linear,
                     uint8_t* out_rgba, rt_counts* counts, int32_t use_bvh);

/* Scheduling analysis (dev tool, scripts/path_stats.py): the bounces of every
 * sample's path (traceRay calls, clamped at 255) of the whole frame,
 * out[(y*W + x)*samples + s]; no image. */
int oracle_path_lengths(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* settings,
                        int32_t nthreads, uint8_t* out);

/* Building blocks exposed for known-answer tests. */
double oracle_go_pow(double x, double y);            /* math.Pow */
double oracle_go_max(double x, double y);            /* math.Max */
double oracle_go_min(double x, double y);            /* math.Min */
void oracle_tonemap(const double in[3], double out[3]);          /* renderer.go:348-367 */
void oracle_to_rgb(const double in[3], uint8_t out[3]);          /* vector.go:106-109 */
/* vector ops (vector.go): op 0 add,1 sub,2 mul,3 cross,4 normalize,5 reflect(a,b),
 * 6 refract(a, b, eta), 7 clamp(a, eta_lo=0..1) */
void oracle_vec_op(int op, const double a[3], const double b[3], double eta, double out[3]);
double oracle_vec_dot(const double a[3], const double b[3]);
double oracle_vec_length(const double a[3]);
/* Sphere.Hit (sphere.go:22-59). Returns 1 on hit; rec = {t, px,py,pz, nx,ny,nz, front} */
int oracle_sphere_hit(const double center[3], double radius, const double o[3], const double d[3],
                      double tmin, double tmax, double rec[8]);
/* Triangle.Hit via NewTriangle (triangle.go:13-88). */
int oracle_triangle_hit(const double v0[3], const double v1[3], const double v2[3], const double o[3],
                        const double d[3], double tmin, double tmax, double rec[8]);
/* Material.Scatter for one material on a given hit, with the RNG stream
 * (seed_key, pixel, sample) advanced by `skip` draws first.  Returns
 * scattered flag; out = {dir x,y,z, atten r,g,b}; *draws = draws consumed. */
int oracle_scatter(const rt_material* m, const double ray_o[3], const double ray_d[3], const double rec[8],
                   uint64_t seed, uint32_t pixel, uint32_t sample, int32_t skip, double out[6], int32_t* draws);
/* First n draws of stream (seed, pixel, sample) — RNG known answers. */
void oracle_rng_draws(uint64_t seed, uint32_t pixel, uint32_t sample, int32_t n, double* out, uint64_t* raw);
void oracle_soft_points(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t depth, uint32_t light, double out[48],
                        int32_t* tries);
/* AtmosphereConfig.GetSkyColor of preset `sky` (RT_SKY_DEFAULT..NIGHT) for a ray direction. */
void oracle_sky_color(int sky, const double dir[3], double out[3]);
/* Flattened cube triangles (createCube, scene.go:150-190): 12 x 9 doubles. */
void oracle_cube_triangles(const double position[3], const double size[3], double out[108]);

#ifdef __cplusplus
}
#endif
#endif
