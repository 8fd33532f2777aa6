/*
 * rt_api.h — C ABI of the MI355X-native renderer core (librtgo.so).
 *
 * Drop-in boundary for the per-pixel ray-trace hot path of
 * JoshElkind/concurrent-raytracer-go.  The reference has no FFI; its seam is
 * the Go method set of *renderer.ParallelRenderer, called only from
 * cmd/raytracer/main.go:40-69.  Each entry point below names the reference
 * symbol (file:line, relative to the reference root) it replaces.
 *
 * Conventions:
 *   - every function returns 0 (RT_OK) on success and a negative RT_E* code
 *     on failure; rt_last_error() returns a thread-local message.  Nothing
 *     here aborts the process (the Go loader panics on a bad material;
 *     internal/scene/scene.go:105,109-145).
 *   - buffers are caller-owned; no pointer is retained after a call returns,
 *     except the scene a context uploads (copied to device memory).
 *   - rt_render is synchronous and blocking like Go's Render
 *     (internal/renderer/renderer.go:67-126).  A context is not safe for
 *     concurrent use from several threads (neither is the Go renderer: it
 *     mutates benchmarkData, renderer.go:103-112).
 *   - all arithmetic on the path is IEEE binary64, like the Go float64 code.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 5  /* 5: rt_tuning tail_* fields; 4: rt_renderer_rank_seconds takes a capacity */

/* status codes */
#define RT_OK 0
#define RT_E_INVALID (-1)   /* bad argument */
#define RT_E_IO (-2)        /* file read/write failed */
#define RT_E_PARSE (-3)     /* scene JSON malformed */
#define RT_E_DEVICE (-4)    /* HIP runtime / device error */
#define RT_E_NOMEM (-5)
#define RT_E_TIMEOUT (-6)   /* a multi-device frame did not finish in time (rt_renderer_set_watchdog) */

/* Object kinds — internal/scene/scene.go:69-82 ("sphere", "cube"; any other
 * type string is skipped by the loader with "Unknown object type"). */
#define RT_OBJ_SPHERE 0
#define RT_OBJ_CUBE 1

/* Material kinds reachable from JSON — internal/scene/scene.go:104-148. */
#define RT_MAT_LAMBERTIAN 0    /* material.go:18-55 (also the default case) */
#define RT_MAT_METAL 1         /* material.go:57-149 */
#define RT_MAT_SHINY 2         /* material.go:151-225 */
#define RT_MAT_PERFECTMIRROR 3 /* advanced_materials.go:111-171 */
#define RT_MAT_GLASS 4         /* advanced_materials.go:9-66 */
#define RT_MAT_DIELECTRIC 5    /* material.go:227-286 */
#define RT_MAT_DIFFUSELIGHT 6  /* material.go:288-318 */

/* Material parameters exactly as the JSON loader hands them to the Go
 * constructors (scene.go:104-148), i.e. with the loader's defaults already
 * applied (metal: roughness 0, metallic 1, specular 1; shiny: roughness 0,
 * metallic 0, specular 1; perfectmirror: roughness 0; glass/dielectric:
 * refractionIndex 1.5).  The constructors' clamps (NewMetal's
 * Min(x,1.0), material.go:65-73 etc.) are applied by the renderer, not here. */
typedef struct {
  int32_t kind;          /* RT_MAT_* */
  int32_t _pad;
  double color[3];       /* "color" (emit colour for diffuselight) */
  double roughness;
  double metallic;
  double specular;
  double refraction_index;
} rt_material;

/* One scene object — internal/scene/scene.go:26-32 (type Object). */
typedef struct {
  int32_t type;          /* RT_OBJ_* */
  int32_t _pad;
  double position[3];    /* sphere centre / cube centre */
  double size[3];        /* cube edge lengths (unused for spheres) */
  double radius;         /* sphere radius (unused for cubes) */
  rt_material material;
} rt_object;

/* Point light — scene.go:34-39.  "type" is ignored by the renderer
 * (renderer.go:248-294 treats every light as a point light). */
typedef struct {
  double position[3];
  double color[3];
  double intensity;
} rt_light;

/* Camera — scene.go:18-24.  Only position and aspect_ratio are used by the
 * reference's getRay (renderer.go:377-390); the others are carried for
 * fidelity. */
typedef struct {
  double position[3];
  double look_at[3];
  double up[3];
  double fov;
  double aspect_ratio;
} rt_camera;

/* Scene view — scene.go:12-16 (type Scene). */
typedef struct {
  rt_camera camera;
  const rt_object* objects;
  int32_t num_objects;
  int32_t _pad0;
  const rt_light* lights;
  int32_t num_lights;
  int32_t _pad1;
} rt_scene;

/* Renderer settings — the ParallelRenderer fields (renderer.go:20-29) and
 * their setters (settings.go:3-25).  Defaults: rt_settings_default(). */
typedef struct {
  int32_t samples;               /* SetSamples; default 100; any count in [0, 2^24] with W*H*samples < 2^40
                                    (past 1024 the linear-scan kernel renders in sample passes) */
  int32_t max_depth;             /* SetMaxDepth; default 50 */
  int32_t anti_aliasing;         /* SetAntiAliasing; inert in the reference (jitter is unconditional, renderer.go:155-156) */
  int32_t recursive_reflections; /* SetRecursiveReflections; default 1 */
  int32_t soft_shadows;          /* SetSoftShadows; default 1 */
  int32_t depth_of_field;        /* SetDepthOfField; inert (advanced.go unused) */
  int32_t num_workers;           /* NewParallelRenderer(n) (the Go CLI passes runtime.NumCPU(),
                                    cmd/raytracer/main.go:46); recorded in benchmark data only */
  int32_t num_devices;           /* rt_render: GPUs 0..n-1 render tiles t % n (0 or 1: device 0 only) */
  uint64_t seed;                 /* counter-based RNG seed (include/rt_rng.h); default 1 */
  int32_t sky;                   /* RT_SKY_*: radiance of a ray that hits nothing; default RT_SKY_NONE */
  int32_t _pad2;
} rt_settings;

/* What a ray that hits nothing returns.  The reference's live path returns
 * black (traceRay, renderer.go:170-173): RT_SKY_NONE, the default and the
 * parity setting.  The others are OPT-IN and follow the reference's
 * (unlinked) atmosphere package: AtmosphereConfig.GetSkyColor
 * (internal/atmosphere/atmosphere.go:100-135) with the presets
 * NewDefaultAtmosphere / NewWhiteAtmosphere / NewSunsetAtmosphere /
 * NewNightAtmosphere (atmosphere.go:28-98); its undefined FastVec3* helpers
 * are taken as the Vec3 methods of the same name (Normalize, a.Lerp(b, t) =
 * a + (b - a) t, Dot, MulScalar; internal/math/vector.go). */
#define RT_SKY_NONE 0
#define RT_SKY_DEFAULT 1
#define RT_SKY_WHITE 2
#define RT_SKY_SUNSET 3
#define RT_SKY_NIGHT 4

typedef struct {
  double render_seconds;    /* wall time of rt_render, upload + kernels + download (Go Render semantics) */
  double kernel_seconds;    /* device time of the render kernels (HIP events) */
  double rays_per_second;   /* W*H*spp / render_seconds — the published metric (README.md:61) */
  double pixels_per_second; /* W*H / render_seconds (README.md:60) */
  int32_t objects;          /* len(hittables): a cube counts as one (renderer.go:109) */
  int32_t lights;
  /* Where render_seconds went (host wall clock): device state created
   * (rt_render only: contexts, streams, RCCL), scene flattened and uploaded
   * (0 when the renderer already holds it), of which building the BVH (the
   * published benchmark JSON's bvh_build_time / setup_time), the launches
   * enqueued (with a new work schedule: the pilot render and the scheduler,
   * DESIGN.md §4.1), the image copied to the host after the kernels, and
   * the device state freed again (rt_render only). */
  double create_seconds;
  double scene_seconds;
  double bvh_build_seconds;
  double launch_seconds;
  double download_seconds;
  double destroy_seconds;
} rt_stats;

/* Per-launch operation counts (for the roofline's algorithmic FLOPs). */
typedef struct {
  uint64_t camera_rays;      /* primary samples traced */
  uint64_t bounce_rays;      /* closest-hit queries (primary + scattered) */
  uint64_t shadow_rays;      /* any-hit queries (hard + soft) */
  uint64_t sphere_tests;     /* ray/sphere intersection tests executed */
  uint64_t triangle_tests;   /* ray/triangle tests executed */
  uint64_t box_tests;        /* BVH node slab tests executed */
  uint64_t shade_events;     /* surface hits shaded (direct lighting + scatter) */
  uint64_t light_evals;      /* per-light direct-lighting evaluations */
  uint64_t rng_draws;        /* uniform draws */
  /* The part of the nine counts above that the product never executes: the
   * counting variant walks every camera sample so that its counts are the
   * reference's (tracePixel traces them all, renderer.go:150-163), but the
   * product skips the samples of pixels whose camera rays provably miss
   * everything (primary-ray culling).  Executed work =
   * count - culled, in the same order (camera_rays .. rng_draws). */
  uint64_t culled[9];
  /* The wavefront path's soft-shadow traversal kernel alone (wf_occlude<soft>,
   * calculateSmartShadow's 16 jittered rays, renderer.go:311-327): its share
   * of the counts, for that kernel's own roofline (shadow_rays: the rays it
   * traced).  Zero on the megakernel. */
  uint64_t soft_occlusion[9];
  /* The wavefront path's closest-hit traversal (wf_extend, hitWorld
   * renderer.go:333-346) and hard-ray traversal (wf_occlude<hard>,
   * renderer.go:305) alone: their shares of the counts (box and sphere tests;
   * bounce_rays / shadow_rays: the rays each traversed), for each kernel's own
   * roofline.  Zero on the megakernel. */
  uint64_t extend[9];
  uint64_t hard_occlusion[9];
} rt_counts;

void rt_settings_default(rt_settings* s);
/* The library keeps device buffers freed by destroyed contexts and renderers
 * for reuse (rt_render creates and frees its device state every call), at
 * most 4 GB per device; this returns them to the device.  A caller that also
 * allocates device memory elsewhere (PyTorch, RCCL) and runs short should
 * call it: the cached blocks are invisible to other allocators. */
int rt_release_cached_memory(void);
int32_t rt_abi_version(void);
/* Debug: __shfl reads of the kernels whose source lane was inactive (they
 * return no data) since the last reset, on `device`.  Only the checking build
 * (`make xlane`, build/xlane/librtgo.so) counts them; a normal build returns
 * RT_E_INVALID. */
int rt_debug_xlane_faults(int32_t device, int32_t reset, uint64_t* out);
const char* rt_last_error(void);

/* ---------------------------------------------------------------- scene */

typedef struct rt_scene_buf rt_scene_buf; /* owns a parsed scene */

/* scene.LoadFromFile — internal/scene/scene.go:45-57 (+ Vec3.UnmarshalJSON,
 * internal/math/vector.go:176-193, and the material defaults of
 * createMaterial, scene.go:104-148).  Unknown object types are dropped like
 * GetHittables does (scene.go:80-82).  A material without "color" (Go
 * panics, scene.go:113) is loaded with colour (0,0,0) and counted in
 * rt_scene_warnings(). `verbose` != 0 prints the reference's stdout lines
 * (scene.go:62-88). */
int rt_scene_load_json(const char* path, int32_t verbose, rt_scene_buf** out);
int rt_scene_parse_json(const char* text, size_t len, int32_t verbose, rt_scene_buf** out);
const rt_scene* rt_scene_view(const rt_scene_buf* buf);
int32_t rt_scene_warnings(const rt_scene_buf* buf);
void rt_scene_free(rt_scene_buf* buf);
/* Print the lines (*Scene).GetHittables prints (scene.go:62-88), in Go's
 * fmt formatting, for a CLI that mirrors cmd/raytracer. */
int rt_scene_print_hittables(const rt_scene_buf* buf);

/* ------------------------------------------------------- blocking render */

/* (*ParallelRenderer).Render — internal/renderer/renderer.go:67-126.
 * out_linear_rgb: W*H*3 floats (may be NULL), pixel (x,y) at (y*W+x)*3, i.e.
 *   the Go image row y (row 0 is the BOTTOM of the viewport: the image is
 *   vertically flipped vs world up, exactly like the reference).  Value =
 *   mean radiance over samples before tone mapping.
 * out_rgba: W*H*4 bytes (may be NULL) — toneMap + ToRGB, alpha 255
 *   (renderer.go:92-97,348-367; vector.go:106-109).
 * stats may be NULL.  Renders on HIP device 0; returns RT_E_DEVICE (and a
 * message) when no device is present — there is no CPU fallback. */
int rt_render(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* settings,
              float* out_linear_rgb, uint8_t* out_rgba, rt_stats* stats);
/* The argument checks rt_render makes before it touches a device (scene
 * arrays and kinds; 1 <= W, H <= 65536; samples range): RT_OK or RT_E_INVALID. */
int rt_validate(const rt_scene* scene, int32_t width, int32_t height, const rt_settings* settings);

/* ------------------------------------------ persistent multi-GPU renderer */

/* The ParallelRenderer object itself (NewParallelRenderer, renderer.go:54-65,
 * then Render per frame, renderer.go:67-126), on GPUs instead of goroutines.
 * One process drives `num_devices` ranks; rank r renders the 32x32 tiles
 * t with t % num_devices == r on devices[r] (devices NULL: 0..n-1).  Ranks
 * whose device is devices[0] render straight into the gather buffer there;
 * the others send their packed tiles (float3 + RGBA8, 16 B per pixel) to
 * devices[0] in ONE RCCL group over xGMI (ncclCommInitAll over the distinct
 * devices), where one kernel scatters them into the image.  Output is
 * bit-identical for every device count (the random stream is keyed by
 * global pixel and sample).  The renderer keeps each device's scene, work
 * schedule and buffers between calls: a call with the same scene content,
 * size and settings (any seed) re-uploads nothing.  A call drives every rank
 * from its own host thread (joined before it returns).  Not thread-safe
 * itself: one call at a time per renderer (nor is the Go renderer:
 * renderer.go:103-112). */
typedef struct rt_renderer rt_renderer;
int rt_renderer_create(const int32_t* devices, int32_t num_devices, rt_renderer** out);
/* Render with the renderer's devices (settings->num_devices is ignored). */
int rt_renderer_render(rt_renderer* r, const rt_scene* scene, int32_t width, int32_t height,
                       const rt_settings* settings, float* out_linear_rgb, uint8_t* out_rgba, rt_stats* stats);
void rt_renderer_destroy(rt_renderer* r);
/* Watchdog of a multi-rank Render (more than one rank): the frame gets one
 * deadline, `seconds` after Render starts (after the scene upload).  Every
 * host wait of the frame is bounded by it: each rank's waits inside its share
 * render (its previous render, the schedule build, a BVH scene's bounce loop),
 * the partition's measuring render, and the waits for the ranks' streams, the
 * RCCL gather into the first device (renderer.go:398-436 is the tile farm-out
 * it replaces) and the unpack.  Past it, Render stops waiting, aborts the
 * renderer's RCCL communicators and returns RT_E_TIMEOUT with the rank,
 * device, frame and partition in rt_last_error().  The renderer is then
 * unusable: later calls return RT_E_TIMEOUT, and rt_renderer_destroy releases
 * only what does not wait on the stalled work (exit the process to reclaim the
 * rest).  Default 0: no bound, as Go's Render (a large frame may take
 * minutes); callers opt in (the CLI: --watchdog SECONDS).  One-rank renders
 * have no collective and are never bounded. */
int rt_renderer_set_watchdog(rt_renderer* r, double seconds);
/* Test hook for the watchdog: the renderer's next multi-rank frame first
 * runs, on `rank`'s stream, one workgroup that sleeps for `ms` (0..60000)
 * milliseconds of device time and then exits -- a stall that always ends. */
int rt_renderer_test_stall(rt_renderer* r, int32_t rank, double ms);

/* ------------------------------------------- resident context (bench/MGPU) */

typedef struct rt_context rt_context;

int rt_context_create(int32_t device, rt_context** out);
void rt_context_destroy(rt_context* ctx);

/* Flatten (GetHittables, scene.go:59-90; createCube, scene.go:150-190) and
 * upload the scene to device memory.  Builds the BVH when the scene is
 * large (or when force_bvh > 0; force_bvh < 0 forbids it). */
int rt_context_set_scene(rt_context* ctx, const rt_scene* scene, int32_t force_bvh);

/* Work-partition tuning.  No setting changes a single output bit (the GPU
 * parity tests render with each and compare against the oracle): they only
 * choose how the same work is cut into blocks and ordered, and exist for the
 * tests that force every kind of work block and for experiments.  The
 * library never reads the environment. */
#define RT_PATH_AUTO 0        /* wavefront kernels for BVH scenes, else the megakernel */
#define RT_PATH_MEGAKERNEL 1  /* the megakernel also for BVH scenes */
typedef struct {
  int32_t path;           /* RT_PATH_* */
  int32_t pilot;          /* 1: block sizes from a one-sample pilot render; 0: geometric estimate */
  int32_t frustum;        /* 1: primary-ray candidate masks (cull, black tiles) */
  int32_t stage;          /* 1: small scenes staged into LDS */
  double block_work;      /* path bounces x samples per block; 0: default (one frame per launch: 384, 256 with
                             triangles; several frames per launch: 1024, 2048 with triangles; BVH scenes 8192) */
  int32_t block_samples;  /* pixels x samples of a large block at most; 0: 1024 */
  int32_t bvh_bins;       /* SAH bins per axis; 0: 32 */
  int32_t bvh_leaf;       /* spheres per BVH leaf at most (1..7); 0: 4 */
  int32_t wf_paths;       /* wavefront path slots (at most 2^24); 0: 2^24, fewer when the frame has fewer samples */
  int64_t wf_chunk;       /* wavefront samples per chunk; 0: 2^30 */
  int32_t wf_lds_nodes;   /* BVH nodes staged into LDS; -1: as many as fit */
  int32_t wf_trav_block;  /* threads per traversal workgroup (64..1024); 0: 1024 */
  int32_t wf_trav_wgs;    /* traversal workgroups sharing a CU's LDS; 0: 1 */
  int32_t pilot_depth;    /* bounces the pilot render follows a path at most (default 12); 0: max_depth */
  int32_t split_samples;  /* samples per sub-block of a split (heavy) pixel, 1..64; 0: 64 */
  int32_t measure;        /* 1: the first frame of a schedule measures every pixel's path lengths and the
                             next frame re-cuts the blocks from them; 0: pilot schedule only (default) */
  int32_t split_depth;    /* measured schedules split a pixel with a path of more bounces than this; 0: 16 */
  int32_t partition;      /* rt_renderer with N > 1 ranks: RT_PARTITION_*; 0: auto (balanced for linear-scan
                             scenes, strided for BVH scenes, whose frames have thousands of busy tiles) */
  int32_t wf_list_tries;  /* wavefront list test: rejection tries a listed cone's accepted-try mask covers
                             (1..64; 0: 64); later points continue the sequential loop (tests force it low) */
  /* tail helpers (megakernel, staged scenes): a block's last
   * few long paths are handed to extra one-wave workgroups at the end of the
   * launch that run each alone, at the latency of a lone bounce */
  int32_t tail_helpers;   /* helper workgroups per launch; 0: 64; -1: none, the paths stay in their blocks
                             (rt_tuning_default: -1; DESIGN.md §4.6 measures 64 as a net loss) */
  int32_t tail_paths;     /* a block exports once at most this many paths are left; 0: 4 */
  int32_t tail_depth;     /* ... each at least this many bounces deep; 0: 2 */
  int32_t tail_every;     /* ... checked every this many iterations of the block's drain (rounded up to a power of 2, at most 64); 0: 4 */
  int32_t tail_at;        /* the helpers follow this percentage of the launch's main workgroups (1..100); 0: 100 */
  int32_t _tail_pad;
} rt_tuning;
#define RT_PARTITION_AUTO 0
#define RT_PARTITION_STRIDED 1
#define RT_PARTITION_BALANCED 2
void rt_tuning_default(rt_tuning* t);
/* Applies to later rt_context_set_scene (BVH shape) and render calls. */
int rt_context_set_tuning(rt_context* ctx, const rt_tuning* t);
int rt_renderer_set_tuning(rt_renderer* r, const rt_tuning* t);

#define RT_LAYOUT_IMAGE 0        /* write pixels of this rank's tiles into a W*H image */
#define RT_LAYOUT_PACKED_TILES 1 /* write this rank's tiles packed: [local_tile][32*32] */

/* Number of 32x32 tiles of a W*H image (createRenderTasks, renderer.go:398-436). */
int32_t rt_num_tiles(int32_t width, int32_t height);
/* Tiles owned by `rank` of `world` under strided assignment t -> t % world. */
int32_t rt_tiles_for_rank(int32_t width, int32_t height, int32_t rank, int32_t world);

/* Enqueue a render of the tiles t with t % world == rank on `hip_stream`
 * (a hipStream_t, NULL = default stream).  d_linear (float3 per pixel) and
 * d_rgba (4 B per pixel, may be NULL) are DEVICE pointers sized for the
 * layout: W*H pixels (IMAGE) or rt_tiles_for_rank()*1024 pixels (PACKED).
 * Asynchronous: returns after the launches are queued.  If counts != NULL a
 * counting variant runs instead and the counts are returned (synchronous). */
int rt_context_render_async(rt_context* ctx, int32_t width, int32_t height, const rt_settings* settings,
                            int32_t rank, int32_t world, int32_t layout, float* d_linear, uint8_t* d_rgba,
                            void* hip_stream, rt_counts* counts);

/* Several frames of the same scene, size and settings that differ only in
 * their seed (seeds[f]), rendered by ONE launch: the reference's Render
 * called nframes times (renderer.go:67-126), each frame bit-identical to its
 * own rt_context_render_async.  The frames share the work schedule; the
 * launch's workgroups interleave them (every frame's heaviest blocks first),
 * so the low-occupancy tail of long paths is paid once per launch instead of
 * once per frame.  d_linear[f] / d_rgba[f] (d_rgba may
 * be NULL, entries may be NULL) are laid out as in rt_context_render_async.
 * BVH scenes, sample passes and measuring frames render frame by frame. */
#define RT_MAX_FRAMES 32
int rt_context_render_frames_async(rt_context* ctx, int32_t width, int32_t height, const rt_settings* settings,
                                   int32_t nframes, const uint64_t* seeds, int32_t rank, int32_t world,
                                   int32_t layout, float* const* d_linear, uint8_t* const* d_rgba, void* hip_stream);

/* What a context has done so far (diagnostics): work schedules built (a new
 * scene, frame, rank or settings key; a measured re-cut counts too),
 * measuring frames (rt_tuning.measure), frames rendered, render launches,
 * and the launches that rendered several frames at once. */
typedef struct {
  int64_t schedules_built, measuring_frames, frames, launches, batched_launches;
  int64_t blocks, split_pixels;  /* of the schedule last used: work blocks, pixels split over sub-blocks */
  /* tail helpers (rt_tuning.tail_*): paths exported to them since the
   * context's tail buffers were laid out, and a helper error word (0: none);
   * reading them waits for the context's last render */
  int64_t tail_exported, tail_errors;
} rt_context_stats;
int rt_context_get_stats(const rt_context* ctx, rt_context_stats* out);
/* Debug (tail helpers), cumulative since the context's tail
 * buffers were laid out: out[0] paths exported, [1] paths the helpers ran,
 * [2] helpers' ticks running paths, [3] exporting waves' ticks in the export,
 * [4] helpers' lifetime ticks, [5] error word (ticks: s_memrealtime, 100 MHz).
 * Waits for the context's last render; all zero when no launch used helpers. */
int rt_context_tail_debug(const rt_context* ctx, uint64_t out[6]);

/* Packed share of one rank, as rt_comm_gather_tiles_async moves it:
 * [max_local_tiles * 1024 float3][max_local_tiles * 1024 RGBA8] = 16 B per
 * pixel of the largest share (rank 0's).  Render a share with layout
 * RT_LAYOUT_PACKED_TILES, d_linear = share, d_rgba = share + rt_packed_rgba_offset(). */
int32_t rt_max_local_tiles(int32_t width, int32_t height, int32_t world);
size_t rt_packed_bytes(int32_t width, int32_t height, int32_t world);
size_t rt_packed_rgba_offset(int32_t width, int32_t height, int32_t world);

/* Scatter the gathered shares [world][rt_packed_bytes] into W*H images
 * (d_linear float3 and/or d_rgba; either may be NULL). */
int rt_unpack_tiles_async(int32_t width, int32_t height, int32_t world, const void* d_gathered, float* d_linear,
                          uint8_t* d_rgba, void* hip_stream);

/* ---------------------------------------------- RCCL tile gather (xGMI) */

/* One communicator per process for multi-process runs (one process per GPU,
 * e.g. torch.distributed.run): rank 0 makes the id (ncclGetUniqueId), the
 * caller broadcasts its RT_COMM_ID_BYTES bytes, every rank calls
 * rt_comm_create (ncclCommInitRank) on its device. */
#define RT_COMM_ID_BYTES 128
typedef struct rt_comm rt_comm;
int rt_comm_unique_id(uint8_t* id);
int rt_comm_create(const uint8_t* id, int32_t world, int32_t rank, int32_t device, rt_comm** out);
void rt_comm_destroy(rt_comm* comm);
/* The frame's one collective: rank r > 0 sends its packed share
 * (rt_packed_bytes, device pointer d_share) to rank 0, which receives it
 * into d_gathered + r * rt_packed_bytes (one ncclSend/ncclRecv group on
 * `hip_stream`).  Rank 0 renders its own share into d_gathered directly
 * (d_share == d_gathered: nothing to copy). */
int rt_comm_gather_tiles_async(rt_comm* comm, int32_t width, int32_t height, const void* d_share, void* d_gathered,
                               void* hip_stream);

/* ------------------------------------------------ tile partitions (N ranks) */

/* createRenderTasks hands 32x32 tiles to the goroutines through one channel
 * (renderer.go:398-436), so a slow tile never holds the others up.  Ranks on
 * separate GPUs share no queue: each renders a fixed set of tiles.  The
 * default set is strided (t % world == rank).  A frame whose work sits in a
 * few tiles (the headline scene: 23 of its 475 tiles hold all the shading)
 * is better dealt by work: rt_partition_balanced renders the whole frame
 * once on ctx's device with every sample's path length recorded (DESIGN.md
 * §5; frames with more than 1024 samples, a sky or a BVH: the schedule's
 * one-sample pilot estimate instead), sums each tile's path work and deals
 * the tiles heaviest first to the least loaded rank.  Both are
 * deterministic, so every rank that plans the same frame derives the same
 * partition.  Every
 * pixel stays on one rank and the random stream is keyed by global pixel and
 * sample: the image is the same for every partition.
 * A rank's packed share holds its tiles in ascending order (local tile lt =
 * the lt-th of its tiles); every share is sized for the largest. */
typedef struct rt_partition rt_partition;
/* owner[t] = rank of tile t (rt_num_tiles entries, each in [0, world)); NULL: strided. */
int rt_partition_create(int32_t width, int32_t height, int32_t world, const int32_t* owner, rt_partition** out);
/* ctx must hold the scene (rt_context_set_scene); synchronous. */
int rt_partition_balanced(rt_context* ctx, int32_t width, int32_t height, const rt_settings* settings, int32_t world,
                          rt_partition** out);
void rt_partition_destroy(rt_partition* p);
int32_t rt_partition_world(const rt_partition* p);
int32_t rt_partition_owner(const rt_partition* p, int32_t tile);      /* -1: no such tile */
int32_t rt_partition_local_tiles(const rt_partition* p, int32_t rank); /* tiles of `rank` */
int32_t rt_partition_tile(const rt_partition* p, int32_t rank, int32_t local); /* its local-th tile, -1: none */
int32_t rt_partition_max_local(const rt_partition* p);
size_t rt_partition_packed_bytes(const rt_partition* p);  /* one share: max_local * 1024 * 16 */
size_t rt_partition_rgba_offset(const rt_partition* p);   /* max_local * 1024 * 12 */
/* Work of rank's tiles (path bounces summed over samples; balanced partitions, else 0). */
double rt_partition_work(const rt_partition* p, int32_t rank);
/* Later renders of ctx with the partition's (W, H, world) render rank's tiles
 * of it (packed: in its order); NULL (or other sizes): strided.  The
 * partition is copied: it may be destroyed afterwards. */
int rt_context_set_partition(rt_context* ctx, const rt_partition* p);
/* rt_unpack_tiles_async for a partition's shares ([world][rt_partition_packed_bytes]). */
int rt_unpack_partition_async(const rt_partition* p, const void* d_gathered, float* d_linear, uint8_t* d_rgba,
                              void* hip_stream);
/* The same for nframes frames gathered as [world][nframes][packed bytes] (each
 * rank's frames contiguous: one send per rank) into [nframes][W*H] images. */
int rt_unpack_partition_frames_async(const rt_partition* p, int32_t nframes, const void* d_gathered, float* d_linear,
                                     uint8_t* d_rgba, void* hip_stream);
/* rt_comm_gather_tiles_async with shares of share_bytes (a partition's packed bytes). */
int rt_comm_gather_bytes_async(rt_comm* comm, size_t share_bytes, const void* d_share, void* d_gathered,
                               void* hip_stream);
/* Per rank of the renderer's last render: device seconds of its render launches
 * (out[capacity], capacity >= rt_renderer_num_ranks(r), else RT_E_INVALID) --
 * the load balance of a multi-GPU frame. */
int rt_renderer_rank_seconds(const rt_renderer* r, double* out, int32_t capacity);
/* The renderer's rank count (the device list given to rt_renderer_create). */
int32_t rt_renderer_num_ranks(const rt_renderer* r);

/* Debug hook: a device buffer of 48 u64 per workgroup that
 * RT_WG_TIMING builds of the kernel fill: s_memrealtime at start / loop end
 * / end, then s_memtime clocks spent in closest hit, lighting and soft
 * shadows, coop/sequential soft-shadow counts and loop iterations
 * (scripts/wg_timing.py).  Product builds ignore it. */
int rt_context_set_debug_buffer(rt_context* ctx, void* d_buf);

/* Per-kernel device time of the wavefront path (BVH scenes):
 * with profiling on, HIP events are recorded at every kernel boundary of the
 * bounce loop on the render's stream; rt_context_kernel_seconds waits for
 * them and returns each kernel class's total seconds and launches since
 * profiling was switched on, in the order of RT_WF_*.  (The megakernel path
 * records nothing here: rt_context_last_kernel_seconds is its one launch.) */
#define RT_WF_EXTEND 0       /* closest hit of the live paths (hitWorld, renderer.go:333-346) */
#define RT_WF_SHADE1 1       /* hit records + hard shadow rays queued */
#define RT_WF_OCCLUDE_HARD 2 /* any-hit of the hard shadow rays (renderer.go:305) */
#define RT_WF_CONE 3         /* shadow cones of the clear hard rays: candidate lists (renderer.go:311-320) */
#define RT_WF_SOFTGEN 4      /* the 16 jittered points per clear light (renderer.go:311-318) */
#define RT_WF_CONE_RAYS 5    /* the soft rays of cones with a candidate list, against the list */
#define RT_WF_OCCLUDE_SOFT 6 /* any-hit of the other soft shadow rays through the BVH (renderer.go:320) */
#define RT_WF_SHADE 7        /* direct lighting + scatter (renderer.go:181-297) */
#define RT_WF_REGEN 8        /* new camera samples + loop bookkeeping */
#define RT_WF_RESOLVE 9      /* per-pixel in-order sums, tone map, write */
#define RT_WF_KERNELS 10
int rt_context_profile(rt_context* ctx, int32_t on);  /* on / off; resets the totals */
int rt_context_kernel_seconds(rt_context* ctx, double* seconds /* RT_WF_KERNELS */,
                              int64_t* launches /* RT_WF_KERNELS or NULL */);

/* Device time (seconds) of the last render launch enqueued on this context
 * (HIP events recorded around it on its stream); waits for it. */
int rt_context_last_kernel_seconds(rt_context* ctx, double* seconds);

/* ------------------------------------------------------------ output */

/* toneMap + ToRGB on host (renderer.go:348-367; vector.go:106-109). */
void rt_tonemap_rgba(const float* linear_rgb, int32_t npix, uint8_t* out_rgba);
/* SaveImage — renderer.go:438-451 (PNG, opaque 8-bit RGB like Go's encoder). */
int rt_write_png(const char* path, const uint8_t* rgba, int32_t width, int32_t height);
/* SavePPMFromVec3-style P3 writer (internal/output/ppm.go:34-59), from RGBA8. */
int rt_write_ppm(const char* path, const uint8_t* rgba, int32_t width, int32_t height);

#ifdef __cplusplus
}
#endif
#endif /* RT_API_H */
