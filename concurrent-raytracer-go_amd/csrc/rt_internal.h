// rt_internal.h — host-side interfaces between the C ABI (rt_api.cpp), the
// kernels (rt_kernel.hip), the scene loader (scene_json.cpp), the BVH
// builder (bvh.cpp) and the output writers (image_io.cpp).
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/rt_api.h"
#include "rt_scene_dev.h"

namespace rtgo {

void set_error(const std::string& msg);

// Device memory through a per-device cache of freed blocks (dev_pool.cpp):
// hipMalloc / hipFree semantics (hipError_t as int), the block must no longer
// be in use by any stream when it is freed.
int dev_alloc(void** p, size_t n);
void dev_free(void* p);
// pinned host staging buffers, cached per process (dev_pool.cpp)
int host_alloc(void** p, size_t n, bool* fresh = nullptr);  // fresh: newly pinned (not from the cache)
void host_free(void* p);
// non-blocking streams and timing events, reused the same way (current device)
int dev_stream_get(hipStream_t* s);
void dev_stream_put(hipStream_t s);
int dev_event_get(hipEvent_t* e);
void dev_event_put(hipEvent_t e);

// ---------------------------------------------------------------- scene
struct FlatScene {
  std::vector<DSphere> spheres;
  std::vector<DTri> tris;
  std::vector<DBox> boxes;    // one per cube, over its 12 triangles
  std::vector<DMat> mats;
  std::vector<DLight> lights;
  std::vector<DBVHNode> bvh;  // empty => linear scan
  int32_t bvh_depth = 0;      // levels of the BVH (root = 1): the traversal stack holds fewer entries
  std::vector<DQNode> qbvh;   // the BVH with quantized bounds (same node order)
  // the same tree collapsed to groups of 2..4 nodes (bvh.cpp): DQNode slots,
  // groups back to back, breadth-first; the root group's code
  std::vector<DQNode> qbvh4;
  int32_t bvh4_stack = 0;     // the most pending children a 4-wide traversal holds
  int32_t bvh4_root = 0;
  double q0[3] = {0, 0, 0}, qd[3] = {1, 1, 1};  // its grid: coordinate = q0 + q * qd
  double cam_pos[3] = {0, 0, 0};
  double aspect = 0;
  int32_t objects = 0;        // len(hittables)
};

// The AtmosphereConfig presets of RT_SKY_DEFAULT .. RT_SKY_NIGHT
// (internal/atmosphere/atmosphere.go:28-98), index sky - 1.
constexpr int kSkies = 4;
void sky_presets(DSky out[kSkies]);

// GetHittables + createCube + material constructors (scene.go:59-190).
void flatten_scene(const rt_scene& s, FlatScene* out);
// Binned-SAH BVH over out->spheres (reorders spheres). Requires no triangles.
// bins / leaf: SAH bins per axis and spheres per leaf at most (0: defaults).
void build_sphere_bvh(FlatScene* fs, int bins, int leaf);
// The global tiles a rank renders, in local-tile order (local tile lt is
// tiles[lt]): t % world == rank (strided, createRenderTasks order dealt
// round-robin) or a partition's list (rt_partition, rt_multi.cpp).
void strided_tiles(int32_t W, int32_t H, int32_t rank, int32_t world, std::vector<int32_t>* tiles);
// Per local tile: primitives whose projected bounds overlap it (the work
// estimate of a schedule without a pilot render).
void tile_cost(const FlatScene& fs, int32_t W, int32_t H, const std::vector<int32_t>& tiles,
               std::vector<float>* local_cost);
constexpr int32_t kBlockBlack = 1;  // block flag (8th int): black tile, nothing to trace
constexpr int kBlockInts = 16;      // ints per work block record (KParams::blocks)
// Primary-ray candidate masks per local tile (2 x u64: spheres, triangles;
// scenes with <= 64 of each): bit i set unless primitive i's bounding sphere
// provably misses the cone of the tile's camera rays.
void tile_primary_masks(const FlatScene& fs, int32_t W, int32_t H, const std::vector<int32_t>& tiles,
                        std::vector<unsigned long long>* masks);

// The GPU work scheduler (rt_schedule.hip).
struct SchedParams {
  const DSphere* spheres;
  const DTri* tris;
  double cam[3];
  double vw;                   // viewport width 2 * aspect (getRay, renderer.go:377-390)
  int32_t W, H, rank, world, tiles_x, ntiles, local;
  int32_t spp, big_pixels, frustum;
  int32_t split_samples;       // samples per sub-block of a split pixel (<= 64: one path per lane)
  double block_work;
  const unsigned long long* tile_masks;  // per local tile (2 u64) or null (no primary culling)
  const float* tile_cost;      // per local tile: projected primitives (estimate without a pilot)
  const int32_t* tile_list;    // per local tile: its global tile (a partition), or null: rank + lt * world
  const unsigned int* work_max;  // measured per local pixel: the longest path (bounces + 1) ...
  const unsigned int* work_sum;  // ... and the sum over the measured samples, or null (no measurement)
  int32_t work_n;              // samples measured per pixel (1..16: a pilot; spp: a whole frame)
  int32_t work_mean;           // 1: work_n < spp samples of every pixel measured: use their mean (partitions)
  int32_t split_depth;         // a pixel whose longest path has this many bounces is split (measured frames)
  // scratch (sched_layout)
  unsigned long long* pixmask; // per local pixel: 2 u64
  float* est;                  // per local pixel: estimated work of one sample
  int32_t* pilot_blocks;       // 16 records per local tile: the pilot's 64-pixel blocks
  int32_t* hist;               // per weight class: blocks (pass 1)
  int32_t* cursor;             // per weight class: next record (pass 2)
  int32_t* totals;             // [0] blocks, [1] split pixels, [2] split-slot cursor
  int32_t* blocks;             // the records, heaviest class first (pass 2)
};
size_t sched_scratch_bytes(int local);
void sched_layout(void* scratch, int local, SchedParams* p);
// masks + pilot blocks (zeroes the class counters first)
int sched_launch_pixels(const SchedParams& p, void* stream);
// write = false: estimates, pass 1 (class counts, split count), scan;
// write = true: pass 2 (the records)
int sched_launch_blocks(const SchedParams& p, bool write, void* stream);

// ---------------------------------------------------------------- kernels
// PCG jump-ahead entries: cooperative soft shadows evaluate up to 64
// rejection tries (3 draws each) per round and then advance by 3*used
// draws; entry h holds (A_3h, C_3h), h = 0..64 (draws 3h+1, 3h+2 are plain
// steps from 3h).
constexpr int kJump = 64 + 1;
// Largest block (pixels x spp) a workgroup renders (its hit list and
// radiance slots live in LDS: 24 KB); the host picks P = floor(1024 / spp)
// pixels per block (at most 64), so spp <= 1024.
constexpr int kMaxBlockSamples = 1024;
constexpr int kMaxFrames = RT_MAX_FRAMES;  // frames per launch at most (rt_context_render_frames_async)
constexpr int kDbgStride = 48;  // RT_WG_TIMING: 64-bit words per workgroup in the debug buffer
// Counters of the counting variants: the nine of rt_counts, then the same
// nine for the work the counting variant walks only to report the
// reference's counts (camera samples of culled pixels, rt_counts.culled),
// then the soft-shadow traversal kernel's share (rt_counts.soft_occlusion).
constexpr int kCounters = 9;
constexpr int kCountSlots = 5 * kCounters;
// count groups after the totals (rt_counts): culled, then the wavefront
// kernels' own shares -- soft-shadow stage, closest hit, hard occlusion
constexpr int kGroupSoft = 2, kGroupExtend = 3, kGroupHard = 4;
// Deepest BVH the kernels accept (per-lane LDS stack entries; bvh.cpp keeps
// the linear scan for deeper trees).  The stacks are allocated per launch for
// the scene's actual depth (10k spheres: 15 levels).
constexpr int kStack = 40;

// ---- tail helpers: a launch's long paths handed to idle waves
// When a block's wave has started every entry of its hit list and only a
// few paths are left (at most tail_kmax, each at least tail_dmin bounces
// deep), it EXPORTS them: each path's state goes to a queue, and one of
// tail_helpers extra one-wave workgroups at the end of the grid runs it to
// its end with the whole wave (solo_path: ~5 us per bounce against ~9-17
// us for a few paths sharing a wave).  Its radiance goes to a per-sample row
// of its pixel (the block's own pixels: a dynamic row; split pixels: the
// split row), and the last contributor of a pixel -- the block or a helper --
// sums the row in sample order and writes the pixel, so the image is the
// same bit for bit.  Main blocks never wait for a helper; helpers leave when
// every main block is done and the queue is empty, so the launch always
// drains.
constexpr int kTailShards = 64;
// Every word that many waves touch sits on a 128-B line of its own
// (`unsigned int x[32]`, word 0 used): polling helpers and draining blocks
// on one shared line made each of their accesses wait on the others
// (measured: a draining block's iteration 2.4x slower, an export 45 us).
struct TailCtl {
  unsigned int tail[32];          // queue entries reserved (exporters add; helpers read)
  unsigned int head[32];          // queue entries taken by helpers (CAS)
  // the export gate, one 64-bit word: helpers started and not yet gone (high
  // half) | exported paths not yet finished (low half); an exporter reads it
  // (one load), then reserves with one add whose returned value decides
  unsigned long long gate[16];
  unsigned int rows_used[32];     // dynamic rows allocated
  unsigned int helpers_gone[32];  // helpers finished (the last one zeroes the block for the next launch)
  // statistics since the layout (ticks: s_memrealtime, 100 MHz): paths
  // exported, helpers' time running paths, exporting waves' time in the
  // export, helper lifetimes, paths run; the error word (never expected)
  unsigned int exported, solo_ticks, export_ticks, helper_ticks, paths_done, err, pad[26];
  // main workgroups finished, sharded (block b adds to shard b % kTailShards,
  // 128 B apart): one counter took every block's add and serialized them
  unsigned int done[kTailShards * 32];
};
// one exported path (its state after `depth` bounces, renderer.go:165-227)
struct TailPath {
  double o[3], d[3], T[3], L[3];
  uint64_t rng, skey;
  int32_t depth, sample;   // bounces so far; its sample within the destination row
  int32_t kind, row;       // kTailRow: dynamic row `row`; kTailSplit: split slot index `row`
  int32_t nsub, frame;     // split pixel: its sub-blocks; the frame of the launch
  int64_t oi;              // output pixel index (layout-resolved, as the epilogue writes it)
};
// the header of a dynamic row: its pixel's running sum over the samples
// before k0 (summed by the block), and who still owes a sample
struct TailRow {
  double prefix[3];
  int32_t counter;         // contributors still to finish: the block (1) + its exported paths
  int32_t k0;              // first sample held by the row
  int32_t frame, _pad;
  int64_t oi;
};
constexpr int kTailRow = 1, kTailSplit = 2;

struct KParams {
  const DSphere* spheres;
  const DTri* tris;
  const DBox* boxes;
  const DMat* mats;
  const DLight* lights;
  const DBVHNode* bvh;
  const uint64_t* jump;        // PCG jump table: (A_3h, C_3h) for h = 0..kJump-1 (rt_rng.h)
  float* out_linear;
  uint8_t* out_rgba;
  unsigned long long* counts;  // kCounters counters (rt_counts order, then the culled ones) or null
  unsigned long long* dbg;     // per-WG timing records (RT_WG_TIMING builds only) or null
  const int32_t* blocks;       // per block, kBlockInts ints: {local tile, first pixel, pixel count, first sample,
                               //   samples, split slot (-1: none), sub-blocks of the split pixel, flags,
                               //   primary masks (spheres u64, tris u64), live pixels u64, 0, 0}
  double* split_rad;           // split pixels: [slot][spp][3] radiance of the hit samples
  uint32_t* split_hits;        // split pixels: [slot][(spp+31)/32] hit-sample bits (zeroed per launch)
  int32_t* split_cnt;          // split pixels: sub-blocks finished (zeroed per launch)
  unsigned int* work_max;      // measuring renders: per local pixel, its longest path (bounces + 1) ...
  unsigned int* work_sum;      // ... and the bounces + 1 of all its samples' paths (else null)
  const unsigned long long* tile_masks;  // per local tile: primary-ray candidate masks (spheres, tris) or null
  const DSky* sky;             // miss radiance (rt_settings.sky) or null: black (renderer.go:170-173)
  const void* stage_src;       // start of the scene prefix staged into LDS (spheres..lights)
  int32_t stage_bytes;         // bytes to stage (multiple of 16); 0 = read the scene from global memory
  int32_t stack_off;           // byte offset of the BVH stacks in dynamic LDS
  int32_t stack_depth;         // entries per lane of a BVH stack (the tree's depth)
  double cam[3];
  double aspect;
  uint64_t seed_key;
  int32_t ns, nt, nl, use_bvh, nb;
  int32_t W, H;
  int32_t spp, max_depth;
  int32_t recursive, soft;
  int32_t rank, world;
  int32_t tiles_x, ntiles;
  int32_t num_blocks;        // this rank's blocks (one workgroup each)
  int32_t layout;     // RT_LAYOUT_*
  int32_t num_wgs;         // = num_blocks * nframes
  // sample passes (more samples per pixel than a block holds, DESIGN.md
  // §4.1): this launch renders samples [sample_base, sample_base + spp) of
  // spp_total; acc holds each local pixel's running sum (lt * 1024 + pixel,
  // 3 doubles) between passes.  acc_mode: bit 0 = start from acc (not the
  // first pass), bit 1 = store the sum to acc instead of writing the image
  // (not the last pass).  Single pass: acc_mode 0, spp_total = spp.
  double* acc;
  int32_t sample_base, spp_total, acc_mode;
  // FRAMES of one launch (rt_context_render_frames_async): the same schedule
  // rendered nframes times, each frame with its own seed and outputs.
  // Workgroup g renders block g / nframes of frame g % nframes, so every
  // frame's heaviest blocks start first and one launch's tail covers all
  // its frames.  launch_render fills entry 0 from seed_key / out_linear /
  // out_rgba when nframes <= 1.  Split pixels: a copy of the split rows and
  // flags per frame, nsplit slots each (split_frames copies in memory).
  int32_t nframes, nsplit, split_frames, _fpad;
  uint64_t frame_key[kMaxFrames];
  float* frame_lin[kMaxFrames];
  uint8_t* frame_rgba[kMaxFrames];
  // tail helpers (null tail: off): the control block, the queue and its
  // ready flags (== tail_epoch when written), the dynamic rows ([row][spp][3]
  // radiance, [row][(spp+31)/32] hit bits, headers); tail_cap entries and rows
  TailCtl* tail;
  TailPath* tail_q;
  unsigned int* tail_ready;
  double* tail_rows;
  uint32_t* tail_bits;
  TailRow* tail_hdr;
  int32_t tail_cap, tail_helpers, tail_kmax, tail_dmin;
  uint32_t tail_epoch;
  int32_t tail_every_mask;  // the drain's iterations between export checks - 1 (a power of 2 - 1)
  int32_t tail_pos, _tpad2; // the helpers are workgroups [tail_pos, tail_pos + tail_helpers) of the grid
};

// Enqueue the render kernel; returns hipError_t as int.
int launch_render(const KParams& p, bool count, void* stream);
size_t render_shmem(const KParams& p);
// device -> mapped pinned host memory by a kernel (16-byte aligned, a multiple of 16 bytes)
int launch_download(const void* d_src, void* h_dst_mapped, size_t bytes, void* stream);
// one workgroup that sleeps for `ms` of device time, then exits (the
// renderer watchdog's test hook, rt_multi.cpp test_stall)
int launch_spin(double ms, void* stream);
// rt_partition_balanced measuring only the first measure_spp samples of every
// pixel (rt_api.cpp measured_tile_work; the renderer's partitions: 16)
int partition_balanced(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t world, int measure_spp,
                       rt_partition** out);
constexpr int kRendererPartitionSpp = 16;
int launch_unpack(int32_t W, int32_t H, int32_t world, const void* gathered, size_t share_bytes, size_t rgba_off,
                  float* ol, uint8_t* orgba, void* stream);
// The same for a partition: slot[t] = {owner rank, local tile} of global tile t;
// nframes frames gathered as [world][nframes][share] into [nframes][W*H] images.
int launch_unpack_map(int32_t W, int32_t H, int32_t nframes, const int32_t* slot, const void* gathered,
                      size_t share_bytes, size_t rgba_off, float* ol, uint8_t* orgba, void* stream);
// Per global tile of a frame, the sum of its pixels' estimated work (rt_schedule.hip
// sched_est of a whole-frame pilot): the input of a balanced partition.
int sched_launch_tile_work(const SchedParams& p, float* tile_work, void* stream);

// The geometry an occlusion / closest-hit query needs (device pointers).
struct Geo {
  const DSphere* spheres;
  const DTri* tris;
  const DBox* boxes;  // one per cube: its 12 consecutive triangles
  const DBVHNode* bvh;
  int32_t ns, nt, use_bvh, nb;
};

// ---------------------------------------------------------------- wavefront path
// (rt_wavefront.hip: BVH scenes)
constexpr int kWfShards = 8;           // queues / path arrays are split in 8 shards (one atomic word each)
constexpr int kWfBlockSlots = 256;     // threads per workgroup of the wavefront kernels
constexpr int kWfTravBlock = 1024;     // ... of the traversal kernels (extend, occlude): one per CU, BVH in LDS
constexpr uint32_t kDeadSid = 0xFFFFFFFFu;  // a slot with no sample (out-of-image pixel of an edge tile)
// soft shadows: candidate spheres kept per shadow cone (more: its rays are
// traced).  Host allocation and kernels must agree: a constant, not a build
// knob (C4: 16 -> 412.6 ms per frame, 24 -> 416.0, 32 -> 421.1; with the
// list tests ordered by length: 16 -> 403.4, 32 -> 405.7)
constexpr int kWfConeK = 16;
// (r05) a cone with kWfConeK < candidates <= kWfConeWide is "wide": its 16 rays
// are tested against its list, one ray per lane (wf_widetest), instead of
// being traced; the candidate lists hold kWfConeWide entries per (path, light)
#ifndef RT_CONE_WIDE
#define RT_CONE_WIDE 32
#endif
constexpr int kWfConeWide = RT_CONE_WIDE;
struct WfCtl {                 // device-resident loop state; counters of shard s at [32 s] (own 128-B line)
  int32_t cur_cnt[kWfShards * 32];   // live paths per shard of the current array
  int32_t next_cnt[kWfShards * 32];  // survivors appended per shard of the next array
  int32_t hard_cnt[kWfShards * 32];  // hard shadow rays queued per shard
  int32_t soft_cnt[kWfShards * 32];  // soft shadow rays queued per shard
  int32_t cone_cnt[kWfShards * 32];  // shadow cones queued per shard
  int32_t list_cnt[kWfShards * 32];  // entries of listed cones per shard (two each, from the far end of the soft queue)
  int32_t wide_cnt[kWfShards * 32];  // entries of wide cones per shard (two each, in the wide queue)
  int32_t job_head[4][kWfShards * 32];  // persistent kernels (extend, hard, soft, cone): jobs taken per range
  unsigned long long next_sample;    // first sample id of the chunk not started yet
  unsigned long long total;          // sample ids in the chunk
  int32_t live;                // live paths after the last bounce (wf_book)
  int32_t dry;                 // every sample started
  int32_t iter;                // bounces done
  int32_t pad;
};
struct WfPaths {             // structure of arrays, kWfShards * shard_cap slots
  double *ox, *oy, *oz, *dx, *dy, *dz;  // ray
  double *tx, *ty, *tz, *lx, *ly, *lz;  // throughput, radiance so far
  uint64_t* rng;             // stream state
  uint32_t* sid;             // sample id within the chunk (local pixel * spp + sample), kDeadSid: none
  int32_t* depth;
};
struct WfParams {
  Geo g;
  const DQNode* qbvh;        // quantized BVH (FlatScene::qbvh) and its grid
  double q0[3], qd[3];
  const DMat* mats;
  const DLight* lights;
  const DSky* sky;           // miss radiance or null (black)
  int32_t nl, max_depth, recursive, soft, spp;
  int32_t W, H, rank, world, tiles_x, ntiles, layout;
  const int32_t* tile_list;  // per local tile: its global tile (a partition), or null: rank + lt * world
  int32_t stack_depth;       // BVH stack entries per lane (the tree's depth - 1)
  int32_t lds_nodes;         // leading quantized nodes (breadth-first: the top levels) staged in LDS
  int32_t bvh_nodes;         // quantized nodes in all
  const DQNode* qbvh4;       // the 4-wide form (FlatScene::qbvh4): wf_occlude4 walks it when use4
  int32_t nodes4, stack4, use4;  // its slots, stack entries per lane; 1: staged whole in LDS and used
  int32_t root4;             // the root group's code
  int32_t trav_block;        // threads per workgroup of the traversal kernels (<= kWfTravBlock)
  int32_t shard_cap;         // path slots per shard
  int32_t live_bound;        // the host's bound on this bounce's live paths (launch sizes only)
  int32_t dry;               // 1: every sample of the chunk has started (no regen work left)
  int64_t hard_cap, soft_cap;  // queue entries per shard
  uint32_t lp0;              // first local pixel of the chunk (local tile * 1024 + pixel in tile)
  double cam[3];
  double aspect;
  uint64_t seed_key;
  WfPaths cur, next;
  WfCtl* ctl;
  int32_t* hidx;             // per slot of the current array: sphere hit (-1: none)
  double *px, *py, *pz;      // hit point
  uint32_t* lstate;          // [slot][light]: kHardBit | blocked soft rays
  uint32_t* hardq;           // kWfShards queues of hard_cap entries: slot * nl + light
  uint32_t* softq;           // kWfShards queues of soft_cap entries, 4 words: {slot * nl + light, draws x, y, z}
                             // (listed cones, from the far end: 2 entries, wf_softgen)
  const uint64_t* jump;      // PCG jump table (KParams::jump)
  int32_t list_tries;        // tries a listed cone's accepted-try mask covers (1..64, rt_tuning.wf_list_tries)
  uint32_t* coneq;           // kWfShards queues of hard_cap entries: slot * nl + light (clear hard ray)
  int32_t* cand;             // [slot * nl + light][kWfConeWide]: the shadow cone's candidate spheres, -1 ends
  uint32_t* wideq;           // kWfShards queues of wide_cap 4-word entries: two per wide cone (as the listed cones')
  int64_t wide_cap;
  double* rad;               // [sample id][3] radiance
  unsigned long long* counts;
  float* out_linear;
  uint8_t* out_rgba;
};
// Kernel classes of one bounce (rt_context_profile): prof, when not null,
// holds kWfProfEvents hipEvent_t recorded at their boundaries (event k opens
// class k, event k + 1 closes it; a skipped kernel takes no time).
enum { kWfExtend = 0, kWfShade1, kWfHard, kWfCone, kWfSoftgen, kWfList, kWfSoft, kWfShade, kWfRegen, kWfResolve, kWfClasses };
constexpr int kWfProfEvents = kWfClasses + 1;  // (one block serves any class range)
int wf_launch_bounce(const WfParams& p, bool first, bool count, void* stream, const void* prof);
// Quantized nodes the traversal kernels can stage in LDS next to their stacks
// (all of them when they fit; else an odd count, so no child pair is split).
// Load each kernel file's code object onto the current device (HIP loads
// them lazily, at a file's first launch otherwise): rt_context_create.
int preload_render_kernels();
// An empty launch and a 4-KB copy each way on the stream (dev4k: 4 KB of
// device memory): the runtime's first-launch and first-copy set-up.
int warm_device(void* stream, void* dev_buf, void* host_pinned, void* host_pageable, size_t bytes);
int preload_sched_kernels();
int preload_wf_kernels();
// RT_CHECK_XLANE builds: inactive-lane __shfl reads per file (-1: not such a build)
long long xlane_faults_kernel(bool reset);
long long xlane_faults_wavefront(bool reset);
int wf_lds_nodes(int stack_depth, int nodes, int block, int wgs_per_cu);
int wf_launch_resolve(const WfParams& p, int npix, void* stream);

// ---------------------------------------------------------------- partitions
// A tile -> rank assignment (rt_partition, include/rt_api.h): every rank's
// tiles ascending, each tile with its owner and its index in the owner's list
// (its local tile: the slot range [local * 1024, local * 1024 + 1024) of the
// owner's packed share).
struct PartitionData {
  int32_t w = 0, h = 0, world = 1;
  std::vector<int32_t> owner;    // per global tile
  std::vector<int32_t> local;    // per global tile
  std::vector<int32_t> offsets;  // world + 1: rank r's tiles are lists[offsets[r], offsets[r + 1])
  std::vector<int32_t> lists;
  std::vector<double> work;      // per rank: the estimated work of its tiles (balanced partitions), else empty
  int32_t max_local = 0;
  uint64_t id = 0;               // unique per partition object (part of a context's schedule key)
};
// Fills local / offsets / lists / max_local / id from w, h, world, owner.
void finish_partition(PartitionData* d);
// owner and work of a balanced partition of tiles with estimated `work` over
// d->world ranks (longest processing time first), then finish_partition.
void lpt_partition(const std::vector<float>& work, PartitionData* d);
rt_partition* make_partition(PartitionData&& d);
bool context_has_bvh(const rt_context* c);
double context_bvh_seconds(const rt_context* c);
void* context_stream(const rt_context* c);  // its own non-blocking stream (hipStream_t)
// A multi-rank renderer's frame deadline on a context (steady_now_s() clock,
// <= 0: none): the context's host waits during a render (the previous render
// before buffers are reused, the schedule's count read-back, the wavefront
// loop's per-bounce state) poll until it and return RT_E_TIMEOUT after it.
void context_set_deadline(rt_context* c, double deadline);
double steady_now_s();
const PartitionData& partition_data(const rt_partition* p);

// ---------------------------------------------------------------- output
double go_pow_tonemap(double x);  // Pow(x, 1/2.2) with Go's special cases
void tonemap_to_rgba(const double c[3], uint8_t out[4]);

}  // namespace rtgo
