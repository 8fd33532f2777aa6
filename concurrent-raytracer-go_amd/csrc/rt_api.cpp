// rt_api.cpp — C ABI of librtgo.so (include/rt_api.h): scene flattening,
// device residency, launches, blocking render.
//
// Replaces the Go seam *renderer.ParallelRenderer (renderer.go:54-126,
// settings.go:3-25).  Compiled with -ffp-contract=off: the host-side
// precomputations (cube vertices, triangle edges and normals, material
// tables) must equal the values the reference computes per test.
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_rng.h"
#include "rt_internal.h"

namespace rtgo {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      set_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));             \
      return RT_E_DEVICE;                                                               \
    }                                                                                   \
  } while (0)

// Pixels per work block.  Tiles without geometry: up to
// kMaxBlockSamples sample ids (the block's hit list lives in LDS), at most
// 64 pixels; tiles with work get smaller blocks (prepare_schedule).
static int big_block_pixels(int spp, const rt_tuning& tn) {
  int cap = kMaxBlockSamples;
  if (tn.block_samples > 0) cap = std::min(cap, tn.block_samples);
  if (spp <= 0) return 64;
  return std::max(1, std::min(64, cap / spp));
}

static int validate_scene(const rt_scene* s) {
  if (!s) {
    set_error("scene is NULL");
    return RT_E_INVALID;
  }
  if (s->num_objects < 0 || s->num_lights < 0 || (s->num_objects > 0 && !s->objects) ||
      (s->num_lights > 0 && !s->lights)) {
    set_error("scene arrays inconsistent");
    return RT_E_INVALID;
  }
  for (int i = 0; i < s->num_objects; ++i) {
    const rt_object& o = s->objects[i];
    if (o.type != RT_OBJ_SPHERE && o.type != RT_OBJ_CUBE) {
      set_error("object " + std::to_string(i) + ": unknown type " + std::to_string(o.type));
      return RT_E_INVALID;
    }
    if (o.material.kind < RT_MAT_LAMBERTIAN || o.material.kind > RT_MAT_DIFFUSELIGHT) {
      set_error("object " + std::to_string(i) + ": unknown material kind");
      return RT_E_INVALID;
    }
  }
  return RT_OK;
}

static int validate_settings(const rt_settings* st, int32_t w, int32_t h) {
  if (!st) {
    set_error("settings is NULL");
    return RT_E_INVALID;
  }
  // (each side at most 65536: the kernel's camera-jitter division relies on it)
  if (w <= 0 || h <= 0 || w > 65536 || h > 65536 || (long long)w * h > (1LL << 31) / 4) {
    set_error("invalid image size " + std::to_string(w) + "x" + std::to_string(h));
    return RT_E_INVALID;
  }
  // (any count: more than kMaxBlockSamples render in sample passes; the
  // bound keeps pixel x sample ids of a frame in 32 bits on every path)
  if (st->samples < 0 || (long long)st->samples * w * h >= (1LL << 40) || st->samples > (1 << 24)) {
    set_error("samples must be in [0, 2^24] with width * height * samples < 2^40");
    return RT_E_INVALID;
  }
  if (st->sky < RT_SKY_NONE || st->sky > RT_SKY_NIGHT) {
    set_error("sky must be one of RT_SKY_*");
    return RT_E_INVALID;
  }
  return RT_OK;
}

}  // namespace rtgo

using namespace rtgo;

// ======================================================================== ABI
struct rt_context {
  int device = 0;
  rt_tuning tun;  // work partition (rt_context_set_tuning); never changes the image
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool have_scene = false;
  FlatScene flat;
  void* d_scene = nullptr;  // one allocation: spheres | tris | mats | lights | jump table | bvh
  size_t d_scene_bytes = 0;
  void* h_stage = nullptr;  // pinned host image of the scene buffer (its upload), made by the constructor
  size_t h_stage_cap = 0;
  const DSphere* d_spheres = nullptr;
  const DTri* d_tris = nullptr;
  const DBox* d_boxes = nullptr;
  const DMat* d_mats = nullptr;
  const DLight* d_lights = nullptr;
  const DBVHNode* d_bvh = nullptr;
  const DQNode* d_qbvh = nullptr;
  const DQNode* d_qbvh4 = nullptr;
  const uint64_t* d_jump = nullptr;
  const DSky* d_sky = nullptr;  // the kSkies presets
  unsigned long long* d_counts = nullptr;
  hipStream_t last_stream = nullptr;
  bool have_timing = false;
  unsigned long long* dbg = nullptr;
  // the work schedule (rt_schedule.hip), cached per (scene, W, H, rank, world, settings)
  uint64_t scene_gen = 0;
  int64_t order_key[14] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
  int32_t* d_blocks = nullptr;  // work blocks, kBlockInts ints each, heaviest first
  size_t d_blocks_cap = 0;  // bytes
  int32_t num_blocks = 0;
  int32_t nsplit = 0;       // split pixels of the current schedule
  int32_t split_frames = 0; // frames whose copies of the split rows are laid out in d_split
  char* d_split = nullptr;  // their per-sample radiance rows + sub-block counters
  size_t split_cap = 0;
  void* d_acc = nullptr;  // sample passes: running per-pixel sums (KParams.acc)
  size_t acc_cap = 0;
  char* d_pilot = nullptr;  // pilot render scratch: packed float3 + rgba + path lengths (max, sum)
  size_t pilot_cap = 0;
  // measured schedule (rt_tuning.measure): 0 none, 1 the next render measures
  // every pixel's paths into d_meas (max | sum), 2 measured (the next
  // schedule is re-cut from them), 3 done
  int meas_state = 0;
  rt_context_stats stats{};  // rt_context_get_stats
  char* d_meas = nullptr;
  size_t meas_cap = 0;
  char* d_sched = nullptr;  // scheduler scratch (sched_layout) + the per-tile inputs
  size_t sched_cap = 0;
  int32_t h_totals[4] = {0, 0, 0, 0};  // block and split counts of the last schedule (12 bytes read back)
  // pinned staging of the schedule's small copies (the counts read back, the
  // per-tile masks and costs uploaded), made by the constructor
  char* h_small = nullptr;
  size_t h_small_cap = 0;
  std::vector<unsigned long long> masks_host;  // per local tile primary-ray masks
  unsigned long long* d_masks = nullptr;       // (inside d_sched)
  int32_t stage_bytes = 0;  // scene prefix staged into LDS per workgroup (0 = none)
  // wavefront path (BVH scenes): path arrays + queues, per-chunk radiance, loop control
  void* wf_mem = nullptr;
  size_t wf_mem_bytes = 0;
  void* wf_rad = nullptr;
  size_t wf_rad_bytes = 0;
  WfCtl* wf_ctl = nullptr;   // device
  WfCtl* wf_host = nullptr;  // pinned ring of kWfRing snapshots
  hipEvent_t wf_ev[4] = {nullptr, nullptr, nullptr, nullptr};
  // tile partition (rt_context_set_partition): its data and every rank's
  // tile list on this device (null: strided)
  std::shared_ptr<const PartitionData> part;
  int32_t* d_part = nullptr;
  size_t d_part_cap = 0;
  double bvh_seconds = 0;  // host time of the last BVH build (rt_stats.bvh_build_seconds)
  // per-kernel device time of the wavefront path (rt_context_profile): an
  // event pool, the blocks of it the last frame recorded ({first event,
  // first class, last class}) and the totals
  bool prof_on = false;
  std::vector<hipEvent_t> prof_pool;
  size_t prof_used = 0;
  struct ProfBlock {
    size_t base;
    int first, last;
  };
  std::vector<ProfBlock> prof_pending;
  double prof_secs[kWfClasses] = {0};
  int64_t prof_launches[kWfClasses] = {0};
  // a multi-rank renderer's frame deadline (steady_now_s() clock; <= 0:
  // none), set by rt_renderer_render for the frame (context_set_deadline)
  double deadline = 0;
  // tail helpers: control block | queue | ready flags | rows
  // | row bits | row headers, laid out for tail_spp samples per pixel
  char* d_tail = nullptr;
  size_t tail_bytes = 0;
  int32_t tail_cap = 0, tail_spp = -1;
  uint32_t tail_epoch = 0;
};

// Events for kernel classes [first, last] of one launch sequence: ev[k] opens
// class k (null when not profiling)
static hipEvent_t* prof_block(rt_context* c, int first, int last) {
  if (!c->prof_on) return nullptr;
  const size_t need = kWfProfEvents;
  while (c->prof_pool.size() < c->prof_used + need) {
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->prof_pool.push_back(e);
  }
  hipEvent_t* ev = c->prof_pool.data() + c->prof_used;
  c->prof_pending.push_back({c->prof_used, first, last});
  c->prof_used += need;
  return ev;
}

// Adds the recorded blocks to the totals (waits for them)
static int prof_collect(rt_context* c) {
  if (c->prof_pending.empty()) return RT_OK;
  const auto& lastb = c->prof_pending.back();
  HIP_TRY(hipEventSynchronize(c->prof_pool[lastb.base + lastb.last + 1]));
  for (const auto& b : c->prof_pending)
    for (int k = b.first; k <= b.last; ++k) {
      float ms = 0;
      HIP_TRY(hipEventElapsedTime(&ms, c->prof_pool[b.base + k], c->prof_pool[b.base + k + 1]));
      c->prof_secs[k] += ms * 1e-3;
      c->prof_launches[k] += 1;
    }
  c->prof_pending.clear();
  c->prof_used = 0;
  return RT_OK;
}

// Does a render of (w, h, world) use the context's partition?
static bool use_partition(const rt_context* c, int w, int h, int world) {
  return c->part && world > 1 && c->part->w == w && c->part->h == h && c->part->world == world;
}
// Tiles of `rank`: the partition's list or the strided set (createRenderTasks's
// tiles t % world == rank)
static int local_tiles(const rt_context* c, int w, int h, int rank, int world) {
  if (use_partition(c, w, h, world)) return c->part->offsets[rank + 1] - c->part->offsets[rank];
  return rt_tiles_for_rank(w, h, rank, world);
}
static void host_tiles(const rt_context* c, int w, int h, int rank, int world, std::vector<int32_t>* out) {
  if (use_partition(c, w, h, world)) {
    const PartitionData& d = *c->part;
    out->assign(d.lists.begin() + d.offsets[rank], d.lists.begin() + d.offsets[rank + 1]);
  } else {
    strided_tiles(w, h, rank, world, out);
  }
}
static const int32_t* dev_tiles(const rt_context* c, int w, int h, int rank, int world) {
  return use_partition(c, w, h, world) ? c->d_part + c->part->offsets[rank] : nullptr;
}

namespace rtgo {
bool context_has_bvh(const rt_context* c) { return c && !c->flat.bvh.empty(); }
double context_bvh_seconds(const rt_context* c) { return c ? c->bvh_seconds : 0.0; }
void* context_stream(const rt_context* c) { return c ? (void*)c->stream : nullptr; }
}  // namespace rtgo

namespace rtgo {
double steady_now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void context_set_deadline(rt_context* c, double deadline) {
  if (c) c->deadline = deadline;
}

// The context's host waits during a render.  Without a deadline they block
// (hipStreamSynchronize / hipEventSynchronize); with one (a multi-rank
// renderer's frame, rt_renderer_set_watchdog) they poll (yield, then 20 us
// sleeps) and return RT_E_TIMEOUT once it has passed, so a stalled rank ends
// the frame instead of blocking its host thread forever.
template <class Query>
int bounded_wait(rt_context* c, Query query, const char* what) {
  for (unsigned spin = 0;; ++spin) {
    const hipError_t e = query();
    if (e == hipSuccess) return RT_OK;
    if (e != hipErrorNotReady) {
      set_error(std::string(what) + " failed: " + hipGetErrorString(e));
      return RT_E_DEVICE;
    }
    if (steady_now_s() > c->deadline) {
      set_error(std::string("watchdog: ") + what + " did not complete before the frame's deadline");
      return RT_E_TIMEOUT;
    }
    if (spin < 256)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

int wait_stream(rt_context* c, hipStream_t s) {
  if (c->deadline <= 0) {
    HIP_TRY(hipStreamSynchronize(s));
    return RT_OK;
  }
  return bounded_wait(c, [s] { return hipStreamQuery(s); }, "a wait for the render stream");
}

int wait_event(rt_context* c, hipEvent_t ev) {
  if (c->deadline <= 0) {
    HIP_TRY(hipEventSynchronize(ev));
    return RT_OK;
  }
  return bounded_wait(c, [ev] { return hipEventQuery(ev); }, "a wait for a render event");
}

}  // namespace rtgo

extern "C" {

int rt_context_set_tuning(rt_context* c, const rt_tuning* t) {
  if (!c || !t) {
    set_error("context or tuning is NULL");
    return RT_E_INVALID;
  }
  if (t->path != RT_PATH_AUTO && t->path != RT_PATH_MEGAKERNEL) {
    set_error("tuning.path must be RT_PATH_AUTO or RT_PATH_MEGAKERNEL");
    return RT_E_INVALID;
  }
  if (t->pilot_depth < 0 || t->split_samples < 0 || t->split_samples > 64 || t->bvh_leaf < 0 || t->bvh_leaf > 7 || t->bvh_bins < 0 || t->block_work < 0 || t->block_samples < 0 ||
      t->wf_paths < 0 || t->wf_chunk < 0 || t->wf_trav_block < 0 || t->wf_trav_block > 1024 || t->wf_trav_wgs < 0 ||
      t->wf_list_tries < 0 || t->wf_list_tries > 64 || t->tail_helpers < -1 || t->tail_helpers > 4096 ||
      t->tail_paths < 0 || t->tail_paths > 64 || t->tail_depth < 0 || t->tail_every < 0 || t->tail_every > 64 ||
      t->tail_at < 0 || t->tail_at > 100) {
    set_error("tuning value out of range");
    return RT_E_INVALID;
  }
  c->tun = *t;
  c->order_key[0] = -1;  // rebuild the schedule
  return RT_OK;
}

int32_t rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_debug_xlane_faults(int32_t device, int32_t reset, uint64_t* out) {
  if (!out) {
    set_error("out is NULL");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  const long long a = xlane_faults_kernel(reset != 0), b = xlane_faults_wavefront(reset != 0);
  if (a == -1 || b == -1) {
    set_error("not a cross-lane checking build (make xlane)");
    return RT_E_INVALID;
  }
  if (a < 0 || b < 0) {
    set_error("reading the cross-lane fault counters failed");
    return RT_E_DEVICE;
  }
  *out = (uint64_t)(a + b);
  return RT_OK;
}

int rt_validate(const rt_scene* scene, int32_t w, int32_t h, const rt_settings* st) {
  int rc = validate_scene(scene);
  if (rc) return rc;
  return validate_settings(st, w, h);
}

const char* rt_last_error(void) { return g_last_error.c_str(); }

// pinned scene staging made by rt_context_create (grown when a scene needs more)
constexpr size_t kStageDefault = 256 * 1024;
// pinned schedule staging: [0, 256) the counts read back, then the masks and
// costs uploaded (grown when a frame has more tiles)
constexpr size_t kSmallDefault = 64 * 1024;

int rt_context_create(int32_t device, rt_context** out) {
  if (!out) {
    set_error("out is NULL");
    return RT_E_INVALID;
  }
  *out = nullptr;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) {
    set_error("device " + std::to_string(device) + " out of range (" + std::to_string(n) + " devices)");
    return RT_E_DEVICE;
  }
  HIP_TRY(hipSetDevice(device));
  {
    // the kernels' code objects, once per device and process: the
    // constructor's work (NewParallelRenderer), not the first Render's
    static std::mutex mu;
    static std::vector<bool> loaded;
    std::lock_guard<std::mutex> lock(mu);
    if ((int)loaded.size() < n) loaded.resize(n, false);
    if (!loaded[device]) {
      hipError_t e = (hipError_t)preload_render_kernels();
      if (e == hipSuccess) e = (hipError_t)preload_sched_kernels();
      if (e == hipSuccess) e = (hipError_t)preload_wf_kernels();
      if (e != hipSuccess) {
        set_error(std::string("kernel code object load failed: ") + hipGetErrorString(e));
        return RT_E_DEVICE;
      }
      loaded[device] = true;
    }
  }
  rt_context* c = new rt_context();
  c->device = device;
  rt_tuning_default(&c->tun);
  hipError_t e = (hipError_t)dev_stream_get(&c->stream);
  if (e == hipSuccess) e = (hipError_t)dev_event_get(&c->ev0);
  if (e == hipSuccess) e = (hipError_t)dev_event_get(&c->ev1);
  {
    // the runtime's first-launch / first-copy set-up, once per device and
    // process, on the context's stream (constructor work, as above)
    static std::mutex mu;
    static std::vector<bool> warmed;
    std::lock_guard<std::mutex> lock(mu);
    if ((int)warmed.size() < n) warmed.resize(n, false);
    if (e == hipSuccess && !warmed[device]) {
      constexpr size_t kWarmBytes = size_t(4) << 20;  // a large copy each way (the copy engines)
      void* dbuf = nullptr;
      void* hbuf = nullptr;
      e = (hipError_t)dev_alloc(&dbuf, kWarmBytes);
      if (e == hipSuccess) e = (hipError_t)host_alloc(&hbuf, kWarmBytes);
      std::vector<char> pageable(kWarmBytes);
      if (e == hipSuccess) e = (hipError_t)warm_device(c->stream, dbuf, hbuf, pageable.data(), kWarmBytes);
      host_free(hbuf);
      dev_free(dbuf);
      if (e == hipSuccess) warmed[device] = true;
    }
  }

  // pinned staging of the scene upload (a copy from pageable memory makes the
  // runtime set up its own staging on first use: 9.6 ms of a fresh process's
  // first Render, profiles/r04_cli_trace.json)
  if (e == hipSuccess) {
    e = (hipError_t)host_alloc(&c->h_stage, kStageDefault);
    if (e == hipSuccess) c->h_stage_cap = kStageDefault;
  }
  if (e == hipSuccess) {
    e = (hipError_t)host_alloc((void**)&c->h_small, kSmallDefault);
    if (e == hipSuccess) c->h_small_cap = kSmallDefault;
  }
  if (e != hipSuccess) {
    set_error(std::string("context init failed: ") + hipGetErrorString(e));
    rt_context_destroy(c);
    return RT_E_DEVICE;
  }
  *out = c;
  return RT_OK;
}

void rt_context_destroy(rt_context* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  // the last render (on the caller's stream) and the context's own stream
  // must be done before the buffers go back to the cache
  if (c->have_timing) (void)hipEventSynchronize(c->ev1);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : {(void*)c->d_scene, (void*)c->d_counts, (void*)c->d_blocks, (void*)c->d_pilot, c->d_acc,
                  (void*)c->d_meas, (void*)c->d_split, (void*)c->d_sched, (void*)c->d_part, c->wf_mem, c->wf_rad,
                  (void*)c->wf_ctl, (void*)c->d_tail})
    dev_free(p);
  host_free(c->h_stage);
  host_free(c->h_small);
  if (c->wf_host) (void)hipHostFree(c->wf_host);
  for (hipEvent_t& e : c->wf_ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->prof_pool) (void)hipEventDestroy(e);
  dev_event_put(c->ev0);  // (complete: ev1 was waited for, ev0 precedes it)
  dev_event_put(c->ev1);
  dev_stream_put(c->stream);  // (idle: synchronized above)
  delete c;
}

// Wait until the last render enqueued on this context has finished: before
// the host overwrites buffers it reads (scene, schedule, wavefront state).
static int quiesce(rt_context* c) {
  int rc = c->have_timing ? wait_event(c, c->ev1) : RT_OK;
  if (!rc && c->stream) rc = wait_stream(c, c->stream);
  return rc;
}

int rt_context_set_scene(rt_context* c, const rt_scene* s, int32_t force_bvh) {
  if (!c) {
    set_error("context is NULL");
    return RT_E_INVALID;
  }
  int rc = validate_scene(s);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  flatten_scene(*s, &c->flat);
  c->bvh_seconds = 0;
  const bool want_bvh = force_bvh > 0 || (force_bvh == 0 && c->flat.spheres.size() > 64);
  if (want_bvh && !c->flat.tris.empty()) {
    if (force_bvh > 0) {
      set_error("BVH supports sphere-only scenes");
      return RT_E_INVALID;
    }
  } else if (want_bvh) {
    const auto t0 = std::chrono::steady_clock::now();
    build_sphere_bvh(&c->flat, c->tun.bvh_bins, c->tun.bvh_leaf);
    c->bvh_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  const FlatScene& f = c->flat;
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  size_t off_s = 0;
  size_t off_t = off_s + al(f.spheres.size() * sizeof(DSphere));
  size_t off_x = off_t + al(f.tris.size() * sizeof(DTri));
  size_t off_m = off_x + al(f.boxes.size() * sizeof(DBox));
  size_t off_l = off_m + al(f.mats.size() * sizeof(DMat));
  size_t off_j = off_l + al(f.lights.size() * sizeof(DLight));
  size_t off_b = off_j + al(kJump * 2 * sizeof(uint64_t));
  size_t off_q = off_b + al(f.bvh.size() * sizeof(DBVHNode));
  size_t off_q4 = off_q + al(f.qbvh.size() * sizeof(DQNode));
  size_t off_sky = off_q4 + al(f.qbvh4.size() * sizeof(DQNode));
  size_t total = off_sky + al(kSkies * sizeof(DSky)) + 256;
  rc = quiesce(c);  // the last render may still read the scene
  if (rc) return rc;
  if (c->d_scene && c->d_scene_bytes < total) {
    dev_free(c->d_scene);
    c->d_scene = nullptr;
  }
  if (!c->d_scene) {
    HIP_TRY((hipError_t)dev_alloc(&c->d_scene, total));
    c->d_scene_bytes = total;
  }
  char* base = (char*)c->d_scene;
  if (total > c->h_stage_cap) {  // (the last upload was synchronized: the buffer is free)
    host_free(c->h_stage);
    c->h_stage = nullptr;
    c->h_stage_cap = 0;
    HIP_TRY((hipError_t)host_alloc(&c->h_stage, total));
    c->h_stage_cap = total;
  }
  char* host = (char*)c->h_stage;
  memset(host, 0, total);
  memcpy(host + off_s, f.spheres.data(), f.spheres.size() * sizeof(DSphere));
  memcpy(host + off_t, f.tris.data(), f.tris.size() * sizeof(DTri));
  memcpy(host + off_x, f.boxes.data(), f.boxes.size() * sizeof(DBox));
  memcpy(host + off_m, f.mats.data(), f.mats.size() * sizeof(DMat));
  memcpy(host + off_l, f.lights.data(), f.lights.size() * sizeof(DLight));
  {
    uint64_t* jt = reinterpret_cast<uint64_t*>(host + off_j);
    uint64_t a = 1, cc = 0;  // x_{i+j} = A_j x_i + C_j, built incrementally (rt_pcg_jump_coeffs)
    for (int j = 0; j < 3 * kJump; ++j) {
      if (j % 3 == 0) {  // entry h = j / 3: the jump by 3h draws
        jt[2 * (j / 3)] = a;
        jt[2 * (j / 3) + 1] = cc;
      }
      cc = cc * RT_PCG_MULT + RT_PCG_INC;
      a = a * RT_PCG_MULT;
    }
  }
  memcpy(host + off_b, f.bvh.data(), f.bvh.size() * sizeof(DBVHNode));
  memcpy(host + off_q, f.qbvh.data(), f.qbvh.size() * sizeof(DQNode));
  memcpy(host + off_q4, f.qbvh4.data(), f.qbvh4.size() * sizeof(DQNode));
  sky_presets(reinterpret_cast<DSky*>(host + off_sky));
  HIP_TRY(hipMemcpyAsync(base, host, total, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->d_spheres = (const DSphere*)(base + off_s);
  c->d_tris = (const DTri*)(base + off_t);
  c->d_boxes = (const DBox*)(base + off_x);
  c->d_mats = (const DMat*)(base + off_m);
  c->d_lights = (const DLight*)(base + off_l);
  c->d_bvh = (const DBVHNode*)(base + off_b);
  c->d_qbvh = (const DQNode*)(base + off_q);
  c->d_qbvh4 = (const DQNode*)(base + off_q4);
  c->d_jump = (const uint64_t*)(base + off_j);
  c->d_sky = (const DSky*)(base + off_sky);
  // small linear-scan scenes are staged into LDS by every workgroup
  // (the 1 KB PCG jump table stays in global memory, L1-cached: only the
  // cooperative soft-shadow form reads it, and scenes near the LDS limit of 12
  // workgroups per CU ran faster without it)
  c->stage_bytes = (f.bvh.empty() && off_j <= 48 * 1024) ? (int32_t)off_j : 0;
  c->have_scene = true;
  c->scene_gen += 1;
  return RT_OK;
}

// Per (scene, frame, rank, settings) schedule, cached in the context: the
// tiles' primary-ray candidate masks (host: tiles x primitives) and the work
// blocks, built on the GPU by rt_schedule.hip from a ONE-SAMPLE PILOT render
// of this rank's pixels (same kernel, kPilot instantiation) that reports
// each pixel's path length: pixels whose paths bounce a lot go into small
// blocks (or are split into sample ranges) dispatched first, empty sky into
// large blocks.  The pilot traces hard shadows only: the soft rays do not
// change how long a path is, only what a bounce costs, and tracing them
// would make the pilot's own tail (one 50-bounce path) several times longer.
// One 12-byte device->host copy (block and split counts) sizes the launch.
// This only partitions and orders the work; every block is rendered by the
// same code, so the image does not depend on it (tests/test_gpu_schedules.py).
static size_t split_flags_bytes(int nsplit, int spp) {
  return (size_t)nsplit * ((spp + 31) / 32) * sizeof(uint32_t) + (size_t)nsplit * sizeof(int32_t);
}

// device buffer *ptr of *cap bytes, grown to at least n bytes.  dev_free
// hands the old block straight to the device cache (no implicit device sync,
// unlike hipFree), where another context may take it at once: the context's
// last render, which may still use it, is waited for first.
static int grow(rt_context* c, void* ptr, size_t* cap, size_t n) {
  void** p = (void**)ptr;
  if (n <= *cap) return RT_OK;
  if (*p) {
    int rc = quiesce(c);
    if (rc) return rc;
  }
  dev_free(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY((hipError_t)dev_alloc(p, n));
  *cap = n;
  return RT_OK;
}

// The launch parameters of a render of (w, h, st) by `rank` of `world`
// (outputs, counters and schedule are filled in by the caller).
static void base_params(const rt_context* c, int w, int h, const rt_settings* st, int rank, int world, int layout,
                        KParams* out) {
  const FlatScene& f = c->flat;
  KParams& p = *out;
  memset(&p, 0, sizeof p);
  p.spheres = c->d_spheres;
  p.tris = c->d_tris;
  p.boxes = c->d_boxes;
  p.mats = c->d_mats;
  p.lights = c->d_lights;
  p.bvh = c->d_bvh;
  p.jump = c->d_jump;
  p.sky = st->sky != RT_SKY_NONE ? c->d_sky + (st->sky - 1) : nullptr;
  p.dbg = c->dbg;
  memcpy(p.cam, f.cam_pos, sizeof p.cam);
  p.aspect = f.aspect;
  p.seed_key = rt_rng_seed_key(st->seed);
  p.ns = (int32_t)f.spheres.size();
  p.nt = (int32_t)f.tris.size();
  p.nl = (int32_t)f.lights.size();
  p.nb = (int32_t)f.boxes.size();
  p.use_bvh = f.bvh.empty() ? 0 : 1;
  p.W = w;
  p.H = h;
  p.spp = st->samples;
  p.max_depth = st->max_depth;
  p.recursive = st->recursive_reflections != 0;
  p.soft = st->soft_shadows != 0;
  p.rank = rank;
  p.world = world;
  p.tiles_x = (w + 31) / 32;
  p.ntiles = rt_num_tiles(w, h);
  p.layout = layout;
  // LDS staging of the scene prefix + BVH stack placement
  p.stage_src = c->d_scene;
  p.stage_bytes = c->tun.stage ? c->stage_bytes : 0;
  p.stack_off = (p.stage_bytes + 15) & ~15;
  p.stack_depth = std::max(1, f.bvh_depth);
}

// Tail helpers for a megakernel launch of p: render_kernel_tail
// (the staged product body) on a linear-scan scene with shadow-cone masks (what
// solo_path needs), one sample pass, no sky, not measuring.  Lays out the
// context's queue and rows for p.spp_total samples per pixel (the control
// block and ready flags zeroed once per layout: each launch's last helper
// leaves the control block zeroed, and a ready flag holds its launch's epoch)
// and sets p's tail fields; leaves them null (off) otherwise.
static int setup_tail(rt_context* c, KParams* p, hipStream_t s) {
  const rt_tuning& tn = c->tun;
  p->tail = nullptr;
  const bool masks = !p->use_bvh && p->ns <= 64 && p->nt <= 64;
  if (tn.tail_helpers < 0 || p->stage_bytes <= 0 || !masks || p->sky || p->work_max || p->counts || p->acc_mode != 0 ||
      p->spp_total < 1 || p->spp_total > kMaxBlockSamples || p->max_depth < 2 || !p->recursive)
    return RT_OK;
  const int spp = p->spp_total, bw = (spp + 31) / 32;
  const size_t per = (size_t)spp * 24 + (size_t)bw * 4 + sizeof(TailPath) + sizeof(TailRow) + 4;
  // one queue entry and at most one row per exported path; 64 MB at most
  const int cap = (int)std::max<size_t>(1024, std::min<size_t>(16384, (size_t(64) << 20) / per));
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t o_q = al(sizeof(TailCtl)), o_ready = o_q + al((size_t)cap * sizeof(TailPath));
  const size_t o_rows = o_ready + al((size_t)cap * 4), o_bits = o_rows + al((size_t)cap * spp * 24);
  const size_t o_hdr = o_bits + al((size_t)cap * bw * 4), total = o_hdr + al((size_t)cap * sizeof(TailRow));
  if (c->tail_spp != spp || c->tail_cap != cap) {
    int rc = grow(c, &c->d_tail, &c->tail_bytes, total);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_tail, 0, o_rows, s));  // control block, queue, ready flags
    c->tail_spp = spp;
    c->tail_cap = cap;
    c->tail_epoch = 0;
  }
  if (++c->tail_epoch == 0) c->tail_epoch = 1;
  char* b = c->d_tail;
  p->tail = (TailCtl*)b;
  p->tail_q = (TailPath*)(b + o_q);
  p->tail_ready = (unsigned int*)(b + o_ready);
  p->tail_rows = (double*)(b + o_rows);
  p->tail_bits = (uint32_t*)(b + o_bits);
  p->tail_hdr = (TailRow*)(b + o_hdr);
  p->tail_cap = cap;
  p->tail_helpers = tn.tail_helpers > 0 ? tn.tail_helpers : 64;
  p->tail_kmax = tn.tail_paths > 0 ? tn.tail_paths : 4;
  p->tail_dmin = tn.tail_depth > 0 ? tn.tail_depth : 2;
  int every = tn.tail_every > 0 ? tn.tail_every : 4, pow2 = 1;
  while (pow2 < every && pow2 < 64) pow2 <<= 1;
  p->tail_every_mask = pow2 - 1;
  const int at = tn.tail_at > 0 ? std::min(tn.tail_at, 100) : 100;
  p->tail_pos = (int32_t)((int64_t)p->num_wgs * at / 100);
  p->tail_epoch = c->tail_epoch;
  return RT_OK;
}

// The scheduler's inputs for `tiles` (host masks and costs uploaded into
// `in`, the scratch layout at `scratch`), as SchedParams.
static SchedParams sched_params(rt_context* c, const KParams& p, const rt_settings* st, const std::vector<int32_t>& tiles,
                                const int32_t* d_tiles, bool masks, bool frustum, double block_work, int bigP,
                                void* scratch, unsigned long long* d_masks, float* d_cost) {
  const FlatScene& f = c->flat;
  const rt_tuning& tn = c->tun;
  SchedParams sp;
  memset(&sp, 0, sizeof sp);
  sched_layout(scratch, (int)tiles.size(), &sp);
  sp.spheres = c->d_spheres;
  sp.tris = c->d_tris;
  memcpy(sp.cam, f.cam_pos, sizeof sp.cam);
  sp.vw = 2.0 * f.aspect;
  sp.W = p.W;
  sp.H = p.H;
  sp.rank = p.rank;
  sp.world = p.world;
  sp.tiles_x = (p.W + 31) / 32;
  sp.ntiles = rt_num_tiles(p.W, p.H);
  sp.local = (int)tiles.size();
  sp.spp = st->samples;
  sp.big_pixels = bigP;
  sp.frustum = frustum;
  sp.split_samples = tn.split_samples > 0 ? std::min(64, tn.split_samples) : 64;
  sp.split_depth = tn.split_depth > 0 ? tn.split_depth : 16;
  sp.block_work = block_work;
  sp.tile_masks = masks ? d_masks : nullptr;
  sp.tile_cost = d_cost;
  sp.tile_list = d_tiles;
  return sp;
}

// The one-sample pilot render of sp's tiles (blocks of 64 pixels, packed
// output into `buf`, npx * 24 bytes): each pixel's longest path and its
// bounces into sp.work_max / work_sum.
static int run_pilot(const rt_context* c, const KParams& p, SchedParams* sp, char* buf, hipStream_t s) {
  const size_t npx = (size_t)sp->local * 1024;
  float* plin = (float*)buf;
  uint8_t* prgba = (uint8_t*)buf + npx * 12;
  unsigned int* plen = (unsigned int*)((uint8_t*)buf + npx * 16);
  KParams q = p;
  q.spp = 1;
  q.blocks = sp->pilot_blocks;
  q.num_blocks = sp->local * 16;
  q.num_wgs = q.num_blocks;
  q.layout = RT_LAYOUT_PACKED_TILES;
  q.out_linear = plin;
  q.out_rgba = prgba;
  q.counts = nullptr;
  q.dbg = nullptr;
  q.work_max = plen;
  q.work_sum = plen + npx;
  q.soft = 0;  // path lengths only (see above)
  if (c->tun.pilot_depth > 0) q.max_depth = std::min(q.max_depth, c->tun.pilot_depth);
  q.tile_masks = sp->tile_masks;
  q.split_rad = nullptr;
  q.split_hits = nullptr;
  q.split_cnt = nullptr;
  q.acc = nullptr;
  q.acc_mode = 0;
  q.sample_base = 0;
  q.spp_total = 1;
  HIP_TRY(hipMemsetAsync(plen, 0, 2 * npx * sizeof(unsigned int), s));
  const int e = launch_render(q, false, s);
  if (e != hipSuccess) {
    set_error(std::string("pilot launch failed: ") + hipGetErrorString((hipError_t)e));
    return RT_E_DEVICE;
  }
  sp->work_max = plen;
  sp->work_sum = plen + npx;
  sp->work_n = 1;
  return RT_OK;
}

// path bounces per block: 8 full-wave bounce steps; 16x that with a BVH,
// whose bounces are long divergent traversals that need full waves more
// than short blocks (C4: 2.10 s at 512, 1.77 s at 8192)
// (triangle scenes: 256 -- a bounce there tests 12 triangles per cube, so
// fewer bounces make a block: silver C3 0.56 -> 0.46 ms; sphere scenes:
// 384 since solo paths (r02, headline 0.785 -> 0.745 ms; 320: 0.755,
// 448: 0.79, 512 was the r01 optimum)
// Blocks' estimated work (bounce-samples).  A launch of ONE frame ends when
// its slowest block does, so its blocks are small: a long path shares its
// wave with few others (the latency schedule).  A launch of several frames
// (rt_context_render_frames_async) is rendered for throughput: its tail is
// paid once for all of them and overlaps the next launch, and larger blocks
// cost less per sample (fewer visibility passes, splits and block starts).
// Measured (bench.py --tuning block_work=..., 2 launches of 8 frames in
// flight, one MI355X): C2 384 -> 128.7 k, 512 135.5 k, 768 141.3 k, 1024
// 144.8 k, 1536 143.0 k, 2048 139.9 k Mrays/s; C3 256 -> 393.9 k, 512
// 419.8 k, 768 461.8 k, 1024 474.9 k, 2048 480.1 k (16 frames per launch:
// C2 896 144.4 k, 1024 146.2 k, 1280 145.4 k; C3 1024 463.7 k, 1536 476.1 k,
// 2048 479.1 k).  (r05, RNG spec v4: a bounce-sample costs less, so blocks
// grow: the driver's 20 frames as 2 launches of 10, C2 1024 -> 212.5 k, 1536
// 223.7 k, 2048 215.0 k, 3072 212.6 k, 4096 208.6 k; 100 frames as 4 of 25:
// 247.8 k, 251.6 k, 251.0 k, 249.6 k, 248.3 k; scripts/k20_tuning.sh)
// (r06, one frame per launch, sphere scenes, scripts/tail_probe.py, median
// of 40 frames: 384 and 512 bounce-samples per block equal when the order of
// the settings is balanced, 0.571-0.583 vs 0.574-0.586 ms -- a first sweep
// that always ran 384 first had put 512 2 % ahead; 768 0.725, 256 0.60-0.62)
static double default_block_work(const rt_context* c, int frames = 1) {
  const FlatScene& f = c->flat;
  double block_work = !f.bvh.empty() ? 8192.0
                      : frames > 1    ? (f.tris.empty() ? 1536.0 : 2048.0)
                                      : (f.tris.empty() ? 384.0 : 256.0);
  if (c->tun.block_work > 0) block_work = std::max(1.0, c->tun.block_work);
  return block_work;
}

// primary-ray candidate masks apply (small linear-scan scenes)
static bool masks_apply(const FlatScene& f) { return f.bvh.empty() && f.spheres.size() <= 64 && f.tris.size() <= 64; }

static int prepare_schedule(rt_context* c, KParams* p, const rt_settings* st, hipStream_t s, int frames = 1) {
  const FlatScene& f = c->flat;
  const int w = p->W, h = p->H, rank = p->rank, world = p->world;
  const rt_tuning& tn = c->tun;
  int bigP = big_block_pixels(st->samples, tn);
  const double block_work = default_block_work(c, frames);
  const bool pilot = tn.pilot != 0;
  // a sky makes every camera sample count (a miss returns the sky, not +0):
  // no primary-ray culling, no black tiles
  const bool sky = st->sky != RT_SKY_NONE;
  const bool frustum = tn.frustum != 0 && !sky;
  const bool part = use_partition(c, w, h, world);
  const int64_t key[14] = {(int64_t)c->scene_gen, w, h, rank, world, st->samples, st->max_depth,
                           st->recursive_reflections, st->soft_shadows, bigP, (int64_t)(block_work * 16),
                           (pilot ? 1 + tn.pilot_depth : 0) | (int64_t)tn.split_samples << 16,
                           (frustum ? 1 : 0) | (sky ? 2 : 0) | (tn.measure ? 4 : 0) | (int64_t)tn.split_depth << 8,
                           part ? (int64_t)c->part->id : 0};
  const bool masks = masks_apply(f);
  const bool new_key = memcmp(key, c->order_key, sizeof key) != 0;
  // a measured re-cut: the previous frame of this key measured every pixel
  const bool remeasured = !new_key && c->meas_state == 2;
  if (new_key || remeasured) {
    int rc = quiesce(c);  // the last render may still read the blocks, masks and split rows
    if (rc) return rc;
    std::vector<int32_t> tiles;
    host_tiles(c, w, h, rank, world, &tiles);
    const int local = (int)tiles.size();
    c->num_blocks = 0;
    c->nsplit = 0;
    c->split_frames = 0;  // (the split rows are laid out again below)
    c->masks_host.clear();
    c->d_masks = nullptr;
    if (local > 0) {
      // per-tile inputs (host): primary-ray candidate masks, projected-primitive counts
      if (masks) tile_primary_masks(f, w, h, tiles, &c->masks_host);
      std::vector<float> cost;
      tile_cost(f, w, h, tiles, &cost);
      const size_t scratch = sched_scratch_bytes(local);
      const size_t mbytes = c->masks_host.size() * sizeof(unsigned long long), cbytes = cost.size() * sizeof(float);
      const size_t inputs = mbytes + cbytes;
      rc = grow(c, &c->d_sched, &c->sched_cap, scratch + inputs + 256);
      if (rc) return rc;
      if (256 + inputs > c->h_small_cap) {  // (its last use was synchronized below)
        host_free(c->h_small);
        c->h_small = nullptr;
        c->h_small_cap = 0;
        HIP_TRY((hipError_t)host_alloc((void**)&c->h_small, 256 + inputs));
        c->h_small_cap = 256 + inputs;
      }
      char* in = (char*)c->d_sched + ((scratch + 255) & ~size_t(255));
      c->d_masks = masks ? (unsigned long long*)in : nullptr;
      float* d_cost = (float*)(in + mbytes);
      // (through pinned staging: a pageable copy sets up the runtime's own
      // staging on first use, milliseconds of a fresh process's first frame)
      memcpy(c->h_small + 256, c->masks_host.data(), mbytes);
      memcpy(c->h_small + 256 + mbytes, cost.data(), cbytes);
      // From the first copy on, h_small may be read by a DMA still in flight:
      // every return before the synchronize below waits for the stream first
      // (the next schedule writes h_small again; host_free hands it to the
      // process-wide cache).
      auto fail_synced = [&](int code) {
        (void)hipStreamSynchronize(s);
        return code;
      };
      auto hip_ok = [&](hipError_t err, const char* what) {
        if (err == hipSuccess) return true;
        set_error(std::string(what) + " failed: " + hipGetErrorString(err));
        return false;
      };
      if (mbytes && !hip_ok(hipMemcpyAsync(c->d_masks, c->h_small + 256, mbytes, hipMemcpyHostToDevice, s),
                            "schedule mask upload"))
        return fail_synced(RT_E_DEVICE);
      if (cbytes && !hip_ok(hipMemcpyAsync(d_cost, c->h_small + 256 + mbytes, cbytes, hipMemcpyHostToDevice, s),
                            "schedule cost upload"))
        return fail_synced(RT_E_DEVICE);
      SchedParams sp = sched_params(c, *p, st, tiles, dev_tiles(c, w, h, rank, world), masks, frustum, block_work,
                                    bigP, c->d_sched, c->d_masks, d_cost);
      int e = sched_launch_pixels(sp, s);
      if (e != hipSuccess) {
        set_error(std::string("schedule launch failed: ") + hipGetErrorString((hipError_t)e));
        return fail_synced(RT_E_DEVICE);
      }
      if (remeasured) {  // every sample's path of the last frame (the measuring render)
        sp.work_max = (const unsigned int*)c->d_meas;
        sp.work_sum = sp.work_max + (size_t)local * 1024;
        sp.work_n = st->samples;
      } else if (pilot && st->samples > 0 && st->max_depth > 0) {
        rc = grow(c, &c->d_pilot, &c->pilot_cap, (size_t)local * 1024 * 24 + 256);
        if (rc) return fail_synced(rc);
        rc = run_pilot(c, *p, &sp, c->d_pilot, s);
        if (rc) return fail_synced(rc);
      }
      e = sched_launch_blocks(sp, false, s);
      if (e != hipSuccess) {
        set_error(std::string("schedule launch failed: ") + hipGetErrorString((hipError_t)e));
        return fail_synced(RT_E_DEVICE);
      }
      if (!hip_ok(hipMemcpyAsync(c->h_small, sp.totals, 3 * sizeof(int32_t), hipMemcpyDeviceToHost, s),
                  "schedule count read-back"))
        return fail_synced(RT_E_DEVICE);
      rc = wait_stream(c, s);  // (bounded under a renderer's deadline)
      if (rc) return rc;
      memcpy(c->h_totals, c->h_small, 3 * sizeof(int32_t));
      const int nblocks = c->h_totals[0], nsplit = c->h_totals[1];
      rc = grow(c, &c->d_blocks, &c->d_blocks_cap, (size_t)std::max(nblocks, 1) * kBlockInts * sizeof(int32_t));
      if (rc) return rc;
      sp.blocks = c->d_blocks;
      e = sched_launch_blocks(sp, true, s);
      if (e != hipSuccess) {
        set_error(std::string("schedule launch failed: ") + hipGetErrorString((hipError_t)e));
        return RT_E_DEVICE;
      }
      c->num_blocks = nblocks;
      c->nsplit = nsplit;
    }
    // (a rank with no tiles -- more ranks than the frame has tiles -- renders
    // nothing: no scheduler launch, no read-back of counts it never wrote)
    memcpy(c->order_key, key, sizeof key);
    c->stats.schedules_built += 1;
    // a new key's first frame measures (state 1), the next re-cuts (2 -> 3)
    c->meas_state = remeasured ? 3 : (tn.measure && local > 0 ? 1 : 0);
  }
  // split pixels: one copy of their radiance rows, hit bits and sub-block
  // counters per frame a launch renders (`frames`), laid out as [copies of
  // the rows][copies of the bits][copies of the counters].  Bits and counters
  // start at zero; each launch's last sub-block of a pixel zeroes them again
  // (rt_kernel.hip), so they are cleared only when the layout changes.
  const size_t rows = (size_t)c->nsplit * st->samples * 3 * sizeof(double);
  const size_t flags = split_flags_bytes(c->nsplit, st->samples);
  if (c->nsplit && c->split_frames < frames) {
    int rc = quiesce(c);  // earlier launches may still use the rows
    if (rc) return rc;
    rc = grow(c, &c->d_split, &c->split_cap, (rows + flags) * (size_t)frames + 256);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync((char*)c->d_split + rows * (size_t)frames, 0, flags * (size_t)frames, s));
    c->split_frames = frames;
  }
  const size_t nf = (size_t)std::max(c->split_frames, 1);
  p->blocks = c->d_blocks;
  p->num_blocks = c->num_blocks;
  p->nsplit = c->nsplit;
  p->split_frames = c->split_frames;
  p->split_rad = c->nsplit ? (double*)c->d_split : nullptr;
  p->split_hits = c->nsplit ? (uint32_t*)((char*)c->d_split + rows * nf) : nullptr;
  p->split_cnt = c->nsplit ? (int32_t*)(p->split_hits + (size_t)c->nsplit * ((st->samples + 31) / 32) * nf) : nullptr;
  p->tile_masks = (masks && frustum) ? c->d_masks : nullptr;
  return RT_OK;
}

// ---------------------------------------------------------------- wavefront path
// BVH scenes render through the staged kernels of rt_wavefront.hip (DESIGN.md
// §4.2).  Buffers live in the context and grow on demand; a frame is cut into
// chunks of whole pixels (all their samples) so the per-sample radiance
// buffer stays below kWfMaxChunkSamples entries (24 B each).
constexpr int kWfRing = 4;
// (each chunk ends in its own drain of long paths: C5 on one GPU, 2.1 G
// samples, took 7.72 s per frame in chunks of 2^28 samples)
constexpr uint64_t kWfMaxChunkSamples = 1ull << 30;  // 24 GB of radiance (HBM: 288 GB)

static bool use_wavefront(const rt_context* c) { return !c->flat.bvh.empty() && c->tun.path != RT_PATH_MEGAKERNEL; }

// path slots per shard (a multiple of kWfBlockSlots: every shard receives the
// survivors of the workgroups b % kWfShards == shard, at most shard_cap)
// More slots mean fewer, longer bounce iterations (each persistent traversal
// launch pays a fill and a drain): C4 with 2^20 slots 680 ms per frame, 2^21
// 589, 2^22 536, 2^23 510, 1.5 * 2^23 501, 2^24 499.  No more slots than the
// chunk has samples (a path slot holds one sample's path).
static int wf_shard_cap(int nl, const rt_tuning& tn, uint64_t samples) {
  long long cap = 1 << 24;
  if (tn.wf_paths > 0) cap = std::min(1ll << 24, (long long)tn.wf_paths);
  cap = std::min<long long>(cap, (long long)std::min<uint64_t>(samples, 1ull << 40));
  // soft queues: cap * nl * 16 entries of 16 B, at most 8 GB; keys slot * nl + light fit 32 bits
  cap = std::min<long long>(cap, (1ll << 29) / (16ll * std::max(nl, 1)));
  const long long per = kWfShards * kWfBlockSlots;
  return (int)(std::max(1ll, cap / per) * kWfBlockSlots);
}

static int render_wavefront(rt_context* c, const KParams& kp, const rt_settings* st, hipStream_t s, bool count) {
  const FlatScene& f = c->flat;
  if (c->prof_on) {  // the last frame's kernel times (its events are reused)
    int rc = prof_collect(c);
    if (rc) return rc;
  }
  const int nl = (int)f.lights.size();
  const int local = local_tiles(c, kp.W, kp.H, kp.rank, kp.world);
  const uint64_t local_px = (uint64_t)local * 1024;
  const uint64_t spp = (uint64_t)std::max(st->samples, 1);
  uint64_t max_chunk = kWfMaxChunkSamples;
  if (c->tun.wf_chunk > 0) max_chunk = std::min<uint64_t>((uint64_t)c->tun.wf_chunk, max_chunk);
  const uint64_t chunk_px = std::max<uint64_t>(1, std::min<uint64_t>(local_px, max_chunk / spp));
  const int shard_cap = wf_shard_cap(nl, c->tun, chunk_px * spp);
  const size_t cap = (size_t)shard_cap * kWfShards;
  const size_t nlk = (size_t)std::max(nl, 1);
  // hard rays per shard: at most every light of every path of the workgroups
  // b % kWfShards == shard of wf_shade1 / wf_softgen, which cover at most
  // shard_cap paths (their grid has at most cap / kWfBlockSlots workgroups)
  const size_t qcap = (size_t)shard_cap * nlk;
  // one allocation: two path arrays | hit records | per-light state | queues
  const size_t need = 2 * cap * (12 * 8 + 8 + 4 + 4)   // path arrays
                      + cap * (3 * 8 + 4)               // hit point, index
                      + cap * nlk * 4                   // lstate
                      + (size_t)kWfShards * qcap * 4    // hard queues
                      + (size_t)kWfShards * qcap * 16 * 16  // soft queues
                      + (size_t)kWfShards * qcap * 4    // cone queues
                      + cap * nlk * kWfConeWide * 4     // cone candidate lists
                      + (size_t)kWfShards * qcap * 2 * 16  // wide-cone queues
                      + 64 * 256;                       // alignment
  if (need > c->wf_mem_bytes) {
    int rq = quiesce(c);
    if (rq) return rq;
    dev_free(c->wf_mem);
    c->wf_mem = nullptr;
    c->wf_mem_bytes = 0;
    HIP_TRY((hipError_t)dev_alloc(&c->wf_mem, need));
    c->wf_mem_bytes = need;
  }
  if (!c->wf_ctl) {
    HIP_TRY((hipError_t)dev_alloc((void**)&c->wf_ctl, sizeof(WfCtl)));
    HIP_TRY(hipHostMalloc((void**)&c->wf_host, kWfRing * sizeof(WfCtl), hipHostMallocDefault));
    for (hipEvent_t& e : c->wf_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const size_t rad_need = (size_t)(chunk_px * spp * 3 * sizeof(double));
  if (rad_need > c->wf_rad_bytes) {
    int rq = quiesce(c);
    if (rq) return rq;
    dev_free(c->wf_rad);
    c->wf_rad = nullptr;
    c->wf_rad_bytes = 0;
    HIP_TRY((hipError_t)dev_alloc(&c->wf_rad, rad_need));
    c->wf_rad_bytes = rad_need;
  }
  WfParams p;
  memset(&p, 0, sizeof p);
  p.g = Geo{kp.spheres, kp.tris, kp.boxes, kp.bvh, kp.ns, kp.nt, kp.use_bvh, kp.nb};
  p.jump = kp.jump;
  p.list_tries = c->tun.wf_list_tries > 0 ? std::min(64, c->tun.wf_list_tries) : 64;
  p.qbvh = c->d_qbvh;
  memcpy(p.q0, f.q0, sizeof p.q0);
  memcpy(p.qd, f.qd, sizeof p.qd);
  p.mats = kp.mats;
  p.lights = kp.lights;
  p.sky = kp.sky;
  p.nl = nl;
  p.max_depth = kp.max_depth;
  p.recursive = kp.recursive;
  p.soft = kp.soft;
  p.spp = st->samples;  // (0: the mean is 0/0 = NaN, as DivScalar(0) in Go)
  p.W = kp.W;
  p.H = kp.H;
  p.rank = kp.rank;
  p.world = kp.world;
  p.tiles_x = kp.tiles_x;
  p.ntiles = kp.ntiles;
  p.layout = kp.layout;
  p.tile_list = dev_tiles(c, kp.W, kp.H, kp.rank, kp.world);
  // a lane holds at most one pending child per internal node above its leaf:
  // depth - 1 entries (leaves at level bvh_depth, the root at level 1)
  p.stack_depth = std::max(1, f.bvh_depth - 1);
  // traversal workgroups: trav_block threads (64..1024), LDS shared by
  // trav_wgs of them per CU (tuning; default one of 1024)
  const rt_tuning& tn = c->tun;
  p.trav_block = kWfTravBlock;
  int trav_wgs = 1;
  if (tn.wf_trav_block > 0) p.trav_block = std::max(1, std::min(16, tn.wf_trav_block / 64)) * 64;
  if (tn.wf_trav_wgs > 0) trav_wgs = std::min(32, tn.wf_trav_wgs);
  p.bvh_nodes = (int)f.qbvh.size();
  p.lds_nodes = wf_lds_nodes(p.stack_depth, (int)f.qbvh.size(), p.trav_block, trav_wgs);
  if (tn.wf_lds_nodes >= 0)  // stage fewer nodes (an odd count: child pairs never split)
    p.lds_nodes = std::min(p.lds_nodes, tn.wf_lds_nodes | 1);
  // the occlusion kernels' 4-wide tree, where it fits the LDS whole beside
  // its stacks (C4: 4,801 slots and 20 stack entries, 157 KB at 1024
  // threads).  RTGO_BVH4=0 (measurement switch) keeps the binary walk.
  p.qbvh4 = c->d_qbvh4;
  p.nodes4 = (int)f.qbvh4.size();
  p.stack4 = std::max(1, f.bvh4_stack);
  p.root4 = f.bvh4_root;
  {
    const char* e4 = getenv("RTGO_BVH4");
    p.use4 = !(e4 && atoi(e4) == 0) && p.nodes4 > 0 && tn.wf_lds_nodes < 0 &&
             wf_lds_nodes(p.stack4, p.nodes4, p.trav_block, trav_wgs) >= p.nodes4;
  }
  p.shard_cap = shard_cap;
  p.hard_cap = (int64_t)qcap;
  p.soft_cap = (int64_t)qcap * 16;
  memcpy(p.cam, kp.cam, sizeof p.cam);
  p.aspect = kp.aspect;
  p.seed_key = kp.seed_key;
  p.ctl = c->wf_ctl;
  p.counts = kp.counts;
  p.out_linear = kp.out_linear;
  p.out_rgba = kp.out_rgba;
  p.rad = (double*)c->wf_rad;
  {
    char* m = (char*)c->wf_mem;
    auto take = [&](size_t bytes) {
      char* r = m;
      m += (bytes + 255) & ~size_t(255);
      return (void*)r;
    };
    for (WfPaths* a : {&p.cur, &p.next}) {
      double** dd[12] = {&a->ox, &a->oy, &a->oz, &a->dx, &a->dy, &a->dz,
                         &a->tx, &a->ty, &a->tz, &a->lx, &a->ly, &a->lz};
      for (double** q : dd) *q = (double*)take(cap * sizeof(double));
      a->rng = (uint64_t*)take(cap * sizeof(uint64_t));
      a->sid = (uint32_t*)take(cap * sizeof(uint32_t));
      a->depth = (int32_t*)take(cap * sizeof(int32_t));
    }
    double** hh[3] = {&p.px, &p.py, &p.pz};
    for (double** q : hh) *q = (double*)take(cap * sizeof(double));
    p.hidx = (int32_t*)take(cap * sizeof(int32_t));
    p.lstate = (uint32_t*)take(cap * nlk * sizeof(uint32_t));
    p.hardq = (uint32_t*)take((size_t)kWfShards * qcap * sizeof(uint32_t));
    p.softq = (uint32_t*)take((size_t)kWfShards * qcap * 16 * 4 * sizeof(uint32_t));
    p.coneq = (uint32_t*)take((size_t)kWfShards * qcap * sizeof(uint32_t));
    p.cand = (int32_t*)take(cap * nlk * kWfConeWide * sizeof(int32_t));
    p.wide_cap = (int64_t)qcap * 2;
    p.wideq = (uint32_t*)take((size_t)kWfShards * qcap * 2 * 4 * sizeof(uint32_t));
    if ((size_t)(m - (char*)c->wf_mem) > c->wf_mem_bytes) {
      set_error("wavefront buffer layout overflow");
      return RT_E_NOMEM;
    }
  }
  auto fail = [&](int e, const char* what) {
    set_error(std::string("wavefront ") + what + " failed: " + hipGetErrorString((hipError_t)e));
    return RT_E_DEVICE;
  };
  for (uint64_t lp0 = 0; lp0 < local_px; lp0 += chunk_px) {
    const uint64_t npx = std::min(chunk_px, local_px - lp0);
    p.lp0 = (uint32_t)lp0;
    const uint64_t total = npx * (uint64_t)st->samples;
    HIP_TRY(hipMemsetAsync(p.rad, 0, (size_t)(npx * spp * 3 * sizeof(double)), s));
    if (total > 0) {
      WfCtl init;
      memset(&init, 0, sizeof init);
      init.total = total;
      HIP_TRY(hipMemcpyAsync(c->wf_ctl, &init, sizeof init, hipMemcpyHostToDevice, s));
      // the first samples, then bounces until every sample has finished; the
      // host reads the loop state one bounce behind the GPU
      p.live_bound = (int32_t)cap;
      p.dry = 0;
      int e = wf_launch_bounce(p, true, count, s, prof_block(c, kWfRegen, kWfRegen));
      if (e) return fail(e, "launch");
      std::swap(p.cur, p.next);
      const long long max_iter = (long long)total + std::max(kp.max_depth, 0) + 8;
      for (long long it = 0;; ++it) {
        if (it > max_iter) {
          set_error("wavefront loop did not terminate");
          return RT_E_DEVICE;
        }
        e = wf_launch_bounce(p, false, count, s, prof_block(c, kWfExtend, kWfRegen));
        if (e) return fail(e, "launch");
        std::swap(p.cur, p.next);
        const int r = (int)(it % kWfRing);
        HIP_TRY(hipMemcpyAsync(c->wf_host + r, c->wf_ctl, sizeof(WfCtl), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipEventRecord(c->wf_ev[r], s));
        if (it >= 1) {
          const int pr = (int)((it - 1) % kWfRing);
          const int rw = wait_event(c, c->wf_ev[pr]);  // (bounded under a renderer's deadline)
          if (rw) return rw;
          const WfCtl& h = c->wf_host[pr];
          if (h.live == 0 && h.dry) break;  // bounce `it` had nothing to do
          // once dry, live counts only fall: bounce it + 1 has at most h.live paths
          if (h.dry) {
            p.live_bound = h.live;
            p.dry = 1;
          }
        }
      }
    }
    hipEvent_t* rev = prof_block(c, kWfResolve, kWfResolve);
    if (rev) HIP_TRY(hipEventRecord(rev[kWfResolve], s));
    int e = wf_launch_resolve(p, (int)npx, s);
    if (e) return fail(e, "resolve launch");
    if (rev) HIP_TRY(hipEventRecord(rev[kWfResolve + 1], s));
  }
  return RT_OK;
}

// One frame (rt_context_render_async).  key_frames: the frames per launch
// whose schedule this frame uses -- 1 for a frame of its own; n when it is
// one of n frames that rt_context_render_frames_async renders one at a time
// (a measuring frame): the schedule key then stays the batched launch's, so
// the measured re-cut is the one the next batched launch reuses.
static int render_one(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t rank, int32_t world,
                      int32_t layout, float* d_linear, uint8_t* d_rgba, void* stream, rt_counts* counts,
                      int key_frames);

int rt_context_render_async(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t rank,
                            int32_t world, int32_t layout, float* d_linear, uint8_t* d_rgba, void* stream,
                            rt_counts* counts) {
  return render_one(c, w, h, st, rank, world, layout, d_linear, d_rgba, stream, counts, 1);
}

static int render_one(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t rank, int32_t world,
                      int32_t layout, float* d_linear, uint8_t* d_rgba, void* stream, rt_counts* counts,
                      int key_frames) {
  if (!c || !c->have_scene) {
    set_error("context has no scene");
    return RT_E_INVALID;
  }
  int rc = validate_settings(st, w, h);
  if (rc) return rc;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid rank/world");
    return RT_E_INVALID;
  }
  if (layout != RT_LAYOUT_IMAGE && layout != RT_LAYOUT_PACKED_TILES) {
    set_error("invalid layout");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  KParams p;
  base_params(c, w, h, st, rank, world, layout, &p);
  p.out_linear = d_linear;
  p.out_rgba = d_rgba;
  if (counts && !c->d_counts) HIP_TRY((hipError_t)dev_alloc((void**)&c->d_counts, kCountSlots * sizeof(unsigned long long)));
  p.counts = counts ? c->d_counts : nullptr;
  // the caller's stream, as given (NULL = the legacy default stream); a
  // render enqueued on another stream than this context's last one waits for
  // that one first (they share the split rows and the wavefront state)
  hipStream_t s = (hipStream_t)stream;
  if (c->have_timing && s != c->last_stream) HIP_TRY(hipStreamWaitEvent(s, c->ev1, 0));
  const bool wf = use_wavefront(c);
  // The megakernel holds at most kMaxBlockSamples samples of a pixel in one
  // block: more samples per pixel render as consecutive SAMPLE PASSES of at
  // most that many, each continuing every pixel's running sum in sample
  // order (KParams.acc), so the sum is tracePixel's bit for bit.
  const int spp = st->samples;
  const int npass = wf ? 1 : std::max(1, (spp + kMaxBlockSamples - 1) / kMaxBlockSamples);
  p.spp_total = spp;
  if (npass > 1) {
    rc = grow(c, &c->d_acc, &c->acc_cap, (size_t)local_tiles(c, w, h, rank, world) * 1024 * 3 * sizeof(double));
    if (rc) return rc;
    p.acc = (double*)c->d_acc;
  }
  unsigned long long total[kCountSlots] = {0};
  bool measuring = false;
  for (int pass = 0; pass < npass; ++pass) {
    rt_settings ps = *st;
    const int s0 = (int)((long long)spp * pass / npass), s1 = (int)((long long)spp * (pass + 1) / npass);
    ps.samples = s1 - s0;
    p.spp = ps.samples;
    p.sample_base = s0;
    p.acc_mode = npass > 1 ? ((pass > 0 ? 1 : 0) | (pass < npass - 1 ? 2 : 0)) : 0;
    if (!wf) {
      rc = prepare_schedule(c, &p, &ps, s, key_frames);
      if (rc) return rc;
    }
    p.num_wgs = p.num_blocks;
    // the first frame of a new schedule measures every pixel's paths (the same
    // image; a separate instantiation records the lengths): the next frame's
    // blocks are cut from them (prepare_schedule)
    if (!wf && npass == 1 && c->meas_state == 1 && !counts && st->sky == RT_SKY_NONE && p.num_blocks > 0) {
      const size_t npx = (size_t)local_tiles(c, w, h, rank, world) * 1024;
      rc = grow(c, &c->d_meas, &c->meas_cap, npx * 8);
      if (rc) return rc;
      p.work_max = (unsigned int*)c->d_meas;
      p.work_sum = p.work_max + npx;
      measuring = true;
    }
    if (counts) HIP_TRY(hipMemsetAsync(c->d_counts, 0, kCountSlots * sizeof(unsigned long long), s));
    if (measuring) HIP_TRY(hipMemsetAsync(c->d_meas, 0, (size_t)local_tiles(c, w, h, rank, world) * 1024 * 8, s));
    if (pass == 0) HIP_TRY(hipEventRecord(c->ev0, s));
    if (wf) {
      rc = render_wavefront(c, p, st, s, counts != nullptr);
      if (rc) return rc;
    } else {
      if (npass == 1 && !counts) {
        rc = setup_tail(c, &p, s);
        if (rc) return rc;
      }
      int e = launch_render(p, counts != nullptr, s);
      if (e != hipSuccess) {
        set_error(std::string("render launch failed: ") + hipGetErrorString((hipError_t)e));
        return RT_E_DEVICE;
      }
    }
    if (counts) {
      unsigned long long h_c[kCountSlots];
      HIP_TRY(hipMemcpyAsync(h_c, c->d_counts, sizeof h_c, hipMemcpyDeviceToHost, s));
      HIP_TRY(hipStreamSynchronize(s));
      for (int i = 0; i < kCountSlots; ++i) total[i] += h_c[i];
    }
  }
  HIP_TRY(hipEventRecord(c->ev1, s));
  if (measuring) {
    c->meas_state = 2;
    c->stats.measuring_frames += 1;
  }
  c->stats.frames += 1;
  c->stats.launches += npass;
  c->last_stream = s;
  c->have_timing = true;
  if (counts) {
    const unsigned long long* h_c = total;
    counts->camera_rays = h_c[0];
    counts->bounce_rays = h_c[1];
    counts->shadow_rays = h_c[2];
    counts->sphere_tests = h_c[3];
    counts->triangle_tests = h_c[4];
    counts->box_tests = h_c[5];
    counts->shade_events = h_c[6];
    counts->light_evals = h_c[7];
    counts->rng_draws = h_c[8];
    for (int i = 0; i < kCounters; ++i) {
      counts->culled[i] = h_c[kCounters + i];
      counts->soft_occlusion[i] = h_c[kGroupSoft * kCounters + i];
      counts->extend[i] = h_c[kGroupExtend * kCounters + i];
      counts->hard_occlusion[i] = h_c[kGroupHard * kCounters + i];
    }
  }
  return RT_OK;
}

// ------------------------------------------------------------ partitions
int rt_context_set_partition(rt_context* c, const rt_partition* p) {
  if (!c) {
    set_error("context is NULL");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc = quiesce(c);  // the last render may still read the tile lists
  if (rc) return rc;
  if (!p) {
    c->part.reset();
    return RT_OK;
  }
  auto d = std::make_shared<const PartitionData>(partition_data(p));
  rc = grow(c, &c->d_part, &c->d_part_cap, std::max<size_t>(d->lists.size(), 1) * sizeof(int32_t));
  if (rc) return rc;
  if (!d->lists.empty())
    HIP_TRY(hipMemcpy(c->d_part, d->lists.data(), d->lists.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  c->part = std::move(d);
  return RT_OK;
}

// Balanced partition (include/rt_api.h): a one-sample pilot of the whole
// frame (the schedule's pilot, prepare_schedule, over all tiles as one rank),
// each tile's estimated work (spp x the sum of its pixels' estimates,
// sched_tile_work), then longest-processing-time-first: tiles by decreasing
// work (ties: lower tile first) to the least loaded rank (ties: lower rank).
// The measured work of every tile of the frame (r04): the frame rendered
// once at its full sample count through the context's own (one-rank)
// schedule, with the measuring instantiation recording every sample's path
// length; a tile weighs the sum of its pixels' mean path lengths x spp.  The
// one-sample pilot's estimate (the neighbourhood's longest path, which the
// block cutting wants) misjudges whole tiles: with it the slowest of 8 ranks
// of the headline frame took 1.22x the mean share.  Path lengths are
// integers of an exact render, so every rank that measures the same frame on
// its own device derives the same partition.  (r05) measure_spp < spp: the
// measuring render takes only the frame's first measure_spp samples of every
// pixel; a tile weighs its pixels' mean path length over them x spp.  The
// renderer (rt_renderer_render) plans its partition that way with 16
// samples, because its first Render -- and every one-shot rt_render with
// num_devices > 1 -- pays this render before its own frame (at
// the full 100 samples it cost a whole one-GPU frame); the public
// rt_partition_balanced, which a caller plans once for many frames, measures
// every sample (8 ranks of the headline frame, rank shares alone on one GPU:
// predicted 874 k Mrays/s with all 100 samples, 853 k with 16, 815 k with the
// one-sample pilot; profiles/r04_rank_share_probe.json, r05_rank_share_probe.json).
static int measured_tile_work(rt_context* c, int w, int h, const rt_settings* st, int measure_spp,
                              std::vector<float>* work) {
  hipStream_t s = c->stream;
  rt_settings sm = *st;
  sm.samples = std::min(st->samples, measure_spp);
  KParams p;
  base_params(c, w, h, &sm, 0, 1, RT_LAYOUT_PACKED_TILES, &p);
  p.spp = sm.samples;
  p.spp_total = sm.samples;
  p.sample_base = 0;
  p.acc_mode = 0;
  p.acc = nullptr;
  p.counts = nullptr;
  int rc = prepare_schedule(c, &p, &sm, s);
  if (rc) return rc;
  p.num_wgs = p.num_blocks;
  const int ntiles = rt_num_tiles(w, h);
  const size_t npx = (size_t)ntiles * 1024;
  std::vector<int32_t> tiles;
  strided_tiles(w, h, 0, 1, &tiles);
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t o_meas = al(npx * 16);  // [linear | rgba] image, packed tiles
  const size_t o_sched = o_meas + al(npx * 8);
  const size_t o_tw = o_sched + al(sched_scratch_bytes(ntiles));
  const size_t total = o_tw + al((size_t)ntiles * sizeof(float));
  char* buf = nullptr;
  HIP_TRY((hipError_t)dev_alloc((void**)&buf, total));
  auto done = [&](int code) {
    (void)hipStreamSynchronize(s);
    dev_free(buf);
    return code;
  };
  p.out_linear = (float*)buf;
  p.out_rgba = (uint8_t*)(buf + npx * 12);
  unsigned int* meas = (unsigned int*)(buf + o_meas);
  p.work_max = meas;
  p.work_sum = meas + npx;
  if (hipMemsetAsync(meas, 0, npx * 8, s) != hipSuccess) return done(RT_E_DEVICE);
  if (p.num_blocks > 0) {
    const int e = launch_render(p, false, s);
    if (e != hipSuccess) {
      set_error(std::string("partition measuring launch failed: ") + hipGetErrorString((hipError_t)e));
      return done(RT_E_DEVICE);
    }
  }
  SchedParams sp = sched_params(c, p, st, tiles, nullptr, false, false, default_block_work(c),
                                big_block_pixels(st->samples, c->tun), buf + o_sched, nullptr, nullptr);
  sp.work_max = meas;
  sp.work_sum = meas + npx;
  sp.work_n = sm.samples;
  sp.work_mean = 1;          // (the measured samples' mean, times the frame's spp)
  sp.split_depth = 1 << 30;  // (weights only: no pixel is marked heavy)
  float* d_tw = (float*)(buf + o_tw);
  int e = sched_launch_tile_work(sp, d_tw, s);
  if (e == hipSuccess) e = hipMemcpyAsync(work->data(), d_tw, (size_t)ntiles * sizeof(float), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    set_error(std::string("partition measurement failed: ") + hipGetErrorString((hipError_t)e));
    return done(RT_E_DEVICE);
  }
  return done(RT_OK);
}

static int partition_balanced_impl(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t world,
                                   int measure_spp, rt_partition** out);

int rt_partition_balanced(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t world,
                          rt_partition** out) {
  return partition_balanced_impl(c, w, h, st, world, st ? st->samples : 0, out);
}

static int partition_balanced_impl(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t world,
                                   int measure_spp, rt_partition** out) {
  if (!c || !c->have_scene || !out) {
    set_error("rt_partition_balanced: context without a scene, or out is NULL");
    return RT_E_INVALID;
  }
  *out = nullptr;
  int rc = validate_settings(st, w, h);
  if (rc) return rc;
  if (world < 1 || world > 65536) {
    set_error("rt_partition_balanced: world must be in [1, 65536]");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  const FlatScene& f = c->flat;
  const rt_tuning& tn = c->tun;
  hipStream_t s = c->stream;
  const int ntiles = rt_num_tiles(w, h);
  if (tn.pilot != 0 && !use_wavefront(c) && st->sky == RT_SKY_NONE && st->samples > 0 &&
      st->samples <= kMaxBlockSamples && st->max_depth > 0) {
    std::vector<float> work(ntiles, 0.0f);
    rc = measured_tile_work(c, w, h, st, std::max(1, measure_spp), &work);
    if (rc) return rc;
    PartitionData d;
    d.w = w;
    d.h = h;
    d.world = world;
    lpt_partition(work, &d);
    finish_partition(&d);
    *out = make_partition(std::move(d));
    return RT_OK;
  }
  std::vector<int32_t> tiles;
  strided_tiles(w, h, 0, 1, &tiles);
  KParams p;
  base_params(c, w, h, st, 0, 1, RT_LAYOUT_PACKED_TILES, &p);
  const bool masks = masks_apply(f);
  const bool frustum = tn.frustum != 0 && st->sky == RT_SKY_NONE;
  std::vector<unsigned long long> mh;
  if (masks) tile_primary_masks(f, w, h, tiles, &mh);
  std::vector<float> cost;
  tile_cost(f, w, h, tiles, &cost);
  auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t npx = (size_t)ntiles * 1024;
  const size_t o_in = al(sched_scratch_bytes(ntiles));
  const size_t o_cost = o_in + al(mh.size() * sizeof(unsigned long long));
  const size_t o_pilot = o_cost + al(cost.size() * sizeof(float));
  const size_t o_tw = o_pilot + al(npx * 24);
  const size_t total = o_tw + al((size_t)ntiles * sizeof(float));
  char* buf = nullptr;
  HIP_TRY((hipError_t)dev_alloc((void**)&buf, total));
  auto fail = [&](int code) {
    (void)hipStreamSynchronize(s);
    dev_free(buf);
    return code;
  };
  std::vector<float> work(ntiles, 0.0f);
  {
    unsigned long long* d_masks = masks ? (unsigned long long*)(buf + o_in) : nullptr;
    float* d_cost = (float*)(buf + o_cost);
    float* d_tw = (float*)(buf + o_tw);
    if (!mh.empty() &&
        hipMemcpyAsync(d_masks, mh.data(), mh.size() * sizeof(unsigned long long), hipMemcpyHostToDevice, s))
      return fail(RT_E_DEVICE);
    if (!cost.empty() && hipMemcpyAsync(d_cost, cost.data(), cost.size() * sizeof(float), hipMemcpyHostToDevice, s))
      return fail(RT_E_DEVICE);
    SchedParams sp = sched_params(c, p, st, tiles, nullptr, masks, frustum, default_block_work(c),
                                  big_block_pixels(st->samples, tn), buf, d_masks, d_cost);
    int e = sched_launch_pixels(sp, s);
    if (e != hipSuccess) {
      set_error(std::string("partition pilot launch failed: ") + hipGetErrorString((hipError_t)e));
      return fail(RT_E_DEVICE);
    }
    if (tn.pilot != 0 && st->samples > 0 && st->max_depth > 0) {
      rc = run_pilot(c, p, &sp, buf + o_pilot, s);
      if (rc) return fail(rc);
    }
    e = sched_launch_tile_work(sp, d_tw, s);
    if (e != hipSuccess) {
      set_error(std::string("partition estimate launch failed: ") + hipGetErrorString((hipError_t)e));
      return fail(RT_E_DEVICE);
    }
    if (hipMemcpyAsync(work.data(), d_tw, (size_t)ntiles * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      set_error("partition estimate read-back failed");
      return fail(RT_E_DEVICE);
    }
  }
  (void)fail(RT_OK);
  PartitionData d;
  d.w = w;
  d.h = h;
  d.world = world;
  lpt_partition(work, &d);
  finish_partition(&d);
  *out = make_partition(std::move(d));
  return RT_OK;
}

int rt_context_profile(rt_context* c, int32_t on) {
  if (!c) {
    set_error("context is NULL");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc = prof_collect(c);
  if (rc) return rc;
  c->prof_on = on != 0;
  for (int k = 0; k < kWfClasses; ++k) {
    c->prof_secs[k] = 0;
    c->prof_launches[k] = 0;
  }
  return RT_OK;
}

int rt_context_kernel_seconds(rt_context* c, double* seconds, int64_t* launches) {
  if (!c || !seconds) {
    set_error("context or seconds is NULL");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc = prof_collect(c);
  if (rc) return rc;
  for (int k = 0; k < kWfClasses; ++k) {
    seconds[k] = c->prof_secs[k];
    if (launches) launches[k] = c->prof_launches[k];
  }
  return RT_OK;
}

// Several frames of one schedule in ONE launch (include/rt_api.h).
int rt_context_render_frames_async(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t nframes,
                                   const uint64_t* seeds, int32_t rank, int32_t world, int32_t layout,
                                   float* const* d_linear, uint8_t* const* d_rgba, void* stream) {
  if (!c || !c->have_scene) {
    set_error("context has no scene");
    return RT_E_INVALID;
  }
  if (nframes < 1 || nframes > RT_MAX_FRAMES || !seeds || !d_linear) {
    set_error("rt_context_render_frames_async: nframes must be in [1, RT_MAX_FRAMES] with seeds and d_linear given");
    return RT_E_INVALID;
  }
  int rc = validate_settings(st, w, h);
  if (rc) return rc;
  if (world < 1 || rank < 0 || rank >= world) {
    set_error("invalid rank/world");
    return RT_E_INVALID;
  }
  if (layout != RT_LAYOUT_IMAGE && layout != RT_LAYOUT_PACKED_TILES) {
    set_error("invalid layout");
    return RT_E_INVALID;
  }
  // one frame at a time where a launch cannot hold several: the wavefront
  // path (host-driven bounce loop), sample passes, a measuring frame
  const int npass = std::max(1, (st->samples + kMaxBlockSamples - 1) / kMaxBlockSamples);
  // (frame by frame under the batched launch's schedule key: a measuring
  // frame then measures the schedule the next batched launch uses)
  auto one_by_one = [&]() {
    for (int f = 0; f < nframes; ++f) {
      rt_settings sf = *st;
      sf.seed = seeds[f];
      int r = render_one(c, w, h, &sf, rank, world, layout, d_linear[f], d_rgba ? d_rgba[f] : nullptr, stream,
                         nullptr, nframes);
      if (r) return r;
    }
    return (int)RT_OK;
  };
  if (nframes == 1 || use_wavefront(c) || npass > 1 || (c->tun.measure && c->meas_state != 3)) return one_by_one();
  HIP_TRY(hipSetDevice(c->device));
  KParams p;
  base_params(c, w, h, st, rank, world, layout, &p);
  hipStream_t s = (hipStream_t)stream;
  if (c->have_timing && s != c->last_stream) HIP_TRY(hipStreamWaitEvent(s, c->ev1, 0));
  rc = prepare_schedule(c, &p, st, s, nframes);
  if (rc) return rc;
  // a new schedule key whose first frame is to measure (rt_tuning.measure):
  // that frame goes through the single-frame path, which records the paths
  if (c->tun.measure && c->meas_state == 1) return one_by_one();
  p.spp_total = st->samples;
  p.nframes = nframes;
  for (int f = 0; f < nframes; ++f) {
    p.frame_key[f] = rt_rng_seed_key(seeds[f]);
    p.frame_lin[f] = d_linear[f];
    p.frame_rgba[f] = d_rgba ? d_rgba[f] : nullptr;
  }
  p.num_wgs = p.num_blocks * nframes;
  rc = setup_tail(c, &p, s);
  if (rc) return rc;
  HIP_TRY(hipEventRecord(c->ev0, s));
  const int e = launch_render(p, false, s);
  if (e != hipSuccess) {
    set_error(std::string("render launch failed: ") + hipGetErrorString((hipError_t)e));
    return RT_E_DEVICE;
  }
  HIP_TRY(hipEventRecord(c->ev1, s));
  c->last_stream = s;
  c->have_timing = true;
  c->stats.frames += nframes;
  c->stats.launches += 1;
  c->stats.batched_launches += 1;
  return RT_OK;
}

int rt_context_get_stats(const rt_context* c, rt_context_stats* out) {
  if (!c || !out) {
    set_error("context or out is NULL");
    return RT_E_INVALID;
  }
  *out = c->stats;
  out->blocks = c->num_blocks;
  out->split_pixels = c->nsplit;
  out->tail_exported = out->tail_errors = 0;
  if (c->d_tail) {
    rt_context* m = const_cast<rt_context*>(c);
    int rc = quiesce(m);
    if (rc) return rc;
    TailCtl h;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy(&h, c->d_tail, sizeof h, hipMemcpyDeviceToHost));
    out->tail_exported = h.exported;
    out->tail_errors = h.err;
  }
  return RT_OK;
}

int rt_context_tail_debug(const rt_context* c, uint64_t out[6]) {
  if (!c || !out) {
    set_error("context or out is NULL");
    return RT_E_INVALID;
  }
  for (int i = 0; i < 6; ++i) out[i] = 0;
  if (!c->d_tail) return RT_OK;
  rt_context* m = const_cast<rt_context*>(c);
  int rc = quiesce(m);
  if (rc) return rc;
  TailCtl h;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpy(&h, c->d_tail, sizeof h, hipMemcpyDeviceToHost));
  out[0] = h.exported;
  out[1] = h.paths_done;
  out[2] = h.solo_ticks;
  out[3] = h.export_ticks;
  out[4] = h.helper_ticks;
  out[5] = h.err;
  return RT_OK;
}

int rt_context_set_debug_buffer(rt_context* c, void* d_buf) {
  if (!c) {
    set_error("context is NULL");
    return RT_E_INVALID;
  }
  c->dbg = (unsigned long long*)d_buf;
  return RT_OK;
}

int rt_context_last_kernel_seconds(rt_context* c, double* seconds) {
  if (!c || !seconds || !c->have_timing) {
    set_error("no timed launch on this context");
    return RT_E_INVALID;
  }
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(c->ev1));
  float ms = 0;
  HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  *seconds = ms * 1e-3;
  return RT_OK;
}

}  // extern "C"

int rtgo::partition_balanced(rt_context* c, int32_t w, int32_t h, const rt_settings* st, int32_t world,
                             int measure_spp, rt_partition** out) {
  return partition_balanced_impl(c, w, h, st, world, measure_spp, out);
}
