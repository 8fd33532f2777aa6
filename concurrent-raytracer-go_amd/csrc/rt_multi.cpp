// rt_multi.cpp — the multi-GPU side of the C ABI (include/rt_api.h):
// the persistent renderer (rt_renderer_*, one process driving N devices),
// the one-shot rt_render on top of it, and the RCCL tile gather for
// one-process-per-GPU runs (rt_comm_*).
//
// Reference: (*ParallelRenderer).Render fans 32x32 tiles out to goroutines
// and collects their pixels on the main goroutine (renderer.go:67-126,
// createRenderTasks :398-436).  Here tiles t are dealt to ranks t % N (one
// rank per GPU), every rank renders its share into a packed buffer (float3
// + RGBA8, 16 B per pixel, rt_packed_bytes), and the shares meet on the
// first device in ONE RCCL send/recv group over xGMI, where one kernel
// scatters them into the image.  The random stream is keyed
// by global pixel and sample, so the image is the same for every N.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <utility>
#include <vector>

#include "rt_internal.h"

using namespace rtgo;

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) {                                                             \
      set_error(std::string(#expr) + " failed: " + hipGetErrorString(e_));             \
      return RT_E_DEVICE;                                                               \
    }                                                                                   \
  } while (0)

#define NCCL_TRY(expr)                                                                  \
  do {                                                                                  \
    ncclResult_t e_ = (expr);                                                           \
    if (e_ != ncclSuccess) {                                                            \
      set_error(std::string(#expr) + " failed: " + ncclGetErrorString(e_));            \
      return RT_E_DEVICE;                                                               \
    }                                                                                   \
  } while (0)

// Inside ncclGroupStart / ncclGroupEnd: the first failing call is recorded
// and the rest are skipped, but the group is always closed, so a failure
// leaves the communicator usable (NCCL_TRY would return with the group open).
#define NCCL_GROUP_TRY(err, expr)                                                       \
  do {                                                                                  \
    if ((err) == ncclSuccess) {                                                         \
      (err) = (expr);                                                                   \
      if ((err) != ncclSuccess) set_error(std::string(#expr) + " failed: " + ncclGetErrorString(err)); \
    }                                                                                   \
  } while (0)

namespace {

struct Rank {
  int device = 0;
  int comm_idx = 0;             // index of its device in the distinct-device list (0: the root device)
  rt_context* ctx = nullptr;
  hipStream_t stream = nullptr;  // its context's own stream
  hipEvent_t done = nullptr;    // its share is rendered
  void* share = nullptr;        // its own share buffer (devices other than the root's)
  size_t share_cap = 0;
};

// Device buffer that grows on demand.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int grow(int device, size_t bytes) {
    if (bytes <= cap) return RT_OK;
    HIP_TRY(hipSetDevice(device));
    dev_free(p);
    p = nullptr;
    cap = 0;
    HIP_TRY((hipError_t)dev_alloc(&p, bytes));
    cap = bytes;
    return RT_OK;
  }
  void release(int device) {
    if (p) {
      (void)hipSetDevice(device);
      dev_free(p);
    }
    p = nullptr;
    cap = 0;
  }
};

// The scene's content as bytes, field by field (padding is left out: caller
// padding that differs must not force a re-upload): two calls with equal
// bytes render the same image, so the second one re-uploads nothing.
void scene_bytes(const rt_scene& s, std::vector<uint8_t>* out) {
  out->clear();
  auto put = [&](const void* p, size_t n) {
    const uint8_t* b = (const uint8_t*)p;
    out->insert(out->end(), b, b + n);
  };
  const rt_camera& c = s.camera;
  put(c.position, sizeof c.position);
  put(c.look_at, sizeof c.look_at);
  put(c.up, sizeof c.up);
  put(&c.fov, sizeof c.fov);
  put(&c.aspect_ratio, sizeof c.aspect_ratio);
  put(&s.num_objects, sizeof s.num_objects);
  put(&s.num_lights, sizeof s.num_lights);
  for (int i = 0; i < s.num_objects; ++i) {
    const rt_object& o = s.objects[i];
    put(&o.type, sizeof o.type);
    put(o.position, sizeof o.position);
    put(o.size, sizeof o.size);
    put(&o.radius, sizeof o.radius);
    const rt_material& m = o.material;
    put(&m.kind, sizeof m.kind);
    put(m.color, sizeof m.color);
    put(&m.roughness, sizeof m.roughness);
    put(&m.metallic, sizeof m.metallic);
    put(&m.specular, sizeof m.specular);
    put(&m.refraction_index, sizeof m.refraction_index);
  }
  if (s.num_lights > 0) put(s.lights, sizeof(rt_light) * (size_t)s.num_lights);  // (no padding)
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct rt_partition {
  PartitionData d;
  std::mutex mu;
  std::vector<std::pair<int, int32_t*>> slots;  // per device: {owner, local tile} per global tile (unpack)
};

namespace rtgo {

rt_partition* make_partition(PartitionData&& d) {
  rt_partition* p = new rt_partition();
  p->d = std::move(d);
  return p;
}

const PartitionData& partition_data(const rt_partition* p) { return p->d; }

}  // namespace rtgo

struct rt_renderer {
  std::vector<Rank> ranks;
  std::vector<int> devices;        // distinct devices, the root's first
  std::vector<ncclComm_t> comms;   // one per distinct device (empty when there is one)
  std::vector<hipStream_t> comm_streams;  // per distinct device: the stream of its first rank
  DevBuf gathered;                 // root: [world][share bytes]
  DevBuf img_lin, img_rgba;        // root: the W*H image
  std::vector<uint8_t> scene_key;  // content of the scene the contexts hold
  bool have_scene = false;
  uint64_t scene_gen = 0;          // bumped per upload
  rt_tuning tun;
  // the partition of the last multi-rank frame and its key (scene, frame, settings)
  rt_partition* part = nullptr;
  std::vector<int64_t> part_key;
  std::vector<double> rank_secs;   // device seconds of each rank's last render
  // the first Render's image download: pinned staging written by a kernel
  // (launch_download), made by the constructor
  void* h_img = nullptr;
  size_t h_img_cap = 0;
  int64_t frames = 0;              // Render calls so far
  double watchdog_s = 0;           // bound on a multi-rank frame (rt_renderer_set_watchdog; 0: none, as Go's Render)
  std::string stalled;             // set when the watchdog fired: the renderer is unusable
  int stall_rank = -1;             // test hook (rt_renderer_test_stall)
  double stall_ms = 0;
};

struct rt_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1, device = 0;
};

namespace {

// Waits until stream s (of `device`) is idle or `deadline` (now_s() clock,
// <= 0: none) passes: RT_OK, RT_E_TIMEOUT, or RT_E_DEVICE.  Polls the
// stream (yield, then 20 us sleeps), so a collective that never completes
// leaves the caller in control instead of in hipStreamSynchronize forever.
int bounded_sync(int device, hipStream_t s, double deadline) {
  HIP_TRY(hipSetDevice(device));
  if (deadline <= 0) {
    HIP_TRY(hipStreamSynchronize(s));
    return RT_OK;
  }
  for (unsigned spin = 0;; ++spin) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return RT_OK;
    if (e != hipErrorNotReady) {
      set_error(std::string("hipStreamQuery failed: ") + hipGetErrorString(e));
      return RT_E_DEVICE;
    }
    if (now_s() > deadline) return RT_E_TIMEOUT;
    if (spin < 256)
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// Test hook (rt_renderer_test_stall): the next frame's rank k stream first
// runs a kernel that sleeps for ms milliseconds of device time and then
// exits, so a short watchdog fires while every wave still ends on its own
// (tests/test_gpu_watchdog.py).  Armed for one frame.
void test_stall(rt_renderer* r, int n) {
  const int k = r->stall_rank;
  const double ms = r->stall_ms;
  r->stall_rank = -1;
  if (k < 0 || k >= n || ms <= 0) return;
  const Rank& q = r->ranks[k];
  if (hipSetDevice(q.device) == hipSuccess) (void)launch_spin(ms, q.stream);
}

int renderer_fail_cleanup(rt_renderer* r, int rc) {
  rt_renderer_destroy(r);
  return rc;
}

// Ranks on devices other than the root's send their shares; the root receives
// each into its slot of the gather buffer (one group, in rank order, so the
// sends and receives of one device pair match in order).
int group_gather(rt_renderer* r, size_t share_bytes) {
  const int n = (int)r->ranks.size();
  hipStream_t root_s = r->ranks[0].stream;
  for (int k = 1; k < n; ++k) {
    Rank& q = r->ranks[k];
    if (q.comm_idx == 0) continue;
    HIP_TRY(hipSetDevice(q.device));
    HIP_TRY(hipEventRecord(q.done, q.stream));
    HIP_TRY(hipStreamWaitEvent(r->comm_streams[q.comm_idx], q.done, 0));
  }
  NCCL_TRY(ncclGroupStart());
  ncclResult_t ge = ncclSuccess;
  for (int k = 1; k < n; ++k) {
    Rank& q = r->ranks[k];
    if (q.comm_idx == 0) continue;
    NCCL_GROUP_TRY(ge, ncclSend(q.share, share_bytes, ncclUint8, 0, r->comms[q.comm_idx], r->comm_streams[q.comm_idx]));
    NCCL_GROUP_TRY(ge, ncclRecv((uint8_t*)r->gathered.p + (size_t)k * share_bytes, share_bytes, ncclUint8,
                                q.comm_idx, r->comms[0], root_s));
  }
  const ncclResult_t ee = ncclGroupEnd();
  if (ge != ncclSuccess) return RT_E_DEVICE;
  NCCL_TRY(ee);
  return RT_OK;
}

// The tile partition of a multi-rank frame (rt_tuning.partition): balanced
// for linear-scan scenes by default, whose work sits in a few tiles (the
// headline scene: 23 of 475 tiles), strided for BVH scenes (thousands of
// busy tiles).  A balanced partition is planned on the first rank's device
// once per (scene, frame, settings) and set on every rank's context.
int renderer_partition(rt_renderer* r, const rt_scene* scene, int32_t w, int32_t h, const rt_settings* st) {
  const int n = (int)r->ranks.size();
  int mode = r->tun.partition;
  if (mode == RT_PARTITION_AUTO)
    mode = context_has_bvh(r->ranks[0].ctx) ? RT_PARTITION_STRIDED : RT_PARTITION_BALANCED;
  if (mode != RT_PARTITION_BALANCED) {
    if (r->part) {
      for (Rank& q : r->ranks) {
        int rc = rt_context_set_partition(q.ctx, nullptr);
        if (rc) return rc;
      }
      rt_partition_destroy(r->part);
      r->part = nullptr;
      r->part_key.clear();
    }
    return RT_OK;
  }
  const std::vector<int64_t> key = {(int64_t)r->scene_gen, w, h, n, st->samples, st->max_depth,
                                    st->recursive_reflections, st->soft_shadows, st->sky};
  if (r->part && key == r->part_key) return RT_OK;
  rt_partition* p = nullptr;
  int rc = partition_balanced(r->ranks[0].ctx, w, h, st, n, kRendererPartitionSpp, &p);
  if (rc) return rc;
  for (Rank& q : r->ranks) {
    rc = rt_context_set_partition(q.ctx, p);
    if (rc) {
      rt_partition_destroy(p);
      return rc;
    }
  }
  rt_partition_destroy(r->part);
  r->part = p;
  r->part_key = key;
  return RT_OK;
}

}  // namespace

extern "C" {

int32_t rt_max_local_tiles(int32_t w, int32_t h, int32_t world) { return rt_tiles_for_rank(w, h, 0, world); }

size_t rt_packed_bytes(int32_t w, int32_t h, int32_t world) {
  return (size_t)std::max(rt_max_local_tiles(w, h, world), 0) * 1024 * 16;
}

size_t rt_packed_rgba_offset(int32_t w, int32_t h, int32_t world) {
  return (size_t)std::max(rt_max_local_tiles(w, h, world), 0) * 1024 * 12;
}

int rt_unpack_tiles_async(int32_t w, int32_t h, int32_t world, const void* d_gathered, float* d_linear,
                          uint8_t* d_rgba, void* stream) {
  if (w <= 0 || h <= 0 || world < 1 || !d_gathered) {
    set_error("invalid unpack arguments");
    return RT_E_INVALID;
  }
  int e = launch_unpack(w, h, world, d_gathered, rt_packed_bytes(w, h, world), rt_packed_rgba_offset(w, h, world),
                        d_linear, d_rgba, stream);
  if (e != hipSuccess) {
    set_error(std::string("unpack launch failed: ") + hipGetErrorString((hipError_t)e));
    return RT_E_DEVICE;
  }
  return RT_OK;
}

int rt_renderer_create(const int32_t* devices, int32_t n, rt_renderer** out) {
  if (!out || n < 1 || n > 1024) {
    set_error("rt_renderer_create: out is NULL or num_devices not in [1, 1024]");
    return RT_E_INVALID;
  }
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  rt_renderer* r = new rt_renderer();
  rt_tuning_default(&r->tun);
  r->ranks.resize(n);
  for (int k = 0; k < n; ++k) {
    const int d = devices ? devices[k] : k;
    if (d < 0 || d >= ndev) {
      set_error("device " + std::to_string(d) + " out of range (" + std::to_string(ndev) + " devices)");
      return renderer_fail_cleanup(r, RT_E_DEVICE);
    }
    Rank& q = r->ranks[k];
    q.device = d;
    auto it = std::find(r->devices.begin(), r->devices.end(), d);
    q.comm_idx = (int)(it - r->devices.begin());
    if (it == r->devices.end()) r->devices.push_back(d);
    int rc = rt_context_create(d, &q.ctx);
    if (rc) return renderer_fail_cleanup(r, rc);
    q.stream = (hipStream_t)context_stream(q.ctx);  // the rank renders on its context's own stream
    if (hipSetDevice(d) != hipSuccess || hipEventCreateWithFlags(&q.done, hipEventDisableTiming) != hipSuccess) {
      set_error("rt_renderer_create: stream / event creation failed");
      return renderer_fail_cleanup(r, RT_E_DEVICE);
    }
  }
  for (int k = 0; k < n; ++k) {
    Rank& q = r->ranks[k];
    if ((int)r->comm_streams.size() <= q.comm_idx) r->comm_streams.push_back(q.stream);
  }
  {
    // 16 MB (an 800x600 frame's float3 + RGBA8 twice over; grown on demand),
    // its mapped pages touched once by the download kernel when newly pinned
    const size_t cap = size_t(16) << 20;
    bool fresh = false;
    int e = hipSetDevice(r->ranks[0].device);
    if (e == hipSuccess) e = host_alloc(&r->h_img, cap, &fresh);
    if (e == hipSuccess) r->h_img_cap = cap;
    if (e == hipSuccess && fresh) {
      void* d = nullptr;
      void* h_map = nullptr;
      hipStream_t s = r->ranks[0].stream;
      e = dev_alloc(&d, cap);
      if (e == hipSuccess) e = hipHostGetDevicePointer(&h_map, r->h_img, 0);
      if (e == hipSuccess) e = launch_download(d, h_map, cap, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      dev_free(d);
    }
    if (e != hipSuccess) {
      set_error(std::string("rt_renderer_create: pinned staging failed: ") + hipGetErrorString((hipError_t)e));
      return renderer_fail_cleanup(r, RT_E_DEVICE);
    }
  }
  if (r->devices.size() > 1) {
    r->comms.resize(r->devices.size());
    ncclResult_t e = ncclCommInitAll(r->comms.data(), (int)r->devices.size(), r->devices.data());
    if (e != ncclSuccess) {
      r->comms.clear();
      set_error(std::string("ncclCommInitAll failed: ") + ncclGetErrorString(e));
      return renderer_fail_cleanup(r, RT_E_DEVICE);
    }
  }
  *out = r;
  return RT_OK;
}

void rt_renderer_destroy(rt_renderer* r) {
  if (!r) return;
  for (Rank& q : r->ranks) {
    if (q.stream && r->stalled.empty()) {
      (void)hipSetDevice(q.device);
      (void)hipStreamSynchronize(q.stream);
    }
  }
  if (!r->stalled.empty()) {
    // the watchdog fired: the communicators are aborted and the stalled
    // work may never end -- nothing that waits on it is released
    delete r;
    return;
  }
  for (ncclComm_t c : r->comms) (void)ncclCommDestroy(c);
  host_free(r->h_img);
  rt_partition_destroy(r->part);
  const int root = r->ranks.empty() ? 0 : r->ranks[0].device;
  r->gathered.release(root);
  r->img_lin.release(root);
  r->img_rgba.release(root);
  for (Rank& q : r->ranks) {
    (void)hipSetDevice(q.device);
    dev_free(q.share);
    if (q.done) (void)hipEventDestroy(q.done);
    rt_context_destroy(q.ctx);  // (and its stream, the rank's)
  }
  delete r;
}

int rt_renderer_set_tuning(rt_renderer* r, const rt_tuning* t) {
  if (!r || !t) {
    set_error("renderer or tuning is NULL");
    return RT_E_INVALID;
  }
  for (Rank& q : r->ranks) {
    int rc = rt_context_set_tuning(q.ctx, t);
    if (rc) return rc;
  }
  r->tun = *t;
  r->have_scene = false;  // the BVH shape may change
  return RT_OK;
}

int rt_renderer_set_watchdog(rt_renderer* r, double seconds) {
  if (!r) {
    set_error("renderer is NULL");
    return RT_E_INVALID;
  }
  r->watchdog_s = seconds;
  return RT_OK;
}

int rt_renderer_test_stall(rt_renderer* r, int32_t rank, double ms) {
  if (!r || rank < 0 || rank >= (int32_t)r->ranks.size() || !(ms >= 0 && ms <= 60000)) {
    set_error("rt_renderer_test_stall: invalid arguments");
    return RT_E_INVALID;
  }
  r->stall_rank = rank;
  r->stall_ms = ms;
  return RT_OK;
}

int rt_renderer_render(rt_renderer* r, const rt_scene* scene, int32_t w, int32_t h, const rt_settings* st,
                       float* out_linear, uint8_t* out_rgba, rt_stats* stats) {
  if (!r) {
    set_error("renderer is NULL");
    return RT_E_INVALID;
  }
  if (!r->stalled.empty()) {
    set_error(r->stalled);
    return RT_E_TIMEOUT;
  }
  int rc = rt_validate(scene, w, h, st);
  if (rc) return rc;
  const double t0 = now_s();
  const int n = (int)r->ranks.size();
  const int root = r->ranks[0].device;
  // scene upload (flatten + BVH) only when its content changed
  std::vector<uint8_t> key;
  scene_bytes(*scene, &key);
  double bvh_s = 0;
  if (!r->have_scene || key != r->scene_key) {
    r->have_scene = false;
    for (Rank& q : r->ranks) {
      int rc = rt_context_set_scene(q.ctx, scene, 0);
      if (rc) return rc;
      bvh_s += context_bvh_seconds(q.ctx);
    }
    r->scene_key.swap(key);
    r->have_scene = true;
    r->scene_gen += 1;
  }
  const double t_scene = now_s();
  const size_t npix = (size_t)w * h;
  rc = r->img_lin.grow(root, npix * 3 * sizeof(float));
  if (!rc) rc = r->img_rgba.grow(root, npix * 4);
  if (rc) return rc;
  hipStream_t root_s = r->ranks[0].stream;
  // A multi-rank frame with a watchdog (rt_renderer_set_watchdog) has one
  // deadline, taken here before anything of the frame runs: every host wait
  // of the frame is bounded by it -- each rank's own waits inside its render
  // (its previous render, the schedule build, a BVH scene's bounce loop: the
  // rank contexts poll, context_set_deadline) and the waits for the ranks'
  // streams after the launches (bounded_sync, below).
  const double deadline = n > 1 && r->watchdog_s > 0 ? now_s() + r->watchdog_s : 0.0;
  for (Rank& q : r->ranks) context_set_deadline(q.ctx, deadline);
  struct ClearDeadline {
    rt_renderer* r;
    ~ClearDeadline() {
      for (Rank& q : r->ranks) context_set_deadline(q.ctx, 0.0);
    }
  } clear_deadline{r};
  // the watchdog fired for rank k: the communicators are aborted and the
  // renderer refuses later calls (the stalled work may never end)
  auto timed_out = [&](int k, const char* where) {
    const std::string part =
        r->part ? "balanced, " + std::to_string(rt_partition_local_tiles(r->part, k)) + " tiles on this rank"
                : "strided t % " + std::to_string(n) + ", " + std::to_string(rt_tiles_for_rank(w, h, k, n)) +
                      " tiles on this rank";
    r->stalled = "rt_renderer_render: watchdog: rank " + std::to_string(k) + " (device " +
                 std::to_string(r->ranks[k].device) + ") did not finish frame " + std::to_string(r->frames) + " (" +
                 std::to_string(w) + "x" + std::to_string(h) + ", " + std::to_string(st->samples) + " spp) within " +
                 std::to_string(r->watchdog_s) + " s: " + where + " (partition " + part +
                 "); communicators aborted, the renderer is unusable";
    for (ncclComm_t c : r->comms) (void)ncclCommAbort(c);
    r->comms.clear();
    set_error(r->stalled);
    return RT_E_TIMEOUT;
  };
  if (n == 1) {
    rc = rt_context_render_async(r->ranks[0].ctx, w, h, st, 0, 1, RT_LAYOUT_IMAGE, (float*)r->img_lin.p,
                                 (uint8_t*)r->img_rgba.p, root_s, nullptr);
    if (rc) return rc;
  } else {
    rc = renderer_partition(r, scene, w, h, st);
    if (rc == RT_E_TIMEOUT) return timed_out(0, "the partition's measuring render stalled");
    if (rc) return rc;
    const size_t share = r->part ? rt_partition_packed_bytes(r->part) : rt_packed_bytes(w, h, n);
    const size_t rgba_off = r->part ? rt_partition_rgba_offset(r->part) : rt_packed_rgba_offset(w, h, n);
    rc = r->gathered.grow(root, share * (size_t)n);
    if (rc) return rc;
    std::vector<uint8_t*> bufs(n);
    for (int k = 0; k < n; ++k) {
      Rank& q = r->ranks[k];
      if (q.comm_idx == 0) {  // the root's device: straight into the gather buffer
        bufs[k] = (uint8_t*)r->gathered.p + (size_t)k * share;
      } else {
        if (share > q.share_cap) {
          HIP_TRY(hipSetDevice(q.device));
          dev_free(q.share);
          q.share = nullptr;
          q.share_cap = 0;
          HIP_TRY((hipError_t)dev_alloc(&q.share, share));
          q.share_cap = share;
        }
        bufs[k] = (uint8_t*)q.share;
      }
    }
    // One host thread per rank: a BVH scene's wavefront loop is driven from
    // the host bounce by bounce (rt_context_render_async returns when its
    // frame is done), so the ranks must not wait for each other.  The
    // megakernel's launches return at once either way.
    std::vector<int> rcs(n, RT_OK);
    std::vector<std::string> errs(n);
    auto render_rank = [&](int k) {
      Rank& q = r->ranks[k];
      rcs[k] = rt_context_render_async(q.ctx, w, h, st, k, n, RT_LAYOUT_PACKED_TILES, (float*)bufs[k],
                                       bufs[k] + rgba_off, q.stream, nullptr);
      if (rcs[k]) errs[k] = rt_last_error();  // (the error text is per thread)
    };
    test_stall(r, n);
    std::vector<std::thread> pool;
    try {
      for (int k = 1; k < n; ++k) pool.emplace_back(render_rank, k);
    } catch (const std::system_error& ex) {  // no thread: the remaining ranks run on this one
      for (int k = (int)pool.size() + 1; k < n; ++k) render_rank(k);
    }
    render_rank(0);
    for (std::thread& t : pool) t.join();
    for (int k = 1; k <= n; ++k)  // (the other ranks first, as below)
      if (rcs[k % n] == RT_E_TIMEOUT) return timed_out(k % n, "its share render stalled before its launches");
    for (int k = 0; k < n; ++k)
      if (rcs[k]) {
        set_error(errs[k]);
        return rcs[k];
      }
    if (r->devices.size() > 1) {
      rc = group_gather(r, share);
      if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(root));
    for (int k = 1; k < n; ++k) {  // the root's other ranks (their own streams)
      Rank& q = r->ranks[k];
      if (q.comm_idx != 0) continue;
      HIP_TRY(hipEventRecord(q.done, q.stream));
      HIP_TRY(hipStreamWaitEvent(root_s, q.done, 0));
    }
    rc = r->part ? rt_unpack_partition_async(r->part, r->gathered.p, (float*)r->img_lin.p, (uint8_t*)r->img_rgba.p,
                                             root_s)
                 : rt_unpack_tiles_async(w, h, n, r->gathered.p, (float*)r->img_lin.p, (uint8_t*)r->img_rgba.p, root_s);
    if (rc) return rc;
  }
  HIP_TRY(hipSetDevice(root));
  const double t_launch = now_s();
  // Wait for every rank first, then copy the image straight into the
  // caller's buffers from an idle stream.  A device->host copy into pageable
  // memory queued behind the render kernels made the runtime wait for them
  // itself, and in a fresh process its copy started ~8-9 ms after they ended
  // (the CLI's first Render, profiles/r04_cli_trace.json); from an idle
  // stream it starts at once.
  double ks = 0;
  r->rank_secs.assign(n, 0.0);
  // (a multi-rank frame waits at most until its deadline: a stalled rank or
  // collective ends the wait)
  // (the other ranks first: the root's stream waits for every rank's share
  // before its unpack, so a stalled rank is named as itself, not as the root)
  for (int i = 1; i <= n; ++i) {
    const int k = i % n;
    Rank& q = r->ranks[k];
    rc = bounded_sync(q.device, q.stream, deadline);
    if (rc == RT_E_TIMEOUT)
      return timed_out(k, r->devices.size() > 1 ? "its share render, the RCCL gather or the unpack stalled"
                                                 : "its share render or the unpack stalled");
    if (rc) return rc;
    double s = 0;
    rc = rt_context_last_kernel_seconds(q.ctx, &s);
    if (rc) return rc;
    r->rank_secs[k] = s;
    ks = std::max(ks, s);
  }
  HIP_TRY(hipSetDevice(root));
  const size_t lin_b = out_linear ? npix * 3 * sizeof(float) : 0, rgba_b = out_rgba ? npix * 4 : 0;
  const size_t rgba_at = (lin_b + 255) & ~size_t(255);
  const bool by_kernel = r->frames == 0 && lin_b % 16 == 0 && rgba_b % 16 == 0 && rgba_at + rgba_b <= r->h_img_cap;
  if (by_kernel) {
    // The first Render of a renderer (a fresh `raytracer` process renders
    // once): a copy-engine transfer then started 7-15 ms after it was issued,
    // whatever was warmed before (profiles/r04_cli_trace.json,
    // scripts/copy_probe.hip); a kernel writing the pinned staging through its
    // mapping does not wait for that, and the host copies it on.  Later
    // Renders copy straight into the caller's buffers (no host copy).
    void* h_map = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&h_map, r->h_img, 0));
    if (lin_b) HIP_TRY((hipError_t)launch_download(r->img_lin.p, h_map, lin_b, root_s));
    if (rgba_b) HIP_TRY((hipError_t)launch_download(r->img_rgba.p, (char*)h_map + rgba_at, rgba_b, root_s));
    HIP_TRY(hipStreamSynchronize(root_s));
    if (lin_b) memcpy(out_linear, r->h_img, lin_b);
    if (rgba_b) memcpy(out_rgba, (char*)r->h_img + rgba_at, rgba_b);
  } else {
    if (lin_b) HIP_TRY(hipMemcpyAsync(out_linear, r->img_lin.p, lin_b, hipMemcpyDeviceToHost, root_s));
    if (rgba_b) HIP_TRY(hipMemcpyAsync(out_rgba, r->img_rgba.p, rgba_b, hipMemcpyDeviceToHost, root_s));
    HIP_TRY(hipStreamSynchronize(root_s));
  }
  r->frames += 1;
  const double t_end = now_s();
  const double secs = t_end - t0;
  if (stats) {
    memset(stats, 0, sizeof *stats);
    stats->render_seconds = secs;
    stats->scene_seconds = t_scene - t0;
    stats->bvh_build_seconds = bvh_s;
    stats->launch_seconds = t_launch - t_scene;
    // (the time after the launches were enqueued until the image was on the
    // host: the kernels, then the copies)
    stats->download_seconds = t_end - t_launch;
    stats->kernel_seconds = ks;
    stats->rays_per_second = (double)npix * st->samples / secs;
    stats->pixels_per_second = (double)npix / secs;
    stats->objects = scene->num_objects;  // len(hittables): a cube counts once (renderer.go:109)
    stats->lights = scene->num_lights;
  }
  return RT_OK;
}

int rt_render(const rt_scene* scene, int32_t w, int32_t h, const rt_settings* st, float* out_linear,
              uint8_t* out_rgba, rt_stats* stats) {
  int rc = rt_validate(scene, w, h, st);  // before touching a device
  if (rc) return rc;
  const double t0 = now_s();
  rt_renderer* r = nullptr;
  rc = rt_renderer_create(nullptr, std::max(1, st->num_devices), &r);
  if (rc) return rc;
  const double t_created = now_s();
  rc = rt_renderer_render(r, scene, w, h, st, out_linear, out_rgba, stats);
  const double t_rendered = now_s();
  rt_renderer_destroy(r);  // (after a watchdog timeout it releases only what does not wait on the stall)
  if (!rc && stats) {  // Go's Render time covers everything (renderer.go:68,101)
    stats->create_seconds = t_created - t0;
    stats->destroy_seconds = now_s() - t_rendered;
    stats->render_seconds = now_s() - t0;
    stats->rays_per_second = (double)w * h * st->samples / stats->render_seconds;
    stats->pixels_per_second = (double)w * h / stats->render_seconds;
  }
  return rc;
}


// ------------------------------------------------------------ partitions

int rt_partition_create(int32_t w, int32_t h, int32_t world, const int32_t* owner, rt_partition** out) {
  if (!out || w <= 0 || h <= 0 || world < 1 || world > 65536) {
    set_error("rt_partition_create: invalid arguments");
    return RT_E_INVALID;
  }
  *out = nullptr;
  PartitionData d;
  d.w = w;
  d.h = h;
  d.world = world;
  const int ntiles = rt_num_tiles(w, h);
  d.owner.resize(ntiles);
  for (int t = 0; t < ntiles; ++t) {
    const int o = owner ? owner[t] : t % world;
    if (o < 0 || o >= world) {
      set_error("rt_partition_create: owner of tile " + std::to_string(t) + " out of range");
      return RT_E_INVALID;
    }
    d.owner[t] = o;
  }
  finish_partition(&d);
  *out = make_partition(std::move(d));
  return RT_OK;
}

void rt_partition_destroy(rt_partition* p) {
  if (!p) return;
  for (auto& ds : p->slots) {
    (void)hipSetDevice(ds.first);
    (void)hipFree(ds.second);
  }
  delete p;
}

int32_t rt_partition_world(const rt_partition* p) { return p ? p->d.world : 0; }

int32_t rt_partition_owner(const rt_partition* p, int32_t t) {
  return (p && t >= 0 && t < (int32_t)p->d.owner.size()) ? p->d.owner[t] : -1;
}

int32_t rt_partition_local_tiles(const rt_partition* p, int32_t rank) {
  if (!p || rank < 0 || rank >= p->d.world) return 0;
  return p->d.offsets[rank + 1] - p->d.offsets[rank];
}

int32_t rt_partition_tile(const rt_partition* p, int32_t rank, int32_t local) {
  if (!p || local < 0 || local >= rt_partition_local_tiles(p, rank)) return -1;
  return p->d.lists[p->d.offsets[rank] + local];
}

int32_t rt_partition_max_local(const rt_partition* p) { return p ? p->d.max_local : 0; }
size_t rt_partition_packed_bytes(const rt_partition* p) { return p ? (size_t)p->d.max_local * 1024 * 16 : 0; }
size_t rt_partition_rgba_offset(const rt_partition* p) { return p ? (size_t)p->d.max_local * 1024 * 12 : 0; }

double rt_partition_work(const rt_partition* p, int32_t rank) {
  if (!p || rank < 0 || rank >= (int32_t)p->d.work.size()) return 0.0;
  return p->d.work[rank];
}

int rt_unpack_partition_frames_async(const rt_partition* pc, int32_t nframes, const void* d_gathered,
                                     float* d_linear, uint8_t* d_rgba, void* stream) {
  if (!pc || !d_gathered || nframes < 1) {
    set_error("rt_unpack_partition_frames_async: invalid arguments");
    return RT_E_INVALID;
  }
  rt_partition* p = const_cast<rt_partition*>(pc);  // (the per-device slot maps are a cache)
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  int32_t* slot = nullptr;
  {
    std::lock_guard<std::mutex> lock(p->mu);
    for (auto& ds : p->slots)
      if (ds.first == dev) slot = ds.second;
    if (!slot) {
      const int ntiles = (int)p->d.owner.size();
      std::vector<int32_t> h(2 * (size_t)std::max(ntiles, 1), 0);
      for (int t = 0; t < ntiles; ++t) {
        h[2 * t] = p->d.owner[t];
        h[2 * t + 1] = p->d.local[t];
      }
      HIP_TRY(hipMalloc((void**)&slot, h.size() * sizeof(int32_t)));
      if (hipMemcpy(slot, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(slot);
        set_error("rt_unpack_partition_frames_async: slot map upload failed");
        return RT_E_DEVICE;
      }
      p->slots.emplace_back(dev, slot);
    }
  }
  int e = launch_unpack_map(p->d.w, p->d.h, nframes, slot, d_gathered, rt_partition_packed_bytes(p),
                            rt_partition_rgba_offset(p), d_linear, d_rgba, stream);
  if (e != hipSuccess) {
    set_error(std::string("unpack launch failed: ") + hipGetErrorString((hipError_t)e));
    return RT_E_DEVICE;
  }
  return RT_OK;
}

int rt_unpack_partition_async(const rt_partition* p, const void* d_gathered, float* d_linear, uint8_t* d_rgba,
                              void* stream) {
  return rt_unpack_partition_frames_async(p, 1, d_gathered, d_linear, d_rgba, stream);
}

int rt_renderer_rank_seconds(const rt_renderer* r, double* out, int32_t capacity) {
  if (!r || !out) {
    set_error("renderer or out is NULL");
    return RT_E_INVALID;
  }
  if (capacity < (int64_t)r->ranks.size()) {
    set_error("rt_renderer_rank_seconds: out holds " + std::to_string(capacity) + " values, the renderer has " +
              std::to_string(r->ranks.size()) + " ranks");
    return RT_E_INVALID;
  }
  if (r->rank_secs.size() != r->ranks.size()) {
    set_error("the renderer has not rendered a frame yet");
    return RT_E_INVALID;
  }
  for (size_t k = 0; k < r->rank_secs.size(); ++k) out[k] = r->rank_secs[k];
  return RT_OK;
}

int32_t rt_renderer_num_ranks(const rt_renderer* r) { return r ? (int32_t)r->ranks.size() : 0; }

// ------------------------------------------------------------ multi-process

int rt_comm_unique_id(uint8_t* id) {
  if (!id) {
    set_error("id is NULL");
    return RT_E_INVALID;
  }
  static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES != NCCL_UNIQUE_ID_BYTES");
  ncclUniqueId u;
  NCCL_TRY(ncclGetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return RT_OK;
}

int rt_comm_create(const uint8_t* id, int32_t world, int32_t rank, int32_t device, rt_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) {
    set_error("rt_comm_create: invalid arguments");
    return RT_E_INVALID;
  }
  *out = nullptr;
  HIP_TRY(hipSetDevice(device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  rt_comm* c = new rt_comm();
  c->rank = rank;
  c->world = world;
  c->device = device;
  ncclResult_t e = ncclCommInitRank(&c->comm, world, u, rank);
  if (e != ncclSuccess) {
    delete c;
    set_error(std::string("ncclCommInitRank failed: ") + ncclGetErrorString(e));
    return RT_E_DEVICE;
  }
  *out = c;
  return RT_OK;
}

void rt_comm_destroy(rt_comm* c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int rt_comm_gather_bytes_async(rt_comm* c, size_t share, const void* d_share, void* d_gathered, void* stream) {
  if (!c || !d_share || (c->rank == 0 && !d_gathered)) {
    set_error("rt_comm_gather_bytes_async: invalid arguments");
    return RT_E_INVALID;
  }
  if (c->world == 1 || share == 0) return RT_OK;
  hipStream_t s = (hipStream_t)stream;
  HIP_TRY(hipSetDevice(c->device));
  NCCL_TRY(ncclGroupStart());
  ncclResult_t ge = ncclSuccess;
  if (c->rank == 0) {
    for (int k = 1; k < c->world; ++k)
      NCCL_GROUP_TRY(ge, ncclRecv((uint8_t*)d_gathered + (size_t)k * share, share, ncclUint8, k, c->comm, s));
  } else {
    NCCL_GROUP_TRY(ge, ncclSend(d_share, share, ncclUint8, 0, c->comm, s));
  }
  const ncclResult_t ee = ncclGroupEnd();
  if (ge != ncclSuccess) return RT_E_DEVICE;
  NCCL_TRY(ee);
  return RT_OK;
}

int rt_comm_gather_tiles_async(rt_comm* c, int32_t w, int32_t h, const void* d_share, void* d_gathered,
                               void* stream) {
  if (!c || w <= 0 || h <= 0) {
    set_error("rt_comm_gather_tiles_async: invalid arguments");
    return RT_E_INVALID;
  }
  return rt_comm_gather_bytes_async(c, rt_packed_bytes(w, h, c->world), d_share, d_gathered, stream);
}

}  // extern "C"
