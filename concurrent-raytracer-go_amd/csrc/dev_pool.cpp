// dev_pool.cpp — device memory through a per-device cache of freed blocks.
//
// A context's buffers (scene, schedule, split rows, pilot scratch, wavefront
// arrays) and a renderer's image and gather buffers are allocated with
// dev_alloc and returned with dev_free.  hipMalloc / hipFree cost tens to
// hundreds of microseconds each, and hipFree waits for the device: the
// one-shot rt_render, which creates and destroys its device state every
// call (like one `raytracer` process per frame), spent 1.7 of its 3.4 ms in
// rt_renderer_destroy (scripts/oneshot_probe.py).  A freed block is kept for
// the next allocation of a similar size on the same device instead; at most
// kCacheCap bytes per device stay cached, and rt_release_cached_memory()
// returns them all.  Callers free a block only when no stream still uses it
// (a context waits for its last render first).  Idle streams and events of
// destroyed contexts are kept the same way.
#include <hip/hip_runtime_api.h>

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

namespace {

constexpr size_t kGrain = 256 * 1024;              // sizes are rounded up to this
// cached bytes per device at most.  The cache is invisible to the process's
// other allocators (PyTorch's caching allocator, RCCL), so it holds only what
// a one-shot render of a linear-scan scene re-allocates every call (a few MB
// to a few hundred MB); a BVH scene's wavefront arrays (GBs) go back to
// hipFree.  Mixed-allocator callers can empty it with rt_release_cached_memory.
constexpr size_t kCacheCap = size_t(4) << 30;

struct Pool {
  std::multimap<size_t, void*> free_blocks;  // size -> block
  size_t cached = 0;
};

std::mutex g_mu;
std::map<int, Pool> g_pools;
std::map<int, std::vector<hipStream_t>> g_streams;  // idle non-blocking streams per device
std::map<int, std::vector<hipEvent_t>> g_events;    // idle timing events per device
std::unordered_map<void*, std::pair<int, size_t>> g_live;  // block -> (device, size)

size_t round_up(size_t n) { return ((n + kGrain - 1) / kGrain) * kGrain; }

}  // namespace

int dev_alloc(void** p, size_t n) {
  *p = nullptr;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  const size_t sz = round_up(n == 0 ? 1 : n);
  {
    std::lock_guard<std::mutex> lock(g_mu);
    Pool& pool = g_pools[dev];
    // the smallest cached block that fits, if it is not much larger
    auto it = pool.free_blocks.lower_bound(sz);
    if (it != pool.free_blocks.end() && it->first <= 2 * sz + (size_t(64) << 20)) {
      *p = it->second;
      pool.cached -= it->first;
      g_live[*p] = {dev, it->first};
      pool.free_blocks.erase(it);
      return hipSuccess;
    }
  }
  e = hipMalloc(p, sz);
  if (e != hipSuccess) {  // out of memory: give the cache back and try once more
    (void)hipGetLastError();
    rt_release_cached_memory();
    e = hipMalloc(p, sz);
    if (e != hipSuccess) return (int)e;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  g_live[*p] = {dev, sz};
  return hipSuccess;
}

void dev_free(void* p) {
  if (!p) return;
  std::unique_lock<std::mutex> lock(g_mu);
  auto it = g_live.find(p);
  if (it == g_live.end()) {  // (not ours)
    lock.unlock();
    (void)hipFree(p);
    return;
  }
  const int dev = it->second.first;
  const size_t sz = it->second.second;
  g_live.erase(it);
  Pool& pool = g_pools[dev];
  if (pool.cached + sz <= kCacheCap) {
    pool.free_blocks.emplace(sz, p);
    pool.cached += sz;
    return;
  }
  lock.unlock();
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(dev);
  (void)hipFree(p);
  (void)hipSetDevice(cur);
}

// Streams and events of destroyed contexts, kept for the next context on the
// same device (creating and destroying them cost ~0.1-0.2 ms per rt_render).
int dev_stream_get(hipStream_t* s) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto& v = g_streams[dev];
    if (!v.empty()) {
      *s = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  return (int)hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

void dev_stream_put(hipStream_t s) {  // (idle: the caller synchronized it)
  if (!s) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lock(g_mu);
  g_streams[dev].push_back(s);
}

int dev_event_get(hipEvent_t* ev) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto& v = g_events[dev];
    if (!v.empty()) {
      *ev = v.back();
      v.pop_back();
      return hipSuccess;
    }
  }
  return (int)hipEventCreate(ev);
}

void dev_event_put(hipEvent_t ev) {  // (complete: the caller waited for it)
  if (!ev) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lock(g_mu);
  g_events[dev].push_back(ev);
}

// Pinned (page-locked) host staging buffers, cached the same way.  A copy
// between device memory and PAGEABLE host memory makes the runtime set up
// its own staging the first time (the fresh `raytracer` process's first
// Render waited 9.6 ms in the scene's hipMemcpy and 8 ms before the image's
// device->host copy started, profiles/r04_cli_trace.json); the contexts and
// renderers copy through these instead, allocated by their constructors.
namespace {
std::multimap<size_t, void*> g_host_free;  // size -> pinned block
std::unordered_map<void*, size_t> g_host_live;
size_t g_host_cached = 0;
constexpr size_t kHostCacheCap = size_t(256) << 20;
}  // namespace

int host_alloc(void** p, size_t n, bool* fresh) {
  *p = nullptr;
  if (fresh) *fresh = false;
  const size_t sz = round_up(n == 0 ? 1 : n);
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_host_free.lower_bound(sz);
    if (it != g_host_free.end() && it->first <= 2 * sz + (size_t(16) << 20)) {
      *p = it->second;
      g_host_cached -= it->first;
      g_host_live[*p] = it->first;
      g_host_free.erase(it);
      return hipSuccess;
    }
  }
  const hipError_t e = hipHostMalloc(p, sz, hipHostMallocDefault);
  if (e != hipSuccess) {
    *p = nullptr;
    return (int)e;
  }
  if (fresh) *fresh = true;
  std::lock_guard<std::mutex> lock(g_mu);
  g_host_live[*p] = sz;
  return hipSuccess;
}

void host_free(void* p) {  // (no copy may still use it: the caller synchronized)
  if (!p) return;
  std::unique_lock<std::mutex> lock(g_mu);
  auto it = g_host_live.find(p);
  if (it == g_host_live.end()) return;
  const size_t sz = it->second;
  g_host_live.erase(it);
  if (g_host_cached + sz <= kHostCacheCap) {
    g_host_free.emplace(sz, p);
    g_host_cached += sz;
    return;
  }
  lock.unlock();
  (void)hipHostFree(p);
}

}  // namespace rtgo

extern "C" int rt_release_cached_memory(void) {
  std::vector<std::pair<int, void*>> blocks;
  {
    std::lock_guard<std::mutex> lock(rtgo::g_mu);
    for (auto& dp : rtgo::g_pools) {
      for (auto& b : dp.second.free_blocks) blocks.emplace_back(dp.first, b.second);
      dp.second.free_blocks.clear();
      dp.second.cached = 0;
    }
  }
  std::vector<void*> host_blocks;
  {
    std::lock_guard<std::mutex> lock(rtgo::g_mu);
    for (auto& b : rtgo::g_host_free) host_blocks.push_back(b.second);
    rtgo::g_host_free.clear();
    rtgo::g_host_cached = 0;
  }
  for (void* b : host_blocks) (void)hipHostFree(b);
  std::vector<std::pair<int, hipStream_t>> streams;
  std::vector<std::pair<int, hipEvent_t>> events;
  {
    std::lock_guard<std::mutex> lock(rtgo::g_mu);
    for (auto& ds : rtgo::g_streams)
      for (hipStream_t s : ds.second) streams.emplace_back(ds.first, s);
    for (auto& de : rtgo::g_events)
      for (hipEvent_t e : de.second) events.emplace_back(de.first, e);
    rtgo::g_streams.clear();
    rtgo::g_events.clear();
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& b : blocks) {
    (void)hipSetDevice(b.first);
    (void)hipFree(b.second);
  }
  for (auto& s : streams) {
    (void)hipSetDevice(s.first);
    (void)hipStreamDestroy(s.second);
  }
  for (auto& e : events) {
    (void)hipSetDevice(e.first);
    (void)hipEventDestroy(e.second);
  }
  (void)hipSetDevice(cur);
  return RT_OK;
}
