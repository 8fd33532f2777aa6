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
// (a context waits for its last render first).
#include <hip/hip_runtime_api.h>

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

namespace {

constexpr size_t kGrain = 256 * 1024;              // sizes are rounded up to this
constexpr size_t kCacheCap = size_t(32) << 30;     // cached bytes per device at most (HBM: 288 GB)

struct Pool {
  std::multimap<size_t, void*> free_blocks;  // size -> block
  size_t cached = 0;
};

std::mutex g_mu;
std::map<int, Pool> g_pools;
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
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& b : blocks) {
    (void)hipSetDevice(b.first);
    (void)hipFree(b.second);
  }
  (void)hipSetDevice(cur);
  return RT_OK;
}
