// sanitize_driver.cpp — the host code of librtgo and the CPU oracle under
// AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on
// host code; GPU sanitizers are not available on this pool).
//
// Built by tests/c/Makefile from the host-only sources (scene_json.cpp,
// scene_flat.cpp, bvh.cpp, schedule.cpp, image_io.cpp) and oracle/oracle.c;
// run by tests/test_sanitizers.py.  It drives every host path with real and
// malformed input: every committed scene and the 10k-sphere scene through
// the loader, the flattening, the BVH builder (default and extreme leaf /
// bin settings) and the schedule's per-tile inputs; truncated and ill-typed
// JSON; the PNG / PPM writers and the tone map; and small multi-threaded
// oracle renders (the tile queue of renderer.go:67-148).
//   usage: sanitize_driver <scenes dir> <10k scene json> <tmp dir>
#include <dirent.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../concurrent-raytracer-go_amd/csrc/rt_internal.h"
#include "../../oracle/oracle.h"

namespace rtgo {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
}  // namespace rtgo

using namespace rtgo;

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      fprintf(stderr, "CHECK failed at line %d: %s\n", __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static void exercise_scene(const rt_scene* s, const char* name) {
  FlatScene f;
  flatten_scene(*s, &f);
  std::vector<unsigned long long> masks;
  std::vector<float> cost;
  std::vector<int32_t> tiles;
  for (int world : {1, 3, 8}) {
    for (int rank = 0; rank < world; rank += 2) {
      strided_tiles(800, 600, rank, world, &tiles);
      if (f.spheres.size() <= 64 && f.tris.size() <= 64) tile_primary_masks(f, 800, 600, tiles, &masks);
      tile_cost(f, 800, 600, tiles, &cost);
      strided_tiles(33, 17, rank, world, &tiles);
      tile_cost(f, 33, 17, tiles, &cost);
    }
    // a balanced partition of the frame from the projected-primitive costs
    strided_tiles(800, 600, 0, 1, &tiles);
    tile_cost(f, 800, 600, tiles, &cost);
    PartitionData pd;
    pd.w = 800;
    pd.h = 600;
    pd.world = world;
    lpt_partition(cost, &pd);
    CHECK((int)pd.lists.size() == rt_num_tiles(800, 600) && pd.offsets[world] == (int)pd.lists.size());
    for (int r = 0; r < world; ++r)
      for (int k = pd.offsets[r]; k < pd.offsets[r + 1]; ++k)
        CHECK(pd.owner[pd.lists[k]] == r && pd.local[pd.lists[k]] == k - pd.offsets[r]);
  }
  if (f.tris.empty() && !f.spheres.empty()) {
    for (int leaf : {0, 1, 7})
      for (int bins : {0, 2, 64}) {
        FlatScene g = f;
        build_sphere_bvh(&g, bins, leaf);
        CHECK(!g.bvh.empty() && g.qbvh.size() == g.bvh.size());
      }
  }
  printf("%s: %zu spheres, %zu triangles, %zu lights\n", name, f.spheres.size(), f.tris.size(), f.lights.size());
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const std::string dir = argv[1], big = argv[2], tmp = argv[3];
  // every committed scene
  DIR* d = opendir(dir.c_str());
  CHECK(d != nullptr);
  while (dirent* e = d ? readdir(d) : nullptr) {
    std::string n = e->d_name;
    if (n.size() < 5 || n.substr(n.size() - 5) != ".json") continue;
    rt_scene_buf* sb = nullptr;
    CHECK(rt_scene_load_json((dir + "/" + n).c_str(), 0, &sb) == RT_OK);
    if (sb) {
      exercise_scene(rt_scene_view(sb), n.c_str());
      rt_scene_free(sb);
    }
  }
  if (d) closedir(d);
  rt_scene_buf* bigsb = nullptr;
  CHECK(rt_scene_load_json(big.c_str(), 0, &bigsb) == RT_OK);
  if (bigsb) exercise_scene(rt_scene_view(bigsb), "10k spheres");
  // malformed input: errors, never crashes
  const char* bad[] = {
      "", "{", "[]", "{\"objects\": [", "{\"objects\": [{\"type\": \"sphere\", \"position\": [1, 2]}]}",
      "{\"objects\": [{\"type\": \"sphere\", \"position\": {\"X\": \"a\"}}]}", "{\"camera\": 5}",
      "{\"objects\": [{\"type\": \"cube\", \"size\": [1e400, -1e400, 0], \"material\": {\"type\": 7}}]}",
      "{\"objects\": [{\"type\": \"sphere\", \"radius\": 1, \"material\": {\"type\": \"metal\"}}]} x",
      "{\"lights\": [{\"position\": [1,2,3], \"intensity\": \"loud\"}]}", "{\"a\": \"\\ud800\"}",
      "{\"a\": [[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[[]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]]}",
      "{\"objects\": [{\"type\": \"sphere\", \"position\": [0,0,-1], \"radius\": -2, \"material\": {}}]}",
      "{\"objects\": [null, 3, \"x\", {\"type\": \"sphere\"}]}", "\xff\xfe{}", "{\"a\":1e99999}",
  };
  for (const char* t : bad) {
    rt_scene_buf* sb = nullptr;
    const int rc = rt_scene_parse_json(t, strlen(t), 0, &sb);
    if (rc == RT_OK && sb) {  // some of these are valid JSON for the Go loader's rules
      exercise_scene(rt_scene_view(sb), "malformed-but-accepted");
      rt_scene_free(sb);
    }
  }
  // tone map and writers
  const int w = 37, h = 23;
  std::vector<float> lin((size_t)w * h * 3);
  for (size_t i = 0; i < lin.size(); ++i) lin[i] = (float)((i % 17) - 3) * 0.37f;
  lin[5] = NAN;
  lin[6] = INFINITY;
  std::vector<uint8_t> rgba((size_t)w * h * 4);
  rt_tonemap_rgba(lin.data(), w * h, rgba.data());
  CHECK(rt_write_png((tmp + "/a/b/out.png").c_str(), rgba.data(), w, h) == RT_OK);
  CHECK(rt_write_ppm((tmp + "/out.ppm").c_str(), rgba.data(), w, h) == RT_OK);
  CHECK(rt_write_png((tmp + "/x.png").c_str(), rgba.data(), 0, h) != RT_OK);
  // the oracle: small renders of every committed scene, several threads
  d = opendir(dir.c_str());
  while (dirent* e = d ? readdir(d) : nullptr) {
    std::string n = e->d_name;
    if (n.size() < 5 || n.substr(n.size() - 5) != ".json") continue;
    rt_scene_buf* sb = nullptr;
    if (rt_scene_load_json((dir + "/" + n).c_str(), 0, &sb) != RT_OK) continue;
    rt_settings st;
    rt_settings_default(&st);
    st.samples = 2;
    st.max_depth = 8;
    for (int sky : {RT_SKY_NONE, RT_SKY_SUNSET}) {
      st.sky = sky;
      std::vector<double> out((size_t)40 * 30 * 3);
      std::vector<uint8_t> o8((size_t)40 * 30 * 4);
      rt_counts c;
      CHECK(oracle_render(rt_scene_view(sb), 40, 30, &st, 0, 1, 4, -1, out.data(), o8.data(), &c) == 0);
      CHECK(oracle_render(rt_scene_view(sb), 40, 30, &st, 1, 3, 3, 2, out.data(), o8.data(), nullptr) == 0);
    }
    rt_scene_free(sb);
  }
  if (d) closedir(d);
  if (bigsb) {
    rt_settings st;
    rt_settings_default(&st);
    st.samples = 1;
    std::vector<double> out((size_t)64 * 36 * 3);
    CHECK(oracle_render(rt_scene_view(bigsb), 64, 36, &st, 5, 7, 2, 1, out.data(), nullptr, nullptr) == 0);
    std::vector<double> outb((size_t)64 * 36 * 3);  // the BVH baseline variant renders the same pixels
    CHECK(oracle_render_ex(rt_scene_view(bigsb), 64, 36, &st, 5, 7, 2, 1, outb.data(), nullptr, nullptr, 1) == 0);
    for (size_t i = 0; i < out.size(); ++i) CHECK(memcmp(&out[i], &outb[i], sizeof(double)) == 0 || (out[i] != out[i]));
    rt_scene_free(bigsb);
  }
  printf("sanitize_driver: %d failures\n", failures);
  return failures ? 1 : 0;
}
