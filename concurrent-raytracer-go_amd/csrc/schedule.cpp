// schedule.cpp — the per-tile inputs of the work schedule, on the host.
//
// The schedule itself (per-pixel masks, pilot render, blocks, dispatch
// order) is built on the GPU (rt_schedule.hip).  Its per-TILE inputs are
// cheap (tiles x primitives) and stay here:
//   - tile_primary_masks: the primitives whose bounding sphere meets the cone
//     of a tile's camera rays (the per-pixel masks refine these);
//   - tile_cost: primitives projected onto each tile, the work estimate of a
//     schedule built without a pilot render.
#include <math.h>

#include <algorithm>
#include <atomic>
#include <numeric>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

void strided_tiles(int32_t W, int32_t H, int32_t rank, int32_t world, std::vector<int32_t>* tiles) {
  tiles->clear();
  const int ntiles = rt_num_tiles(W, H);
  for (int t = rank; t < ntiles; t += world) tiles->push_back(t);
}

void tile_cost(const FlatScene& fs, int32_t W, int32_t H, const std::vector<int32_t>& tiles,
               std::vector<float>* local_cost) {
  const int tiles_x = (W + 31) / 32, tiles_y = (H + 31) / 32, ntiles = tiles_x * tiles_y;
  std::vector<float> cost(ntiles, 0.0f);
  const double vw = 2.0 * fs.aspect;
  auto add_sphere = [&](const double* c, double r) {
    const double R = fabs(r);
    const double cx = c[0] - fs.cam_pos[0], cy = c[1] - fs.cam_pos[1], cz = c[2] - fs.cam_pos[2];
    if (cz - R >= 0) return;  // entirely behind the camera: no camera ray reaches it
    if (cz + R > -1e-9 || !(fabs(vw) > 0)) {  // straddles the camera plane: everywhere
      for (auto& v : cost) v += 1.0f;
      return;
    }
    // image bounds of the bounding box corners (perspective keeps convexity)
    double u0 = INFINITY, u1 = -INFINITY, v0 = INFINITY, v1 = -INFINITY;
    for (int k = 0; k < 8; ++k) {
      const double qx = cx + ((k & 1) ? R : -R), qy = cy + ((k & 2) ? R : -R), qz = cz + ((k & 4) ? R : -R);
      const double u = 0.5 + qx / (-qz * vw), v = 0.5 + qy / (-qz * 2.0);
      u0 = fmin(u0, u);
      u1 = fmax(u1, u);
      v0 = fmin(v0, v);
      v1 = fmax(v1, v);
    }
    const double px0 = u0 * W, px1 = u1 * W, py0 = v0 * H, py1 = v1 * H;
    if (px1 < 0 || py1 < 0 || px0 >= W || py0 >= H) return;
    const int tx0 = std::max(0, (int)floor(px0) / 32), tx1 = std::min(tiles_x - 1, (int)floor(fmin(px1, W - 1)) / 32);
    const int ty0 = std::max(0, (int)floor(py0) / 32), ty1 = std::min(tiles_y - 1, (int)floor(fmin(py1, H - 1)) / 32);
    for (int ty = ty0; ty <= ty1; ++ty)
      for (int tx = tx0; tx <= tx1; ++tx) cost[ty * tiles_x + tx] += 1.0f;
  };
  for (const DSphere& s : fs.spheres) add_sphere(s.c, s.r);
  for (const DTri& t : fs.tris) add_sphere(t.bc, t.br);

  local_cost->clear();
  for (int32_t t : tiles) local_cost->push_back(cost[t]);
}

// Does the cone (apex, unit axis, cos/sin of its half-angle) meet the sphere
// (c, r)?  Same conservative test as the kernel's cone_meets_sphere: radius
// inflated by ~1e-7, far above binary64 rounding of the ray directions.
static bool cone_meets_sphere(const double c[3], double r, const double apex[3], const double axis[3], double cos_t,
                              double sin_t) {
  const double v[3] = {c[0] - apex[0], c[1] - apex[1], c[2] - apex[2]};
  const double dc2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  const double dc = sqrt(dc2);
  const double ra = fabs(r) * (1.0 + 1e-7) + 1e-7 * dc + 1e-12;
  if (dc <= ra) return true;
  const double tl = sqrt(fmax(dc2 - ra * ra, 0.0));
  const double vd = v[0] * axis[0] + v[1] * axis[1] + v[2] * axis[2];
  return vd >= cos_t * (1.0 - 1e-9) * tl - (sin_t + 1e-9) * ra - 1e-7 * dc;
}

// The cone around the camera rays of the image rectangle [x0, x1) x [y0, y1)
// (pixels): getRay direction (vw*(u-1/2), 2*(v-1/2), -1) with u in
// [x0/W, x1/W], v in [y0/H, y1/H] (renderer.go:155-156,377-390): unit axis
// and the cosine / sine of its half-angle.
static void rect_cone(double vw, int32_t W, int32_t H, int x0, int x1, int y0, int y1, double axis[3], double* cmin,
                      double* smax) {
  const double dx0 = vw * ((double)x0 / W - 0.5), dx1 = vw * ((double)x1 / W - 0.5);
  const double dy0 = 2.0 * ((double)y0 / H - 0.5), dy1 = 2.0 * ((double)y1 / H - 0.5);
  axis[0] = 0.5 * (dx0 + dx1);
  axis[1] = 0.5 * (dy0 + dy1);
  axis[2] = -1.0;
  const double al = sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  for (int k = 0; k < 3; ++k) axis[k] /= al;
  double c = 1.0;  // the widest corner: the angle is quasiconvex on the image plane
  for (int k = 0; k < 4; ++k) {
    const double cx = (k & 1) ? dx1 : dx0, cy = (k & 2) ? dy1 : dy0;
    const double cl = sqrt(cx * cx + cy * cy + 1.0);
    c = fmin(c, (axis[0] * cx + axis[1] * cy - axis[2]) / cl);
  }
  *cmin = c;
  *smax = sqrt(fmax(0.0, 1.0 - c * c));
}

// candidates among `cand` (bit i: sphere / triangle i) whose bounding sphere
// meets the cone
static void cone_masks(const FlatScene& fs, const double axis[3], double cmin, double smax, unsigned long long cand_s,
                       unsigned long long cand_t, unsigned long long* ms, unsigned long long* mt) {
  *ms = 0;
  *mt = 0;
  for (unsigned long long b = cand_s; b; b &= b - 1) {
    const int i = __builtin_ctzll(b);
    if (cone_meets_sphere(fs.spheres[i].c, fs.spheres[i].r, fs.cam_pos, axis, cmin, smax)) *ms |= 1ull << i;
  }
  for (unsigned long long b = cand_t; b; b &= b - 1) {
    const int i = __builtin_ctzll(b);
    if (cone_meets_sphere(fs.tris[i].bc, fs.tris[i].br, fs.cam_pos, axis, cmin, smax)) *mt |= 1ull << i;
  }
}

static unsigned long long low_bits(int n) { return n >= 64 ? ~0ull : (1ull << n) - 1ull; }

void tile_primary_masks(const FlatScene& fs, int32_t W, int32_t H, const std::vector<int32_t>& tiles,
                        std::vector<unsigned long long>* masks) {
  masks->clear();
  const int tiles_x = (W + 31) / 32;
  const int ns = (int)fs.spheres.size(), nt = (int)fs.tris.size();
  const double vw = 2.0 * fs.aspect;
  for (int32_t t : tiles) {
    const int tx = t % tiles_x, ty = t / tiles_x;
    double axis[3], cmin, smax;
    rect_cone(vw, W, H, tx * 32, std::min(tx * 32 + 32, (int)W), ty * 32, std::min(ty * 32 + 32, (int)H), axis, &cmin,
              &smax);
    unsigned long long ms, mt;
    cone_masks(fs, axis, cmin, smax, low_bits(std::min(ns, 64)), low_bits(std::min(nt, 64)), &ms, &mt);
    masks->push_back(ms);
    masks->push_back(mt);
  }
}

// ------------------------------------------------------------ partitions
void finish_partition(PartitionData* d) {
  static std::atomic<uint64_t> next_id{1};
  const int ntiles = (int)d->owner.size();
  d->offsets.assign(d->world + 1, 0);
  for (int t = 0; t < ntiles; ++t) d->offsets[d->owner[t] + 1] += 1;
  d->max_local = 0;
  for (int r = 0; r < d->world; ++r) {
    d->max_local = std::max(d->max_local, d->offsets[r + 1]);
    d->offsets[r + 1] += d->offsets[r];
  }
  d->lists.assign(ntiles, 0);
  d->local.assign(ntiles, 0);
  std::vector<int32_t> fill(d->offsets.begin(), d->offsets.end() - 1);
  for (int t = 0; t < ntiles; ++t) {  // ascending within each rank
    const int r = d->owner[t];
    d->local[t] = fill[r] - d->offsets[r];
    d->lists[fill[r]++] = t;
  }
  d->id = next_id.fetch_add(1);
}

// Longest processing time first: tiles by decreasing estimated work (ties:
// the lower tile first) to the least loaded rank (ties: the lower rank).
// Each tile weighs its estimate + 1: tiles with no estimated work still cost
// a launch slot, and spread evenly instead of piling onto one rank.
void lpt_partition(const std::vector<float>& work, PartitionData* d) {
  const int ntiles = (int)work.size(), world = d->world;
  d->owner.assign(ntiles, 0);
  std::vector<int32_t> order(ntiles);
  std::iota(order.begin(), order.end(), 0);
  auto wt = [&](int t) { return (double)work[t] + 1.0; };
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return wt(a) > wt(b); });
  d->work.assign(world, 0.0);
  for (int t : order) {
    int r = 0;
    for (int k = 1; k < world; ++k)
      if (d->work[k] < d->work[r]) r = k;
    d->owner[t] = r;
    d->work[r] += wt(t);
  }
  finish_partition(d);
}

}  // namespace rtgo
