// schedule.cpp — how a rank's 32x32 tiles become work blocks.
//
// The reference hands tiles to goroutines in row-major order through a
// channel (createRenderTasks, internal/renderer/renderer.go:398-436); a
// goroutine that draws a slow tile just keeps it while the others continue.
// On the GPU a workgroup is dispatched once and runs to completion, so a
// slow block dispatched late (long multi-bounce paths between mirrors and
// inside glass) runs alone at the end of the launch.  The host therefore
//   - estimates each tile's cost from the primitives projected onto it
//     (tile_dispatch_order) and each tile's primary-ray candidates
//     (tile_primary_masks),
//   - and, from a one-sample pilot render (rt_api.cpp prepare_schedule),
//     each pixel's path length; build_blocks cuts the pixels into blocks of
//     about equal work, splits the heaviest pixels into sample ranges, and
//     orders the blocks most expensive first.
// This only partitions and orders work: every block is rendered by the same
// code and every pixel's samples are summed in sample order, so the image
// does not depend on the schedule.
#include <math.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

void tile_dispatch_order(const FlatScene& fs, int32_t W, int32_t H, int32_t rank, int32_t world,
                         std::vector<int32_t>* order, std::vector<float>* local_cost) {
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

  order->clear();
  local_cost->clear();
  for (int t = rank, lt = 0; t < ntiles; t += world, ++lt) {
    order->push_back(lt);
    local_cost->push_back(cost[t]);
  }
  std::stable_sort(order->begin(), order->end(), [&](int32_t a, int32_t b) {
    return cost[rank + a * world] > cost[rank + b * world];
  });
}

int build_blocks(const std::vector<float>& pixel_work, int spp, int big_pixels, double block_work,
                 const std::vector<uint8_t>& black_tiles, std::vector<int32_t>* blocks) {
  // pixel_work[lt * 1024 + p]: estimated path work per sample of pixel p
  // (row-major) of local tile lt.  Pixels are taken in row-major order and
  // grouped into blocks of consecutive pixels while the block's work
  // spp * sum(work) stays within block_work (at most big_pixels pixels).  A
  // pixel whose own work exceeds block_work is split into sample ranges of
  // at most 64 samples (one path per lane), each its own block; the pixel
  // is resolved by whichever of its blocks finishes last.  Blocks are
  // dispatched most expensive first, so the longest paths start at once.
  // A tile flagged in black_tiles (no camera ray of it can hit anything,
  // tile_primary_masks) becomes 16 blocks of 64 pixels marked kBlockBlack,
  // dispatched last: the kernel writes their black pixels without tracing.
  struct B {
    double est;
    int32_t lt, p0, np, s0, ns, slot, nsub, flags;
  };
  std::vector<B> v;
  int nsplit = 0;
  const double S = std::max(spp, 1);
  const int local = (int)(pixel_work.size() / 1024);
  for (int lt = 0; lt < local; ++lt) {
    if (spp > 0 && lt < (int)black_tiles.size() && black_tiles[lt]) {
      for (int p0 = 0; p0 < 1024; p0 += 64) v.push_back(B{0.0, lt, p0, 64, 0, spp, -1, 1, kBlockBlack});
      continue;
    }
    const float* w = pixel_work.data() + (size_t)lt * 1024;
    int p = 0;
    while (p < 1024) {
      const double e = S * w[p];
      if (spp > 1 && e > block_work) {  // split this pixel
        const int k = (spp + 63) / 64;  // ranges of <= 64 samples: one path per lane
        const int slot = nsplit++;
        for (int j = 0; j < k; ++j) {
          const int s0 = (int)((long long)spp * j / k), s1 = (int)((long long)spp * (j + 1) / k);
          v.push_back(B{(s1 - s0) * (double)w[p], lt, p, 1, s0, s1 - s0, slot, k, 0});
        }
        ++p;
        continue;
      }
      int np = 1;
      double sum = e;
      while (p + np < 1024 && np < big_pixels && S * w[p + np] <= block_work && sum + S * w[p + np] <= block_work) {
        sum += S * w[p + np];
        ++np;
      }
      v.push_back(B{sum, lt, p, np, 0, spp, -1, 1, 0});
      p += np;
    }
  }
  std::stable_sort(v.begin(), v.end(), [](const B& a, const B& b) { return a.est > b.est; });
  blocks->clear();
  for (const B& b : v)
    blocks->insert(blocks->end(), {b.lt, b.p0, b.np, b.s0, b.ns, b.slot, b.nsub, b.flags, 0, 0, 0, 0, 0, 0, 0, 0});
  return nsplit;
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

void tile_primary_masks(const FlatScene& fs, int32_t W, int32_t H, int32_t rank, int32_t world,
                        std::vector<unsigned long long>* masks) {
  masks->clear();
  const int tiles_x = (W + 31) / 32, tiles_y = (H + 31) / 32, ntiles = tiles_x * tiles_y;
  const int ns = (int)fs.spheres.size(), nt = (int)fs.tris.size();
  const double vw = 2.0 * fs.aspect;
  for (int t = rank; t < ntiles; t += world) {
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

void pixel_primary_masks(const FlatScene& fs, int32_t W, int32_t H, int32_t rank, int32_t world,
                         const std::vector<unsigned long long>& tile_masks, std::vector<unsigned long long>* pix) {
  const int tiles_x = (W + 31) / 32, ntiles = tiles_x * ((H + 31) / 32);
  const double vw = 2.0 * fs.aspect;
  const int local = (int)(tile_masks.size() / 2);
  pix->assign((size_t)local * 1024 * 2, 0ull);
  for (int lt = 0; lt < local; ++lt) {
    const int t = rank + lt * world;
    const unsigned long long ts = tile_masks[2 * lt], tt = tile_masks[2 * lt + 1];
    if (t >= ntiles || (ts | tt) == 0) continue;
    const int tx = t % tiles_x, ty = t / tiles_x;
    for (int q = 0; q < 1024; ++q) {
      const int x = tx * 32 + (q & 31), y = ty * 32 + (q >> 5);
      if (x >= W || y >= H) continue;
      double axis[3], cmin, smax;
      rect_cone(vw, W, H, x, x + 1, y, y + 1, axis, &cmin, &smax);
      unsigned long long* m = pix->data() + ((size_t)lt * 1024 + q) * 2;
      cone_masks(fs, axis, cmin, smax, ts, tt, &m[0], &m[1]);
    }
  }
}

void fill_block_masks(const std::vector<unsigned long long>& pix, std::vector<int32_t>* blocks) {
  for (size_t b = 0; b + kBlockInts <= blocks->size(); b += kBlockInts) {
    int32_t* r = blocks->data() + b;
    const int lt = r[0], p0 = r[1], np = std::min(r[2], 64);
    unsigned long long ms = 0, mt = 0, live = 0;
    for (int k = 0; k < np && p0 + k < 1024; ++k) {
      const unsigned long long* m = pix.data() + ((size_t)lt * 1024 + p0 + k) * 2;
      ms |= m[0];
      mt |= m[1];
      if (m[0] | m[1]) live |= 1ull << k;
    }
    r[8] = (int32_t)(uint32_t)ms;
    r[9] = (int32_t)(uint32_t)(ms >> 32);
    r[10] = (int32_t)(uint32_t)mt;
    r[11] = (int32_t)(uint32_t)(mt >> 32);
    r[12] = (int32_t)(uint32_t)live;
    r[13] = (int32_t)(uint32_t)(live >> 32);
  }
}

}  // namespace rtgo
