// bvh.cpp — binned-SAH bounding volume hierarchy over spheres.
//
// The reference's live path has no acceleration structure: hitWorld is a
// linear closest-hit scan (internal/renderer/renderer.go:333-346), and its
// only BVH (internal/optimization/spatial_acceleration.go:9-69) does not
// compile.  This BVH is a pure accelerator introduced by the build for the
// 10k-sphere configurations: traversal returns the
// same closest hit as the linear scan (same Sphere.Hit arithmetic, exact-t
// ties resolved by hittable index, as in the scan).
//
// Layout: nodes in breadth-first order with the two children of an internal
// node adjacent (left = i, right = i + 1), 32 B each, float bounds rounded
// outward by one ulp so a box never excludes a point of its spheres.  Every
// sphere box is also padded by pad = 2^-18 * M, M the largest coordinate
// magnitude of the scene (sphere extents and the camera): the kernel's slab
// test runs in binary32 on the ray origin rounded to float, an error of at
// most 2^-24 * M per axis, which the padding covers 64 times over.
// Spheres are reordered so every leaf is a contiguous range.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "rt_internal.h"

namespace rtgo {

namespace {

struct Box {
  double lo[3], hi[3];
  void reset() {
    for (int k = 0; k < 3; ++k) {
      lo[k] = INFINITY;
      hi[k] = -INFINITY;
    }
  }
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow_pt(const double p[3]) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  double area() const {
    double e[3];
    for (int k = 0; k < 3; ++k) e[k] = std::max(0.0, hi[k] - lo[k]);
    return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
  }
};

float down(double v) {
  float f = (float)v;
  if ((double)f > v) f = nextafterf(f, -INFINITY);
  return nextafterf(f, -INFINITY);
}
float up(double v) {
  float f = (float)v;
  if ((double)f < v) f = nextafterf(f, INFINITY);
  return nextafterf(f, INFINITY);
}

constexpr int kMaxBins = 64;
constexpr int kDefaultBins = 32;  // SAH bins per axis (C4: 807 ms at 16, 796 at 32)
constexpr int kDefaultLeaf = 4;   // spheres per leaf at most (C4: 872 ms at 2, 840 at 3, 825 at 6)

}  // namespace

void build_sphere_bvh(FlatScene* fs, int bins, int leaf) {
  // rt_tuning: bins, leaf (<= 7: a 3-bit count); 0 = the defaults
  const int kBins = bins > 0 ? std::max(2, std::min(kMaxBins, bins)) : kDefaultBins;
  const int kLeafMax = leaf > 0 ? std::min(7, leaf) : kDefaultLeaf;
  fs->bvh.clear();
  fs->qbvh.clear();
  fs->qbvh4.clear();
  fs->bvh4_stack = 0;
  fs->bvh4_root = 0;
  const int n = (int)fs->spheres.size();
  if (n == 0) return;
  std::vector<Box> pb(n);
  std::vector<double> cen(3 * (size_t)n);
  double M = 1.0;
  for (int k = 0; k < 3; ++k) M = std::max(M, fabs(fs->cam_pos[k]));
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) M = std::max(M, fabs(fs->spheres[i].c[k]) + fabs(fs->spheres[i].r));
  const double pad = ldexp(M, -18);
  for (int i = 0; i < n; ++i) {
    const DSphere& s = fs->spheres[i];
    double r = fabs(s.r);
    for (int k = 0; k < 3; ++k) {
      pb[i].lo[k] = s.c[k] - r - pad;
      pb[i].hi[k] = s.c[k] + r + pad;
      cen[3 * (size_t)i + k] = s.c[k];
    }
  }
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;

  struct Task {
    int node, first, count;
  };
  std::vector<DBVHNode> nodes;
  nodes.reserve(2 * (size_t)n);
  nodes.push_back(DBVHNode{});
  std::vector<Task> stack;
  stack.push_back({0, 0, n});
  while (!stack.empty()) {
    Task t = stack.back();
    stack.pop_back();
    Box b, cb;
    b.reset();
    cb.reset();
    for (int i = t.first; i < t.first + t.count; ++i) {
      b.grow(pb[idx[i]]);
      cb.grow_pt(&cen[3 * (size_t)idx[i]]);
    }
    DBVHNode& nd = nodes[t.node];
    for (int k = 0; k < 3; ++k) {
      nd.lo[k] = down(b.lo[k]);
      nd.hi[k] = up(b.hi[k]);
    }
    auto make_leaf = [&]() {
      nodes[t.node].left_or_first = t.first;
      nodes[t.node].count = t.count;
    };
    if (t.count <= kLeafMax) {
      make_leaf();
      continue;
    }
    // binned SAH along each axis
    double best_cost = INFINITY;
    int best_axis = -1, best_split = -1;
    for (int ax = 0; ax < 3; ++ax) {
      double ext = cb.hi[ax] - cb.lo[ax];
      if (!(ext > 0)) continue;
      Box bins[kMaxBins];
      int cnt[kMaxBins] = {0};
      for (int k = 0; k < kBins; ++k) bins[k].reset();
      const double scale = kBins / ext;
      for (int i = t.first; i < t.first + t.count; ++i) {
        int bi = (int)((cen[3 * (size_t)idx[i] + ax] - cb.lo[ax]) * scale);
        bi = std::min(std::max(bi, 0), kBins - 1);
        bins[bi].grow(pb[idx[i]]);
        cnt[bi]++;
      }
      double la[kMaxBins], ra[kMaxBins];
      int lc[kMaxBins], rc[kMaxBins];
      Box acc;
      acc.reset();
      int c = 0;
      for (int k = 0; k < kBins; ++k) {
        acc.grow(bins[k]);
        c += cnt[k];
        la[k] = acc.area();
        lc[k] = c;
      }
      acc.reset();
      c = 0;
      for (int k = kBins - 1; k >= 0; --k) {
        acc.grow(bins[k]);
        c += cnt[k];
        ra[k] = acc.area();
        rc[k] = c;
      }
      for (int k = 0; k < kBins - 1; ++k) {
        if (lc[k] == 0 || rc[k + 1] == 0) continue;
        double cost = la[k] * lc[k] + ra[k + 1] * rc[k + 1];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = ax;
          best_split = k;
        }
      }
    }
    int mid;
    if (best_axis < 0) {
      // all centroids coincide: split by count
      mid = t.first + t.count / 2;
    } else {
      const double ext = cb.hi[best_axis] - cb.lo[best_axis];
      const double scale = kBins / ext;
      auto it = std::partition(idx.begin() + t.first, idx.begin() + t.first + t.count, [&](int i) {
        int bi = (int)((cen[3 * (size_t)i + best_axis] - cb.lo[best_axis]) * scale);
        bi = std::min(std::max(bi, 0), kBins - 1);
        return bi <= best_split;
      });
      mid = (int)(it - idx.begin());
      if (mid == t.first || mid == t.first + t.count) mid = t.first + t.count / 2;
    }
    const int left = (int)nodes.size();
    nodes.push_back(DBVHNode{});
    nodes.push_back(DBVHNode{});
    nodes[t.node].left_or_first = left;
    nodes[t.node].count = 0;
    stack.push_back({left + 1, mid, t.first + t.count - mid});
    stack.push_back({left, t.first, mid - t.first});
  }
  // breadth-first renumbering (child pairs stay adjacent): the top levels of
  // the tree become a prefix of the node array, which the wavefront traversal
  // kernels stage in LDS (rt_wavefront.hip stage_tree)
  {
    std::vector<DBVHNode> bfs;
    bfs.reserve(nodes.size());
    bfs.push_back(nodes[0]);
    for (size_t i = 0; i < bfs.size(); ++i) {
      if (bfs[i].count != 0) continue;
      const int old = bfs[i].left_or_first;
      bfs[i].left_or_first = (int)bfs.size();
      bfs.push_back(nodes[old]);
      bfs.push_back(nodes[old + 1]);
    }
    nodes.swap(bfs);
  }
  // depth check: traversal keeps at most depth-1 pending children on its
  // per-lane LDS stack, which the kernels size to the tree's depth (at most
  // kStack = 40 entries)
  {
    std::vector<std::pair<int, int>> st = {{0, 1}};
    int maxd = 0;
    while (!st.empty()) {
      auto [ni, dep] = st.back();
      st.pop_back();
      maxd = std::max(maxd, dep);
      if (nodes[ni].count == 0) {
        st.push_back({nodes[ni].left_or_first, dep + 1});
        st.push_back({nodes[ni].left_or_first + 1, dep + 1});
      }
    }
    if (maxd > kStack) {
      fs->bvh.clear();  // too deep for the stack: keep the linear scan
      return;
    }
    fs->bvh_depth = maxd;
  }
  // quantized copy: a grid of 65000 steps per axis over the root box with 4
  // steps of margin; lo rounded down, hi up, one more step each way, and the
  // decoded box checked to contain the float box
  {
    const DBVHNode& r = nodes[0];
    for (int k = 0; k < 3; ++k) {
      const double ext = (double)r.hi[k] - (double)r.lo[k];
      fs->qd[k] = ext > 0 ? ext / 65000.0 : 1.0;
      fs->q0[k] = (double)r.lo[k] - 4 * fs->qd[k];
    }
    fs->qbvh.resize(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) {
      const DBVHNode& nd = nodes[i];
      uint32_t ql[3], qh[3];
      for (int k = 0; k < 3; ++k) {
        double a = floor(((double)nd.lo[k] - fs->q0[k]) / fs->qd[k]) - 1;
        double b = ceil(((double)nd.hi[k] - fs->q0[k]) / fs->qd[k]) + 1;
        a = std::min(std::max(a, 0.0), 65535.0);
        b = std::min(std::max(b, 0.0), 65535.0);
        if (!(fs->q0[k] + a * fs->qd[k] <= (double)nd.lo[k]) || !(fs->q0[k] + b * fs->qd[k] >= (double)nd.hi[k])) {
          fs->bvh.clear();  // cannot happen for finite boxes; keep the linear scan rather than cull wrongly
          fs->qbvh.clear();
          return;
        }
        ql[k] = (uint32_t)a;
        qh[k] = (uint32_t)b;
      }
      DQNode& q = fs->qbvh[i];
      q.w[0] = ql[0] | (qh[0] << 16);  // per axis (lo, hi): the kernel picks near / far per ray
      q.w[1] = ql[1] | (qh[1] << 16);
      q.w[2] = ql[2] | (qh[2] << 16);
      q.w[3] = (uint32_t)((nd.left_or_first << 3) | nd.count);
    }
  }
  // 4-wide form for the closest-hit and occlusion traversals (rt_wavefront.hip
  // descend4): every group holds 2..4 nodes of the binary tree that cover one
  // internal node's subtree (its children, then the largest internal one
  // among them replaced by its own children), with the quantized boxes and
  // codes of qbvh.  Groups are stored back to back, breadth-first, without
  // empty slots; an internal slot's code is (its group's first slot << 5) |
  // (its size - 1) << 3, so the low 3 bits stay 0 as in qbvh; 3 padding slots
  // at the end keep a group's 4-slot load inside the array.  Same leaves,
  // same boxes: the spheres a ray tests are the binary traversal's.
  {
    auto area = [&](int i) {
      const DBVHNode& b = nodes[i];
      const double x = (double)b.hi[0] - b.lo[0], y = (double)b.hi[1] - b.lo[1], z = (double)b.hi[2] - b.lo[2];
      return x * y + y * z + z * x;
    };
    fs->qbvh4.clear();
    fs->bvh4_stack = 0;
    fs->bvh4_root = 0;
    if (nodes[0].count == 0) {
      std::vector<int> bin = {0}, pend = {0};
      std::vector<std::vector<int>> kids;
      std::vector<std::vector<int>> sub;  // per kid: its group, or -1 (a leaf)
      for (size_t g = 0; g < bin.size(); ++g) {
        std::vector<int> k = {nodes[bin[g]].left_or_first, nodes[bin[g]].left_or_first + 1};
        while (k.size() < 4) {
          int best = -1;
          for (int i = 0; i < (int)k.size(); ++i)
            if (nodes[k[i]].count == 0 && (best < 0 || area(k[i]) > area(k[best]))) best = i;
          if (best < 0) break;
          const int b = k[best];
          k[best] = nodes[b].left_or_first;
          k.insert(k.begin() + best + 1, nodes[b].left_or_first + 1);
        }
        const int pd = pend[g] + (int)k.size() - 1;
        fs->bvh4_stack = std::max(fs->bvh4_stack, pd);
        std::vector<int> sg(k.size(), -1);
        for (size_t i = 0; i < k.size(); ++i)
          if (nodes[k[i]].count == 0) {
            sg[i] = (int)bin.size();
            bin.push_back(k[i]);
            pend.push_back(pd);
          }
        kids.push_back(std::move(k));
        sub.push_back(std::move(sg));
      }
      std::vector<int> base(kids.size() + 1, 0);
      for (size_t g = 0; g < kids.size(); ++g) base[g + 1] = base[g] + (int)kids[g].size();
      auto code = [&](int g) { return (uint32_t)(base[g] << 5) | (uint32_t)((kids[g].size() - 1) << 3); };
      fs->qbvh4.resize(base[kids.size()] + 3);
      for (size_t g = 0; g < kids.size(); ++g)
        for (size_t i = 0; i < kids[g].size(); ++i) {
          DQNode e = fs->qbvh[kids[g][i]];
          if (sub[g][i] >= 0) e.w[3] = code(sub[g][i]);
          fs->qbvh4[base[g] + i] = e;
        }
      for (int i = 0; i < 3; ++i) {
        DQNode& e = fs->qbvh4[base[kids.size()] + i];
        e.w[0] = e.w[1] = e.w[2] = 0x0000FFFFu;
        e.w[3] = ~0u;
      }
      fs->bvh4_root = (int32_t)code(0);
    }
  }
  std::vector<DSphere> reordered(n);
  for (int i = 0; i < n; ++i) reordered[i] = fs->spheres[idx[i]];
  fs->spheres.swap(reordered);
  fs->bvh.swap(nodes);
}

}  // namespace rtgo
