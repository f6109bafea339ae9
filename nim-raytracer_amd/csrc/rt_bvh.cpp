// rt_bvh.cpp — binned-SAH BVH2 builder (see rt_bvh.h).
#include "rt_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>

namespace rtmi {
namespace {

struct Box {
  double lo[3], hi[3];
  void reset() {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::numeric_limits<double>::infinity();
      hi[a] = -std::numeric_limits<double>::infinity();
    }
  }
  void grow(const Box& b) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], b.lo[a]);
      hi[a] = std::max(hi[a], b.hi[a]);
    }
  }
  void grow(const double* p) {
    for (int a = 0; a < 3; ++a) {
      lo[a] = std::min(lo[a], p[a]);
      hi[a] = std::max(hi[a], p[a]);
    }
  }
  bool empty() const { return !(lo[0] <= hi[0]); }
  double area() const {
    if (empty()) return 0.0;
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

struct ChildRef {
  int32_t c = -1;  // node index (internal) or first triangle (leaf)
  int32_t n = 0;   // 0 = internal, > 0 = leaf count
  Box box;
};

constexpr int kMedianDepth = 38;  // past this depth: object-median splits

struct Builder {
  const BvhBuildParams& prm;
  std::vector<Box> tri_box;
  std::vector<double> cen;  // nf*3 centroids
  std::vector<int32_t>& idx;
  std::vector<BvhNode>& nodes;
  double inflate = 0.0;
  int max_depth = 0;

  Builder(const BvhBuildParams& p, std::vector<int32_t>& order, std::vector<BvhNode>& n)
      : prm(p), idx(order), nodes(n) {}

  // Round a float64 bound outward to float32 after inflating by `inflate`.
  float lo32(double v) const {
    const double x = v - inflate;
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -std::numeric_limits<float>::infinity());
    return f;
  }
  float hi32(double v) const {
    const double x = v + inflate;
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, std::numeric_limits<float>::infinity());
    return f;
  }

  void set_child(BvhNode& nd, int which, const ChildRef& r) const {
    float* lo = which == 0 ? nd.lo0 : nd.lo1;
    float* hi = which == 0 ? nd.hi0 : nd.hi1;
    for (int a = 0; a < 3; ++a) {
      lo[a] = lo32(r.box.lo[a]);
      hi[a] = hi32(r.box.hi[a]);
    }
    if (which == 0) {
      nd.c0 = r.c;
      nd.n0 = r.n;
    } else {
      nd.c1 = r.c;
      nd.n1 = r.n;
    }
  }

  ChildRef make_leaf(int b, int e, const Box& bb) const {
    ChildRef r;
    r.c = b;
    r.n = e - b;
    r.box = bb;
    return r;
  }

  // Returns the split position in [b, e) or -1 to make a leaf.
  int split(int b, int e, int depth, const Box& bb) {
    const int n = e - b;
    Box cb;
    cb.reset();
    for (int i = b; i < e; ++i) cb.grow(&cen[3 * (size_t)idx[i]]);
    int axis = 0;
    double ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = cb.hi[a] - cb.lo[a];
    if (ext[1] > ext[axis]) axis = 1;
    if (ext[2] > ext[axis]) axis = 2;
    const auto median = [&](int ax) {
      const int mid = b + n / 2;
      std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e, [&](int32_t x, int32_t y) {
        const double cx = cen[3 * (size_t)x + ax], cy = cen[3 * (size_t)y + ax];
        return cx < cy || (cx == cy && x < y);
      });
      return mid;
    };
    if (!(ext[axis] > 0.0)) return n <= prm.max_leaf ? -1 : median(axis);
    if (depth >= kMedianDepth) return n <= prm.max_leaf ? -1 : median(axis);
    if (n <= prm.max_leaf) return -1;

    const int NB = prm.bins;
    double best_cost = std::numeric_limits<double>::infinity();
    int best_axis = -1, best_bin = -1;
    std::vector<Box> bin_box(NB);
    std::vector<int> bin_cnt(NB);
    std::vector<double> right_area(NB);
    std::vector<int> right_cnt(NB);
    for (int a = 0; a < 3; ++a) {
      if (!(ext[a] > 0.0)) continue;
      const double scale = NB / ext[a];
      for (int k = 0; k < NB; ++k) {
        bin_box[k].reset();
        bin_cnt[k] = 0;
      }
      for (int i = b; i < e; ++i) {
        const int32_t t = idx[i];
        int k = (int)((cen[3 * (size_t)t + a] - cb.lo[a]) * scale);
        k = std::min(std::max(k, 0), NB - 1);
        bin_box[k].grow(tri_box[t]);
        bin_cnt[k]++;
      }
      Box acc;
      acc.reset();
      int cnt = 0;
      for (int k = NB - 1; k > 0; --k) {
        acc.grow(bin_box[k]);
        cnt += bin_cnt[k];
        right_area[k] = acc.area();
        right_cnt[k] = cnt;
      }
      acc.reset();
      cnt = 0;
      for (int k = 0; k < NB - 1; ++k) {
        acc.grow(bin_box[k]);
        cnt += bin_cnt[k];
        const int rc = right_cnt[k + 1];
        if (cnt == 0 || rc == 0) continue;
        const double cost = acc.area() * cnt + right_area[k + 1] * rc;
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = a;
          best_bin = k;
        }
      }
    }
    const double parent_area = bb.area();
    const double leaf_cost = prm.cost_tri * n;
    const double split_cost =
        prm.cost_node + (parent_area > 0.0 ? prm.cost_tri * best_cost / parent_area : 0.0);
    if (best_axis < 0) return median(axis);
    if (n <= prm.max_leaf && leaf_cost <= split_cost) return -1;
    const double scale = NB / ext[best_axis];
    const auto mid_it = std::partition(idx.begin() + b, idx.begin() + e, [&](int32_t t) {
      int k = (int)((cen[3 * (size_t)t + best_axis] - cb.lo[best_axis]) * scale);
      k = std::min(std::max(k, 0), NB - 1);
      return k <= best_bin;
    });
    const int mid = (int)(mid_it - idx.begin());
    if (mid == b || mid == e) return median(axis);
    return mid;
  }

  Box range_box(int b, int e) const {
    Box bb;
    bb.reset();
    for (int i = b; i < e; ++i) bb.grow(tri_box[idx[i]]);
    return bb;
  }

  // Builds [b, e) below a node at `depth` (root = depth 1).
  ChildRef build(int b, int e, int depth) {
    const Box bb = range_box(b, e);
    const int s = split(b, e, depth, bb);
    if (s < 0) return make_leaf(b, e, bb);
    const int32_t me = (int32_t)nodes.size();
    nodes.emplace_back();
    max_depth = std::max(max_depth, depth);
    const ChildRef l = build(b, s, depth + 1);
    const ChildRef r = build(s, e, depth + 1);
    set_child(nodes[me], 0, l);
    set_child(nodes[me], 1, r);
    ChildRef out;
    out.c = me;
    out.n = 0;
    out.box = bb;
    return out;
  }
};

}  // namespace

bool build_bvh(const double* v, const int32_t* f, int64_t nf, const BvhBuildParams& prm, BvhResult* out,
               const char** err) {
  out->nodes.clear();
  out->order.clear();
  out->max_depth = 0;
  if (nf <= 0) return true;
  if (nf > (int64_t)1 << 30) {
    *err = "mesh too large (> 2^30 faces)";
    return false;
  }
  out->order.resize((size_t)nf);
  for (int64_t i = 0; i < nf; ++i) out->order[(size_t)i] = (int32_t)i;
  Builder B(prm, out->order, out->nodes);
  B.tri_box.resize((size_t)nf);
  B.cen.resize((size_t)nf * 3);
  double mag = 0.0;
  Box all;
  all.reset();
  for (int64_t i = 0; i < nf; ++i) {
    Box& tb = B.tri_box[(size_t)i];
    tb.reset();
    for (int k = 0; k < 3; ++k) tb.grow(&v[3 * (size_t)f[3 * i + k]]);
    all.grow(tb);
    for (int a = 0; a < 3; ++a) {
      B.cen[3 * (size_t)i + a] = 0.5 * (tb.lo[a] + tb.hi[a]);
      mag = std::max(mag, std::max(std::fabs(tb.lo[a]), std::fabs(tb.hi[a])));
    }
  }
  double extent = 0.0;
  for (int a = 0; a < 3; ++a) extent = std::max(extent, all.hi[a] - all.lo[a]);
  if (!std::isfinite(mag) || !std::isfinite(extent)) {
    *err = "mesh has non-finite vertices";
    return false;
  }
  // conservative margin: ~2^-20 of the mesh scale (see rt_bvh.h)
  B.inflate = std::ldexp(std::max(extent, mag), -20) + 1e-30;
  out->nodes.reserve((size_t)(2 * nf / std::max(1, prm.max_leaf) + 2));
  const int32_t root = 0;
  out->nodes.emplace_back();
  const Box bb = B.range_box(0, (int)nf);
  const int s = B.split(0, (int)nf, 1, bb);
  ChildRef l, r;
  if (s < 0) {
    // a single leaf: the root's second slot repeats it, so every child of
    // every node is valid (the kernels skip no-child checks); a repeated
    // triangle can only tie with itself and never changes the closest hit
    l = B.make_leaf(0, (int)nf, bb);
    r = l;
  } else {
    l = B.build(0, s, 2);
    r = B.build(s, (int)nf, 2);
  }
  B.set_child(out->nodes[root], 0, l);
  B.set_child(out->nodes[root], 1, r);
  out->max_depth = std::max(1, B.max_depth);
  if (out->max_depth > kMaxBvhDepth) {
    *err = "BVH deeper than the traversal stack";
    return false;
  }
  return validate_bvh(*out, nf, err);
}

bool validate_bvh(const BvhResult& r, int64_t nf, const char** err) {
  const int32_t nn = (int32_t)r.nodes.size();
  if (nf > 0 && nn == 0) {
    *err = "BVH has no root";
    return false;
  }
  std::vector<unsigned char> seen((size_t)nf, 0);
  int64_t covered = 0;
  const bool single = nn == 1 && r.nodes[0].n0 > 0 && r.nodes[0].c0 == r.nodes[0].c1 &&
                      r.nodes[0].n0 == r.nodes[0].n1;  // one leaf, repeated in both slots
  for (const BvhNode& nd : r.nodes) {
    const int32_t cs[2] = {nd.c0, nd.c1}, ns[2] = {nd.n0, nd.n1};
    for (int k = 0; k < 2; ++k) {
      if (ns[k] > 0) {
        if (cs[k] < 0 || (int64_t)cs[k] + ns[k] > nf) {
          *err = "BVH leaf out of range";
          return false;
        }
        if (single && k == 1) continue;
        for (int32_t i = cs[k]; i < cs[k] + ns[k]; ++i) {
          if (seen[(size_t)i]) {
            *err = "BVH leaves overlap";
            return false;
          }
          seen[(size_t)i] = 1;
          ++covered;
        }
      } else if (cs[k] >= nn || cs[k] <= 0) {  // internal: never the root, never empty
        *err = "BVH child out of range";
        return false;
      }
    }
  }
  if (covered != nf || (int64_t)r.order.size() != nf) {
    *err = "BVH leaves do not cover every face";
    return false;
  }
  std::fill(seen.begin(), seen.end(), 0);
  for (int32_t f : r.order) {
    if (f < 0 || f >= nf || seen[(size_t)f]) {
      *err = "BVH face order is not a permutation";
      return false;
    }
    seen[(size_t)f] = 1;
  }
  return true;
}

}  // namespace rtmi
