// rt_bvh.h — host BVH2 builder (binned SAH) for one triangle mesh.
//
// The reference has no acceleration structure: TriangleMesh.intersect loops
// over every face (src/renderer/geom.nim:339-358). This BVH is new; it is
// built so that traversal returns exactly the brute-force answer (closest
// t >= 0, lowest face index on ties): node boxes are the exact float64 face
// bounds inflated by a small relative margin and rounded outward to float32,
// so box culling is conservative in both precisions.
#pragma once
#include <cstdint>
#include <vector>

#include "rt_common.h"

namespace rtmi {

struct BvhBuildParams {
  int max_leaf = kLeafMax;  // triangles per leaf, SAH may stop earlier
  int bins = 32;            // SAH bins per axis
  float cost_node = 1.0f;   // relative cost of one node fetch (two boxes)
  float cost_tri = 1.0f;    // relative cost of one triangle test
};

struct BvhResult {
  std::vector<BvhNode> nodes;       // nodes[0] = root, depth-first order
  std::vector<int32_t> order;       // leaf-ordered original face indices
  int max_depth = 0;
};

// Collapse a BVH2 into a BVH4 (greedy: expand the internal child with the
// largest surface area until four slots are used). Leaves keep their triangle
// ranges; boxes are copied from the BVH2 (already conservative fp32).
bool collapse_bvh4(const BvhResult& b2, std::vector<Bvh4Node>* out, int* max_depth, const char** err);

// vertices: nv*3 doubles; faces: nf*3 indices (validated by the caller).
bool build_bvh(const double* vertices, const int32_t* faces, int64_t nf, const BvhBuildParams& prm,
               BvhResult* out, const char** err);

}  // namespace rtmi
