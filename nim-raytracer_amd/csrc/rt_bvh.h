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
  int max_leaf = kLeafMax;  // triangles per leaf, SAH may stop earlier (4 measured best:
                            // C3 8.45 ms vs 8.54 at 6 and 8.73 at 8)
  int bins = 32;            // SAH bins per axis
  float cost_node = 1.0f;   // relative cost of one node fetch (two boxes)
  float cost_tri = 1.0f;    // relative cost of one triangle test
};

struct BvhResult {
  std::vector<BvhNode> nodes;       // nodes[0] = root, depth-first order
  std::vector<int32_t> order;       // leaf-ordered original face indices
  int max_depth = 0;
};


// vertices: nv*3 doubles; faces: nf*3 indices (validated by the caller).
bool build_bvh(const double* vertices, const int32_t* faces, int64_t nf, const BvhBuildParams& prm,
               BvhResult* out, const char** err);

}  // namespace rtmi
