// rt_bvh.h — BVH2 builders for one triangle mesh: host binned SAH, device PLOC.
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

// Device builder (rt_bvh_gpu.hip): PLOC clustering + SAH collapse on the
// current HIP device, same node format, leaf limit and conservative bounds.
// d_vertices / d_faces are device copies of the mesh arrays.
bool build_bvh_device(const double* d_vertices, const int32_t* d_faces, int64_t nf, const BvhBuildParams& prm,
                      BvhResult* out, const char** err);

// Device packing of one mesh's triangle records in BVH leaf order (d_order:
// leaf slot -> face): rt_common.h TriFast for the float32 kernel and TriF64
// for the float64 one, rounded exactly as a host loop would. All pointers are
// device pointers; stream is a hipStream_t.
bool pack_triangles_device(const double* d_vertices, const int32_t* d_faces, const int32_t* d_order, int64_t nf,
                           TriFast* d_fast, TriF64* d_f64, void* stream);

// Structure check shared by both builders: every child reference in range,
// no inner node points at the root, leaves cover every face exactly once.
bool validate_bvh(const BvhResult& r, int64_t nf, const char** err);

}  // namespace rtmi
