// rt_bins.h — triangle lists for coherent ray families of the float32 kernel.
//
// The BVH answers "which faces can this ray hit" for any ray. Two ray
// families of the reference's renderer are much more regular:
//   * camera rays (castPrimaryRay, renderer.nim:31-44) all leave the camera
//     origin, and the samples of one pixel stay inside that pixel's square;
//   * shadow rays to a distant light (renderer.nim:93-104 with
//     light.nim:46-50) are parallel.
// For each, the faces of the scene's mesh are binned once by their
// conservative projection — onto the image (pixel lists) or onto the plane
// orthogonal to the light (light grids) — and a ray tests only its bin's
// faces. A bin holds every face whose projection, grown by a margin far above
// the float32 error of the ray set-up and of the triangle test, touches the
// bin; faces that can never pass the single-sided det cull for that family
// (back faces w.r.t. the camera or the light, geom.nim:306) are left out.
// The search over a bin uses the same (t, face) key as the BVH search, so the
// closest hit, the shadow early exit and every Stats count are those of the
// BVH path (bit-identical frames, tests/test_gpu_bins.py).
#pragma once
#include <stdint.h>

#include <vector>

#include "rt_common.h"

namespace rtmi {

// One face of the binned mesh: object-space vertices (float64, as given) and
// the byte offset of its TriFast record in FastData.tree.
struct BinTri {
  double v[3][3];
  int32_t rec;
};

// Pixel lists: off[y * w + x] .. off[y * w + x + 1] index ent[] (record byte
// offsets); ent[] is padded with kBinPad entries so a kernel may read ahead.
constexpr int kBinPad = 4;
struct PixelBinsHost {
  std::vector<int32_t> off, ent;
};
// o2w / w2o: the mesh object's transforms, c2w: camera, column-major (glm).
// Returns false (with *why) when the camera set-up does not allow binning
// (a face vertex at or behind the camera plane).
bool build_pixel_bins(const std::vector<BinTri>& tris, const double o2w[16], const double w2o[16],
                      const double c2w[16], double fov_deg, int width, int height, PixelBinsHost* out,
                      const char** why);

// Light grid of one distant light (rt_common.h LightGrid), host side.
struct LightGridHost {
  LightGrid g;
  std::vector<int32_t> off, ent;  // off: gu * gv + 1 (entry indices local to ent)
};
// dir: the light's travel direction (world); shadow rays go along -dir.
bool build_light_grid(const std::vector<BinTri>& tris, const double w2o[16], const double dir[3],
                      LightGridHost* out, const char** why);

}  // namespace rtmi
