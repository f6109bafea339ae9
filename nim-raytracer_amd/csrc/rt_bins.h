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

#include "rt_bins_geom.h"
#include "rt_common.h"

namespace rtmi {

// Growth of a pixel's square (in pixels) in every camera-ray bin: a pixel's
// bins (face lists, object masks, shadow skips) cover every ray through
// [x - kPixelMargin, x + 1 + kPixelMargin] x [y - ..., y + 1 + ...]. That
// holds for the kernels' camera rays as long as every sample offset lies in
// [0, 1) — true for all of sampling.nim's samplers (akNone: 0, grid:
// (i + 1/2)/m, jittered / multi-jittered / correlated: [0, 1)), checked on
// the host (rtmi.cpp sampler_in_pixel) before any bin is handed to a kernel —
// and the margin is far above the float32 error of the ray set-up.
constexpr double kPixelMargin = 0.05;

// One face of the binned mesh: object-space vertices (float64, as given) and
// the byte offset of its TriFast record in FastData.tree.
struct BinTri {
  double v[3][3];
  int32_t rec;
  int32_t face;  // the face's index in its mesh (TriFast.id)
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
  // per face (leaf order, record rec0 + 64 i): its projection's bounding box
  // grown by the lists' margin (u0, u1, v0, v1), NaN for faces never listed
  std::vector<double> box;
  int32_t rec0 = 0;
};
// dir: the light's travel direction (world); shadow rays go along -dir.
bool build_light_grid(const std::vector<BinTri>& tris, const double w2o[16], const double dir[3],
                      LightGridHost* out, const char** why);

// Shadow skips. Per pixel, bit l (l < 8): every shadow ray to distant light
// l that leaves a camera hit of this pixel provably meets no face of the mesh,
// so the kernel drops the mesh from that wave's shadow trace (the mesh could
// only have answered "miss"). Built for scenes of one mesh and planes: a pixel
// qualifies when its camera-ray list is empty (its rays hit planes or
// nothing), and the footprint of its rays on every plane they reach — the
// quad of the pixel's (grown) corner rays, moved by the shadow-ray bias and
// grown by a float32 error margin — covers only empty cells of the light's
// grid (a cell range checked on the grid's occupancy prefix sums) or lies off
// the grid. Pixels whose corner rays straddle a plane's horizon do not
// qualify.
struct GridOcc {
  LightGrid g{};                 // g.gu == 0: no grid for this light
  std::vector<int32_t> sat;      // (gu + 1) x (gv + 1) prefix counts of non-empty cells
  const LightGridHost* lists = nullptr;  // the grid's cell lists and face boxes (shadow lists)
};
void grid_occupancy(const LightGridHost& lg, GridOcc* out);
void skip_grid(const GridOcc& go, bg::SkipGrid* out);  // the skip test's view (sat points into go)
struct SkipPlane {
  double o2w[16], w2o[16];       // a plane object's transforms (y = 0 in object space)
};
// Per-camera constants of the camera-ray bins (rt_bins_geom.h PixCam) and of
// the shadow skips (SkipCam + one SkipPlaneC per plane); false: a singular
// camera (pixel_camera) or a camera on a plane (skip_camera: no pixel
// qualifies).
bool pixel_camera(const double o2w[16], const double w2o[16], const double c2w[16], double fov_deg, int width,
                  int height, bg::PixCam* out);
bool skip_camera(const std::vector<SkipPlane>& planes, const double mesh_w2o[16], const double c2w[16],
                 double fov_deg, int width, int height, double bias, bg::SkipCam* cam,
                 std::vector<bg::SkipPlaneC>* pc);
// pix_off: the pixel lists' offsets (w * h + 1); out: one byte per pixel,
// packed four to a dword (pixel 4i + k in byte k of out[i]).
//
// Per-pixel shadow lists (sl != nullptr, the grids' `lists` set): for a
// qualifying pixel and a light l whose skip bit stays clear, the faces whose
// grown projected box meets the grown footprint of the pixel's shadow-ray
// origins on the planes it reaches — every face any such shadow ray can hit —
// deduplicated, those covering most of the footprint first, at most
// kShadowListMax. sl[2 (pix * nl + l)] = start in *sl_ent, sl[.. + 1] =
// count, -1: no list (the kernel searches the light's grid cells).
constexpr int kShadowListMax = 48;
bool build_shadow_skips(const std::vector<int32_t>& pix_off, const std::vector<SkipPlane>& planes,
                        const double mesh_w2o[16], const std::vector<GridOcc>& grids, const double c2w[16],
                        double fov_deg, int width, int height, double bias, std::vector<uint32_t>* out,
                        const char** why, std::vector<int32_t>* sl = nullptr, std::vector<int32_t>* sl_ent = nullptr,
                        int sl_nl = 0);

}  // namespace rtmi

namespace rtmi {

// Object bins (scenes of 4..64 objects): per pixel / per light-grid cell a
// 64-bit mask of the objects whose world bounding box can meet the bin's rays
// (bit i = object i, so the trace visits the listed objects in scene order).
// An object that can only be hit by rays through its bounding box in front of
// the ray origin (spheres, boxes, meshes: geom.nim:76-96, 215-237, 339-358)
// and is not hit contributes nothing to the closest hit or to Stats' hit count,
// so skipping it is exact; planes (unbounded) are in every bin.
struct ObjBox {
  bool always;       // in every bin (planes, boxes that cannot be projected)
  double lo[3], hi[3];  // world-space bounding box
  // the object box's 8 corners in world space (through the inverse of the
  // world_to_object the kernel transforms rays with); the light grids bin
  // the convex hull of their projection instead of its bounding rectangle
  double corner[8][3];
};
bool build_object_pixel_masks(const std::vector<ObjBox>& objs, const double c2w[16], double fov_deg, int width,
                              int height, std::vector<unsigned long long>* masks, const char** why);
struct ObjGridHost {
  LightGrid g;                           // off_base unused; rmax: float32-safe origin radius
  std::vector<unsigned long long> masks; // gu * gv cell masks
  unsigned long long off_grid = 0;       // mask of a safe lane outside the grid (planes)
};
bool build_object_light_grid(const std::vector<ObjBox>& objs, const double dir[3], ObjGridHost* out,
                             const char** why);

}  // namespace rtmi
