// rt_frame.h — per-call (per-frame) device builders of the float32 kernel's
// camera-dependent data: the camera-ray face lists of the launch's pixels,
// their pixel records (list length + shadow skip bits), the lean / general
// lists of a two-class launch, and the object masks of analytic scenes.
//
// The reference does every per-pixel piece of work on every renderLine call
// (renderer.nim:162-211); so does this build: nothing that depends on the
// camera is kept from one render call to the next. What is built once per
// scene (rt_scene_create) depends only on the scene's geometry and lights:
// the BVH, the light grids and their occupancy prefix sums, the faces'
// float64 vertices. Each render call runs, on its own stream, three build
// launches before its render kernels (round 4; round 3 took ten):
//   k_frame_build1   blocks [0, face_blocks): per face (one thread) its
//                    pixel rectangle, a launch-row test and the cull, then
//                    the block's (face, pixel) pairs dealt out over its
//                    threads: for a face of <= kBigFace pixels a SAT test
//                    per pixel of the launch; a listed
//                    pixel's counter hands out its slot (atomicAdd) and the
//                    face's record offset goes straight into the pixel's
//                    fixed block of 2^slot_lg slots — no count / scan / fill
//                    passes. Larger faces go onto the huge list.
//                    the other blocks: per 64 x 4 tile of the launch, the
//                    shadow skips its pixels share (one test for the tile);
//                    block 0 also zeroes the render kernels' queue heads +
//                    Stats words.
//   k_frame_build2   one block per tile: per pixel its huge faces (the tile's
//                    share of the huge list, a SAT test each, appended after
//                    the small faces), its record (list length + skip bits:
//                    the tile's, or the pixel's own test), its counter zeroed
//                    for the next call; with a split, the tile's lean /
//                    general counts.
//   k_frame_lists    (two-class launches) one block per 16 tiles: its offsets
//                    summed by the block itself from every earlier tile's
//                    counts (no inter-block hand-off, no scan launch), its
//                    pixels written to the lean / general lists in tile order.
// A pixel with more listed faces than its 2^slot_lg slots keeps its true
// count in the record; the render kernels then traverse the BVH for that
// pixel's camera rays (the same answers, rt_fast.h mesh_search) — exact, no
// failure mode.
//   k_frame_obj_masks    (scenes of 4..64 objects) per pixel: 64-bit object mask
// Every geometric bound is rt_bins_geom.h's, shared with the host builders
// the tests compare against (float64, no FMA contraction on either side).
#pragma once
#include <stdint.h>

#include "rt_bins_geom.h"
#include "rt_common.h"

namespace rtmi {

constexpr int kFrameMaxPlanes = 8;

// The image rows of one launch (rtmi.cpp Mapping): mode 0 rows
// y0 + k * step (k < nrows) and columns x = j * step, mode 1 the rank's
// round-robin bands (every column).
struct FrameRows {
  int32_t mode, y0, nrows, step, band_h, rank, world, height;
};
__host__ __device__ inline bool frame_has_row(const FrameRows& r, int y) {
  if (y < 0 || y >= r.height) return false;
  if (r.mode == 0) {
    const int d = y - r.y0;
    return d >= 0 && d < r.nrows * r.step && d % r.step == 0;
  }
  return (y / r.band_h) % r.world == r.rank;
}
// some launch row in [ylo, yhi] (ylo <= yhi)
__host__ __device__ inline bool frame_meets_rows(const FrameRows& r, int ylo, int yhi) {
  ylo = ylo < 0 ? 0 : ylo;
  yhi = yhi < r.height - 1 ? yhi : r.height - 1;
  if (ylo > yhi) return false;
  if (r.mode == 0) {
    const int last = r.y0 + (r.nrows - 1) * r.step;
    if (r.nrows <= 0 || yhi < r.y0 || ylo > last) return false;
    const int d = ylo > r.y0 ? ylo - r.y0 : 0;
    const int first = r.y0 + (d + r.step - 1) / r.step * r.step;  // first launch row >= ylo
    return first <= yhi && first <= last;
  }
  const int b0 = ylo / r.band_h, b1 = yhi / r.band_h;
  const int b = b0 + ((r.rank - b0 % r.world) % r.world + r.world) % r.world;  // first own band >= b0
  return b <= b1;
}
// a column of the launch (its pixels: launch rows x launch columns)
__host__ __device__ inline bool frame_has_col(const FrameRows& r, int x) {
  return r.mode != 0 || x % r.step == 0;
}
// image row of launch row k (k < nrows), or -1 past the image
__host__ __device__ inline int frame_row(const FrameRows& r, int k) {
  if (r.mode == 0) return r.y0 + k * r.step;
  const int y = (k / r.band_h * r.world + r.rank) * r.band_h + k % r.band_h;
  return y < r.height ? y : -1;
}

// a face of the binned mesh (rt_bins.h BinTri, the same layout)
struct DevBinTri {
  double v[3][3];
  int32_t rec;
  int32_t face;
};

// frame counters (one small device array). FC_HUGE0 / FC_HUGE1: the huge-face
// list's length of calls of even / odd parity (k_frame_build1 appends to its
// call's word and zeroes the other one, which the next call uses).
// Word 0 is unused: the build has no failure mode (a list past its slots
// keeps its true length and the render kernels take the BVH for that pixel;
// huge faces past kHugeCap are walked by their blocks).
enum : int32_t { FC_RESERVED = 0, FC_HEAVY = 1, FC_LEAN = 2, FC_HUGE0 = 3, FC_HUGE1 = 4, FC_WORDS = 8 };

// Faces whose pixel rectangle holds more than kBigFace pixels are not walked
// by k_frame_build1's blocks (a few large faces, e.g. a 576-face torus
// filling a quarter of a 1080p frame, left a handful of blocks looping over
// thousands of pixels each: 3 ms per call); they go to the huge list, whose
// faces k_frame_build2 tests per tile (each tile culls the list against its
// pixel rectangle, then each pixel tests the tile's share). Past kHugeCap
// faces the rest are walked by their blocks (slow, exact).
#ifndef RTMI_BIG_FACE
#define RTMI_BIG_FACE 64
#endif
constexpr int kBigFace = RTMI_BIG_FACE, kHugeCap = 4096;

// Per-pixel list slots: at least 2^kSlotLg record offsets per pixel (the
// host gives small images more, up to 256, and 4K frames 128: rtmi.cpp
// slot_lg_for). C3 at 1080p lists at most 28 faces per pixel, p99 11; the
// 1M-face torus at 4K 99, p999 34. Round 6: 64 at least (was 32): the torus
// pixels past 32 took the BVH for their camera rays, and with them a rank of
// 8 ran at 80 % of its share of the whole frame; with 64 the ranks' mean is
// 10.1 ms against 11.3 and the whole frame 72.1 → 71.7 ms (`RTMI_SLOT_LG`
// A/B, profiles/r6/ab_slots/); with 128 at 4K no torus pixel is left to the
// BVH and every rank of 8 runs 9.6 ms (profiles/r6/ab_slots/lg7_*).
#ifndef RTMI_SLOT_LG
#define RTMI_SLOT_LG 6
#endif
constexpr int kSlotLg = RTMI_SLOT_LG;

struct HugeFace {
  int32_t rec, pad;
  int32_t r[4];    // pixel rectangle x0, x1, y0, y1
  double pr[6];    // projected vertices (rt_bins_geom.h tri_meets_box)
};

struct RecordsLaunch {
  // the launch's one-pixel groups (rt_fast.h lane_pixel / group_pixel, tile 1 x 1)
  int32_t mode, y0, nrows, ncols, step, max_step, band_h, rank, world, width, height, ngroups;
  uint32_t* info;           // out: per pixel min(list length, kPixCount) | skip bits << 24
  // shadow skips (have == 0: none)
  int32_t nplanes, nl;
  uint32_t have;
  bg::SkipCam cam;
  bg::SkipPlaneC planes[kFrameMaxPlanes];
  const LightGrid* grids;   // per light (rt_scene::grids)
  const int32_t* sat;       // occupancy prefix sums of every light's grid, back to back
  int64_t sat_off[8];
  int32_t records;          // 1: skip bits (one-pixel launches); 0: list lengths only
  // two-class split (split == 0: records only)
  int32_t split;
  uint32_t full;            // every light's bit: (1 << nlight) - 1
  int32_t* lean;            // capacity ngroups + 64
  int32_t* heavy;           // capacity ngroups
  int32_t* ctr;
};

struct FrameLaunch {
  // faces (k_frame_build1)
  const DevBinTri* tris;
  int32_t nf;
  bg::PixCam cam;
  FrameRows rows;
  int32_t* cnt;             // per pixel: zero between calls (k_frame_build2 zeroes the launch's)
  int32_t* slots;           // per pixel 2^slot_lg list entries (TriFast byte offsets), + kBinPad
  int32_t slot_lg;
  HugeFace* huge;           // kHugeCap
  int32_t parity;           // the call's FC_HUGE word: FC_HUGE0 + parity
  // tiles / records / lists (k_frame_build1 tile blocks, k_frame_build2)
  RecordsLaunch r;
  uint8_t* tile_bits;       // per skip cell (kSkipCells per tile): 1 = every light skipped for the whole cell
  unsigned long long* tile_cls;  // per tile: lean << 32 | general pixel counts (split)
  int32_t tiles_x, ntiles;
  unsigned int* zero;       // words k_frame_build1 zeroes (queue heads + Stats), or nullptr
  int32_t nzero;
  int32_t diag;             // TEMP diagnostic (RTMI_DIAG_B2): 1 = no per-pixel skip tests, 2 = no faces, 3 = no skip cells (wrong data)
};

// object bins (rt_bins.h build_object_pixel_masks): world boxes of the objects
struct DevObjBox {
  double lo[3], hi[3];
  int32_t always;
  int32_t pad;
};
struct ObjMaskLaunch {
  const DevObjBox* objs;
  int32_t nobj, width, height;
  double w2c[16];
  double cam_a, cam_c, margin;
  FrameRows rows;
  unsigned long long* masks;  // per pixel
  int32_t* rects;             // scratch: 4 x 64 rectangle ints, then the 64-bit always mask (kObjRectInts)
};
constexpr int kObjRectInts = 4 * 64 + 2;

}  // namespace rtmi

extern "C" {
// The call's build launches (k_frame_build1, k_frame_build2 and, with a
// split, k_frame_lists) on `stream`.
int rtmi_frame_build(const rtmi::FrameLaunch* a, void* stream);
long long rtmi_frame_tile_bytes(int ncols, int nrows);
long long rtmi_frame_skip_cells(int ncols, int nrows);
int rtmi_frame_obj_masks(const rtmi::ObjMaskLaunch* a, void* stream);
}
