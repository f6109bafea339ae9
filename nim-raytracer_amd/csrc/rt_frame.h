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
// float64 vertices. Each render call runs, on its own stream, in order:
//   k_frame_bins_count   per face: its pixel rectangle, a SAT test per pixel
//                        of the launch's rows, one atomic count per listed pixel
//                        (faces of more than kBigFace pixels: onto the big list)
//   k_frame_bins_big     the big faces' pixels spread over the whole grid
//   rocprim exclusive scan of the counts -> per-pixel list offsets
//   k_frame_bins_fill    per face again: scatter its record offset into each
//                        listed pixel's list (the pixels are the count pass's
//                        per-face bit mask; the counts return to zero)
//   k_frame_bins_big     the same for the big faces
//   k_frame_tiles        per 64 x 4 tile of the launch: the shadow skips the
//                        tile's pixels share (one test for the whole tile)
//   k_frame_records      per pixel of the launch: the record (the tile's skip
//                        bits, or the pixel's own test)
//   k_frame_class_count  per block of groups in launch order: its lean and
//                        general counts; a rocprim scan of them; then
//   k_frame_class_write  the groups written to the lean and general lists at
//                        their blocks' offsets (wave ballot + mbcnt ranks) —
//                        the lists in launch order, no global atomics
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
// y0 + k * step (k < nrows), mode 1 the rank's round-robin bands.
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
  int32_t pad;
};

// frame counters (one small device array; cleared by k_frame_bins_count,
// the list lengths written by k_frame_class_write)
// (FC_BIG: the big-face list's length, appended by k_frame_bins_count,
// moved to FC_BIG_N and cleared by k_frame_bins_fill)
enum : int32_t { FC_OVERFLOW = 0, FC_HEAVY = 1, FC_LEAN = 2, FC_DONE = 3, FC_BIG = 4, FC_BIG_N = 5, FC_WORDS = 6 };

// Faces whose pixel rectangle holds more than kBigFace pixels are not walked
// by their own kFaceLanes threads (a few large faces, e.g. a 576-face torus
// filling a quarter of a 1080p frame, left a handful of threads looping over
// thousands of pixels each: 3 ms per call); they go to a list of up to
// kBigCap faces whose pixels the whole grid shares (k_frame_bins_big).
#ifndef RTMI_BIG_FACE
#define RTMI_BIG_FACE 64
#endif
constexpr int kBigFace = RTMI_BIG_FACE, kBigCap = 4096;
// rect[4 * face] of a face on the big list carries this bit
constexpr int32_t kRectBig = 1 << 30;

struct BinsLaunch {
  const DevBinTri* tris;
  int32_t nf;
  bg::PixCam cam;
  FrameRows rows;
  int32_t* rect;   // 4 per face (scratch)
  double* proj;    // 6 per face (scratch)
  int32_t* cnt;    // per pixel + 1: zero between calls (the fill pass counts back down)
  int32_t* off;    // per pixel + 1: list offsets (the scan of cnt over [scan_lo, scan_lo + scan_n))
  int32_t* ent;    // list entries (TriFast byte offsets), capacity cap
  int64_t cap;
  int32_t* ctr;    // FC_* counters
  int32_t* big;    // the big-face list (kBigCap faces)
  unsigned long long* fmask;  // per face (not big): its listed pixels, bit = index in its rectangle
  int64_t scan_lo, scan_n;
  int32_t pad_rec; // a valid record offset for the read-ahead padding
};

struct RecordsLaunch {
  // the launch's one-pixel groups (rt_fast.h lane_pixel / group_pixel, tile 1 x 1)
  int32_t mode, y0, nrows, ncols, step, max_step, band_h, rank, world, width, height, ngroups;
  const int32_t* order;     // launch order (group_order), or nullptr
  const int32_t* off;       // pixel lists (per pixel + 1)
  uint32_t* info;           // out: FastParams.pix_info records
  // shadow skips (have == 0: none)
  int32_t nplanes, nl;
  uint32_t have;
  bg::SkipCam cam;
  bg::SkipPlaneC planes[kFrameMaxPlanes];
  const LightGrid* grids;   // per light (rt_scene::grids)
  const int32_t* sat;       // occupancy prefix sums of every light's grid, back to back
  int64_t sat_off[8];
  // two-class split (split == 0: records only)
  int32_t split;
  uint32_t full;            // every light's bit: (1 << nlight) - 1
  int32_t* lean;            // capacity ngroups + 64
  int32_t* heavy;           // capacity ngroups
  int32_t* ctr;
  int32_t tiles_done;       // host: the tile bits were written by the count launch
  int32_t records_done;     // host: the records (+ tile class counts) were written by the fill launch
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
// count + scan; *scan_tmp_bytes in/out: the scan's scratch size (query with scan_tmp == nullptr)
// tr / tile_bits (optional): the call's pixel-record launch; its tiles
// (k_frame_tiles) then run in the count launch and *tiles_done = 1
int rtmi_frame_bins_count(const rtmi::BinsLaunch* a, void* scan_tmp, size_t* scan_tmp_bytes, void* stream,
                          const rtmi::RecordsLaunch* tr = nullptr, void* tile_bits = nullptr,
                          int* tiles_done = nullptr);
// r (optional): the call's pixel-record launch (its tiles done); the
// records then run in the fill launch (tile_cls: the tile-ordered lists'
// class counts, or nullptr) and *records_done = 1
int rtmi_frame_bins_fill(const rtmi::BinsLaunch* a, void* stream, const rtmi::RecordsLaunch* r = nullptr,
                         const void* tile_bits = nullptr, void* tile_cls = nullptr, int* records_done = nullptr);
// records (+ lists); tile_bits: rtmi_frame_tile_bytes(ncols, nrows) bytes;
// scratch: *scratch_bytes (query with scratch == nullptr)
int rtmi_frame_records(const rtmi::RecordsLaunch* a, void* tile_bits, void* scratch, size_t* scratch_bytes,
                       void* stream);
long long rtmi_frame_tile_bytes(int ncols, int nrows);
int rtmi_frame_obj_masks(const rtmi::ObjMaskLaunch* a, void* stream);
}
