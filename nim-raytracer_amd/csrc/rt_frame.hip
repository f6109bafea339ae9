// rt_frame.hip — per-call device builders of the camera-dependent data of
// the float32 kernels (rt_frame.h). float64 geometry (rt_bins_geom.h), built
// with -ffp-contract=off like the host builders the tests compare against.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <rocprim/device/device_scan.hpp>

#include "rt_bins.h"
#include "rt_frame.h"

namespace rtmi {
namespace {

__device__ __forceinline__ unsigned lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// kFaceLanes threads per face: each takes every kFaceLanes-th pixel of the
// face's rectangle (a face covers a few pixels; one thread per face left the
// GPU a quarter of a wave per SIMD — latency-bound at 69 k faces).
constexpr int kFaceLanes = 4;

// Per face: its pixel rectangle and projected vertices (kept for the fill
// pass), and one count per pixel of the launch's rows that the face's grown
// projection meets (rt_bins.cpp build_pixel_bins, the same bounds).
__device__ __forceinline__ void bins_count_body(const BinsLaunch& a, const int t) {
  if (t == 0) {  // (not FC_BIG: other blocks append to it now; k_frame_bins_fill zeroes it;
                 // not FC_OVERFLOW: kept until the host reports it, rtmi.cpp report_overflow)
#pragma unroll
    for (int k = 0; k < FC_BIG; ++k)
      if (k != FC_OVERFLOW) a.ctr[k] = 0;
  }
  const int i = t / kFaceLanes, q = t % kFaceLanes;
  if (i >= a.nf) return;
  double v[3][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k) v[p][k] = a.tris[i].v[p][k];
  double pr[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int r[4];
  // (a vertex at or behind the camera plane: the host checked the mesh box
  // against the camera plane before launching, so this never fails)
  if (!bg::face_pixel_rect(a.cam, v, pr, r)) r[0] = -1;
  if (q == 0) {
    reinterpret_cast<int4*>(a.rect)[i] = make_int4(r[0], r[1], r[2], r[3]);
#pragma unroll
    for (int k = 0; k < 6; ++k) a.proj[6 * (size_t)i + k] = pr[k];
  }
  const int rw = r[1] - r[0] + 1, area = r[0] < 0 ? 0 : rw * (r[3] - r[2] + 1);
  // a big face goes onto the big list (its first thread takes the slot;
  // the face's kFaceLanes threads are adjacent lanes of one wave)
  int slot = kBigCap;
  if (q == 0 && area > kBigFace) slot = atomicAdd(&a.ctr[FC_BIG], 1);
  slot = __shfl(slot, (int)(threadIdx.x & 63u) - q);
  const bool big = slot < kBigCap;
  if (q == 0) {
    reinterpret_cast<int4*>(a.rect)[i] = make_int4(big ? (r[0] | kRectBig) : r[0], r[1], r[2], r[3]);
#pragma unroll
    for (int k = 0; k < 6; ++k) a.proj[6 * (size_t)i + k] = pr[k];
    if (big) a.big[slot] = i;
  }
  if (r[0] < 0 || big) return;
  const double m = a.cam.margin;
  // the listed pixels as a bit mask over the rectangle, kept for the fill
  // pass: it scatters without re-testing (faces of <= 64 pixels)
  unsigned long long bits = 0ull;
  for (int idx = q; idx < area; idx += kFaceLanes) {
    const int y = r[2] + idx / rw, x = r[0] + idx % rw;
    if (frame_has_row(a.rows, y) && bg::tri_meets_box(pr, x - m, y - m, x + 1 + m, y + 1 + m)) {
      atomicAdd(&a.cnt[(size_t)y * a.cam.width + x], 1);
      if (idx < 64) bits |= 1ull << idx;
    }
  }
#pragma unroll
  for (int k = 1; k < kFaceLanes; k <<= 1) {
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)bits, k), hi = (unsigned)__shfl_xor((int)(unsigned)(bits >> 32), k);
    bits |= ((unsigned long long)hi << 32) | lo;
  }
  if (q == 0) a.fmask[i] = bits;  // (unused for a face of more than 64 pixels: the fill pass tests again)
}
__global__ __launch_bounds__(256) void k_frame_bins_count(const BinsLaunch a) {
  bins_count_body(a, (int)(blockIdx.x * 256u + threadIdx.x));
}

// The big faces' pixels (FILL false: counted, true: filled), spread over the
// whole grid: each block scans the list's rectangle areas in LDS, then its
// threads take every (gridDim * 256)-th pixel of the concatenated rectangles
// (a binary search finds the face).
template <bool FILL>
__global__ __launch_bounds__(256) void k_frame_bins_big(const BinsLaunch a) {
  __shared__ int32_t pre[kBigCap + 1];
  __shared__ int32_t part[256];
  const int n = min(a.ctr[FILL ? FC_BIG_N : FC_BIG], kBigCap);
  if (n == 0) return;
  const int t = (int)threadIdx.x;
  // exclusive scan of the areas: 16 per thread, then the 256 partial sums
  constexpr int kPer = kBigCap / 256;
  int32_t loc[kPer];
  int32_t sum = 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int e = t * kPer + k;
    int32_t ar = 0;
    if (e < n) {
      const int4 r = reinterpret_cast<const int4*>(a.rect)[a.big[e]];
      ar = ((r.x & ~kRectBig) <= r.y) ? (r.y - (r.x & ~kRectBig) + 1) * (r.w - r.z + 1) : 0;
    }
    loc[k] = sum;
    sum += ar;
  }
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    const int32_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  const int32_t base = t > 0 ? part[t - 1] : 0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) pre[t * kPer + k] = base + loc[k];
  if (t == 255) pre[kBigCap] = part[255];
  __syncthreads();
  const int32_t total = pre[kBigCap];
  const double m = a.cam.margin;
  for (int32_t idx = (int32_t)(blockIdx.x * 256u) + t; idx < total; idx += (int32_t)(gridDim.x * 256u)) {
    int lo = 0, hi = n - 1;  // the last face e with pre[e] <= idx
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= idx) lo = mid;
      else hi = mid - 1;
    }
    const int i = a.big[lo];
    const int4 r = reinterpret_cast<const int4*>(a.rect)[i];
    const int x0 = r.x & ~kRectBig, rw = r.y - x0 + 1, local = idx - pre[lo];
    const int y = r.z + local / rw, x = x0 + local % rw;
    if (!frame_has_row(a.rows, y)) continue;
    double pr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) pr[k] = a.proj[6 * (size_t)i + k];
    if (!bg::tri_meets_box(pr, x - m, y - m, x + 1 + m, y + 1 + m)) continue;
    const size_t pix = (size_t)y * a.cam.width + x;
    if (!FILL) {
      atomicAdd(&a.cnt[pix], 1);
    } else {
      const int64_t slot = (int64_t)a.off[pix] + atomicSub(&a.cnt[pix], 1) - 1;
      if (slot < a.cap) a.ent[slot] = a.tris[i].rec;
      else atomicOr(&a.ctr[FC_OVERFLOW], 1);
    }
  }
}

// Per face again: its record offset into each listed pixel's list. The
// slot comes from counting the pixel's count back down, so the counts are
// zero again for the next call (no clearing pass).
__device__ __forceinline__ void bins_fill_body(const BinsLaunch& a, const int t) {
  if (t == 0) {  // read-ahead padding after the last list (rt_bins.h kBinPad)
    const int64_t total = a.off[a.scan_lo + a.scan_n - 1];
    for (int k = 0; k < kBinPad; ++k)
      if (total + k < a.cap) a.ent[total + k] = a.pad_rec;
    if (total + kBinPad > a.cap) atomicOr(&a.ctr[FC_OVERFLOW], 1);
    a.ctr[FC_BIG_N] = a.ctr[FC_BIG];  // the count pass's big list, for the big fill pass
    a.ctr[FC_BIG] = 0;
  }
  const int i = t / kFaceLanes, q = t % kFaceLanes;
  if (i >= a.nf) return;
  const int4 r = reinterpret_cast<const int4*>(a.rect)[i];
  if (r.x < 0 || (r.x & kRectBig)) return;  // off screen / the big fill pass's
  const int32_t rec = a.tris[i].rec;
  const int rw = r.y - r.x + 1, area = rw * (r.w - r.z + 1);
  if (area > 64) {  // no mask (a big face the full big list left here, or kBigFace > 64): test again
    double pr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) pr[k] = a.proj[6 * (size_t)i + k];
    const double m = a.cam.margin;
    for (int idx = q; idx < area; idx += kFaceLanes) {
      const int y = r.z + idx / rw, x = r.x + idx % rw;
      if (frame_has_row(a.rows, y) && bg::tri_meets_box(pr, x - m, y - m, x + 1 + m, y + 1 + m)) {
        const size_t pix = (size_t)y * a.cam.width + x;
        const int64_t slot = (int64_t)a.off[pix] + atomicSub(&a.cnt[pix], 1) - 1;
        if (slot < a.cap) a.ent[slot] = rec;
        else atomicOr(&a.ctr[FC_OVERFLOW], 1);
      }
    }
    return;
  }
  // the count pass's mask: lane q takes the listed pixels idx = q mod kFaceLanes
  unsigned long long bits = a.fmask[i] & (0x1111111111111111ull << q);
  while (bits != 0ull) {
    const int idx = (int)__builtin_ctzll(bits);
    bits &= bits - 1ull;
    const int y = r.z + idx / rw, x = r.x + idx % rw;
    const size_t pix = (size_t)y * a.cam.width + x;
    const int64_t slot = (int64_t)a.off[pix] + atomicSub(&a.cnt[pix], 1) - 1;
    if (slot < a.cap) a.ent[slot] = rec;
    else atomicOr(&a.ctr[FC_OVERFLOW], 1);
  }
}
__global__ __launch_bounds__(256) void k_frame_bins_fill(const BinsLaunch a) {
  bins_fill_body(a, (int)(blockIdx.x * 256u + threadIdx.x));
}

// The launch's pixel at launch column j, launch row k (rt_fast.h lane_pixel
// for one-pixel groups); valid = inside the launch and the image.
struct LaunchPix {
  int x, y;
  bool valid, drawn;  // drawn: not skipped by a progressive pass
};
__device__ __forceinline__ LaunchPix launch_pixel(const RecordsLaunch& a, int j, int k) {
  LaunchPix r;
  r.x = j * a.step;
  r.valid = j < a.ncols && k < a.nrows;
  if (a.mode == 0) {
    r.y = a.y0 + k * a.step;
  } else {
    r.y = (k / a.band_h * a.world + a.rank) * a.band_h + k % a.band_h;
    r.valid = r.valid && r.y < a.height;
  }
  r.drawn = r.valid;
  if (a.step < a.max_step) {  // progressive refinement skip (renderer.nim:175-178)
    const int mask = a.step * 2 - 1;
    if ((r.x & mask) == 0 && (r.y & mask) == 0) r.drawn = false;
  }
  return r;
}

__device__ __forceinline__ void load_skip_grids(const RecordsLaunch& a, bg::SkipGrid* sg) {
  if ((int)threadIdx.x < a.nl) {
    const LightGrid& G = a.grids[threadIdx.x];
    bg::SkipGrid& s = sg[threadIdx.x];
    for (int c = 0; c < 3; ++c) {
      s.e1[c] = G.e1[c];
      s.e2[c] = G.e2[c];
    }
    s.u0 = G.u0;
    s.v0 = G.v0;
    s.inv_h = G.inv_h;
    s.gu = G.gu;
    s.gv = G.gv;
    s.sat = a.sat + a.sat_off[threadIdx.x];
  }
  __syncthreads();
}

// Records are built per tile of kTileW launch columns x kTileH launch rows
// (one block, one wave per launch row). The tile's shadow skips are tested
// once for the rectangle its pixels span (rt_bins_geom.h rect_skip_bits:
// the tile's grown corner rays bound every pixel's, so a tile whose bits
// cover every light gives each of its pixels exactly the bits the per-pixel
// test would); the pixels of other tiles take the per-pixel test.
constexpr int kTileW = 64, kTileH = 4;

// One thread per tile: the tile's skip bits (0 when not every light is skipped).
__device__ __forceinline__ void tiles_body(const RecordsLaunch& a, const int t, int tiles_x, int ntiles,
                                           uint8_t* tile_bits, const bg::SkipGrid* sg) {
  if (t >= ntiles) return;
  const int tj = t % tiles_x, tk = t / tiles_x;
  const int j0 = tj * kTileW, j1 = min(j0 + kTileW, a.ncols) - 1;
  int ylo = 0x7fffffff, yhi = -1;
  for (int k = tk * kTileH; k < min(tk * kTileH + kTileH, a.nrows); ++k) {
    const LaunchPix p = launch_pixel(a, j0, k);
    if (!p.valid) continue;
    ylo = min(ylo, p.y);
    yhi = max(yhi, p.y);
  }
  unsigned bits = 0u;
  if (yhi >= 0) bits = bg::rect_skip_bits(a.cam, a.planes, a.nplanes, sg, a.nl, a.have, j0 * a.step, ylo, j1 * a.step, yhi);
  tile_bits[t] = (uint8_t)(bits == a.have ? 1u : 0u);
}
__global__ __launch_bounds__(256) void k_frame_tiles(const RecordsLaunch a, int tiles_x, int ntiles, uint8_t* tile_bits) {
  __shared__ bg::SkipGrid sg[8];
  load_skip_grids(a, sg);
  tiles_body(a, (int)(blockIdx.x * 256u + threadIdx.x), tiles_x, ntiles, tile_bits, sg);
}

// k_frame_bins_count and k_frame_tiles in one launch (the tiles depend on
// the camera and the light grids only): blocks [0, face_blocks) count the
// faces' pixels, the rest test the 64 x 4 tiles — one launch fewer per call
// (each costs 4-10 us however little it does; 8 ranks' band sets are
// dominated by such fixed costs).
__global__ __launch_bounds__(256) void k_frame_bins_count_tiles(const BinsLaunch a, const RecordsLaunch r,
                                                                int face_blocks, int tiles_x, int ntiles,
                                                                uint8_t* tile_bits) {
  __shared__ bg::SkipGrid sg[8];
  if ((int)blockIdx.x < face_blocks) {
    bins_count_body(a, (int)(blockIdx.x * 256u + threadIdx.x));
    return;
  }
  load_skip_grids(r, sg);
  tiles_body(r, (int)((blockIdx.x - (unsigned)face_blocks) * 256u + threadIdx.x), tiles_x, ntiles, tile_bits, sg);
}

// Per pixel of one tile (block (tile column, tile row)): the pixel record —
// list length, and for an empty list the shadow skip bits (the tile's, or
// the pixel's own test).
// tile_cls (split launches in screen order, a.order == nullptr): the tile's
// lean / general pixel counts (lean << 32 | general) for the tile-ordered
// lists (k_frame_class_write_tiles), or nullptr.
__device__ __forceinline__ int pixel_class(const RecordsLaunch& a, const LaunchPix& p, uint32_t info) {
  if (!p.drawn) return 0;
  return (info & kPixCount) == 0u && ((info >> 24) & a.full) == a.full ? 1 : 2;
}
// (bx, by): the block's tile; tiles_x tiles per launch row
__device__ __forceinline__ void records_body(const RecordsLaunch& a, const uint8_t* tile_bits,
                                             unsigned long long* tile_cls, int bx, int by, int tiles_x,
                                             const bg::SkipGrid* sg, unsigned long long* wsum) {
  const int j = bx * kTileW + (int)(threadIdx.x & 63u);
  const int k = by * kTileH + (int)(threadIdx.x >> 6);
  const LaunchPix p = launch_pixel(a, j, k);
  int c = 0;
  if (p.valid) {
    const size_t pix = (size_t)p.y * a.width + p.x;
    const int32_t n = a.off[pix + 1] - a.off[pix];
    uint32_t info = n < (int32_t)kPixCount ? (uint32_t)n : kPixCount;
    if (n == 0 && a.have != 0u) {
      const bool tile = tile_bits[by * tiles_x + bx] != 0;
      const unsigned bits = tile ? a.have : bg::pixel_skip_bits(a.cam, a.planes, a.nplanes, sg, a.nl, a.have, p.x, p.y);
      info |= bits << 24;
    }
    a.info[pix] = info;
    c = pixel_class(a, p, info);
  }
  if (!tile_cls) return;
  const unsigned long long ml = __ballot(c == 1), mh = __ballot(c == 2);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  __syncthreads();
  if (threadIdx.x == 0) tile_cls[by * tiles_x + bx] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}
__global__ __launch_bounds__(256) void k_frame_records(const RecordsLaunch a, const uint8_t* tile_bits,
                                                       unsigned long long* tile_cls) {
  __shared__ bg::SkipGrid sg[8];
  __shared__ unsigned long long wsum[4];
  load_skip_grids(a, sg);
  records_body(a, tile_bits, tile_cls, (int)blockIdx.x, (int)blockIdx.y, (int)gridDim.x, sg, wsum);
}

// k_frame_bins_fill and k_frame_records in one launch: the records read the
// list offsets and the tile bits (both written by earlier launches), never
// the entries the fill pass writes, so the two are independent. Blocks
// [0, fill_blocks) fill, the rest build one tile's records each.
__global__ __launch_bounds__(256) void k_frame_fill_records(const BinsLaunch a, const RecordsLaunch r, int fill_blocks,
                                                            int tiles_x, const uint8_t* tile_bits,
                                                            unsigned long long* tile_cls) {
  __shared__ bg::SkipGrid sg[8];
  __shared__ unsigned long long wsum[4];
  if ((int)blockIdx.x < fill_blocks) {
    bins_fill_body(a, (int)(blockIdx.x * 256u + threadIdx.x));
    return;
  }
  load_skip_grids(r, sg);
  const int b = (int)blockIdx.x - fill_blocks;
  records_body(r, tile_bits, tile_cls, b % tiles_x, b / tiles_x, tiles_x, sg, wsum);
}

// Exclusive scan of n packed counts by one block (n = the launch's tiles:
// 8,100 at 1080p; rocPRIM's scan took two launches, ~10 us): per round of
// 8 x 1024 values, every thread loads its 8 (coalesced, all in flight at
// once), wave scans of each, then one wave scans the 128 wave totals.
__device__ __forceinline__ unsigned long long shfl_up_u64(unsigned long long x, int off) {
  const unsigned lo = (unsigned)__shfl_up((int)(unsigned)x, off), hi = (unsigned)__shfl_up((int)(unsigned)(x >> 32), off);
  return ((unsigned long long)hi << 32) | lo;
}
__global__ __launch_bounds__(1024) void k_scan_tiles(const unsigned long long* __restrict__ in,
                                                     unsigned long long* __restrict__ out, int n) {
  constexpr int C = 8;
  __shared__ unsigned long long wtot[C * 16];
  __shared__ unsigned long long carry;
  const int t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry = 0ull;
  for (int base = 0; base < n; base += 1024 * C) {
    unsigned long long v[C], x[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int i = base + c * 1024 + t;
      v[c] = i < n ? in[i] : 0ull;
      x[c] = v[c];
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const unsigned long long y = shfl_up_u64(x[c], off);
        x[c] += lane >= off ? y : 0ull;
      }
    if (lane == 63)
#pragma unroll
      for (int c = 0; c < C; ++c) wtot[c * 16 + w] = x[c];
    __syncthreads();
    if (t < 64) {  // the 128 wave totals in order (chunk-major), two per lane
      const unsigned long long a0 = wtot[2 * t], a1 = wtot[2 * t + 1];
      unsigned long long y = a0 + a1;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const unsigned long long z = shfl_up_u64(y, off);
        y += lane >= off ? z : 0ull;
      }
      const unsigned long long ex = carry + y - a0 - a1;  // before wave total 2 t
      wtot[2 * t] = ex;
      wtot[2 * t + 1] = ex + a0;
      if (t == 63) carry += y;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const int i = base + c * 1024 + t;
      if (i < n) out[i] = wtot[c * 16 + w] + x[c] - v[c];
    }
    __syncthreads();
  }
}

// The lean / general lists in tile order (the records kernel's tiles, its
// counts scanned): each tile's groups at its offsets, wave ballots + mbcnt
// ranks; the last tile writes the lengths and the lean list's -1 padding.
__global__ __launch_bounds__(256) void k_frame_class_write_tiles(const RecordsLaunch a,
                                                                 const unsigned long long* tile_cls,
                                                                 const unsigned long long* tile_off) {
  __shared__ unsigned long long wsum[4];
  const int j = (int)blockIdx.x * kTileW + (int)(threadIdx.x & 63u);
  const int k = (int)blockIdx.y * kTileH + (int)(threadIdx.x >> 6);
  const LaunchPix p = launch_pixel(a, j, k);
  const int c = p.valid ? pixel_class(a, p, a.info[(size_t)p.y * a.width + p.x]) : 0;
  const unsigned long long ml = __ballot(c == 1), mh = __ballot(c == 2);
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63u) == 0) wsum[w] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  __syncthreads();
  const int tile = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  unsigned long long base = tile_off[tile];
  for (int i = 0; i < w; ++i) base += wsum[i];
  const int g = k * a.ncols + j;
  if (c == 1) a.lean[(int)(base >> 32) + (int)lane_rank(ml)] = g;
  if (c == 2) a.heavy[(int)(base & 0xffffffffu) + (int)lane_rank(mh)] = g;
  if (tile != (int)(gridDim.x * gridDim.y) - 1) return;
  const unsigned long long tot = tile_off[tile] + tile_cls[tile];
  const int nl = (int)(tot >> 32), nh = (int)(tot & 0xffffffffu);
  if (threadIdx.x == 0) {
    a.ctr[FC_LEAN] = nl;
    a.ctr[FC_HEAVY] = nh;
  }
  const int end = nl == 0 ? 64 : (nl + 63) / 64 * 64;
  for (int e = nl + (int)threadIdx.x; e < end; e += 256) a.lean[e] = -1;
}

// The class of the gi-th group of the launch order (order, or screen order):
// 1 lean (empty list, every light skipped), 2 general, 0 not drawn.
__device__ __forceinline__ int group_class(const RecordsLaunch& a, int gi, int* g_out) {
  if (gi >= a.ngroups) return 0;
  const int g = a.order ? a.order[gi] : gi;
  *g_out = g;
  const int k = g / a.ncols, j = g - k * a.ncols;
  const LaunchPix p = launch_pixel(a, j, k);
  if (!p.drawn) return 0;
  const uint32_t info = a.info[(size_t)p.y * a.width + p.x];
  return (info & kPixCount) == 0u && ((info >> 24) & a.full) == a.full ? 1 : 2;
}

// The lean / general lists in launch order, without a global atomic per wave
// (one counter takes ~90 atomics/us: 32 k waves would serialise on it):
// k_frame_class_count counts each block's lean and general groups (packed
// lean << 32 | general), an exclusive scan gives every block its offsets,
// k_frame_class_write writes each block's groups there (wave ballots, mbcnt
// ranks, the waves' counts through LDS).
__global__ __launch_bounds__(256) void k_frame_class_count(const RecordsLaunch a, unsigned long long* blk) {
  __shared__ unsigned long long wsum[4];
  int g = 0;
  const int c = group_class(a, (int)(blockIdx.x * 256u + threadIdx.x), &g);
  const unsigned long long ml = __ballot(c == 1), mh = __ballot(c == 2);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void k_frame_class_write(const RecordsLaunch a, const unsigned long long* blk,
                                                           const unsigned long long* blk_off) {
  __shared__ unsigned long long wsum[4];
  int g = 0;
  const int c = group_class(a, (int)(blockIdx.x * 256u + threadIdx.x), &g);
  const unsigned long long ml = __ballot(c == 1), mh = __ballot(c == 2);
  const int w = (int)(threadIdx.x >> 6);
  if ((threadIdx.x & 63u) == 0) wsum[w] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  __syncthreads();
  unsigned long long base = blk_off[blockIdx.x];
  for (int i = 0; i < w; ++i) base += wsum[i];
  if (c == 1) a.lean[(int)(base >> 32) + (int)lane_rank(ml)] = g;
  if (c == 2) a.heavy[(int)(base & 0xffffffffu) + (int)lane_rank(mh)] = g;
  if (blockIdx.x != gridDim.x - 1) return;
  // the last block: the list lengths, and the lean list padded with -1 to
  // whole 64-entry runs (the lean kernels read items of 4 / 16 entries)
  const unsigned long long tot = blk_off[blockIdx.x] + blk[blockIdx.x];
  const int nl = (int)(tot >> 32), nh = (int)(tot & 0xffffffffu);
  if (threadIdx.x == 0) {
    a.ctr[FC_LEAN] = nl;
    a.ctr[FC_HEAVY] = nh;
  }
  const int end = nl == 0 ? 64 : (nl + 63) / 64 * 64;
  for (int e = nl + (int)threadIdx.x; e < end; e += 256) a.lean[e] = -1;
}

// Object masks (rt_bins.cpp build_object_pixel_masks). k_frame_obj_rects
// projects every object's world box once, one thread per (object, corner)
// (the corners' float64 projections in parallel, min / max over each
// object's 8 lanes): its pixel rectangle (x0, x1, y0, y1; -1s: off screen)
// into rects[4 i ..], and after them the mask of the objects with no bounded
// projection (in every pixel's mask).
__global__ __launch_bounds__(512) void k_frame_obj_rects(const ObjMaskLaunch a) {
  __shared__ int alw[64];
  const int t = (int)threadIdx.x, i = t >> 3, c = t & 7;
  bool proj = false, bad = false;
  double px = 0.0, py = 0.0;
  if (i < a.nobj) {
    const DevObjBox& b = a.objs[i];
    proj = !b.always;
    const double pw[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
    double pc[3];
    bg::xform_point(a.w2c, pw, pc);
    // a corner at or behind the camera plane: no bounded projection
    bad = !(pc[2] < -1e-9 * (1.0 + fabs(pc[0]) + fabs(pc[1])));
    if (!bad) {
      px = 0.5 * a.width + (pc[0] / -pc[2]) / a.cam_a;
      py = 0.5 * a.height - (pc[1] / -pc[2]) / a.cam_c;
    }
  }
  double xmin = px, xmax = px, ymin = py, ymax = py;
#pragma unroll
  for (int k = 1; k < 8; k <<= 1) {  // the object's 8 lanes (aligned groups of one wave)
    xmin = bg::dmin(xmin, __shfl_xor(xmin, k));
    xmax = bg::dmax(xmax, __shfl_xor(xmax, k));
    ymin = bg::dmin(ymin, __shfl_xor(ymin, k));
    ymax = bg::dmax(ymax, __shfl_xor(ymax, k));
    bad = bad || __shfl_xor((int)bad, k) != 0;
  }
  if (i < a.nobj && c == 0) {
    proj = proj && !bad;
    alw[i] = proj ? 0 : 1;
    int4 r = make_int4(-1, -1, -1, -1);
    const double m = a.margin;
    if (proj && xmax + m >= 0.0 && ymax + m >= 0.0 && xmin - m < a.width && ymin - m < a.height)
      r = make_int4((int)bg::dmax(0.0, floor(xmin - m)), (int)bg::dmin((double)a.width - 1, floor(xmax + m)),
                    (int)bg::dmax(0.0, floor(ymin - m)), (int)bg::dmin((double)a.height - 1, floor(ymax + m)));
    reinterpret_cast<int4*>(a.rects)[i] = r;
  }
  __syncthreads();
  if (t == 0) {
    unsigned long long am = 0ull;
    for (int k = 0; k < a.nobj; ++k) am |= alw[k] ? 1ull << k : 0ull;
    *reinterpret_cast<unsigned long long*>(a.rects + 4 * 64) = am;
  }
}

// Per pixel of a 256-column segment (blockIdx.x) of every gridDim.y-th launch
// row: lane i of each wave holds object i's rectangle in registers, a ballot
// gives the row's objects, and each pixel tests its x against theirs
// (read back from the holding lanes as uniform values).
__global__ __launch_bounds__(256) void k_frame_obj_masks(const ObjMaskLaunch a) {
  const int lane = (int)(threadIdx.x & 63u);
  const int4 mine = lane < a.nobj ? reinterpret_cast<const int4*>(a.rects)[lane] : make_int4(-1, -1, -1, -1);
  const unsigned long long always = *reinterpret_cast<const unsigned long long*>(a.rects + 4 * 64);
  const int x = (int)(blockIdx.x * 256u + threadIdx.x);
  for (int k = (int)blockIdx.y; k < a.rows.nrows; k += (int)gridDim.y) {
    const int y = frame_row(a.rows, k);
    if (y < 0) continue;
    unsigned long long row = __ballot(mine.x >= 0 && y >= mine.z && y <= mine.w);
    unsigned long long mk = always;
    while (row != 0ull) {
      const int i = (int)__builtin_ctzll(row);
      row &= row - 1ull;
      const int x0 = __builtin_amdgcn_readlane(mine.x, i), x1 = __builtin_amdgcn_readlane(mine.y, i);
      mk |= (x >= x0 && x <= x1) ? 1ull << i : 0ull;
    }
    if (x < a.width) a.masks[(size_t)y * a.width + x] = mk;
  }
}

// The face lists' offsets: an exclusive scan of the per-pixel counts in two
// launches (rocPRIM's took an init launch and a 14 us scan for 2 M counts):
// k_scan_sums sums each kScanChunk-count chunk; k_scan_apply gives each
// chunk its offset (the sum of the earlier chunks' sums, one wave) and scans
// the chunk through LDS (coalesced loads and stores, 32 consecutive counts
// per thread, wave scans of the thread sums).
constexpr int kScanPer = 32, kScanChunk = 256 * kScanPer;
__global__ __launch_bounds__(256) void k_scan_sums(const int32_t* __restrict__ in, long long n, int32_t* __restrict__ sums) {
  __shared__ int32_t ws[4];
  const long long base = (long long)blockIdx.x * kScanChunk;
  int32_t v = 0;
#pragma unroll 8
  for (int j = 0; j < kScanPer; ++j) {
    const long long i = base + (long long)j * 256 + threadIdx.x;
    v += i < n ? in[i] : 0;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}
__global__ __launch_bounds__(256) void k_scan_apply(const int32_t* __restrict__ in, long long n,
                                                    const int32_t* __restrict__ sums, int32_t* __restrict__ out) {
  // the chunk in LDS with one pad word per 32 (P(e) = e + e / 32): the
  // coalesced passes and the per-thread runs of 32 are both conflict-free
  __shared__ int32_t buf[kScanChunk + kScanChunk / 32];
  __shared__ int32_t wtot[4];
  __shared__ int32_t before;
  const int t = (int)threadIdx.x, lane = t & 63, w = t >> 6;
  const long long base = (long long)blockIdx.x * kScanChunk;
  if (w == 0) {  // this chunk's offset: the earlier chunks' sums
    int32_t p = 0;
    for (int i = lane; i < (int)blockIdx.x; i += 64) p += sums[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) p += __shfl_xor(p, off);
    if (lane == 0) before = p;
  }
#pragma unroll 8
  for (int j = 0; j < kScanPer; ++j) {
    const int e = j * 256 + t;
    const long long i = base + e;
    buf[e + (e >> 5)] = i < n ? in[i] : 0;
  }
  __syncthreads();
  int32_t x[kScanPer], sum = 0;  // this thread's 32 consecutive counts
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    x[j] = buf[t * (kScanPer + 1) + j];
    sum += x[j];
  }
  int32_t inc = sum;  // inclusive scan of the thread sums within the wave
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int32_t y = __shfl_up(inc, off);
    inc += lane >= off ? y : 0;
  }
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int32_t run = before + inc - sum;
  for (int k = 0; k < w; ++k) run += wtot[k];
#pragma unroll
  for (int j = 0; j < kScanPer; ++j) {
    buf[t * (kScanPer + 1) + j] = run;
    run += x[j];
  }
  __syncthreads();
#pragma unroll 8
  for (int j = 0; j < kScanPer; ++j) {
    const int e = j * 256 + t;
    const long long i = base + e;
    if (i < n) out[i] = buf[e + (e >> 5)];
  }
}

}  // namespace
}  // namespace rtmi

namespace {
constexpr int kBigBlocks = 512;  // the big-face passes' grid (their blocks exit at once on an empty list)
}

extern "C" int rtmi_frame_bins_count(const rtmi::BinsLaunch* a, void* scan_tmp, size_t* scan_tmp_bytes,
                                     void* stream, const rtmi::RecordsLaunch* tr, void* tile_bits, int* tiles_done) {
  hipStream_t st = (hipStream_t)stream;
  const long long nchunk = ((long long)a->scan_n + rtmi::kScanChunk - 1) / rtmi::kScanChunk;
  if (!scan_tmp) {
    *scan_tmp_bytes = (size_t)std::max(1LL, nchunk) * sizeof(int32_t);
    return 0;
  }
  if (*scan_tmp_bytes < (size_t)nchunk * sizeof(int32_t)) return (int)hipErrorInvalidValue;
  const int blocks = std::max(1, (int)(((long long)a->nf * rtmi::kFaceLanes + 255) / 256));
  const int tiles_x = tr ? (tr->ncols + rtmi::kTileW - 1) / rtmi::kTileW : 0;
  const int ntiles = tr ? tiles_x * ((tr->nrows + rtmi::kTileH - 1) / rtmi::kTileH) : 0;
  if (tiles_done) *tiles_done = 0;
  if (tr && tile_bits && tiles_done && tr->have != 0u && ntiles > 0) {
    hipLaunchKernelGGL(rtmi::k_frame_bins_count_tiles, dim3(blocks + (ntiles + 255) / 256), dim3(256), 0, st, *a, *tr,
                       blocks, tiles_x, ntiles, (uint8_t*)tile_bits);
    *tiles_done = 1;
  } else {
    hipLaunchKernelGGL(rtmi::k_frame_bins_count, dim3(blocks), dim3(256), 0, st, *a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rtmi::k_frame_bins_big<false>, dim3(kBigBlocks), dim3(256), 0, st, *a);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if (nchunk == 0) return 0;
  hipLaunchKernelGGL(rtmi::k_scan_sums, dim3((unsigned)nchunk), dim3(256), 0, st, a->cnt + a->scan_lo, (long long)a->scan_n,
                     (int32_t*)scan_tmp);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rtmi::k_scan_apply, dim3((unsigned)nchunk), dim3(256), 0, st, a->cnt + a->scan_lo,
                     (long long)a->scan_n, (const int32_t*)scan_tmp, a->off + a->scan_lo);
  return (int)hipGetLastError();
}

extern "C" int rtmi_frame_bins_fill(const rtmi::BinsLaunch* a, void* stream, const rtmi::RecordsLaunch* r,
                                    const void* tile_bits, void* tile_cls, int* records_done) {
  const int blocks = std::max(1, (int)(((long long)a->nf * rtmi::kFaceLanes + 255) / 256));
  const int tiles_x = r ? (r->ncols + rtmi::kTileW - 1) / rtmi::kTileW : 0;
  const int ntiles = r ? tiles_x * ((r->nrows + rtmi::kTileH - 1) / rtmi::kTileH) : 0;
  if (records_done) *records_done = 0;
  if (r && records_done && ntiles > 0) {
    hipLaunchKernelGGL(rtmi::k_frame_fill_records, dim3(blocks + ntiles), dim3(256), 0, (hipStream_t)stream, *a, *r,
                       blocks, tiles_x, (const uint8_t*)tile_bits, (unsigned long long*)tile_cls);
    *records_done = 1;
  } else {
    hipLaunchKernelGGL(rtmi::k_frame_bins_fill, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *a);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(rtmi::k_frame_bins_big<true>, dim3(kBigBlocks), dim3(256), 0, (hipStream_t)stream, *a);
  return (int)hipGetLastError();
}

extern "C" int rtmi_frame_records(const rtmi::RecordsLaunch* a, void* tile_bits, void* scratch, size_t* scratch_bytes,
                                  void* stream) {
  using namespace rtmi;
  hipStream_t st = (hipStream_t)stream;
  const int nblk = std::max(1, (a->ngroups + 255) / 256);
  // scratch: the per-block class counts, their scan, the scan's temporary storage
  const size_t cnt_bytes = ((size_t)nblk * sizeof(unsigned long long) + 255) / 256 * 256;
  size_t scan_bytes = 0;
  hipError_t e = rocprim::exclusive_scan(nullptr, scan_bytes, (unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, 0ull, (size_t)nblk,
                                         rocprim::plus<unsigned long long>(), st);
  if (e != hipSuccess) return (int)e;
  const int tiles_x = (a->ncols + kTileW - 1) / kTileW, tiles_y = (a->nrows + kTileH - 1) / kTileH;
  const int ntiles = tiles_x * tiles_y;
  const size_t tile_bytes = ((size_t)std::max(ntiles, 1) * sizeof(unsigned long long) + 255) / 256 * 256;
  if (!scratch) {
    *scratch_bytes = std::max(2 * cnt_bytes + scan_bytes, 2 * tile_bytes);
    return 0;
  }
  if (*scratch_bytes < 2 * cnt_bytes + scan_bytes && !(a->split && !a->order)) return (int)hipErrorInvalidValue;
  if (ntiles <= 0) return 0;
  if (a->have != 0u && !a->tiles_done) {
    hipLaunchKernelGGL(k_frame_tiles, dim3((ntiles + 255) / 256), dim3(256), 0, st, *a, tiles_x, ntiles,
                       (uint8_t*)tile_bits);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  }
  if (a->split && !a->order) {  // tile-ordered lists: counts from the records kernel, one-block scan
    if (*scratch_bytes < 2 * tile_bytes) return (int)hipErrorInvalidValue;
    unsigned long long* tc = (unsigned long long*)scratch;
    unsigned long long* to = (unsigned long long*)((char*)scratch + tile_bytes);
    if (!a->records_done) {
      hipLaunchKernelGGL(k_frame_records, dim3(tiles_x, tiles_y), dim3(256), 0, st, *a, (const uint8_t*)tile_bits, tc);
      if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    }
    hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(1024), 0, st, (const unsigned long long*)tc, to, ntiles);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
    hipLaunchKernelGGL(k_frame_class_write_tiles, dim3(tiles_x, tiles_y), dim3(256), 0, st, *a,
                       (const unsigned long long*)tc, (const unsigned long long*)to);
    return (int)hipGetLastError();
  }
  if (!a->records_done) {
    hipLaunchKernelGGL(k_frame_records, dim3(tiles_x, tiles_y), dim3(256), 0, st, *a, (const uint8_t*)tile_bits,
                       (unsigned long long*)nullptr);
    if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  }
  if (!a->split) return 0;
  unsigned long long* blk = (unsigned long long*)scratch;
  unsigned long long* blk_off = (unsigned long long*)((char*)scratch + cnt_bytes);
  void* tmp = (char*)scratch + 2 * cnt_bytes;
  hipLaunchKernelGGL(k_frame_class_count, dim3(nblk), dim3(256), 0, st, *a, blk);
  if ((e = hipGetLastError()) != hipSuccess) return (int)e;
  if ((e = rocprim::exclusive_scan(tmp, scan_bytes, blk, blk_off, 0ull, (size_t)nblk,
                                   rocprim::plus<unsigned long long>(), st)) != hipSuccess)
    return (int)e;
  hipLaunchKernelGGL(k_frame_class_write, dim3(nblk), dim3(256), 0, st, *a, (const unsigned long long*)blk,
                     (const unsigned long long*)blk_off);
  return (int)hipGetLastError();
}

// Tile-bit bytes rtmi_frame_records needs for a launch of ncols x nrows groups.
extern "C" long long rtmi_frame_tile_bytes(int ncols, int nrows) {
  using namespace rtmi;
  return (long long)((ncols + kTileW - 1) / kTileW) * ((nrows + kTileH - 1) / kTileH);
}

extern "C" int rtmi_frame_obj_masks(const rtmi::ObjMaskLaunch* a, void* stream) {
  if (a->nobj > 64 || a->rows.nrows <= 0 || a->width <= 0) return a->nobj > 64 ? (int)hipErrorInvalidValue : 0;
  hipLaunchKernelGGL(rtmi::k_frame_obj_rects, dim3(1), dim3(512), 0, (hipStream_t)stream, *a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const unsigned segs = (unsigned)((a->width + 255) / 256);
  const unsigned rows = (unsigned)std::min<long long>(a->rows.nrows, std::max<long long>(1, 2048 / segs));
  hipLaunchKernelGGL(rtmi::k_frame_obj_masks, dim3(segs, rows), dim3(256), 0, (hipStream_t)stream, *a);
  return (int)hipGetLastError();
}
