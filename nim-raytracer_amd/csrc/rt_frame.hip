// rt_frame.hip — per-call device builders of the camera-dependent data of
// the float32 kernels (rt_frame.h). float64 geometry (rt_bins_geom.h), built
// with -ffp-contract=off like the host builders the tests compare against.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rt_bins.h"
#include "rt_frame.h"

namespace rtmi {
namespace {

__device__ __forceinline__ unsigned lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
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
// (one block, one wave per launch row). The shadow skips are tested once per
// cell of kSkipW columns of a tile for the rectangle its pixels span
// (rt_bins_geom.h rect_skip_bits: the cell's grown corner rays bound every
// pixel's, so a cell whose bits cover every light gives each of its pixels
// exactly the bits the per-pixel test would); the pixels of other cells take
// the per-pixel test (a long float64 chain: a whole 64-column tile's test
// failed wherever any of its pixels neared the object's shadow or a
// horizon, and its 256 pixels then each ran the chain).
constexpr int kTileW = 64, kTileH = 4, kSkipW = 16, kSkipCells = kTileW / kSkipW;

// One thread per skip cell: its bits (1 = every light skipped).
__device__ __forceinline__ void tiles_body(const RecordsLaunch& a, const int t, int tiles_x, int ntiles,
                                           uint8_t* tile_bits, const bg::SkipGrid* sg) {
  if (t >= ntiles * kSkipCells) return;
  const int tile = t / kSkipCells, c = t % kSkipCells;
  const int tj = tile % tiles_x, tk = tile / tiles_x;
  const int j0 = tj * kTileW + c * kSkipW;
  if (j0 >= a.ncols) {
    tile_bits[t] = 0;
    return;
  }
  const int j1 = min(j0 + kSkipW, a.ncols) - 1;
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

// ---- k_frame_build1: faces (slot appends, huge list) + tiles -------------

// kFacesPerBlock faces per block, one per thread of its first wave for the
// projection (each face's rectangle, cull and row tests run once), then the
// block's (face, rectangle pixel) pairs are dealt out evenly over all its
// threads (a face covers a few pixels, a few cover dozens: a face per thread
// for the pixel loop left most lanes idle behind the largest face of their
// wave; 256 faces per block left one wave per SIMD for the pixel loop).
constexpr int kFacesPerBlock = 64;

// Per face: its pixel rectangle (rt_bins.cpp build_pixel_bins, the same
// bounds); every launch pixel its grown projection meets gets the face's
// record offset in its next slot (the pixel's counter hands slots out). A
// face of more than kBigFace pixels goes onto the huge list instead. The
// projection comes before the cull: a face with no launch row in its
// rectangle (a band launch of a multi-GPU frame) is dropped without the
// cull's square roots — it lists no launch pixel either way.
__device__ __forceinline__ void faces_block(const FrameLaunch& a) {
  __shared__ double s_pr[kFacesPerBlock][6];
  __shared__ int s_pre[kFacesPerBlock + 1], s_x0[kFacesPerBlock], s_y0[kFacesPerBlock], s_rw[kFacesPerBlock];
  __shared__ int32_t s_rec[kFacesPerBlock];
  const int tid = (int)threadIdx.x, i = (int)blockIdx.x * kFacesPerBlock + tid;
  int area = 0;
  if (tid < kFacesPerBlock && i < a.nf) {
    double v[3][3];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int k = 0; k < 3; ++k) v[p][k] = a.tris[i].v[p][k];
    double pr[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int r[4];
    // (a vertex at or behind the camera plane: the host checked the mesh box
    // against the camera plane before launching, so this never fails)
    if (bg::face_project_rect(a.cam, v, pr, r) && r[0] >= 0 && frame_meets_rows(a.rows, r[2], r[3]) &&
        !bg::face_is_back(a.cam, v)) {
      const int rw = r[1] - r[0] + 1;
      area = rw * (r[3] - r[2] + 1);
      const int32_t rec = a.tris[i].rec;
      if (area > kBigFace) {
        const int slot = atomicAdd(&a.r.ctr[FC_HUGE0 + a.parity], 1);
        if (slot < kHugeCap) {
          HugeFace& h = a.huge[slot];
          h.rec = rec;
#pragma unroll
          for (int k = 0; k < 4; ++k) h.r[k] = r[k];
#pragma unroll
          for (int k = 0; k < 6; ++k) h.pr[k] = pr[k];
          area = 0;
        }
        // the list is full: the block's threads walk this face (slow, exact)
      }
      if (area > 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) s_pr[tid][k] = pr[k];
        s_x0[tid] = r[0];
        s_y0[tid] = r[2];
        s_rw[tid] = rw;
        s_rec[tid] = rec;
      }
    }
  }
  // exclusive prefix of the areas (Hillis-Steele over the block)
  if (tid < kFacesPerBlock) s_pre[tid + 1] = area;
  if (tid == 0) s_pre[0] = 0;
  __syncthreads();
  for (int d = 1; d < kFacesPerBlock; d <<= 1) {
    const int add = tid < kFacesPerBlock && tid + 1 > d ? s_pre[tid + 1 - d] : 0;
    __syncthreads();
    if (tid < kFacesPerBlock) s_pre[tid + 1] += add;
    __syncthreads();
  }
  const int total = s_pre[kFacesPerBlock];
  const double m = a.cam.margin;
  for (int idx = tid; idx < total; idx += (int)blockDim.x) {
    int lo = 0, hi = kFacesPerBlock - 1;  // the last face whose range starts at or before idx
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= idx) lo = mid;
      else hi = mid - 1;
    }
    const int local = idx - s_pre[lo], rw = s_rw[lo];
    const int y = s_y0[lo] + local / rw, x = s_x0[lo] + local % rw;
    if (!frame_has_row(a.rows, y) || !frame_has_col(a.rows, x)) continue;
    double pr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) pr[k] = s_pr[lo][k];
    if (bg::tri_meets_box(pr, x - m, y - m, x + 1 + m, y + 1 + m)) {
      const size_t pix = (size_t)y * a.cam.width + x;
      const int s = atomicAdd(&a.cnt[pix], 1);
      if (s < (1 << a.slot_lg)) a.slots[(pix << a.slot_lg) + s] = s_rec[lo];
    }
  }
}

// blocks [0, face_blocks): faces; the rest: one tile per thread (its skip
// bits). Block 0 also clears
// the next call's huge-list counter and the render kernels' queue heads +
// Stats words (one launch fewer than a memset).
__global__ __launch_bounds__(256) void k_frame_build1(const FrameLaunch a, int face_blocks) {
  __shared__ bg::SkipGrid sg[8];
  if (blockIdx.x == 0) {
    for (int k = (int)threadIdx.x; k < a.nzero; k += 256) a.zero[k] = 0u;
    if (threadIdx.x == 0) a.r.ctr[FC_HUGE0 + (a.parity ^ 1)] = 0;
  }
  if ((int)blockIdx.x < face_blocks) {
    if (a.diag != 2) faces_block(a);
    return;
  }
  if (a.diag == 3) return;
  const int t = (int)((blockIdx.x - (unsigned)face_blocks) * 256u + threadIdx.x);
  if (a.r.records && a.r.have != 0u) {
    load_skip_grids(a.r, sg);
    tiles_body(a.r, t, a.tiles_x, a.ntiles, a.tile_bits, sg);
  }
}

// ---- k_frame_build2: huge faces, records, counters, lean / general lists --

// Tiles per block of k_frame_lists, by launch size: every block sums the
// counts of all earlier tiles (~ntiles^2 / (2 chunk) loads per launch, L2
// hits) and then writes its chunk's pixels, so small launches want small
// chunks (more blocks, each chunk's records and writes short) and large ones
// large chunks (the summing grows with the square of the tiles). Measured
// (C3, interleaved A/Bs, `profiles/r5/ab/r5aa_*`, `r5ab_*`): rank 0 of 8
// (1,012 tiles) back to back 0.142 ms with 16 tiles per block, 0.137 with 4,
// 0.136 with 2 or 1; the whole 1080p frame (8,100 tiles) 0.823 ms with 16,
// 0.816 with 4. 4K frames (32,400 tiles) keep 16. RTMI_LISTS_CHUNK=1|2|4|16
// forces one (diagnostic builds).
__host__ __forceinline__ int lists_chunk(int ntiles) { return ntiles <= 2048 ? 2 : ntiles <= 8192 ? 4 : 16; }

// The class of a launch pixel: 1 lean (empty list, every light skipped), 2
// general, 0 not drawn (a progressive pass skips it).
__device__ __forceinline__ int pixel_class(const RecordsLaunch& a, const LaunchPix& p, uint32_t info) {
  if (!p.drawn) return 0;
  return (info & kPixCount) == 0u && ((info >> 24) & a.full) == a.full ? 1 : 2;
}

// One tile's pixels (one per thread): their huge faces, records, counters.
// Returns the thread's pixel class (0 none, 1 lean, 2 general).
__device__ __forceinline__ int build2_tile(const FrameLaunch& a, int t, int nhuge, const bg::SkipGrid* sg,
                                           int32_t* hl, int* hn) {
  const RecordsLaunch& r = a.r;
  const int bx = t % a.tiles_x, by = t / a.tiles_x;
  const int j = bx * kTileW + (int)(threadIdx.x & 63u), k = by * kTileH + (int)(threadIdx.x >> 6);
  const LaunchPix p = launch_pixel(r, j, k);
  size_t pix = 0;
  int32_t n0 = 0, n = 0;
  if (p.valid) {
    pix = (size_t)p.y * r.width + p.x;
    n0 = a.cnt[pix];
    n = n0;
  }
  if (nhuge > 0) {  // the tile's share of the huge list, in rounds of 256 faces
    const int x0 = bx * kTileW * r.step, x1 = (min(bx * kTileW + kTileW, r.ncols) - 1) * r.step;
    int ylo = 0x7fffffff, yhi = -1;
    for (int kk = by * kTileH; kk < min(by * kTileH + kTileH, r.nrows); ++kk) {
      const LaunchPix q = launch_pixel(r, bx * kTileW, kk);
      if (!q.valid) continue;
      ylo = min(ylo, q.y);
      yhi = max(yhi, q.y);
    }
    const double m = a.cam.margin;
    for (int h0 = 0; h0 < nhuge; h0 += 256) {
      if (threadIdx.x == 0) *hn = 0;
      __syncthreads();
      const int h = h0 + (int)threadIdx.x;
      if (h < nhuge && yhi >= 0) {
        const HugeFace& f = a.huge[h];
        if (f.r[0] <= x1 && f.r[1] >= x0 && f.r[2] <= yhi && f.r[3] >= ylo) hl[atomicAdd(hn, 1)] = h;
      }
      __syncthreads();
      const int cnt = *hn;
      for (int e = 0; e < cnt; ++e) {
        const HugeFace& f = a.huge[hl[e]];
        if (p.valid && p.x >= f.r[0] && p.x <= f.r[1] && p.y >= f.r[2] && p.y <= f.r[3] &&
            bg::tri_meets_box(f.pr, p.x - m, p.y - m, p.x + 1 + m, p.y + 1 + m)) {
          if (n < (1 << a.slot_lg)) a.slots[(pix << a.slot_lg) + n] = f.rec;
          ++n;
        }
      }
      __syncthreads();
    }
  }
  if (!p.valid) return 0;
  if (n0 != 0) a.cnt[pix] = 0;  // zero for the next call
  uint32_t info = n < (int32_t)kPixCount ? (uint32_t)n : kPixCount;
  if (n == 0 && r.records && r.have != 0u) {
    const bool tile = a.tile_bits[t * kSkipCells + (int)(threadIdx.x & 63u) / kSkipW] != 0;
    const unsigned bits = tile || a.diag == 1 ? r.have : bg::pixel_skip_bits(r.cam, r.planes, r.nplanes, sg, r.nl, r.have, p.x, p.y);
    info |= bits << 24;
  }
  r.info[pix] = info;
  return r.split ? pixel_class(r, p, info) : 0;
}

// k_frame_build2: one tile per block, all of them at once (a pixel's own
// skip test is a long float64 chain: tiles taken in turn by a persistent
// grid serialised those chains, 90 us per C3 call).
// With split, the tile's lean / general pixel counts (lean << 32 | general)
// go to tile_cls for k_frame_lists.
template <int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void k_frame_build2(const FrameLaunch a) {
  __shared__ bg::SkipGrid sg[8];
  __shared__ int32_t hl[256];
  __shared__ int hn;
  __shared__ unsigned long long wsum[4];
  const RecordsLaunch& r = a.r;
  if (r.records && r.have != 0u) load_skip_grids(r, sg);
  const int nhuge = min(r.ctr[FC_HUGE0 + a.parity], kHugeCap);
  const int cl = build2_tile(a, (int)blockIdx.x, nhuge, sg, hl, &hn);
  if (!r.split) return;
  const unsigned long long ml = __ballot(cl == 1), mh = __ballot(cl == 2);
  if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  __syncthreads();
  if (threadIdx.x == 0) a.tile_cls[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// k_frame_lists: the lean / general lists (two-class launches) in tile
// order. One block per chunk of kChunkTiles tiles (above): its offsets are the sum of
// every earlier tile's counts (k_frame_build2's tile_cls), summed by the
// block itself — each block re-reads the earlier counts (8,100 x 8 B at
// 1080p, L2-resident) instead of waiting on other blocks: no inter-block
// hand-off, no spin, no scan launch. Then each thread loads its pixel's
// record in each of the chunk's tiles (all loads in flight), and the chunk's
// pixels are written at their offsets (wave ballots, mbcnt ranks).
template <int kChunkTiles>
__global__ __launch_bounds__(256) void k_frame_lists(const FrameLaunch a) {
  __shared__ unsigned long long wpart[4];
  __shared__ unsigned long long wsum[kChunkTiles][4];
  const RecordsLaunch& r = a.r;
  const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int t0 = (int)blockIdx.x * kChunkTiles;
  uint32_t inf[kChunkTiles];
  LaunchPix px[kChunkTiles];
#pragma unroll
  for (int i = 0; i < kChunkTiles; ++i) {
    const int t = t0 + i;
    const int bx = t % a.tiles_x, by = t / a.tiles_x;
    px[i] = launch_pixel(r, bx * kTileW + lane, by * kTileH + w);
    px[i].valid = px[i].valid && t < a.ntiles;
    inf[i] = px[i].valid ? r.info[(size_t)px[i].y * r.width + px[i].x] : 0u;
  }
  // every earlier tile's counts (lean << 32 | general)
  // (kSumUnroll independent loads in flight per thread: a load-add chain of
  // t0 / 256 steps was most of the kernel's time)
  constexpr int kSumUnroll = 8;
  unsigned long long v = 0ull;
  for (int t = tid; t < t0; t += 256 * kSumUnroll) {
    unsigned long long part[kSumUnroll];
#pragma unroll
    for (int u = 0; u < kSumUnroll; ++u) part[u] = t + u * 256 < t0 ? a.tile_cls[t + u * 256] : 0ull;
#pragma unroll
    for (int u = 0; u < kSumUnroll; ++u) v += part[u];
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, off);
    const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(v >> 32), off);
    v += ((unsigned long long)hi << 32) | lo;
  }
  if (lane == 0) wpart[w] = v;
  int cls[kChunkTiles];
#pragma unroll
  for (int i = 0; i < kChunkTiles; ++i) {
    cls[i] = px[i].valid ? pixel_class(r, px[i], inf[i]) : 0;
    const unsigned long long ml = __ballot(cls[i] == 1), mh = __ballot(cls[i] == 2);
    if (lane == 0) wsum[i][w] = ((unsigned long long)__popcll(ml) << 32) | __popcll(mh);
  }
  __syncthreads();
  unsigned long long base = wpart[0] + wpart[1] + wpart[2] + wpart[3];
#pragma unroll
  for (int i = 0; i < kChunkTiles; ++i) {
    const int t = t0 + i;
    const unsigned long long ml = __ballot(cls[i] == 1), mh = __ballot(cls[i] == 2);
    unsigned long long b = base;
    for (int q = 0; q < w; ++q) b += wsum[i][q];
    const int bx = t % a.tiles_x, by = t / a.tiles_x;
    const int g = (by * kTileH + w) * r.ncols + bx * kTileW + lane;
    if (cls[i] == 1) r.lean[(int)(b >> 32) + (int)lane_rank(ml)] = g;
    if (cls[i] == 2) r.heavy[(int)(b & 0xffffffffull) + (int)lane_rank(mh)] = g;
    base += wsum[i][0] + wsum[i][1] + wsum[i][2] + wsum[i][3];
  }
  if ((int)blockIdx.x == (int)gridDim.x - 1) {  // the last chunk: the list lengths, the lean list's -1 padding
    const int nl = (int)(base >> 32), nh = (int)(base & 0xffffffffull);
    if (tid == 0) {
      r.ctr[FC_LEAN] = nl;
      r.ctr[FC_HEAVY] = nh;
    }
    const int end = nl == 0 ? 64 : (nl + 63) / 64 * 64;
    for (int e = nl + tid; e < end; e += 256) r.lean[e] = -1;
  }
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

}  // namespace
}  // namespace rtmi

extern "C" int rtmi_frame_build(const rtmi::FrameLaunch* a, void* stream) {
  using namespace rtmi;
  static_assert(sizeof(FrameLaunch) <= 4096, "kernel argument size");
  hipStream_t st = (hipStream_t)stream;
  const int face_blocks = std::max(1, (a->nf + kFacesPerBlock - 1) / kFacesPerBlock);
  const int tile_blocks = (a->ntiles * kSkipCells + 255) / 256;
  hipLaunchKernelGGL(k_frame_build1, dim3(face_blocks + tile_blocks), dim3(256), 0, st, *a, face_blocks);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || a->ntiles <= 0) return (int)e;
  static const int b2w = rtmi::diag_env("RTMI_B2_WAVES") ? std::atoi(rtmi::diag_env("RTMI_B2_WAVES")) : 4;  // diagnostic
  if (b2w == 8)
    hipLaunchKernelGGL(k_frame_build2<8>, dim3((unsigned)a->ntiles), dim3(256), 0, st, *a);
  else
    hipLaunchKernelGGL(k_frame_build2<4>, dim3((unsigned)a->ntiles), dim3(256), 0, st, *a);
  if ((e = hipGetLastError()) != hipSuccess || !a->r.split) return (int)e;
  static const int chunk_env = rtmi::diag_env("RTMI_LISTS_CHUNK") ? std::atoi(rtmi::diag_env("RTMI_LISTS_CHUNK")) : 0;
  const int chunk = chunk_env == 1 || chunk_env == 2 || chunk_env == 4 || chunk_env == 16 ? chunk_env
                                                                                          : lists_chunk(a->ntiles);
  const int nchunks = (a->ntiles + chunk - 1) / chunk;
  if (chunk == 1)
    hipLaunchKernelGGL(k_frame_lists<1>, dim3((unsigned)nchunks), dim3(256), 0, st, *a);
  else if (chunk == 2)
    hipLaunchKernelGGL(k_frame_lists<2>, dim3((unsigned)nchunks), dim3(256), 0, st, *a);
  else if (chunk == 4)
    hipLaunchKernelGGL(k_frame_lists<4>, dim3((unsigned)nchunks), dim3(256), 0, st, *a);
  else
    hipLaunchKernelGGL(k_frame_lists<16>, dim3((unsigned)nchunks), dim3(256), 0, st, *a);
  return (int)hipGetLastError();
}

extern "C" long long rtmi_frame_skip_cells(int ncols, int nrows) {
  using namespace rtmi;
  return (long long)((ncols + kTileW - 1) / kTileW) * ((nrows + kTileH - 1) / kTileH) * kSkipCells;
}

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
