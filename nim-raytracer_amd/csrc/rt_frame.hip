// rt_frame.hip — per-call device builders of the camera-dependent data of
// the float32 kernels (rt_frame.h). float64 geometry (rt_bins_geom.h), built
// with -ffp-contract=off like the host builders the tests compare against.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>

#include "rt_bins.h"
#include "rt_frame.h"

namespace rtmi {
namespace {

__device__ __forceinline__ unsigned lane_rank(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Per face: its pixel rectangle and projected vertices (kept for the fill
// pass), and one count per pixel of the launch's rows that the face's grown
// projection meets (rt_bins.cpp build_pixel_bins, the same bounds).
__global__ __launch_bounds__(256) void k_frame_bins_count(const BinsLaunch a) {
  const int i = (int)(blockIdx.x * 256u + threadIdx.x);
  if (i == 0) {
#pragma unroll
    for (int k = 0; k < FC_WORDS; ++k) a.ctr[k] = 0;
  }
  if (i >= a.nf) return;
  double v[3][3];
#pragma unroll
  for (int p = 0; p < 3; ++p)
#pragma unroll
    for (int k = 0; k < 3; ++k) v[p][k] = a.tris[i].v[p][k];
  double q[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  int r[4];
  // (a vertex at or behind the camera plane: the host checked the mesh box
  // against the camera plane before launching, so this never fails)
  if (!bg::face_pixel_rect(a.cam, v, q, r)) r[0] = -1;
  reinterpret_cast<int4*>(a.rect)[i] = make_int4(r[0], r[1], r[2], r[3]);
#pragma unroll
  for (int k = 0; k < 6; ++k) a.proj[6 * (size_t)i + k] = q[k];
  if (r[0] < 0) return;
  const double m = a.cam.margin;
  for (int y = r[2]; y <= r[3]; ++y) {
    if (!frame_has_row(a.rows, y)) continue;
    for (int x = r[0]; x <= r[1]; ++x)
      if (bg::tri_meets_box(q, x - m, y - m, x + 1 + m, y + 1 + m))
        atomicAdd(&a.cnt[(size_t)y * a.cam.width + x], 1);
  }
}

// Per face again: its record offset into each listed pixel's list. The
// slot comes from counting the pixel's count back down, so the counts are
// zero again for the next call (no clearing pass).
__global__ __launch_bounds__(256) void k_frame_bins_fill(const BinsLaunch a) {
  const int i = (int)(blockIdx.x * 256u + threadIdx.x);
  if (i == 0) {  // read-ahead padding after the last list (rt_bins.h kBinPad)
    const int64_t total = a.off[a.scan_lo + a.scan_n - 1];
    for (int k = 0; k < kBinPad; ++k)
      if (total + k < a.cap) a.ent[total + k] = a.pad_rec;
    if (total + kBinPad > a.cap) atomicOr(&a.ctr[FC_OVERFLOW], 1);
  }
  if (i >= a.nf) return;
  const int4 r = reinterpret_cast<const int4*>(a.rect)[i];
  if (r.x < 0) return;
  double q[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) q[k] = a.proj[6 * (size_t)i + k];
  const int32_t rec = a.tris[i].rec;
  const double m = a.cam.margin;
  for (int y = r.z; y <= r.w; ++y) {
    if (!frame_has_row(a.rows, y)) continue;
    for (int x = r.x; x <= r.y; ++x)
      if (bg::tri_meets_box(q, x - m, y - m, x + 1 + m, y + 1 + m)) {
        const size_t pix = (size_t)y * a.cam.width + x;
        const int64_t slot = (int64_t)a.off[pix] + atomicSub(&a.cnt[pix], 1) - 1;
        if (slot < a.cap) a.ent[slot] = rec;
        else atomicOr(&a.ctr[FC_OVERFLOW], 1);
      }
  }
}

// Per pixel group of the launch (one pixel each): the pixel record — list
// length, and for an empty list the shadow skip bits (rt_bins_geom.h
// pixel_skip_bits) — and, for a two-class launch, the group appended to the
// lean list (empty list, every light skipped) or the general list: a wave
// ballot per list, the lane's slot its mbcnt prefix, one atomic per wave. The
// last block to finish pads the lean list with -1 to whole 64-entry runs.
__global__ __launch_bounds__(256) void k_frame_records(const RecordsLaunch a) {
  __shared__ bool last;
  __shared__ bg::SkipGrid sg[8];
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
  const int gi = (int)(blockIdx.x * 256u + threadIdx.x);
  bool valid = gi < a.ngroups;
  const int g = valid ? (a.order ? a.order[gi] : gi) : 0;
  const int k = g / a.ncols, j = g - k * a.ncols;
  const int x = j * a.step;
  int y;
  if (a.mode == 0) {
    y = a.y0 + k * a.step;
  } else {
    y = (k / a.band_h * a.world + a.rank) * a.band_h + k % a.band_h;
    valid = valid && y < a.height;
  }
  bool drawn = valid;
  if (a.step < a.max_step) {  // progressive refinement skip (renderer.nim:175-178)
    const int mask = a.step * 2 - 1;
    if ((x & mask) == 0 && (y & mask) == 0) drawn = false;
  }
  uint32_t info = 0u;
  if (valid) {
    const size_t pix = (size_t)y * a.width + x;
    const int32_t n = a.off[pix + 1] - a.off[pix];
    info = n < (int32_t)kPixCount ? (uint32_t)n : kPixCount;
    if (n == 0 && a.have != 0u) info |= bg::pixel_skip_bits(a.cam, a.planes, a.nplanes, sg, a.nl, a.have, x, y) << 24;
    a.info[pix] = info;
  }
  if (!a.split) return;
  const bool lean = drawn && (info & kPixCount) == 0u && ((info >> 24) & a.full) == a.full;
  const bool heavy = drawn && !lean;
  const unsigned long long ml = __ballot(lean), mh = __ballot(heavy);
  const int lane = (int)(threadIdx.x & 63u);
  int bl = 0, bh = 0;
  if (lane == 0) {
    if (ml) bl = atomicAdd(&a.ctr[FC_LEAN], (int)__popcll(ml));
    if (mh) bh = atomicAdd(&a.ctr[FC_HEAVY], (int)__popcll(mh));
  }
  bl = __shfl(bl, 0);
  bh = __shfl(bh, 0);
  if (lean) a.lean[bl + (int)lane_rank(ml)] = g;
  if (heavy) a.heavy[bh + (int)lane_rank(mh)] = g;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&a.ctr[FC_DONE], 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  const int n = atomicAdd(&a.ctr[FC_LEAN], 0);
  const int end = n == 0 ? 64 : (n + 63) / 64 * 64;
  for (int e = n + (int)threadIdx.x; e < end; e += 256) a.lean[e] = -1;
}

// Object masks (rt_bins.cpp build_object_pixel_masks): each block projects
// every object's world box once into LDS, then its threads walk the launch's
// pixels.
__global__ __launch_bounds__(256) void k_frame_obj_masks(const ObjMaskLaunch a) {
  __shared__ int rect[64][4];
  __shared__ int alw[64];
  const int t = (int)threadIdx.x;
  if (t < a.nobj) {
    const DevObjBox& b = a.objs[t];
    bool proj = !b.always;
    double xmin = INFINITY, xmax = -INFINITY, ymin = INFINITY, ymax = -INFINITY;
    for (int c = 0; proj && c < 8; ++c) {
      const double pw[3] = {(c & 1) ? b.hi[0] : b.lo[0], (c & 2) ? b.hi[1] : b.lo[1], (c & 4) ? b.hi[2] : b.lo[2]};
      double pc[3];
      bg::xform_point(a.w2c, pw, pc);
      if (!(pc[2] < -1e-9 * (1.0 + fabs(pc[0]) + fabs(pc[1])))) {
        proj = false;  // a corner at or behind the camera plane: no bounded projection
        break;
      }
      const double px = 0.5 * a.width + (pc[0] / -pc[2]) / a.cam_a;
      const double py = 0.5 * a.height - (pc[1] / -pc[2]) / a.cam_c;
      xmin = bg::dmin(xmin, px);
      xmax = bg::dmax(xmax, px);
      ymin = bg::dmin(ymin, py);
      ymax = bg::dmax(ymax, py);
    }
    alw[t] = proj ? 0 : 1;
    rect[t][0] = rect[t][1] = rect[t][2] = rect[t][3] = -1;
    const double m = a.margin;
    if (proj && xmax + m >= 0.0 && ymax + m >= 0.0 && xmin - m < a.width && ymin - m < a.height) {
      rect[t][0] = (int)bg::dmax(0.0, floor(xmin - m));
      rect[t][1] = (int)bg::dmin((double)a.width - 1, floor(xmax + m));
      rect[t][2] = (int)bg::dmax(0.0, floor(ymin - m));
      rect[t][3] = (int)bg::dmin((double)a.height - 1, floor(ymax + m));
    }
  }
  __syncthreads();
  unsigned long long always = 0ull;
  for (int i = 0; i < a.nobj; ++i) always |= alw[i] ? 1ull << i : 0ull;
  const long long total = (long long)a.rows.nrows * a.width;
  for (long long idx = (long long)blockIdx.x * 256 + t; idx < total; idx += (long long)gridDim.x * 256) {
    const int k = (int)(idx / a.width), x = (int)(idx - (long long)k * a.width);
    const int y = frame_row(a.rows, k);
    if (y < 0) continue;
    unsigned long long mk = always;
    for (int i = 0; i < a.nobj; ++i)
      if (rect[i][0] >= 0 && x >= rect[i][0] && x <= rect[i][1] && y >= rect[i][2] && y <= rect[i][3]) mk |= 1ull << i;
    a.masks[(size_t)y * a.width + x] = mk;
  }
}

}  // namespace
}  // namespace rtmi

extern "C" int rtmi_frame_bins_count(const rtmi::BinsLaunch* a, void* scan_tmp, size_t* scan_tmp_bytes,
                                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!scan_tmp) {
    return (int)rocprim::exclusive_scan(nullptr, *scan_tmp_bytes, a->cnt, a->off, 0, (size_t)a->scan_n,
                                        rocprim::plus<int32_t>(), st);
  }
  const int blocks = (a->nf + 255) / 256;
  hipLaunchKernelGGL(rtmi::k_frame_bins_count, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, *a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)rocprim::exclusive_scan(scan_tmp, *scan_tmp_bytes, a->cnt + a->scan_lo, a->off + a->scan_lo, 0,
                                      (size_t)a->scan_n, rocprim::plus<int32_t>(), st);
}

extern "C" int rtmi_frame_bins_fill(const rtmi::BinsLaunch* a, void* stream) {
  const int blocks = (a->nf + 255) / 256;
  hipLaunchKernelGGL(rtmi::k_frame_bins_fill, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, *a);
  return (int)hipGetLastError();
}

extern "C" int rtmi_frame_records(const rtmi::RecordsLaunch* a, void* stream) {
  const int blocks = (a->ngroups + 255) / 256;
  hipLaunchKernelGGL(rtmi::k_frame_records, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, *a);
  return (int)hipGetLastError();
}

extern "C" int rtmi_frame_obj_masks(const rtmi::ObjMaskLaunch* a, void* stream) {
  if (a->nobj > 64) return (int)hipErrorInvalidValue;
  const long long total = (long long)a->rows.nrows * a->width;
  const long long blocks = std::min<long long>(2048, (total + 255) / 256);
  hipLaunchKernelGGL(rtmi::k_frame_obj_masks, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(256), 0,
                     (hipStream_t)stream, *a);
  return (int)hipGetLastError();
}
