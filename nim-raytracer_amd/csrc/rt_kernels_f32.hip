// rt_kernels_f32.hip — float (performance mode) instantiation of the render
// kernel, plus the precision-independent helper kernels (stats reduction,
// multi-GPU band un-interleave). Built with FMA contraction on.
#include <algorithm>
#include <cstdlib>

#include "rt_fast.h"

namespace rtmi {

// Sum per-wave partial counters into acc (acc accumulates across launches
// until the host clears it). Each block folds kWavesPerBlock waves in
// registers, then one atomic per counter per block.
constexpr int kWavesPerBlock = 256;
__global__ __launch_bounds__(256) void k_reduce_stats(const unsigned long long* __restrict__ partials,
                                                      int num_waves, unsigned long long* __restrict__ acc) {
  __shared__ unsigned long long red[kStatSlots][256];
  const int w = blockIdx.x * kWavesPerBlock + threadIdx.x;
#pragma unroll
  for (int k = 0; k < kStatSlots; ++k) red[k][threadIdx.x] = w < num_waves ? partials[(size_t)w * kStatSlots + k] : 0ull;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
#pragma unroll
      for (int k = 0; k < kStatSlots; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + off];
    }
    __syncthreads();
  }
  if ((int)threadIdx.x < kStatSlots) atomicAdd(&acc[threadIdx.x], red[threadIdx.x][0]);
}

// Rank-0 epilogue of the framebuffer gather: gathered = world compact band
// buffers back to back, each band_rows rows; image row y lives in band
// b = y / band_h owned by rank b % world as local band b / world.
__global__ __launch_bounds__(256) void k_unshard(const float4* __restrict__ gathered, float4* __restrict__ fb,
                                                 int row_f4, int height, int band_h, int world, int band_rows) {
  const int y = blockIdx.x;
  if (y >= height) return;
  const int b = y / band_h, r = y % band_h;
  const int owner = b % world, lb = b / world;
  const size_t src_row = (size_t)owner * band_rows + (size_t)lb * band_h + r;
  const float4* src = gathered + src_row * row_f4;
  float4* dst = fb + (size_t)y * row_f4;
  for (int i = threadIdx.x; i < row_f4; i += blockDim.x) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_unshard_scalar(const float* __restrict__ gathered, float* __restrict__ fb,
                                                        int row_f, int height, int band_h, int world, int band_rows) {
  const int y = blockIdx.x;
  if (y >= height) return;
  const int b = y / band_h, r = y % band_h;
  const int owner = b % world, lb = b / world;
  const size_t src_row = (size_t)owner * band_rows + (size_t)lb * band_h + r;
  for (int i = threadIdx.x; i < row_f; i += blockDim.x) fb[(size_t)y * row_f + i] = gathered[src_row * row_f + i];
}

// After k_render_wave: the framebuffer's pixels += their queued rays'
// radiance (p->sec, 32.32 fixed point), scaled like the pixel's level-0 sum
// (calcPixel's 1 / len, renderer.nim:159).
__global__ __launch_bounds__(256) void k_sec_add(float* __restrict__ fb, const long long* __restrict__ sec, size_t n,
                                                 float scale) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const long long v = sec[i];
    if (v != 0) fb[i] += (float)((double)v * 0x1p-32) * scale;
  }
}

// the instrumented (RT_FLAG_COUNT_TRAVERSAL) kernel: all features
template __global__ void fast::k_render_fast<true, fast::F_ALL>(const FastParams);
// lean pixels of one-plane scenes (rtmi.cpp lean1_ok), one or two lights
template __global__ void fast::k_render_lean1<1>(const FastParams);
template __global__ void fast::k_render_lean1<2>(const FastParams);
template __global__ void fast::k_render_lean1q<1, 4>(const FastParams);
template __global__ void fast::k_render_lean1q<2, 4>(const FastParams);
template __global__ void fast::k_render_lean1q<1, 16>(const FastParams);
template __global__ void fast::k_render_lean1q<2, 16>(const FastParams);
// general pixels of the same scenes
template __global__ void fast::k_render_gen1<1>(const FastParams);
template __global__ void fast::k_render_gen1<2>(const FastParams);
// both classes of a one-plane launch in one kernel
template __global__ void fast::k_render_mix1<1, 4>(const FastParams);
template __global__ void fast::k_render_mix1<2, 4>(const FastParams);
template __global__ void fast::k_render_mix1<1, 16>(const FastParams);
template __global__ void fast::k_render_mix1<2, 16>(const FastParams);

}  // namespace rtmi

// feature-subset specialisations: rt_kernels_f32_part.hip, 16 objects
#define RTMI_PART_DECL(k)                                                                             \
  extern "C" int rtmi_launch_render_f32_part##k(unsigned, const rtmi::FastParams*, int, size_t, void*); \
  extern "C" int rtmi_render_f32_part_blocks_per_cu##k(unsigned, size_t);                              \
  extern "C" int rtmi_launch_lean_f32_part##k(unsigned, const rtmi::FastParams*, int, size_t, void*);   \
  extern "C" int rtmi_lean_f32_part_blocks_per_cu##k(unsigned, size_t);                              \
  extern "C" int rtmi_launch_gen_f32_part##k(unsigned, const rtmi::FastParams*, int, size_t, void*);    \
  extern "C" int rtmi_gen_f32_part_blocks_per_cu##k(unsigned, size_t);                              \
  extern "C" int rtmi_launch_wave_f32_part##k(unsigned, const rtmi::FastParams*, int, size_t, void*);   \
  extern "C" int rtmi_wave_f32_part_blocks_per_cu##k(unsigned, size_t);
RTMI_PART_DECL(0) RTMI_PART_DECL(1) RTMI_PART_DECL(2) RTMI_PART_DECL(3)
RTMI_PART_DECL(4) RTMI_PART_DECL(5) RTMI_PART_DECL(6) RTMI_PART_DECL(7)
RTMI_PART_DECL(8) RTMI_PART_DECL(9) RTMI_PART_DECL(10) RTMI_PART_DECL(11)
RTMI_PART_DECL(12) RTMI_PART_DECL(13) RTMI_PART_DECL(14) RTMI_PART_DECL(15)

namespace {
#define RTMI_L(k) rtmi_launch_render_f32_part##k
#define RTMI_O(k) rtmi_render_f32_part_blocks_per_cu##k
int (*const kLaunch[16])(unsigned, const rtmi::FastParams*, int, size_t, void*) = {
    RTMI_L(0), RTMI_L(1), RTMI_L(2),  RTMI_L(3),  RTMI_L(4),  RTMI_L(5),  RTMI_L(6),  RTMI_L(7),
    RTMI_L(8), RTMI_L(9), RTMI_L(10), RTMI_L(11), RTMI_L(12), RTMI_L(13), RTMI_L(14), RTMI_L(15)};
int (*const kOccupancy[16])(unsigned, size_t) = {
    RTMI_O(0), RTMI_O(1), RTMI_O(2),  RTMI_O(3),  RTMI_O(4),  RTMI_O(5),  RTMI_O(6),  RTMI_O(7),
    RTMI_O(8), RTMI_O(9), RTMI_O(10), RTMI_O(11), RTMI_O(12), RTMI_O(13), RTMI_O(14), RTMI_O(15)};
#define RTMI_LL(k) rtmi_launch_lean_f32_part##k
#define RTMI_LO(k) rtmi_lean_f32_part_blocks_per_cu##k
int (*const kLaunchLean[16])(unsigned, const rtmi::FastParams*, int, size_t, void*) = {
    RTMI_LL(0), RTMI_LL(1), RTMI_LL(2),  RTMI_LL(3),  RTMI_LL(4),  RTMI_LL(5),  RTMI_LL(6),  RTMI_LL(7),
    RTMI_LL(8), RTMI_LL(9), RTMI_LL(10), RTMI_LL(11), RTMI_LL(12), RTMI_LL(13), RTMI_LL(14), RTMI_LL(15)};
int (*const kOccupancyLean[16])(unsigned, size_t) = {
    RTMI_LO(0), RTMI_LO(1), RTMI_LO(2),  RTMI_LO(3),  RTMI_LO(4),  RTMI_LO(5),  RTMI_LO(6),  RTMI_LO(7),
    RTMI_LO(8), RTMI_LO(9), RTMI_LO(10), RTMI_LO(11), RTMI_LO(12), RTMI_LO(13), RTMI_LO(14), RTMI_LO(15)};
#define RTMI_LG(k) rtmi_launch_gen_f32_part##k
#define RTMI_GO(k) rtmi_gen_f32_part_blocks_per_cu##k
int (*const kLaunchGen[16])(unsigned, const rtmi::FastParams*, int, size_t, void*) = {
    RTMI_LG(0), RTMI_LG(1), RTMI_LG(2),  RTMI_LG(3),  RTMI_LG(4),  RTMI_LG(5),  RTMI_LG(6),  RTMI_LG(7),
    RTMI_LG(8), RTMI_LG(9), RTMI_LG(10), RTMI_LG(11), RTMI_LG(12), RTMI_LG(13), RTMI_LG(14), RTMI_LG(15)};
int (*const kOccupancyGen[16])(unsigned, size_t) = {
    RTMI_GO(0), RTMI_GO(1), RTMI_GO(2),  RTMI_GO(3),  RTMI_GO(4),  RTMI_GO(5),  RTMI_GO(6),  RTMI_GO(7),
    RTMI_GO(8), RTMI_GO(9), RTMI_GO(10), RTMI_GO(11), RTMI_GO(12), RTMI_GO(13), RTMI_GO(14), RTMI_GO(15)};
#define RTMI_LW(k) rtmi_launch_wave_f32_part##k
#define RTMI_WO(k) rtmi_wave_f32_part_blocks_per_cu##k
int (*const kLaunchWave[16])(unsigned, const rtmi::FastParams*, int, size_t, void*) = {
    RTMI_LW(0), RTMI_LW(1), RTMI_LW(2),  RTMI_LW(3),  RTMI_LW(4),  RTMI_LW(5),  RTMI_LW(6),  RTMI_LW(7),
    RTMI_LW(8), RTMI_LW(9), RTMI_LW(10), RTMI_LW(11), RTMI_LW(12), RTMI_LW(13), RTMI_LW(14), RTMI_LW(15)};
int (*const kOccupancyWave[16])(unsigned, size_t) = {
    RTMI_WO(0), RTMI_WO(1), RTMI_WO(2),  RTMI_WO(3),  RTMI_WO(4),  RTMI_WO(5),  RTMI_WO(6),  RTMI_WO(7),
    RTMI_WO(8), RTMI_WO(9), RTMI_WO(10), RTMI_WO(11), RTMI_WO(12), RTMI_WO(13), RTMI_WO(14), RTMI_WO(15)};
}  // namespace

// The reflection-compacting kernel of a reflective feature subset.
extern "C" int rtmi_launch_wave_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem,
                                    void* stream) {
  return kLaunchWave[(subset >> 3) & 15u](subset & 127u, p, blocks, shmem, stream);
}

// Resident blocks per CU of the reflection-compacting kernel; 0: none for the subset.
extern "C" int rtmi_wave_f32_blocks_per_cu(unsigned subset, size_t shmem) {
  return kOccupancyWave[(subset >> 3) & 15u](subset & 127u, shmem);
}

// fb[i] += sec[i] (32.32 fixed point) * scale where sec[i] != 0, i < n
extern "C" int rtmi_launch_sec_add(float* fb, const long long* sec, size_t n, float scale, int num_cus, void* stream) {
  const size_t want = (n + 255) / 256;
  const unsigned blocks = (unsigned)std::min<size_t>(want > 0 ? want : 1, (size_t)num_cus * 16);
  hipLaunchKernelGGL(rtmi::k_sec_add, dim3(blocks), dim3(256), 0, (hipStream_t)stream, fb, sec, n, scale);
  return (int)hipGetLastError();
}

// The batched general-pixel kernel of a feature subset (two-class launches).
extern "C" int rtmi_launch_gen_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem,
                                   void* stream) {
  return kLaunchGen[(subset >> 3) & 15u](subset & 127u, p, blocks, shmem, stream);
}

// Resident blocks per CU of the batched general kernel; 0: none for the subset.
extern "C" int rtmi_gen_f32_blocks_per_cu(unsigned subset, size_t shmem) {
  return kOccupancyGen[(subset >> 3) & 15u](subset & 127u, shmem);
}

// The lean-pixel kernel of a feature subset (two-class launches).
extern "C" int rtmi_launch_lean_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem,
                                    void* stream) {
  return kLaunchLean[(subset >> 3) & 15u](subset & 127u, p, blocks, shmem, stream);
}

// Resident blocks per CU of the lean-pixel kernel; 0: no lean kernel for the subset.
extern "C" int rtmi_lean_f32_blocks_per_cu(unsigned subset, size_t shmem) {
  return kOccupancyLean[(subset >> 3) & 15u](subset & 127u, shmem);
}

// k_render_lean1q (lp = 4 or 16 lanes per pixel, 64 / lp pixels per work
// item) instead of k_render_lean1 (lp = 64: one pixel per wave, a run of 4
// per item); RTMI_LEAN1Q=0 picks the latter (diagnostic A/B).
extern "C" int rtmi_lean1_quads() {
  static const int q = [] {
    const char* e = rtmi::diag_env("RTMI_LEAN1Q");
    return e ? std::atoi(e) : 1;
  }();
  return q;
}

// The one-plane lean-pixel kernel for nl (1 or 2) distant lights, lp lanes per pixel.
extern "C" int rtmi_launch_lean1_f32(const rtmi::FastParams* p, int nl, int lp, int blocks, void* stream) {
  if (lp == 4 || lp == 16) {
    using namespace rtmi::fast;
#define RTMI_LQ(nl_, lp_) \
  if (nl == nl_ && lp == lp_) { \
    hipLaunchKernelGGL((k_render_lean1q<nl_, lp_>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p); \
    return (int)hipGetLastError(); \
  }
    RTMI_LQ(1, 4) RTMI_LQ(2, 4) RTMI_LQ(1, 16) RTMI_LQ(2, 16)
#undef RTMI_LQ
    return (int)hipErrorInvalidValue;
  }
  if (nl == 1)
    hipLaunchKernelGGL(rtmi::fast::k_render_lean1<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else if (nl == 2)
    hipLaunchKernelGGL(rtmi::fast::k_render_lean1<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// Resident blocks per CU of the one-plane lean kernel actually launched:
// k_render_lean1q<nl, lp> (lp = 4 or 16), k_render_lean1<nl> (lp = 64).
extern "C" int rtmi_lean1_f32_blocks_per_cu(int nl, int lp) {
  using namespace rtmi::fast;
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
#define RTMI_OQ(nl_, lp_) \
  if (nl == nl_ && lp == lp_) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_render_lean1q<nl_, lp_>, 256, 0);
  RTMI_OQ(1, 4) RTMI_OQ(2, 4) RTMI_OQ(1, 16) RTMI_OQ(2, 16)
#undef RTMI_OQ
  if (lp == 64 && (nl == 1 || nl == 2))
    e = nl == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_render_lean1<1>, 256, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_render_lean1<2>, 256, 0);
  return e == hipSuccess && nb > 0 ? nb : 1;
}

// The one-plane batched general-pixel kernel for nl (1 or 2) distant lights.
extern "C" int rtmi_launch_gen1_f32(const rtmi::FastParams* p, int nl, int blocks, void* stream) {
  if (nl == 1)
    hipLaunchKernelGGL(rtmi::fast::k_render_gen1<1>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else if (nl == 2)
    hipLaunchKernelGGL(rtmi::fast::k_render_gen1<2>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// The one-plane merged kernel (general items, then lean items with lp lanes per pixel).
extern "C" int rtmi_launch_mix1_f32(const rtmi::FastParams* p, int nl, int lp, int blocks, void* stream) {
  using namespace rtmi::fast;
#define RTMI_MX(nl_, lp_) \
  if (nl == nl_ && lp == lp_) { \
    hipLaunchKernelGGL((k_render_mix1<nl_, lp_>), dim3(blocks), dim3(256), 0, (hipStream_t)stream, *p); \
    return (int)hipGetLastError(); \
  }
  RTMI_MX(1, 4) RTMI_MX(2, 4) RTMI_MX(1, 16) RTMI_MX(2, 16)
#undef RTMI_MX
  return (int)hipErrorInvalidValue;
}

// Resident blocks per CU of k_render_mix1<nl, lp> (each launched
// instantiation sized from its own register use).
extern "C" int rtmi_mix1_f32_blocks_per_cu(int nl, int lp) {
  using namespace rtmi::fast;
  int nb = 0;
  hipError_t e = hipErrorInvalidValue;
#define RTMI_OM(nl_, lp_) \
  if (nl == nl_ && lp == lp_) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_render_mix1<nl_, lp_>, 256, 0);
  RTMI_OM(1, 4) RTMI_OM(2, 4) RTMI_OM(1, 16) RTMI_OM(2, 16)
#undef RTMI_OM
  return e == hipSuccess && nb > 0 ? nb : 1;
}

extern "C" int rtmi_gen1_f32_blocks_per_cu(int nl) {
  int nb = 0;
  const hipError_t e = nl == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rtmi::fast::k_render_gen1<1>, 256, 0)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rtmi::fast::k_render_gen1<2>, 256, 0);
  return e == hipSuccess && nb > 0 ? nb : 1;
}

extern "C" int rtmi_launch_render_f32(const rtmi::FastParams* p, unsigned subset, int blocks, size_t shmem,
                                      void* stream) {
  if (p->flags & rtmi::RT_DEV_FLAG_COUNT) {
    hipLaunchKernelGGL((rtmi::fast::k_render_fast<true, rtmi::fast::F_ALL>), dim3(blocks), dim3(256), shmem,
                       (hipStream_t)stream, *p);
    return (int)hipGetLastError();
  }
  return kLaunch[(subset >> 3) & 15u](subset & 127u, p, blocks, shmem, stream);
}

// Resident 256-thread blocks per CU of the render kernel (grid sizing for the
// work-queue loop: launch exactly what fits, waves pull pixel groups).
extern "C" int rtmi_render_f32_blocks_per_cu(int count, unsigned subset, size_t shmem) {
  if (count) {
    int nb = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &nb, rtmi::fast::k_render_fast<true, rtmi::fast::F_ALL>, 256, shmem);
    return e == hipSuccess && nb > 0 ? nb : 1;
  }
  return kOccupancy[(subset >> 3) & 15u](subset & 127u, shmem);
}

extern "C" int rtmi_launch_reduce_stats(const unsigned long long* partials, int num_waves,
                                        unsigned long long* acc, void* stream) {
  const int blocks = (num_waves + rtmi::kWavesPerBlock - 1) / rtmi::kWavesPerBlock;
  hipLaunchKernelGGL(rtmi::k_reduce_stats, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, partials, num_waves, acc);
  return (int)hipGetLastError();
}

extern "C" int rtmi_launch_unshard(const float* gathered, float* fb, int width, int height, int band_h,
                                   int world, void* stream) {
  const int nbands = (height + band_h - 1) / band_h;
  const int band_rows = ((nbands + world - 1) / world) * band_h;
  const int row_f = width * 3;
  if ((row_f % 4) == 0 && (((uintptr_t)gathered | (uintptr_t)fb) & 15) == 0) {
    hipLaunchKernelGGL(rtmi::k_unshard, dim3(height), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)gathered, (float4*)fb, row_f / 4, height, band_h, world, band_rows);
  } else {
    hipLaunchKernelGGL(rtmi::k_unshard_scalar, dim3(height), dim3(256), 0, (hipStream_t)stream, gathered, fb,
                       row_f, height, band_h, world, band_rows);
  }
  return (int)hipGetLastError();
}
